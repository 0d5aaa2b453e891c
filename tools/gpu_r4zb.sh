#!/bin/bash
# Config-5 A/B (tools/gpu_r4za.sh), then the 8-bit literal table: device-decoder tests and the 50M-record end-to-end bench.
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_r4za.sh || exit 1
OUT=gpurun_out/r4zb
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gbam.py tests/test_gbam_count.py tests/test_api_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "FAIL|Error" $OUT/pytest.log | head; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
g++ -O2 -fopenmp -o tools/synthbam tools/synthbam.cpp -lz || exit 1
timeout -k 10 700 python -u tools/e2e_bench.py --synth --records 50000000 --host-decoder --devices 3 > $OUT/e2e_synth50m.json 2> $OUT/e2e_synth50m.err || { tail -30 $OUT/e2e_synth50m.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/e2e_synth50m.json')); print({k: d[k] for k in ('GatherCellMetrics_s', 'GatherCellMetrics_records_per_s', 'device_decode_stages_s', 'csv_gz_s', 'GatherCellMetrics_parts_s', 'parts_and_one_device_csv_identical', 'GatherCellMetrics_host_decoder_s', 'device_and_host_decoder_csv_identical')})"
