#!/bin/bash
# End-of-round GPU call A (round 4): all GPU tests, smoke, the 50M-record end-to-end bench.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/final4a
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -3 $OUT/smoke.log
g++ -O2 -fopenmp -o tools/synthbam tools/synthbam.cpp -lz || exit 1
timeout -k 10 700 python -u tools/e2e_bench.py --synth --records 50000000 --host-decoder --devices 3 > $OUT/e2e_synth50m.json 2> $OUT/e2e_synth50m.err || { tail -30 $OUT/e2e_synth50m.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/e2e_synth50m.json')); print({k: d[k] for k in ('GatherCellMetrics_s', 'GatherCellMetrics_records_per_s', 'device_decode_stages_s', 'csv_gz_s', 'GatherCellMetrics_parts_s', 'parts_and_one_device_csv_identical', 'GatherCellMetrics_host_decoder_s', 'device_and_host_decoder_csv_identical')})"
