#!/bin/bash
# Device dictionaries ranked on the GPU + parallel prefault; fused tag pack+keys; level1_plan
# uniform-run fast path: tests, A/B benches, then the 50M-record e2e.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4i
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gbam.py tests/test_gbam_count.py tests/test_api_gpu.py tests/test_gpu_tagsort.py tests/test_gpu_buckets.py tests/test_gpu_parity.py "tests/test_gpu_configs.py::test_config2_cell_rows_100M" "tests/test_gpu_configs.py::test_config2_grouped_gene_rows_100M" "tests/test_gpu_configs.py::test_config5_gpu_sort_is_the_reference_stable_sort_100M" "tests/test_gpu_configs.py::test_config5_cell_metrics_after_gpu_sort_100M" -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "FAIL|Error" $OUT/pytest.log | head; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
bash tools/gpu_variants.sh r4i/var exp/l1_v1.so exp/gh_off.so exp/ht_nodf.so || exit 1
SCT_NO_AUX_STREAM=1 timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/var/noaux.json 2> $OUT/var/noaux.err || { tail -20 $OUT/var/noaux.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/var/noaux.json')); print('noaux', round(d['ms_per_step'],3), d['kernel_ms_per_step'])"
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/var/base2.json 2> $OUT/var/base2.err || { tail -20 $OUT/var/base2.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/var/base2.json')); print('base2', round(d['ms_per_step'],3), d['kernel_ms_per_step'])"
timeout -k 10 300 python bench.py --no-cpu-baseline --config 5 > $OUT/c5.json 2> $OUT/c5.err || { tail -20 $OUT/c5.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/c5.json')); print('c5', d['ms_per_step'], d['kernel_ms_per_step'])"
g++ -O2 -fopenmp -o tools/synthbam tools/synthbam.cpp -lz || exit 1
timeout -k 10 900 python -u tools/e2e_bench.py --synth --records 50000000 --host-decoder --devices 3 > $OUT/e2e_synth50m.json 2> $OUT/e2e_synth50m.err || { tail -30 $OUT/e2e_synth50m.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/e2e_synth50m.json')); print({k: d[k] for k in ('GatherCellMetrics_s', 'GatherCellMetrics_records_per_s', 'device_decode_stages_s', 'GatherCellMetrics_parts_s', 'parts_and_one_device_csv_identical', 'GatherCellMetrics_host_decoder_s', 'device_and_host_decoder_csv_identical')})"
