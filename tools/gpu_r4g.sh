#!/bin/bash
# 1. onesweep radix sort: tag sort / count matrix / config-5 tests; config-5 bench onesweep vs the
#    reduce-then-scan passes (SCT_RADIX_ONESWEEP=0); Welford ablations.
# 2. End to end on a config-2-shaped 50M-record BAM (tools/synthbam.cpp): GatherCellMetrics with the
#    device decoder, with devices=[0,0,0] (three parts), and with the host decoder; CSVs compared.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4g
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_buckets.py tests/test_gpu_parity.py tests/test_gpu_tagsort.py tests/test_gpu_count.py tests/test_sortorder.py "tests/test_gpu_configs.py::test_config2_cell_rows_100M" "tests/test_gpu_configs.py::test_config2_grouped_gene_rows_100M" "tests/test_gpu_configs.py::test_config5_gpu_sort_is_the_reference_stable_sort_100M" "tests/test_gpu_configs.py::test_config5_cell_metrics_after_gpu_sort_100M" "tests/test_gpu_configs.py::test_config5_gene_metrics_after_gpu_sort_100M" -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "FAIL|Error" $OUT/pytest.log | head; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for v in 1 0; do
  SCT_RADIX_ONESWEEP=$v timeout -k 10 300 python bench.py --no-cpu-baseline --config 5 > $OUT/c5_os$v.json 2> $OUT/c5_os$v.err || { tail -20 $OUT/c5_os$v.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/c5_os$v.json')); print('os$v', d['ms_per_step'], d['kernel_ms_per_step'])"
done
SCT_LIB_PATH=exp/tie_v1.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-check --config 5 > $OUT/c5_tie1.json 2> $OUT/c5_tie1.err || { tail -20 $OUT/c5_tie1.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/c5_tie1.json')); print('tie_v1', d['ms_per_step'], d['kernel_ms_per_step'])"
for L in "" exp/wf_noload.so exp/wf_b16.so; do
  n=$(basename ${L:-tree} .so)
  SCT_LIB_PATH=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-check --steps 5 > $OUT/w_$n.json 2> $OUT/w_$n.err || { tail -20 $OUT/w_$n.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/w_$n.json')); print('$n', d['ms_per_step'], d.get('dropin_cell_welford_ms'))"
done
bash tools/gpu_variants.sh r4g/var exp/ht_v1.so || exit 1
