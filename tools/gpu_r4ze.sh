#!/bin/bash
# Gene reduce: a few changed lanes flush their runs with direct LDS atomics instead of the wave's segmented
# DPP scan (SCT_GENE_FLUSH_LANES 8 in the tree; 24 and 64 as variants; gr_head = the measured engine).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4ze
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_api_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "FAIL|Error" $OUT/pytest.log | head; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
bash tools/gpu_variants.sh r4ze/var exp/gr_head.so exp/gr_fl24.so exp/gr_fl64.so || exit 1
bash tools/gpu_variants.sh r4ze/var2 exp/gr_head.so || exit 1
BENCH_ARGS="--config 4" bash tools/gpu_variants.sh r4ze/c4 exp/gr_head.so || exit 1
