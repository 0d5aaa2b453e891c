#!/bin/bash
# device BAM decode: windows, parts, OOM decline, API paths
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4c
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gbam.py tests/test_gbam_count.py tests/test_api_gpu.py tests/test_gpu_tagsort.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "FAIL|Error|error" $OUT/pytest.log | head -30; tail -60 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
bash tools/gpu_variants.sh r4c/var exp/emit2k.so || exit 1
