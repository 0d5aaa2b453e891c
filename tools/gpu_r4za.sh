#!/bin/bash
# Config 5: tag_unpack with four records per thread and one more tiebreak digit in the field sort; tag-sort tests, then
# the config-5 bench against the previous engine (unpack_old) and the tree without the extra digit (nodigit).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4za
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_tagsort.py tests/test_gpu_configs.py -k "tagsort or sort or config5" -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "FAIL|Error" $OUT/pytest.log | head; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
BENCH_ARGS="--config 5" bash tools/gpu_variants.sh r4za/var exp/unpack_old.so exp/nodigit.so || exit 1
