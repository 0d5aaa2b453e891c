#!/bin/bash
# Round 4, first call: baseline bench + gene_reduce ablations, then the changed GPU test files.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4a
mkdir -p $OUT
bash tools/gpu_variants.sh r4a/var exp/gr_noatom.so exp/gr_nostream.so exp/gr_nouy.so || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_tagsort.py tests/test_gbam.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
