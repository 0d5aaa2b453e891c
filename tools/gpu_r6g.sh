#!/bin/bash
# Round 6: hash tile two-window pipeline (tree: 8 waves/SIMD bound), without the bound (nolb), and the
# single-window kernel (old); then the hash-tile parity tests on the tree.
set -o pipefail
bash tools/gpu_tl_ab.sh r6g tree=tree nolb=exp/ht_nolb.so old=exp/ht_old.so || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_buckets.py > gpurun_out/r6g/pytest.log 2>&1 || { tail -30 gpurun_out/r6g/pytest.log; exit 1; }
tail -2 gpurun_out/r6g/pytest.log
