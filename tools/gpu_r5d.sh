#!/bin/bash
# Round 5: the step's fills merged into one launch (tree) and the classify counter diagnostic, against
# the round-4 engine, by kernel-trace timelines; the parity tests of the tree first.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_buckets.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r5d_pytest.log 2>&1 || { tail -30 gpurun_out/r5d_pytest.log; exit 1; }
tail -1 gpurun_out/r5d_pytest.log
bash tools/gpu_tl_ab.sh r5d base=exp/base_r4.so tree=tree d1=exp/d1_norec.so
