#!/bin/bash
# Round 6 experiment: medium big buckets on 512-thread / 40 KB blocks (exp/patches/r6_big_mid.py):
# bucket parity tests on the patched library, then the timeline A/B against the tree.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_bigmid; mkdir -p $O
SCT_LIB_PATH=$GRAFT_REPO_ROOT/exp/big_mid.so timeout -k 10 400 python -u -m pytest tests/test_gpu_buckets.py tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu_tl_ab.sh r6_bigmid_tl tree=tree mid=exp/big_mid.so mid2=exp/big_mid.so tree2=tree
