#!/bin/bash
# Round 6: the group sort with an MSD pass by K1's top digit + segmented LSD (tree) against the group
# sort over all of K1 (c5lsd); tag-sort tests and config 5 at 100M on the tree.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_tagsort.py tests/test_gpu_configs.py -k "tag or group or config5" > gpurun_out/r6i_pytest.log 2>&1 || { tail -40 gpurun_out/r6i_pytest.log; exit 1; }
tail -2 gpurun_out/r6i_pytest.log
bash tools/gpu_tl_ab.sh r6i --args "--config 5" tree=tree lsd=exp/c5lsd.so
