#!/bin/bash
# Round 6: level-1 counts read back before the key pass (no host wait between the key pass and level 2):
# parity tests, then the config-2 step timeline against HEAD (twice each)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6q; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_buckets.py tests/test_gpu_configs.py tests/test_api_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/gpu_tl_ab.sh r6q tree=tree head=exp/head.so tree2=tree head2=exp/head.so
