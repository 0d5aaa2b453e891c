#!/bin/bash
# Round 5: the hash tiles' payloads loaded speculatively beside the descriptors (tree) against
# round-5 HEAD (base5): bucket/parity tests, timelines at configs 2 and 4, two bench runs each.
set -o pipefail
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_buckets.py > gpurun_out/r5zd_tests.log 2>&1 || { tail -30 gpurun_out/r5zd_tests.log; exit 1; }
tail -2 gpurun_out/r5zd_tests.log
bash tools/gpu_tl_ab.sh sp2 base=exp/base5.so spec=tree || exit 1
bash tools/gpu_tl_ab.sh sp4 --args "--config 4" base=exp/base5.so spec=tree || exit 1
bash tools/gpu_ab.sh spab exp/base5.so skip-tests || exit 1
