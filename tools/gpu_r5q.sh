#!/bin/bash
# Round 5: the stream lanes on a side stream (tree) against round-5 HEAD (base5): engine parity tests,
# then timelines at configs 2 and 4 and two bench runs each.
set -o pipefail
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_buckets.py tests/test_api_gpu.py > gpurun_out/r5q_tests.log 2>&1 || { tail -30 gpurun_out/r5q_tests.log; exit 1; }
tail -2 gpurun_out/r5q_tests.log
bash tools/gpu_tl_ab.sh lanes2 base=exp/base5.so lanes=tree || exit 1
bash tools/gpu_tl_ab.sh lanes4 --args "--config 4" base=exp/base5.so lanes=tree || exit 1
bash tools/gpu_ab.sh lanesab exp/base5.so skip-tests || exit 1
