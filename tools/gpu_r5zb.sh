#!/bin/bash
# Round 5: the gene reduce's first run boundary flushed once per sub-tile by the lanes together
# (tree) against round-5 HEAD (base5): gene/parity tests, timelines at configs 2 and 4, benches.
set -o pipefail
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_buckets.py tests/test_api_gpu.py tests/test_gpu_exchange.py > gpurun_out/r5zb_tests.log 2>&1 || { tail -30 gpurun_out/r5zb_tests.log; exit 1; }
tail -2 gpurun_out/r5zb_tests.log
bash tools/gpu_tl_ab.sh cf2 base=exp/base5.so conv=tree || exit 1
bash tools/gpu_tl_ab.sh cf4 --args "--config 4" base=exp/base5.so conv=tree || exit 1
bash tools/gpu_ab.sh cfab exp/base5.so skip-tests || exit 1
