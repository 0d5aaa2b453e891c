#!/bin/bash
# Round 5: the Welford head kernel by default with the start gate: Welford parity tests, then the
# drop-in timelines at configs 2 and 4.
set -o pipefail
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_api_gpu.py tests/test_gpu_exchange.py tests/test_gpu_buckets.py > gpurun_out/r5m_tests.log 2>&1 || { tail -30 gpurun_out/r5m_tests.log; exit 1; }
tail -3 gpurun_out/r5m_tests.log
bash tools/gpu_tl_ab.sh g2 --args "--welford" tree=tree || exit 1
bash tools/gpu_tl_ab.sh g4 --args "--welford --config 4" tree=tree || exit 1
