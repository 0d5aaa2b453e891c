#!/bin/bash
# Round 5: concurrent Welford pipelines on one device with a side-stream pair per call (tree) against
# shared pairs (base5), then the multi-device GPU tests.
set -o pipefail
echo "== base5 (shared side streams)"; SCT_LIB_PATH=$GRAFT_REPO_ROOT/exp/base5.so timeout -k 10 300 python tools/concurrent_welford_probe.py || exit 1
echo "== tree (pooled pairs)"; timeout -k 10 300 python tools/concurrent_welford_probe.py || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_exchange.py tests/test_gpu_parity.py tests/test_api_gpu.py > gpurun_out/r5ze_tests.log 2>&1 || { tail -30 gpurun_out/r5ze_tests.log; exit 1; }
tail -2 gpurun_out/r5ze_tests.log
