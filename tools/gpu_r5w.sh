#!/bin/bash
# Round 5: the Welford head-entity boundary parity tests.
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "welford_head" > gpurun_out/r5w_tests.log 2>&1 || { tail -40 gpurun_out/r5w_tests.log; exit 1; }
tail -5 gpurun_out/r5w_tests.log
