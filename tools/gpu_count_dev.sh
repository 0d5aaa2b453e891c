#!/bin/bash
# Device count-mode decode: GPU tests, then CreateCountMatrix end to end (24M records).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gbam_count.py tests/test_gpu_count.py tests/test_gbam.py > gpurun_out/count_dev_tests.log 2>&1 || { tail -30 gpurun_out/count_dev_tests.log; exit 1; }
tail -3 gpurun_out/count_dev_tests.log
timeout -k 10 600 python -u tools/e2e_bench.py --count --records 24000000 --host-decoder > gpurun_out/count_e2e.json 2> gpurun_out/count_e2e.err || { tail -20 gpurun_out/count_e2e.err; exit 1; }
cat gpurun_out/count_e2e.json
