#!/bin/bash
# Welford chain A/B (tree vs variants) then the Welford parity tests on the last variant.
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_wf_ab.sh wf_pipe "$@" || exit 1
L=${@: -1}
SCT_LIB_PATH=$L timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_buckets.py -k "welford or Welford" > gpurun_out/wf_pipe/parity.log 2>&1 || { tail -30 gpurun_out/wf_pipe/parity.log; exit 1; }
tail -2 gpurun_out/wf_pipe/parity.log
