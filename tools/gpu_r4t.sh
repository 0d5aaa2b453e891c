#!/bin/bash
# Welford chains fed through an LDS ring by DMA: microbenchmark, byte-identical tests, drop-in time,
# kernel trace.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4t
mkdir -p $OUT
timeout -k 10 60 ./exp/wm_lds 272000 | sed "s/^/lds /" | tee -a $OUT/wm.txt || exit 1
timeout -k 10 600 python -u -m pytest tests/test_api_gpu.py tests/test_gpu_parity.py "tests/test_gpu_configs.py" -k "welford or Welford or api or parity or config2 or config4" -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "FAIL|Error" $OUT/pytest.log | head; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 200 python3 tools/dropin_probe.py > $OUT/dropin.txt 2>&1 || { tail -20 $OUT/dropin.txt; exit 1; }
grep call $OUT/dropin.txt
R=$GRAFT_REPO_ROOT
mkdir -p $R/$OUT/tr
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$OUT/tr -o dropin -- python3 $R/tools/dropin_probe.py > $R/$OUT/probe.log 2>&1 || { tail -20 $R/$OUT/probe.log; exit 1; }
grep call $R/$OUT/probe.log
