#!/bin/bash
# Welford chains without ordering barriers and with ping-pong sample buffers: byte-identical tests,
# the engine-kernel microbenchmark, the drop-in call time.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4q
mkdir -p $OUT
for v in new dpp_noasm; do
  timeout -k 10 60 ./exp/wm_$v 272000 | sed "s/^/$v /" | tee -a $OUT/wm.txt || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_api_gpu.py tests/test_gpu_parity.py "tests/test_gpu_configs.py" -k "welford or Welford or api or parity or config2 or config4" -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "FAIL|Error" $OUT/pytest.log | head; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 200 python3 tools/dropin_probe.py > $OUT/dropin.txt 2>&1 || { tail -20 $OUT/dropin.txt; exit 1; }
grep call $OUT/dropin.txt
