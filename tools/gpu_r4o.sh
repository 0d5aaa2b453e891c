#!/bin/bash
# welford_x first on the caller's stream: Welford byte-identical tests, drop-in A/B, kernel trace.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4o
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_api_gpu.py tests/test_gpu_parity.py "tests/test_gpu_configs.py" -k "welford or Welford or api or parity or config2 or config4" -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "FAIL|Error" $OUT/pytest.log | head; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for e in "SCT_WF_XFIRST=1" "SCT_WF_XFIRST=0" "SCT_WF_XFIRST=1 SCT_WF_PRIO=1"; do
  env $e timeout -k 10 200 python3 tools/dropin_probe.py > $OUT/dropin_ab.tmp 2>&1 || { tail -20 $OUT/dropin_ab.tmp; exit 1; }
  echo "[$e] $(grep call $OUT/dropin_ab.tmp | tr '\n' ' ')" | tee -a $OUT/dropin_ab.txt
done
mkdir -p $GRAFT_REPO_ROOT/gpurun_out/r4o/tr
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r4o/tr -o dropin -- python3 $GRAFT_REPO_ROOT/tools/dropin_probe.py > $GRAFT_REPO_ROOT/gpurun_out/r4o/probe.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r4o/probe.log; exit 1; }
grep call $GRAFT_REPO_ROOT/gpurun_out/r4o/probe.log
for v in base pf; do
  timeout -k 10 60 $GRAFT_REPO_ROOT/exp/wm_$v 272000 | sed "s/^/$v /" | tee -a $GRAFT_REPO_ROOT/gpurun_out/r4o/wm.txt || exit 1
done
cd $GRAFT_REPO_ROOT
SCT_LIB_PATH=exp/wf_pf.so timeout -k 10 200 python3 tools/dropin_probe.py > gpurun_out/r4o/dropin_pf.tmp 2>&1 || { tail -20 gpurun_out/r4o/dropin_pf.tmp; exit 1; }
echo "[wf_pf] $(grep call gpurun_out/r4o/dropin_pf.tmp | tr '\n' ' ')" | tee -a gpurun_out/r4o/dropin_ab.txt
