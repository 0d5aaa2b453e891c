#!/bin/bash
# Kernel trace of the Welford drop-in (config 2): kernel start / end times of one call.
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4n
mkdir -p $OUT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr -o dropin -- python3 $GRAFT_REPO_ROOT/tools/dropin_probe.py > $OUT/probe.log 2>&1 || { tail -20 $OUT/probe.log; exit 1; }
grep "call" $OUT/probe.log
find $OUT/tr -name "*kernel_trace.csv" | head -3
