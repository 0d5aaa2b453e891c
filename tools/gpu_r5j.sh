#!/bin/bash
# Round 5: Welford head chains with / without the LDS reservation (timelines at configs 2 and 4).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
./tools/debug/devattr || exit 1
for cfg in 2 4; do
  for kb in 0 def; do
    OUT=$R/gpurun_out/hog$cfg/$kb
    mkdir -p $OUT
    if [ $kb == def ]; then unset SCT_WF_HEAD_LDS_KB; else export SCT_WF_HEAD_LDS_KB=$kb; fi
    (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT -o tr -- python3 $R/tools/pmc_probe.py --reps 3 --welford --config $cfg > $OUT.log 2>&1) || { tail -20 $OUT.log; exit 1; }
    python3 tools/timeline.py $OUT > $OUT.timeline.txt || exit 1
    echo "== cfg $cfg lds $kb"; grep -E "welford_chains|span" $OUT.timeline.txt
  done
done
