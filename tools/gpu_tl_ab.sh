#!/bin/bash
# Timeline A/B: for each engine build (name=path; "tree" = the in-tree library), one rocprofv3
# kernel-trace run of tools/pmc_probe.py and tools/timeline.py's per-kernel table of the last step.
# Usage: bash tools/gpu_tl_ab.sh <tag> [probe args --] name=path ...
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=$1
shift
ARGS=""
if [ "$1" == "--args" ]; then ARGS=$2; shift 2; fi
OUT=$R/gpurun_out/$T
mkdir -p $OUT
for nv in "$@"; do
  name=${nv%%=*}
  lib=${nv#*=}
  cd /tmp
  if [ "$lib" == "tree" ]; then
    timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/$name -o tr -- python3 $R/tools/pmc_probe.py --reps 3 $ARGS > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; exit 1; }
  else
    SCT_LIB_PATH=$R/$lib timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/$name -o tr -- python3 $R/tools/pmc_probe.py --reps 3 $ARGS > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; exit 1; }
  fi
  cd $R
  python3 tools/timeline.py $OUT/$name > $OUT/$name.timeline.txt || exit 1
  echo "== $name"; tail -1 $OUT/$name.timeline.txt
done
python3 tools/timeline_cmp.py $OUT "$@" > $OUT/compare.txt && cat $OUT/compare.txt
