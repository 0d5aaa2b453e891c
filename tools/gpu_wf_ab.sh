#!/bin/bash
# One GPU call: kernel tables (tools/kernel_times.py --only $ONLY, default cell_welford) for the tree's engine and
# experimental libraries, in A B.. ..B A order.  Usage: bash tools/gpu_wf_ab.sh <tag> exp/a.so exp/b.so ...
set -o pipefail
export TMPDIR=/tmp
T=$1; shift
OUT=gpurun_out/$T
mkdir -p $OUT
LIBS=("" "$@")
N=${#LIBS[@]}
ORDER=$(seq 0 $((N-1))); ORDER="$ORDER $(seq $((N-1)) -1 0)"
i=0
for k in $ORDER; do
  L=${LIBS[$k]}; name=${L:-tree}; name=$(basename $name .so)
  if [ -n "$L" ]; then E="env SCT_LIB_PATH=$L"; else E=""; fi
  timeout -k 10 240 $E python tools/kernel_times.py --only ${ONLY:-cell_welford} --reps 2 > $OUT/kt_${i}_$name.json 2> $OUT/kt_${i}_$name.err || { tail -20 $OUT/kt_${i}_$name.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/kt_${i}_$name.json'))['${ONLY:-cell_welford}']; print('$name', d['_total'], 'wall', d['_wall_ms'], {k: v for k, v in list(d.items())[:4]})"
  i=$((i+1))
done
