#!/bin/bash
# Drop-in call time: tree, chains without sample loads (in situ), 4 x 16-record buffers.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4s
mkdir -p $OUT
for L in "" exp/wf_noload2.so exp/wf_deep.so; do
  n=$(basename ${L:-tree} .so)
  SCT_LIB_PATH=$L timeout -k 10 200 python3 tools/dropin_probe.py > $OUT/d_$n.txt 2>&1 || { tail -20 $OUT/d_$n.txt; exit 1; }
  echo "[$n] $(grep call $OUT/d_$n.txt | tr '\n' ' ')" | tee -a $OUT/dropin_ab.txt
done
