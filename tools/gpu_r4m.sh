#!/bin/bash
set -o pipefail
OUT=gpurun_out/r4m
mkdir -p $OUT
for v in base simple simple_noload; do
  timeout -k 10 60 ./exp/wm_$v 272000 | sed "s/^/$v /" | tee -a $OUT/wm.txt || exit 1
done
bash tools/gpu_r4n.sh
for e in "" "SCT_WF_EARLY=1" "SCT_WF_PRIO=1" "SCT_WF_EARLY=1 SCT_WF_PRIO=1"; do
  env $e timeout -k 10 200 python3 tools/dropin_probe.py > $OUT/dropin_ab.tmp 2>&1 || { tail -20 $OUT/dropin_ab.tmp; exit 1; }
  echo "[$e] $(grep call $OUT/dropin_ab.tmp | tr '\n' ' ')" | tee -a $OUT/dropin_ab.txt
done
