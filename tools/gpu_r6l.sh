#!/bin/bash
# group_wave XCD mapping A/B on config 5's tag sort alone (tools/c5_sort_probe.py), twice each
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6l
mkdir -p $OUT
cd $R
for rep in 1 2; do
  timeout -k 10 240 python3 tools/c5_sort_probe.py > $OUT/tree$rep.txt 2>&1 || { tail -20 $OUT/tree$rep.txt; exit 1; }
  SCT_LIB_PATH=$R/exp/r6_gw_xcd.so timeout -k 10 240 python3 tools/c5_sort_probe.py > $OUT/xcd$rep.txt 2>&1 || { tail -20 $OUT/xcd$rep.txt; exit 1; }
done
tail -n 1 $OUT/*.txt
