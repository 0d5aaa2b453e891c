#!/bin/bash
# group_wave ablations on config 5's tag sort alone (tools/c5_sort_probe.py)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6k
mkdir -p $OUT
cd $R
timeout -k 10 240 python3 tools/c5_sort_probe.py > $OUT/tree.txt 2>&1 || { tail -20 $OUT/tree.txt; exit 1; }
for v in nostore seqrows nosort; do
  SCT_LIB_PATH=$R/exp/r6_gw_$v.so timeout -k 10 240 python3 tools/c5_sort_probe.py > $OUT/$v.txt 2>&1 || { tail -20 $OUT/$v.txt; exit 1; }
done
tail -n 1 $OUT/*.txt
