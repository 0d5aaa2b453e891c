#!/bin/bash
# Round 5: gene reduce work items of 32K / 64K payloads for every bucket (the hot buckets already use
# 64K) against 16K (base5): timelines at configs 2 and 4, and the reduce's PMC writes.
set -o pipefail
bash tools/gpu_tl_ab.sh gc2 base=exp/base5.so gc32k=exp/gc32k.so gc64k=exp/gc64k.so || exit 1
bash tools/gpu_tl_ab.sh gc4 --args "--config 4" base=exp/base5.so gc32k=exp/gc32k.so gc64k=exp/gc64k.so || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in base5 gc32k gc64k; do
  mkdir -p $R/gpurun_out/gcw/$v
  (cd /tmp && SCT_LIB_PATH=$R/exp/$v.so timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/gcw/$v -o write -- python3 $R/tools/pmc_probe.py > $R/gpurun_out/gcw/$v/write.log 2>&1) || exit 1
done
echo pmc done
