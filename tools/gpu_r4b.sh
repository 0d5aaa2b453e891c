#!/bin/bash
# SQ counters of gene_reduce: tree vs ablations (sort only / no streams)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r4b
mkdir -p $OUT
bash tools/gpu_variants.sh r4b/var exp/gr_sortonly.so || exit 1
cd /tmp
for v in base gr_sortonly gr_nouy; do
  if [ $v = base ]; then L=""; else L=$R/exp/$v.so; fi
  SCT_LIB_PATH=$L timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $OUT/$v -o sq1 -- python3 $R/tools/pmc_probe.py --reps 1 > $OUT/$v.sq1.log 2>&1 || exit 1
  SCT_LIB_PATH=$L timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $OUT/$v -o sq2 -- python3 $R/tools/pmc_probe.py --reps 1 > $OUT/$v.sq2.log 2>&1 || exit 1
  python3 $R/tools/sq_summary.py $(find $OUT/$v -name "*counter_collection.csv") | grep -A1 "gene_reduce\|gene_emit\|hash_tile\|build_keys" > $OUT/$v.sq.txt
  echo "== $v"; cat $OUT/$v.sq.txt
done
