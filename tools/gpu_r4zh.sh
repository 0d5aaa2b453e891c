#!/bin/bash
# SQ issue / wait / LDS counters of the final round-4 engine (efe216cf...), config 2 and config 5, for the round-5 plan.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for c in 2 5; do
  O=$R/gpurun_out/r4zh/c$c
  mkdir -p $O
  cd /tmp
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $O -o sq1 -- python3 $R/tools/pmc_probe.py --reps 1 --config $c > $O/sq1.log 2>&1 || { tail -20 $O/sq1.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $O -o sq2 -- python3 $R/tools/pmc_probe.py --reps 1 --config $c > $O/sq2.log 2>&1 || { tail -20 $O/sq2.log; exit 1; }
  cd $R
  python3 tools/sq_summary.py $(find $O -name "*counter_collection.csv") > $O/sq_summary.txt || exit 1
  head -24 $O/sq_summary.txt
done
