# SQ counter passes over tools/pmc_probe.py (per-kernel issue / wait / LDS breakdown)
set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$R/gpurun_out/${1:-pmc_sq}
mkdir -p $O
cd /tmp
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $O -o sq1 -- python3 $R/tools/pmc_probe.py --reps 1 > $O/sq1.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $O -o sq2 -- python3 $R/tools/pmc_probe.py --reps 1 > $O/sq2.log 2>&1
find $O -name "*counter_collection.csv" | head
