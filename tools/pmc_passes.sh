#!/bin/bash
# rocprofv3 --pmc passes (one counter per pass, kernel trace only) over tools/pmc_probe.py.
# Usage: bash tools/pmc_passes.sh <out-dir under gpurun_out> [pmc_probe.py args, e.g. --config 4]
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-pmc}
shift || true
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT -o fetch -- python3 $R/tools/pmc_probe.py "$@" > $OUT/fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT -o write -- python3 $R/tools/pmc_probe.py "$@" > $OUT/write.log 2>&1
python3 $R/tools/pmc_traffic.py $OUT "$@" > $OUT/pmc_traffic.json
