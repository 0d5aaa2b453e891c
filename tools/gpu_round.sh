#!/bin/bash
# One GPU call: parity tests, smoke, PMC traffic passes, bench (JSON line), rocprofv3 kernel stats.
# Usage: bash tools/gpu_round.sh <tag>   (outputs under gpurun_out/<tag>)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-run}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
bash tools/pmc_passes.sh ${1:-run}/pmc || { tail -20 $OUT/pmc/*.log; exit 1; }
timeout -k 10 300 python bench.py --traffic-json $OUT/pmc/pmc_traffic.json > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o sct -- python bench.py --steps 5 --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { tail -30 $OUT/bench_prof.err; exit 1; }
find $OUT/prof -name '*kernel_stats.csv' | head -3
