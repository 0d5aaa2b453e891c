#!/bin/bash
# One GPU call for a kernel iteration: -m gpu parity suite, the config-2 bench line, SQ counters.
# Usage: bash tools/gpu_iter.sh <tag> [skip-tests]   (outputs under gpurun_out/<tag>)
set -o pipefail
export TMPDIR=/tmp
T=${1:-iter}
OUT=gpurun_out/$T
mkdir -p $OUT
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
fi
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print('ms/step %.3f' % d['ms_per_step'], d['kernel_ms_per_step'])"
bash tools/pmc_sq.sh $T/sq > /dev/null && python3 tools/sq_summary.py $(find $OUT/sq -name "*counter_collection.csv") > $OUT/sq_summary.txt && head -8 $OUT/sq_summary.txt
