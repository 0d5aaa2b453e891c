#!/bin/bash
# One GPU call: parity tests (-m gpu), then the config-2 bench (JSON line with the kernel table).
# Usage: bash tools/gpu_test_bench.sh <tag> [skip-tests] [extra bench args...]   (outputs under gpurun_out/<tag>)
set -o pipefail
export TMPDIR=/tmp
T=${1:-tb}
OUT=gpurun_out/$T
mkdir -p $OUT
shift
if [ "$1" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
else
  shift
fi
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print('ms/step %.3f' % d['ms_per_step'], d['kernel_ms_per_step'], d['roofline']['kernel'], round(d['roofline']['frac'],3))"
