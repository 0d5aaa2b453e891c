#!/bin/bash
# One GPU call: parity tests (-m gpu), then the config-2 bench twice -- the tree as built, and with an
# environment switch -- each once per order (A B B A), for a same-box A/B of an engine option.
# Usage: bash tools/gpu_ab_env.sh <tag> <VAR=value> [skip-tests] [bench args...]
set -o pipefail
export TMPDIR=/tmp
T=$1; ENVSW=$2; shift 2
OUT=gpurun_out/$T
mkdir -p $OUT
if [ "$1" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
else
  shift
fi
for r in a1 b1 b2 a2; do
  if [ ${r:0:1} = b ]; then E="env $ENVSW"; else E=""; fi
  timeout -k 10 300 $E python bench.py --no-cpu-baseline "$@" > $OUT/bench_$r.json 2> $OUT/bench_$r.err || { tail -30 $OUT/bench_$r.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$r.json')); k=d['kernel_ms_per_step']; print('$r', 'ms/step %.3f' % d['ms_per_step'], 'welford %.1f' % d.get('dropin_cell_welford_ms', 0), {x: k[x] for x in list(k)[:8]})"
done
