#!/bin/bash
# One GPU call: parity tests (-m gpu) unless "skip-tests", then the config-2 bench for several
# environment variants (name=VAR=value, "tree" = as built) in the order given and then reversed,
# for a same-box A/B/C of engine options.
# Usage: bash tools/gpu_ab_multi.sh <tag> [skip-tests] [--args "bench args"] name=ENV ... 
set -o pipefail
export TMPDIR=/tmp
T=$1; shift
OUT=gpurun_out/$T
mkdir -p $OUT
if [ "$1" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
else
  shift
fi
ARGS=""
if [ "$1" == "--args" ]; then ARGS=$2; shift 2; fi
V=("$@")
ORDER=()
for ((i = 0; i < ${#V[@]}; i++)); do ORDER+=("${V[$i]}:1"); done
for ((i = ${#V[@]} - 1; i >= 0; i--)); do ORDER+=("${V[$i]}:2"); done
for ov in "${ORDER[@]}"; do
  nv=${ov%:*}; r=${ov##*:}
  name=${nv%%=*}; env=${nv#*=}
  if [ "$name" == "tree" ]; then E=""; else E="env ${env//,/ }"; fi
  timeout -k 10 300 $E python bench.py --no-cpu-baseline $ARGS > $OUT/bench_${name}_$r.json 2> $OUT/bench_${name}_$r.err || { tail -30 $OUT/bench_${name}_$r.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_${name}_$r.json')); k=d['kernel_ms_per_step']; print('${name}_$r', 'ms/step %.3f' % d['ms_per_step'], {x: k[x] for x in list(k)[:6]})"
done
