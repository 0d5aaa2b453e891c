#!/bin/bash
# A/B of an experimental engine build (SCT_LIB_PATH) against the in-tree one on the config-2 bench.
# Usage: bash tools/gpu_ab.sh <tag> <exp.so> [skip-tests]   (outputs under gpurun_out/<tag>)
set -o pipefail
T=${1:-ab}
EXP=$2
OUT=gpurun_out/$T
mkdir -p $OUT
if [ "$3" != "skip-tests" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
fi
for r in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_a$r.json 2> $OUT/bench_a$r.err || { tail -30 $OUT/bench_a$r.err; exit 1; }
  SCT_LIB_PATH=$EXP timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_b$r.json 2> $OUT/bench_b$r.err || { tail -30 $OUT/bench_b$r.err; exit 1; }
done
for f in $OUT/bench_a1.json $OUT/bench_b1.json $OUT/bench_a2.json $OUT/bench_b2.json; do
  python -c "import json,sys; d=json.load(open('$f')); k=d['kernel_ms_per_step']; print('$f', 'ms/step %.3f' % d['ms_per_step'], {x: k[x] for x in ('build_keys','hash_tile','gene_reduce','gene_emit')})"
done
