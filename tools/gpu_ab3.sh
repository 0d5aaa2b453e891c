#!/bin/bash
# One GPU call: parity tests, the FP64 dependent-latency microbenchmark, then the config-2 bench for
# three engines on one box: the tree (A), the tree without the planned first level (B,
# SCT_NO_L1_PLAN=1) and an experimental library (C, SCT_LIB_PATH=$2), in the order A B C C B A.
# Usage: bash tools/gpu_ab3.sh <tag> <exp.so> [skip-tests]
set -o pipefail
export TMPDIR=/tmp
T=$1; EXP=$2
OUT=gpurun_out/$T
mkdir -p $OUT
if [ "$3" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
fi
if [ -x tools/debug/fp64_chain ]; then timeout -k 10 60 ./tools/debug/fp64_chain > $OUT/fp64.txt 2>&1 && cat $OUT/fp64.txt; fi
for r in a1 b1 c1 c2 b2 a2; do
  case ${r:0:1} in a) E="";; b) E="env SCT_NO_L1_PLAN=1";; c) E="env SCT_LIB_PATH=$EXP";; esac
  timeout -k 10 300 $E python bench.py --no-cpu-baseline > $OUT/bench_$r.json 2> $OUT/bench_$r.err || { tail -30 $OUT/bench_$r.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$r.json')); k=d['kernel_ms_per_step']; print('$r', 'ms/step %.3f' % d['ms_per_step'], 'welford %.1f' % d.get('dropin_cell_welford_ms', 0), {x: k[x] for x in list(k)[:9]})"
done
