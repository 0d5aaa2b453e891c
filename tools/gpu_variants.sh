#!/bin/bash
# Config-2 bench kernel table for the in-tree engine and each experimental build (SCT_LIB_PATH).
# Usage: [BENCH_ARGS="--config 5"] bash tools/gpu_variants.sh <tag> <exp1.so> [exp2.so ...]
# (outputs under gpurun_out/<tag>)
set -o pipefail
T=$1
shift
OUT=gpurun_out/$T
mkdir -p $OUT
run() {  # name lib
  if [ -z "$2" ]; then
    timeout -k 10 300 python bench.py --no-cpu-baseline $BENCH_ARGS > $OUT/$1.json 2> $OUT/$1.err || { tail -30 $OUT/$1.err; exit 1; }
  else
    SCT_LIB_PATH=$2 timeout -k 10 300 python bench.py --no-cpu-baseline --no-check $BENCH_ARGS > $OUT/$1.json 2> $OUT/$1.err || { tail -30 $OUT/$1.err; exit 1; }
  fi
  python -c "import json; d=json.load(open('$OUT/$1.json')); k=d['kernel_ms_per_step']; print('$1', 'ms/step %.3f' % d['ms_per_step'], k)"
}
run base ""
for lib in "$@"; do run $(basename $lib .so) $lib; done
