#!/bin/bash
# One GPU call: bench configs 4 and 5, the count-matrix bench and the end-to-end gatherer timing
# at the current kernels.  Usage: bash tools/gpu_configs.sh <tag>   (outputs under gpurun_out/<tag>)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-configs}
mkdir -p $OUT
timeout -k 10 300 python bench.py --config 4 --no-cpu-baseline > $OUT/bench_config4.json 2> $OUT/bench_config4.err || { tail -20 $OUT/bench_config4.err; exit 1; }
cat $OUT/bench_config4.json
timeout -k 10 300 python bench.py --config 5 --no-cpu-baseline > $OUT/bench_config5.json 2> $OUT/bench_config5.err || { tail -20 $OUT/bench_config5.err; exit 1; }
cat $OUT/bench_config5.json
timeout -k 10 300 python tools/count_bench.py > $OUT/count_bench.json 2> $OUT/count_bench.err || { tail -20 $OUT/count_bench.err; exit 1; }
cat $OUT/count_bench.json
timeout -k 10 300 python tools/e2e_bench.py > $OUT/e2e.json 2> $OUT/e2e.err || { tail -20 $OUT/e2e.err; exit 1; }
cat $OUT/e2e.json
