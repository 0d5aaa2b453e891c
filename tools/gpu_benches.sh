#!/bin/bash
# One GPU call: the bench at config 2 (default), config 4, config 5 and a 10x-v3 (2^24 UMIs) shard.
# Usage: bash tools/gpu_benches.sh <tag>   (outputs under gpurun_out/<tag>)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-benches}
mkdir -p $OUT
for spec in "c2:" "c4:--config 4" "c5:--config 5" "v3:--umi-bits 24"; do
  name=${spec%%:*}; args=${spec#*:}
  timeout -k 10 300 python bench.py $args > $OUT/bench_$name.json 2> $OUT/bench_$name.err || { tail -30 $OUT/bench_$name.err; exit 1; }
  cat $OUT/bench_$name.json
done
