#!/bin/bash
# One GPU call: the -m gpu suite (full-size config tests included), then one bench line.
# Usage: bash tools/gpu_check.sh <tag>   (outputs under gpurun_out/<tag>)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-check}
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread --durations=15 > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -22 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
