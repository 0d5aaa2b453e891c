#!/bin/bash
# One GPU call: the device BAM decode tests, then (optionally) the end-to-end bench.
set -o pipefail
export TMPDIR=/tmp
T=${1:-gbam}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gbam.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gbam.log 2>&1 || { tail -60 $OUT/pytest_gbam.log; exit 1; }
tail -3 $OUT/pytest_gbam.log
if [ -n "$2" ]; then
  timeout -k 10 600 python -u tools/e2e_bench.py $2 > $OUT/e2e.json 2> $OUT/e2e.err || { tail -30 $OUT/e2e.err; exit 1; }
  cat $OUT/e2e.json
fi
