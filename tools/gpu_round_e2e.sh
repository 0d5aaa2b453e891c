#!/bin/bash
# One GPU call: tools/gpu_round.sh (tests, smoke, PMC, bench, rocprofv3), then the end-to-end
# GatherCellMetrics bench on a generated BAM (device decoder, and the host decoder beside it).
# Usage: bash tools/gpu_round_e2e.sh <tag> [records]
set -o pipefail
T=${1:-run}
bash tools/gpu_round.sh $T || exit 1
OUT=gpurun_out/$T
timeout -k 10 600 python -u tools/e2e_bench.py --records ${2:-24000000} --host-decoder > $OUT/e2e.json 2> $OUT/e2e.err || { tail -30 $OUT/e2e.err; exit 1; }
cat $OUT/e2e.json
