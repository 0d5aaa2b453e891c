#!/bin/bash
# One GPU call: parity tests (-m gpu) then per-kernel times of the bench workload.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-quick}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 200 python tools/kernel_times.py --only cell_and_gene --reps 3 > $OUT/kt.json 2> $OUT/kt.err || { tail -20 $OUT/kt.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/kt.json'))['cell_and_gene']; print(d)"
