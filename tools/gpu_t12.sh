#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/t12; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "gene or config or parity or api or multigpu" > $OUT/pytest.log 2>&1; tail -2 $OUT/pytest.log
grep -q " passed" $OUT/pytest.log && ! grep -q failed $OUT/pytest.log || exit 1
ONLY=cell_and_gene bash tools/gpu_wf_ab.sh gq_ab exp/gq0.so
