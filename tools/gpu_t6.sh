#!/bin/bash
# Round 3 experiments: Welford reciprocal pairs through LDS in groups (tree: 8) vs readlane (ylds0),
# gene_reduce's direct flush of a few changed lanes (tree: <= 8 lanes) vs the DPP scan always (df0).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/t6
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "welford or config or parity or gene or api" > gpurun_out/t6/pytest.log 2>&1; tail -2 gpurun_out/t6/pytest.log
grep -q " passed" gpurun_out/t6/pytest.log && ! grep -q failed gpurun_out/t6/pytest.log || exit 1
bash tools/gpu_wf_ab.sh wf_ylds exp/ylds0.so exp/ylds16.so || exit 1
ONLY=cell_and_gene bash tools/gpu_wf_ab.sh gr_df exp/df0.so exp/df2.so exp/df16.so
