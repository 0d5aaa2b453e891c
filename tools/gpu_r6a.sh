#!/bin/bash
# Round 6 baseline: bench config 2 on the tree + a kernel-trace timeline of the probe.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6a
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r6a/bench_c2.json 2> gpurun_out/r6a/bench_c2.log || { tail -20 gpurun_out/r6a/bench_c2.log; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r6a/bench_c2.json'));print(d['ms_per_step'],d['kernel_ms_per_step'],d.get('dropin_cell_welford_ms'))"
bash tools/gpu_tl_ab.sh r6a_tl tree || exit 1
