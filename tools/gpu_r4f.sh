#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4f
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_api_gpu.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "FAIL|Error" $OUT/pytest.log | head; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for L in "" exp/wf_lds.so exp/wf_readlane.so; do
  n=$(basename ${L:-tree} .so)
  SCT_LIB_PATH=$L timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 > $OUT/b_$n.json 2> $OUT/b_$n.err || { tail -20 $OUT/b_$n.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/b_$n.json')); print('$n', d['ms_per_step'], d.get('dropin_cell_welford_ms'), d.get('dropin_kernel_ms', {}).get('welford_chains') if isinstance(d.get('dropin_kernel_ms'), dict) else '')"
done
