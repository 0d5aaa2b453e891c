#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4e
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_buckets.py tests/test_gpu_parity.py tests/test_api_gpu.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "FAIL|Error" $OUT/pytest.log | head; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
bash tools/gpu_variants.sh r4e/var exp/head.so exp/bk_nostream.so exp/bk_nocount.so exp/gc32768.so exp/gc65536.so || exit 1
for L in "" exp/wf_lds.so exp/wf_readlane.so; do
  n=$(basename ${L:-tree} .so)
  SCT_LIB_PATH=$L timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 > $OUT/w_$n.json 2> $OUT/w_$n.err || { tail -20 $OUT/w_$n.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/w_$n.json')); print('$n', d['ms_per_step'], d.get('dropin_cell_welford_ms'))"
done
