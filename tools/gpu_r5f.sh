#!/bin/bash
# Round 5: the three-wave Welford head chains (tree) -- Welford parity at the fixture sizes and at
# configs 2 / 4, then the drop-in time against the round-4 head chains (exp/wf_old.so).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5f
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_buckets.py tests/test_gpu_configs.py::test_config2_cell_rows_100M tests/test_gpu_configs.py::test_config4_shard_cell_rows_125M -x -q --timeout 400 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for c in 2 4; do
  for v in tree wf_old; do
    if [ $v == tree ]; then L=""; else L="SCT_LIB_PATH=exp/$v.so"; fi
    env $L timeout -k 10 300 python bench.py --config $c --steps 3 --no-cpu-baseline > $OUT/bench_c${c}_$v.json 2> $OUT/bench_c${c}_$v.err || { tail -20 $OUT/bench_c${c}_$v.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/bench_c${c}_$v.json')); print('c$c $v', round(d['ms_per_step'],3), 'dropin_welford_ms', round(d['dropin_cell_welford_ms'],2))"
  done
done
bash tools/gpu_tl_ab.sh r5f_tl tree=tree
