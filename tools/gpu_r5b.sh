#!/bin/bash
# Round 5: the cell-bin exchange for unsorted input -- its GPU tests, then bench.py's N-rank config-5
# path rehearsed on one GPU (ranks share cuda:0, collectives over gloo: not a scaling number).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5b
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_api_gpu.py::test_cell_sorted_pass_refuses_unsorted_input tests/test_gpu_exchange.py -x -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
for n in 2 3; do
  SCT_BENCH_SHARE_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --config 5 --steps 2 --warmup 1 --records $((24000000 / n)) --cells $((3000 / n)) --no-cpu-baseline > $OUT/bench_c5_n$n.json 2> $OUT/bench_c5_n$n.err || { tail -30 $OUT/bench_c5_n$n.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/bench_c5_n$n.json').read().strip().splitlines()[-1]); print('n$n', d['n_gpus'], round(d['ms_per_step'],3), '%.3g' % d['value'], d['config']['workload'])"
done
