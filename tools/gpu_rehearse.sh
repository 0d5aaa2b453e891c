#!/bin/bash
# One GPU call: bench.py's N-rank path rehearsed on one GPU (SCT_BENCH_SHARE_DEVICE=1: ranks share
# cuda:0, collectives over gloo) at N = 2 and 4 -- launch, barriers, the per-step partial all-reduce
# and its record-count check, max-over-ranks timing, allreduce_ms, the JSON line.  Not a scaling number.
set -o pipefail
export TMPDIR=/tmp SCT_BENCH_SHARE_DEVICE=1
OUT=gpurun_out/rehearse; mkdir -p $OUT
for n in 2 4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --steps 3 --warmup 1 --records $((40000000 / n)) --cells $((4000 / n)) --no-cpu-baseline > $OUT/bench_n$n.json 2> $OUT/bench_n$n.err || { tail -30 $OUT/bench_n$n.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/bench_n$n.json').read().strip().splitlines()[-1]); print('n$n', d['n_gpus'], round(d['ms_per_step'],3), '%.3g' % d['value'], d['allreduce_ms'], d['config']['parallelism'])"
done
