#!/bin/bash
# Round 5: rehearsal of the config-5 N-rank path with the cell-bin exchange on a one-GPU box: 2 and 3
# ranks on cuda:0, collectives over gloo (RCCL holds one rank per device).  Correctness of the
# dealing, binning, exchange, per-rank tag sort and the gene all-reduce only -- never a scaling number.
set -o pipefail
export SCT_BENCH_SHARE_DEVICE=1
OUT=gpurun_out/r5z
mkdir -p $OUT
for np in 2 3; do
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus $np --config 5 --records 20000000 --cells 2000 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_c5_n$np.json 2> $OUT/bench_c5_n$np.err || { tail -30 $OUT/bench_c5_n$np.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_c5_n$np.json')); print($np, d['n_gpus'], round(d['ms_per_step'],2), d['config']['workload'][:160])"
done
