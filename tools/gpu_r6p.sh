#!/bin/bash
# Round 6 (9-bit MSD group sort): the N > 1 bench paths rehearsed on one GPU (2 ranks sharing cuda:0
# over gloo): config 5 (cell-bin exchange, then each rank's group sort) and config 3 (strong scaling)
# against N = 1 (gene rows hash).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6p; mkdir -p $O
SCT_BENCH_SHARE_DEVICE=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 2 --config 5 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c5_n2.json 2> $O/bench_c5_n2.log || { tail -30 $O/bench_c5_n2.log; exit 1; }
timeout -k 10 300 python bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c3_n1.json 2> $O/bench_c3_n1.log || { tail -20 $O/bench_c3_n1.log; exit 1; }
SCT_BENCH_SHARE_DEVICE=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29614 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c3_n2.json 2> $O/bench_c3_n2.log || { tail -30 $O/bench_c3_n2.log; exit 1; }
python3 - <<'PY'
import json
def last(p): return json.loads(open(p).read().strip().splitlines()[-1])
c5 = last('gpurun_out/r6p/bench_c5_n2.json')
print('c5 n2', c5['scaling'], c5['config']['records_per_job'], c5['ms_per_step'], c5['config']['parallelism'])
a, b = last('gpurun_out/r6p/bench_c3_n1.json'), last('gpurun_out/r6p/bench_c3_n2.json')
print('c3 n1', a['config']['records_per_job'], a['ms_per_step'], a['gene_rows_sha256'][:16])
print('c3 n2', b['config']['records_per_job'], b['config']['records_per_rank'], b['ms_per_step'], b['gene_rows_sha256'][:16])
print('gene rows equal:', a['gene_rows_sha256'] == b['gene_rows_sha256'])
PY
