#!/bin/bash
# Round 6: GPU tests on the tree (protocol error paths, gate order, record-balanced bins, packed
# exchange), bench config 2, the concurrent Welford probe, and the config-3 strong-scaling split
# rehearsed on one GPU (2 ranks sharing cuda:0 over gloo) against config 3 at N = 1 (gene rows hash).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6b; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.log || { tail -20 $O/bench_c2.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_c2.json'));print('c2', d['ms_per_step'], d['dropin_cell_welford_ms'], d['gene_rows_sha256'])"
timeout -k 10 300 python tools/concurrent_welford_probe.py > $O/concurrent.txt 2>&1 || { tail -20 $O/concurrent.txt; exit 1; }
tail -6 $O/concurrent.txt
timeout -k 10 300 python bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c3_n1.json 2> $O/bench_c3_n1.log || { tail -20 $O/bench_c3_n1.log; exit 1; }
SCT_BENCH_SHARE_DEVICE=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c3_n2.json 2> $O/bench_c3_n2.log || { tail -30 $O/bench_c3_n2.log; exit 1; }
python3 - <<'PY'
import json
a = json.loads(open('gpurun_out/r6b/bench_c3_n1.json').read().strip().splitlines()[-1])
b = json.loads(open('gpurun_out/r6b/bench_c3_n2.json').read().strip().splitlines()[-1])
print('c3 n1', a['scaling'], a['config']['records_per_job'], a['ms_per_step'], a['gene_rows_sha256'][:16])
print('c3 n2', b['scaling'], b['config']['records_per_job'], b['config']['records_per_rank'], b['ms_per_step'], b['gene_rows_sha256'][:16], b['config']['parallelism'])
print('gene rows equal:', a['gene_rows_sha256'] == b['gene_rows_sha256'])
PY
