"""CountMatrix (sct_count_matrix) throughput on one GPU, one JSON line like bench.py's.

python tools/count_bench.py [--records N] [--cells C] [--genes G] [--steps K]   (needs a GPU)

Workload: N records in query-name groups (a record starts a new group with p = 0.75),
C cells, G annotated genes (+1 %% multi-gene values), 2^20 molecule barcodes, XF mixed;
columns resident in HBM.  A step = the full C-ABI call (molecule keys, sort, pairs, rows,
CSR scatter; synchronizes).  cpu_baseline: the oracle's column loop (oracle/count_oracle.py,
one core) on the first records of the same columns.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from sctools_amd import count as C  # noqa: E402
from sctools_amd import engine as E  # noqa: E402

# algorithmic bytes per record (or per item) of each kernel launch
ALG = {
    "count_groups": 4 * 3 + 1 + 1 + 8 + 4,  # cell, umi, gene, xf, qhead in; key, value out
    "radix_downsweep": 24,                  # (8-byte key + 4-byte value) in and out per pass
    "radix_upsweep": 8,
    "count_pairs": 8 + 4,
    "count_emit": 8 + 4 + 4,
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=100_000_000)
    ap.add_argument("--cells", type=int, default=10_000)
    ap.add_argument("--genes", type=int, default=30_000)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--cpu-sample", type=int, default=3_000_000)
    args = ap.parse_args()
    n, nc, ng = args.records, args.cells, args.genes
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(1)
    qhead = (torch.rand(n, device=dev, generator=g) < 0.75).to(torch.uint8)
    qhead[0] = 1
    cell = torch.randint(1, nc, (n,), device=dev, generator=g, dtype=torch.int32)
    cell = torch.sort(cell).values.to(torch.int32)  # cell-grouped, as a tag-sorted BAM is
    umi = torch.randint(1, 1 << 20, (n,), device=dev, generator=g, dtype=torch.int32)
    gene = torch.randint(1, ng + 1, (n,), device=dev, generator=g, dtype=torch.int32)
    xf = torch.tensor([0, 1, 2, 3, 4, 5], dtype=torch.uint8, device=dev)[
        torch.multinomial(torch.tensor([0.03, 0.55, 0.15, 0.12, 0.1, 0.05], device=dev), n, replacement=True,
                          generator=g)]
    genes = [None] + ["G%05d" % i for i in range(1, ng + 1)]
    for i in range(1, ng + 1, 100):
        genes[i] += ",X"
    names = {"G%05d" % i: i - 1 for i in range(1, ng + 1)}
    gc = torch.from_numpy(C.gene_columns(genes, names)).to(dev)
    eng = E.get_engine(dev)
    call = lambda: eng.count_matrix(cell, umi, gene, xf, qhead, gc, nc, 1 << 20, 0, 0, ng)  # noqa: E731
    for _ in range(args.warmup):
        res, _ = call()
    torch.cuda.synchronize()
    eng.profile_enable(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res, unknown = call()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    prof = eng.profile_read()
    eng.profile_enable(False)
    assert unknown == -1
    nnz = int(res[3].numel())
    kms = {k: v[0] / args.steps for k, v in sorted(prof.items(), key=lambda kv: -kv[1][0])}
    dom = max(kms, key=kms.get)
    launches = prof[dom][1] / args.steps
    per_launch_ms = kms[dom] / launches
    # the radix kernels sort the counted groups' molecule keys (eng.count_stats["sorted"] items,
    # cbits + colbits + ubits bits) and then the rows' (first record, cell) keys (rows items,
    # 32 bits): algorithmic bytes per step over the kernel's total time per step
    sorted_items = eng.count_stats["sorted"]
    bitlen = lambda v: max(0, int(v - 1).bit_length())  # noqa: E731
    mol_passes = -(-(bitlen(nc) + bitlen(ng) + bitlen(1 << 20)) // 8)
    row_passes = int(round(launches)) - mol_passes
    items = {"radix_downsweep": sorted_items * mol_passes + int(res[0].numel()) * row_passes,
             "radix_upsweep": sorted_items * mol_passes + int(res[0].numel()) * row_passes}
    step_bytes = ALG.get(dom, 0) * items.get(dom, n * launches)
    achieved = step_bytes / (kms[dom] * 1e-3) / 1e9
    # CPU baseline: the oracle's column restatement, one core, on a leading sample
    from oracle import count_oracle as O

    m = min(args.cpu_sample, n)
    while m < n and qhead[m].item() == 0:
        m += 1
    host = {k: t[:m].cpu().numpy() for k, t in dict(cell=cell, umi=umi, gene=gene, xf=xf, qhead=qhead).items()}
    cells = [None] + ["C%05d" % i for i in range(1, nc)]
    umis = [None] + ["U%07d" % i for i in range(1, 1 << 20)]
    t1 = time.perf_counter()
    O.count_columns(host, cells, umis, genes, names)
    cpu_s = time.perf_counter() - t1
    print(json.dumps({
        "metric": "records/sec for CountMatrix (CreateCountMatrix)", "value": n / dt, "unit": "records/s",
        "n_gpus": 1, "steps": args.steps, "warmup": args.warmup, "ms_per_step": dt * 1e3, "higher_is_better": True,
        "dtype": "int64", "data": "synthetic query-name groups, generated on GPU",
        "config": {"workload": "count matrix: %d records, %d cells, %d genes, 2^20 molecule barcodes" % (n, nc, ng),
                   "rows": int(res[0].numel()), "nnz": nnz},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": 8000.0, "unit": "GB/s",
                     "frac": achieved / 8000.0, "avg_launch_ms": per_launch_ms, "launches_per_step": launches,
                     "alg_bytes_per_item": ALG.get(dom, 0), "items_per_step": items.get(dom, n * launches),
                     "sorted_molecule_keys": sorted_items},
        "kernel_ms_per_step": {k: round(v, 4) for k, v in kms.items()},
        "cpu_baseline": {"value": m / cpu_s, "unit": "records/s", "cores": 1, "kind": "port",
                         "sample": "first %d records: oracle count_columns loop, %.1fs" % (m, cpu_s)},
    }))


if __name__ == "__main__":
    main()
