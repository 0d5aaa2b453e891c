"""Debug: the (CB, UB, GE, qname) GPU sort's permutation at several sizes."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from sctools_amd import engine as E, synth

eng = E.get_engine("cuda:0")
for n in (200_000, 2_000_000, 20_000_000):
    d = synth.generate(synth.SynthConfig(n_reads=n, n_cells=max(10, n // 10000), n_genes=30_000, seed=5, p_nh1=0.7,
                                         p_dup=0.4, p_secondary=0.1), device="cuda:0")
    g = torch.Generator(device="cuda:0"); g.manual_seed(1)
    perm = torch.randperm(n, generator=g, device="cuda:0")
    cols = {c: t[perm].contiguous() for c, t in d.cols.items()}
    tie = d.extra["qname"][perm].contiguous()
    dims = E.Dims(d.n_cell_ids, d.n_gene_ids, d.n_umi_ids)
    probe = dict(cols); probe["pos"] = torch.arange(n, dtype=torch.int32, device="cuda:0")
    out = eng.tag_sort(probe, dims, "cell_umi_gene", tie, int(d.extra["n_qnames"]))
    p = out["pos"].long().cpu().numpy()
    cnt = np.bincount(p, minlength=n)
    bad = np.flatnonzero(cnt != 1)
    k = ((out["cell"].long() << 37) | (out["umi"].long() << 17) | out["gene"].long()).cpu().numpy()
    runs = np.diff(np.flatnonzero(np.r_[True, k[1:] != k[:-1], True]))
    print(n, "dups/missing", len(bad), "max run", runs.max(), "runs>16", int((runs > 16).sum()), flush=True)
    if len(bad):
        dup = np.flatnonzero(cnt > 1)[:5]
        for v in dup:
            where = np.flatnonzero(p == v)
            print("  value", v, "at", where, "keys", k[where], flush=True)
