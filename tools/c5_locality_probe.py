"""Experiments only: config 5's tag sort on the shuffled set as the bench has it, and on the same
records pre-grouped (untimed) by the top bits of the cell id -- what an MSD pass by cell would give
the group sort's row gather (locality of the rows gathered by consecutive output positions)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def main():
    from sctools_amd import engine as E
    from sctools_amd import synth

    dev = torch.device("cuda", 0)
    eng = E.get_engine(dev)
    cfg = synth.SynthConfig(n_reads=100_000_000, n_cells=10_000, n_genes=30_000, seed=0)
    cfg.p_nh1, cfg.p_dup, cfg.p_secondary = 0.70, 0.40, 0.10
    data = synth.generate(cfg, device=dev, chunk=16_000_000)
    dims = E.Dims(data.n_cell_ids, data.n_gene_ids, data.n_umi_ids)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    perm = torch.randperm(cfg.n_reads, generator=g, device=dev)
    cols = {c: t[perm].contiguous() for c, t in data.cols.items()}
    qname, nq = data.extra["qname"][perm].contiguous(), data.extra["n_qnames"]
    del perm
    for shift in (None, 6, 3):
        if shift is None:
            c2, q2, label = cols, qname, "shuffled"
        else:
            o = torch.argsort(cols["cell"] >> shift, stable=True)
            c2 = {c: t[o].contiguous() for c, t in cols.items()}
            q2 = qname[o].contiguous()
            label = "grouped by cell >> %d" % shift
        for _ in range(2):
            eng.tag_sort(c2, dims, "cell_umi_gene", q2, nq)
        torch.cuda.synchronize()
        eng.profile_only("")
        eng.profile_enable(True)
        for _ in range(3):
            eng.tag_sort(c2, dims, "cell_umi_gene", q2, nq)
        torch.cuda.synchronize()
        eng.profile_enable(False)
        t = eng.profile_read_items()
        print(label, {k: round(v[0] / 3, 3) for k, v in sorted(t.items(), key=lambda kv: -kv[1][0])}, flush=True)
        if shift is not None:
            del c2, q2


if __name__ == "__main__":
    main()
