"""Experiments only: config 5's tag sort alone (no metrics after it) on the shuffled set as the bench
has it, per-kernel times from the engine's HIP-event profile.  Safe for timing-only ablation builds
(SCT_LIB_PATH) whose sorted columns are wrong: nothing reads them."""
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
    del perm, data
    for _ in range(2):
        eng.tag_sort(cols, dims, "cell_umi_gene", qname, nq)
    torch.cuda.synchronize()
    eng.profile_only("")
    eng.profile_enable(True)
    for _ in range(3):
        eng.tag_sort(cols, dims, "cell_umi_gene", qname, nq)
    torch.cuda.synchronize()
    eng.profile_enable(False)
    t = eng.profile_read_items()
    print(os.environ.get("SCT_LIB_PATH", "tree"), {k: round(v[0] / 3, 3) for k, v in sorted(t.items(), key=lambda kv: -kv[1][0])},
          flush=True)


if __name__ == "__main__":
    main()
