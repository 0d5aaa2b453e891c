"""Workload for rocprofv3 --pmc passes (HBM traffic per kernel).

Runs the bench step (cell + grouped gene metrics, exact mode) on the config-2
shard (or bench.py's config 4 / 5 with --config) twice, then a calibration copy of a known byte count (torch clone of a
1 GiB int64 tensor: 1 GiB read + 1 GiB written with wide coalesced accesses),
so the counters' units and the gfx950 FETCH_SIZE correction can be checked
against a known figure in the same run.  Run under rocprofv3, e.g.

  rocprofv3 --pmc FETCH_SIZE --output-format csv -d OUT -o fetch -- python3 tools/pmc_probe.py
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=100_000_000)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--config", type=int, default=2, choices=[2, 4, 5],
                    help="bench.py's workloads: 2 (default), 4 (125M records, 62.5k lognormal(0, 2) cells), "
                         "5 (100M shuffled records sorted by (CB, UB, GE, query name) inside the step)")
    ap.add_argument("--welford", action="store_true",
                    help="the drop-in default instead: cell rows only, Welford float mode (bench's dropin_cell_welford_ms)")
    a = ap.parse_args()
    from sctools_amd import engine as E
    from sctools_amd import synth

    dev = torch.device("cuda", 0)
    eng = E.get_engine(dev)
    cells = 10_000
    if a.config == 4:
        a.records, cells = 125_000_000, 62_500
    cfg = synth.SynthConfig(n_reads=a.records, n_cells=cells, n_genes=30_000, sigma=2.0 if a.config == 4 else 1.0,
                            seed=0)
    if a.config == 5:
        cfg.p_nh1, cfg.p_dup, cfg.p_secondary = 0.70, 0.40, 0.10
    data = synth.generate(cfg, device=dev, chunk=16_000_000)
    dims = E.Dims(data.n_cell_ids, data.n_gene_ids, data.n_umi_ids)
    qname, n_qnames = None, 0
    if a.config == 5:  # bench.py's config 5: a global permutation, regrouped inside the step
        g = torch.Generator(device=dev)
        g.manual_seed(1)
        perm = torch.randperm(a.records, generator=g, device=dev)
        data.cols = {c: t[perm].contiguous() for c, t in data.cols.items()}
        qname, n_qnames = data.extra["qname"][perm].contiguous(), data.extra["n_qnames"]
        del perm

    def cols():
        return eng.tag_sort(data.cols, dims, "cell_umi_gene", qname, n_qnames) if a.config == 5 else data.cols

    mito = torch.from_numpy(data.gene_is_mito).to(dev)
    n_ent = eng.count_entities(cols(), "cell", dims)
    for _ in range(a.reps):
        if a.welford:
            eng.compute(cols(), "cell", dims, mito, torch.from_numpy(data.gene_is_multi).to(dev), float_mode="welford", n_entities=n_ent)
            continue
        ci, cf, part = eng.cell_and_gene(cols(), dims, mito, n_entities=n_ent)
        eng.finalize_partials(part)
    torch.cuda.synchronize()
    x = torch.ones(1 << 27, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    y = x.clone()
    torch.cuda.synchronize()
    print("calibration clone bytes read=%d written=%d" % (x.numel() * 8, y.numel() * 8), flush=True)


if __name__ == "__main__":
    main()
