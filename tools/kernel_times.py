"""Per-kernel timings (HIP events in the engine) for each entry point on the bench workload.

python tools/kernel_times.py [--records N] [--cells C]   (needs a GPU)
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from sctools_amd import engine as E  # noqa: E402
from sctools_amd import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=100_000_000)
    ap.add_argument("--cells", type=int, default=10_000)
    ap.add_argument("--genes", type=int, default=30_000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--only", default="", help="comma-separated variant names")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    eng = E.get_engine(dev)
    d = synth.generate(synth.SynthConfig(n_reads=a.records, n_cells=a.cells, n_genes=a.genes), device=dev,
                       chunk=16_000_000)
    dims = E.Dims(d.n_cell_ids, d.n_gene_ids, d.n_umi_ids)
    mito = torch.from_numpy(d.gene_is_mito).to(dev)
    n_ent = eng.count_entities(d.cols, "cell", dims)
    variants = {
        "cell_exact": lambda: eng.compute(d.cols, "cell", dims, mito, mito, float_mode="exact", n_entities=n_ent),
        "cell_welford": lambda: eng.compute(d.cols, "cell", dims, mito, mito, float_mode="welford", n_entities=n_ent),
        "cell_and_gene": lambda: eng.cell_and_gene(d.cols, dims, mito, n_entities=n_ent),
    }
    if a.only:
        variants = {k: v for k, v in variants.items() if k in a.only.split(",")}
    out = {}
    import time

    for name, fn in variants.items():
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            fn()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / a.reps * 1e3
        eng.profile_enable(True)
        for _ in range(a.reps):
            fn()
        torch.cuda.synchronize()
        eng.profile_enable(False)
        prof = eng.profile_read()
        out[name] = {k: round(v[0] / a.reps, 4) for k, v in sorted(prof.items(), key=lambda kv: -kv[1][0])}
        out[name]["_total"] = round(sum(v[0] for v in prof.values()) / a.reps, 4)
        out[name]["_wall_ms"] = round(wall, 4)  # the call's wall time, kernels unprofiled (side streams overlap)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
