"""Workload for a rocprofv3 --kernel-trace of the drop-in default (Welford cell rows, bench.py's
side measurement) at config 2: when does each kernel of one call start and end (the Welford stage
runs on a side stream beside the bucket partition).  Run as
  rocprofv3 --kernel-trace --output-format csv -d OUT -o dropin -- python3 tools/dropin_probe.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    from sctools_amd import engine as E
    from sctools_amd import synth

    dev = torch.device("cuda", 0)
    eng = E.get_engine(dev)
    cfg = synth.SynthConfig(n_reads=100_000_000, n_cells=10_000, n_genes=30_000, sigma=1.0, seed=0)
    data = synth.generate(cfg, device=dev, chunk=16_000_000)
    dims = E.Dims(data.n_cell_ids, data.n_gene_ids, data.n_umi_ids)
    mito = torch.from_numpy(data.gene_is_mito).to(dev)
    multi = torch.zeros_like(mito)
    n_ent = eng.count_entities(data.cols, "cell", dims)
    for i in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.compute(data.cols, "cell", dims, mito, multi, float_mode="welford", n_entities=n_ent)
        torch.cuda.synchronize()
        print("call %d: %.2f ms" % (i, (time.perf_counter() - t0) * 1e3), flush=True)


if __name__ == "__main__":
    main()
