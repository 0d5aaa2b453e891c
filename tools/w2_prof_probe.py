"""Experiments only: the drop-in Welford pass (config 2 or 4) with an engine built with -DSCT_W2_PROF
(SCT_LIB_PATH), then the head kernel's per-wave barrier ticks of the last block to finish."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def main():
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    from sctools_amd import _native as N
    from sctools_amd import engine as E
    from sctools_amd import synth

    dev = torch.device("cuda", 0)
    eng = E.get_engine(dev)
    n, cells = (125_000_000, 62_500) if cfg == 4 else (100_000_000, 10_000)
    data = synth.generate(synth.SynthConfig(n_reads=n, n_cells=cells, n_genes=30_000, sigma=2.0 if cfg == 4 else 1.0,
                                            seed=0), device=dev, chunk=16_000_000)
    dims = E.Dims(data.n_cell_ids, data.n_gene_ids, data.n_umi_ids)
    mito = torch.from_numpy(data.gene_is_mito).to(dev)
    multi = torch.from_numpy(data.gene_is_multi).to(dev)
    n_ent = eng.count_entities(data.cols, "cell", dims)
    lib = N.load()
    for rep in range(3):
        eng.compute(data.cols, "cell", dims, mito, multi, float_mode="welford", n_entities=n_ent)
        torch.cuda.synchronize()
        pr = (ctypes.c_ulonglong * 10)()
        assert lib.sct_debug_w2_prof(pr) == 0
        print("rep %d: " % rep + "  ".join("wave %d %.2f of %.2f ms" % (w, pr[2 * w] / 1e5, pr[2 * w + 1] / 1e5)
                                          for w in range(4)) + "  clock %.0f MHz" % (100.0 * pr[8] / max(pr[1], 1)),
              flush=True)


if __name__ == "__main__":
    main()
