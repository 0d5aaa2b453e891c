"""Run by tests/test_gpu_tagsort.py::test_tag_sort_small_radix_tiles in a child process whose
SCT_LIB_PATH is tests/native/libsct_engine_si4.so: the engine built with 1024-item radix tiles.

Round 3 sized the tag sort's digit counts by the 2048-record row tile; radix_sort's tiles were the
same size only by coincidence, and the 1024-item build overflowed them (an illegal memory access in
config 5's (CB, UB, GE, query name) sort).  Here every radix_sort caller of the tag sort runs on that
build: the one-round tiebreak path, the two-round path (keys wider than 64 bits) and the long-tie
path, each against numpy's stable lexsort.  Exit status 0 = all equal.
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sctools_amd import _native as N  # noqa: E402
from sctools_amd import engine as E  # noqa: E402
from sctools_amd import synth  # noqa: E402

assert os.path.basename(N.LIB_PATH) == "libsct_engine_si4.so", N.LIB_PATH


def host(cols):
    out = {c: t.cpu().numpy() for c, t in cols.items()}
    for c in ("gq_sum", "gq_len", "gq_gt30"):
        out[c] = out[c].view(np.uint16)
    return out


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
    eng = E.get_engine("cuda:0")
    d = synth.generate(synth.SynthConfig(n_reads=n, n_cells=500, n_genes=3000, seed=21), device="cpu")
    arrays = host(d.cols)
    perm = np.random.default_rng(21).permutation(n)
    arrays = {c: np.ascontiguousarray(a[perm]) for c, a in arrays.items()}
    rng = np.random.default_rng(22)
    # long runs of equal (CB, UB, GE) for the compact (run, name) sort
    for L in (17, 300, 5000):
        idx = rng.choice(n, size=L, replace=False)
        for c in ("cell", "umi", "gene"):
            arrays[c][idx] = arrays[c][idx[0]]
    tie = rng.integers(0, 50_000, n).astype(np.int32)
    cases = [("one round + ties", E.Dims(d.n_cell_ids, d.n_gene_ids, d.n_umi_ids)),
             ("two rounds", E.Dims(1 << 28, 1 << 30, 1 << 30))]
    dev = {c: torch.from_numpy(a).to(eng.device) for c, a in arrays.items()}
    idx = np.lexsort((tie, arrays["gene"], arrays["umi"], arrays["cell"]))
    for name, dims in cases:
        out = host(eng.tag_sort(dev, dims, "cell_umi_gene", torch.from_numpy(tie).to(eng.device), 50_000))
        for c in N.RECORD_COLUMNS:
            assert np.array_equal(out[c], arrays[c][idx]), (name, c)
        print("si4 %s: %d records equal numpy's lexsort" % (name, n))
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
