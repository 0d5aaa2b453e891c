"""Record real engine partials for the CPU multi-rank test (tests/test_distributed_cpu.py).

Runs on the GPU box: each synthetic fixture set (tests/golden/synth/<name>.npz) is cut into
`world` cell-disjoint shards (distributed.shard_bounds); for every shard the engine's
cell rows and [n_gene_ids, SCT_NP] gene partials (sct_cell_metrics_gene_partials) are saved,
with the unsharded partials and the GPU-finalized gene rows.  The npz files go to
gpurun_out/partials/ and are committed under tests/golden/partials/.

    python tools/make_partials_fixture.py [world]
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import helpers as H  # noqa: E402
from sctools_amd import distributed as D  # noqa: E402
from sctools_amd import engine as E  # noqa: E402


def main():
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    out_dir = os.path.join(ROOT, "gpurun_out", "partials")
    os.makedirs(out_dir, exist_ok=True)
    eng = E.get_engine("cuda:0")
    for name in ("s0", "s1", "s2"):
        s = H.synth(name)
        d = E.Dims(*s.dims)
        cols = E.to_device(s.arrays, eng.device)
        gm = torch.from_numpy(s.gene_is_mito).to(eng.device)
        _, _, whole = eng.cell_and_gene(cols, d, gm)
        whole = whole.clone()
        gi, gf = eng.finalize_partials(whole.clone())
        rec = {"whole": whole.cpu().numpy(), "gi": gi.cpu().numpy(), "gf": gf.cpu().numpy()}
        bounds = D.shard_bounds(cols["cell"], world)
        rec["bounds"] = np.array(bounds, dtype=np.int64)
        for r, (lo, hi) in enumerate(bounds):
            ci, cf, p = eng.cell_and_gene(D.shard(cols, lo, hi), d, gm)
            rec["ci%d" % r] = ci.cpu().numpy()
            rec["cf%d" % r] = cf.cpu().numpy()
            rec["part%d" % r] = p.cpu().numpy()
        path = os.path.join(out_dir, "%s_ws%d.npz" % (name, world))
        np.savez_compressed(path, **rec)
        print(path, os.path.getsize(path))


if __name__ == "__main__":
    main()
