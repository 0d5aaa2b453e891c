"""Cell-sharded multi-rank path (sctools_amd/distributed.py) on CPU with gloo, world_size 2.

The engine needs a GPU, so the ranks use a test double backed by the oracle:
``cell_and_gene`` returns the oracle's cell rows of the shard and, as the
"partials", the oracle's grouped gene integer columns of the shard scattered
into [n_gene_ids, 64] int64 rows.  Those columns are exactly the additive
counters of the real partial rows, so after the all-reduce they must equal
the oracle on the unsharded records -- the property the RCCL path relies on.
(The exact-sum float lanes' additivity is checked on the GPU in
tests/test_gpu_parity.py::test_sharded_partials_add_up.)
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import helpers as H
from oracle import oracle as O
from sctools_amd import _native as N
from sctools_amd import distributed as D

ADDITIVE = [i for i in range(N.SCT_NI) if i != N.I_ENTITY]


class OracleBackend:
    def __init__(self, n_gene_ids, mito):
        self.n_gene_ids = n_gene_ids
        self.mito = mito

    def cell_and_gene(self, cols, dims, gene_is_mito, n_entities=None, partials=None):
        arrays = {k: v.numpy() for k, v in cols.items()}
        ci, cf = O.run(arrays, "cell", self.mito, self.n_gene_ids)
        gi, _ = O.run(arrays, "gene_grouped", self.mito, self.n_gene_ids)
        part = torch.zeros((self.n_gene_ids, N.SCT_NP), dtype=torch.int64)
        g = torch.from_numpy(gi[:, N.I_ENTITY])
        part[g, : N.SCT_NI] = torch.from_numpy(gi)
        part[:, N.I_ENTITY] = 0
        return torch.from_numpy(ci), torch.from_numpy(cf), part

    def finalize_partials(self, part):
        ints = part[:, : N.SCT_NI].clone()
        ints[:, N.I_ENTITY] = torch.arange(part.shape[0])
        return ints, torch.zeros((part.shape[0], N.SCT_NF), dtype=torch.float64)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, name, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        s = H.synth(name)
        cols = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in s.arrays.items()}
        bounds = D.shard_bounds(cols["cell"], world)
        lo, hi = bounds[rank]
        job = D.ShardedCellGeneMetrics(OracleBackend(len(s.gene_names), s.gene_is_mito))
        (ci, cf), (gi, _) = job.run(D.shard(cols, lo, hi), None, None, record_offset=lo)
        if rank == 0:
            np.savez(os.path.join(outdir, "out.npz"), ci=ci.numpy(), cf=cf.numpy(), gi=gi.numpy(),
                     bounds=np.array(bounds))
        else:
            assert ci is None and cf is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name", ["s0", "s2"])
def test_two_rank_gloo_matches_unsharded(tmp_path, name):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), name, str(tmp_path)), nprocs=world, join=True)
    got = np.load(tmp_path / "out.npz")
    s = H.synth(name)
    ci, cf = O.run(s.arrays, "cell", s.gene_is_mito, len(s.gene_names))
    assert np.array_equal(got["ci"], ci)
    assert np.array_equal(got["cf"].view(np.int64), cf.view(np.int64))
    gi, _ = O.run(s.arrays, "gene_grouped", s.gene_is_mito, len(s.gene_names))
    dense = np.zeros((len(s.gene_names), N.SCT_NI), dtype=np.int64)
    dense[gi[:, N.I_ENTITY]] = gi
    assert np.array_equal(got["gi"][:, ADDITIVE], dense[:, ADDITIVE])
    b = got["bounds"]
    assert b[0][0] == 0 and b[-1][1] == len(s.arrays["cell"]) and b[0][1] == b[1][0]


def test_shard_bounds_cut_at_runs():
    e = np.array([0, 0, 0, 1, 1, 2, 2, 2, 2, 3], dtype=np.int32)
    assert D.shard_bounds(e, 1) == [(0, 10)]
    assert D.shard_bounds(e, 2) == [(0, 5), (5, 10)]
    b = D.shard_bounds(e, 4)
    assert b[0][0] == 0 and b[-1][1] == 10
    heads = {0, 3, 5, 9, 10}
    assert all(lo in heads and hi in heads and lo <= hi for lo, hi in b)
    # one giant run: everything lands on the first rank, others are empty
    assert D.shard_bounds(np.zeros(7, dtype=np.int32), 3) == [(0, 7), (7, 7), (7, 7)]
    assert D.shard_bounds(np.zeros(0, dtype=np.int32), 2) == [(0, 0), (0, 0)]
