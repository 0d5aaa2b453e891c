"""Cell-sharded multi-rank path (sctools_amd/distributed.py) on CPU with gloo, world_size 2.

The ranks run the REAL engine outputs: ``RecordedBackend`` replays, for the rank's shard,
the cell rows and the [n_gene_ids, SCT_NP] int64 gene partials that the HIP engine produced
on an MI355X for exactly this shard (tools/make_partials_fixture.py ->
tests/golden/partials/<set>_ws2.npz; shards from distributed.shard_bounds).  So the gloo
all-reduce sums the engine's real partial layout -- 20 counters and the 4 x 8 exact-sum lanes
of fixedpt.h -- and the test requires:

* the reduced partials equal the engine's partials of the UNSHARDED records, bit for bit;
* finalizing them on the host (the same fixedpt.h, compiled by g++ in tests/native) gives
  the GPU-finalized gene rows bit for bit, and the oracle's grouped gene rows (integers exact,
  floats within 1e-9);
* the gathered cell rows equal the oracle's cell rows of the whole set (integers exact).
"""
import ctypes
import os
import socket
import subprocess

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import helpers as H
from oracle import oracle as O
from sctools_amd import _native as N
from sctools_amd import distributed as D

HERE = os.path.dirname(os.path.abspath(__file__))
PARTIALS = os.path.join(HERE, "golden", "partials")
FXLIB = os.path.join(HERE, "native", "libfxcheck.so")
ADDITIVE = [i for i in range(N.SCT_NI) if i != N.I_ENTITY]

# partial slot -> output int column (finalize.h k_finalize)
P_TO_I = {0: N.I_N_READS, 1: N.I_PERFECT_UMI, 2: N.I_EXONIC, 3: N.I_INTRONIC, 4: N.I_UTR, 5: N.I_UNIQUE,
          6: N.I_MULTIPLE, 7: N.I_DUP, 8: N.I_SPLICED, 9: N.I_N_MOL, 10: N.I_MOL_SINGLE, 11: N.I_N_FRAG,
          12: N.I_FRAG_SINGLE, 13: N.I_N_K1, 14: N.I_K1_MULTI, 15: N.I_PERFECT_CB, 16: N.I_INTERGENIC,
          17: N.I_UNMAPPED, 18: N.I_MITO_GENES, 19: N.I_MITO_READS}


def fxlib():
    if not os.path.exists(FXLIB):
        subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared", "-o", FXLIB,
                        os.path.join(HERE, "native", "fxcheck.cpp")], check=True)
    lib = ctypes.CDLL(FXLIB)
    lib.fx_finalize_lanes.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_double),
                                      ctypes.POINTER(ctypes.c_double)]
    return lib


def host_finalize_gene(part: np.ndarray):
    """Gene rows from partial rows on the host: k_finalize's mapping, fixedpt.h's finalize."""
    lib = fxlib()
    rows = part.shape[0]
    gi = np.zeros((rows, N.SCT_NI), np.int64)
    gf = np.zeros((rows, N.SCT_NF), np.float64)
    for slot, col in P_TO_I.items():
        gi[:, col] = part[:, slot]
    gi[:, N.I_ENTITY] = np.arange(rows)
    n = part[:, 0]
    with np.errstate(divide="ignore", invalid="ignore"):
        gf[:, N.F_RPM] = np.where(part[:, 9] > 0, n / np.maximum(part[:, 9], 1), np.nan)
        gf[:, N.F_RPF] = np.where(part[:, 11] > 0, n / np.maximum(part[:, 11], 1), np.nan)
        gf[:, N.F_FPM] = np.where(part[:, 9] > 0, part[:, 11] / np.maximum(part[:, 9], 1), np.nan)
    m, v = ctypes.c_double(), ctypes.c_double()
    for r in range(rows):
        for st, (fm, fv) in enumerate(((N.F_UY_MEAN, N.F_UY_VAR), (N.F_GQF_MEAN, N.F_GQF_VAR),
                                       (N.F_GQ_MEAN, N.F_GQ_VAR))):
            lanes = np.ascontiguousarray(part[r, N.SCT_P_FLOAT_BASE + 8 * st: N.SCT_P_FLOAT_BASE + 8 * st + 8])
            lib.fx_finalize_lanes(lanes.ctypes.data, int(n[r]), ctypes.byref(m), ctypes.byref(v))
            gf[r, fm], gf[r, fv] = m.value, v.value
    return gi, gf


class RecordedBackend:
    """The engine's outputs for this rank's shard, recorded on an MI355X."""

    def __init__(self, rec, rank):
        self.rec = rec
        self.rank = rank

    def cell_and_gene(self, cols, dims, gene_is_mito, n_entities=None, partials=None):
        r = self.rank
        return (torch.from_numpy(self.rec["ci%d" % r]), torch.from_numpy(self.rec["cf%d" % r]),
                torch.from_numpy(np.array(self.rec["part%d" % r], copy=True)))

    def finalize_partials(self, part):
        gi, gf = host_finalize_gene(part.numpy())
        return torch.from_numpy(gi), torch.from_numpy(gf)


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
        rec = dict(np.load(os.path.join(PARTIALS, "%s_ws%d.npz" % (name, world))))
        s = H.synth(name)
        cols = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in s.arrays.items()}
        bounds = D.shard_bounds(cols["cell"], world)
        assert np.array_equal(np.array(bounds), rec["bounds"])  # the shards the engine saw
        lo, hi = bounds[rank]
        job = D.ShardedCellGeneMetrics(RecordedBackend(rec, rank))
        (ci, cf), (gi, gf) = job.run(D.shard(cols, lo, hi), None, None, record_offset=lo)
        part = torch.from_numpy(np.ascontiguousarray(rec["part%d" % rank])).clone()
        D.allreduce_partials(part)
        if rank == 0:
            np.savez(os.path.join(outdir, "out.npz"), ci=ci.numpy(), cf=cf.numpy(), gi=gi.numpy(), gf=gf.numpy(),
                     part=part.numpy())
        else:
            assert ci is None and cf is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name", ["s0", "s2"])
def test_two_rank_gloo_real_partials_match_unsharded(tmp_path, name):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), name, str(tmp_path)), nprocs=world, join=True)
    got = np.load(tmp_path / "out.npz")
    rec = np.load(os.path.join(PARTIALS, "%s_ws%d.npz" % (name, world)))
    s = H.synth(name)
    # the all-reduced partials ARE the unsharded partials (every lane, exact-sum lanes included)
    assert np.array_equal(got["part"], rec["whole"])
    # host finalize of the reduced rows == the GPU's finalize of the unsharded partials, bit for bit
    assert np.array_equal(got["gi"], rec["gi"])
    assert np.array_equal(got["gf"].view(np.int64), rec["gf"].view(np.int64))
    # ... and the reference semantics: the oracle's grouped gene rows
    oi, of = O.run(s.arrays, "gene_grouped", s.gene_is_mito, len(s.gene_names))
    live = oi[:, 0] > 0
    assert np.array_equal(got["gi"][live][:, ADDITIVE], oi[live][:, ADDITIVE])
    a, b = got["gf"][live][:, :6], of[live][:, :6]
    assert np.array_equal(np.isnan(a), np.isnan(b))
    ok = np.isnan(a) | (np.abs(a - b) <= 1e-9 * np.maximum(np.abs(a), np.abs(b)))
    assert ok.all()
    # gathered cell rows (the MergeCellMetrics step): the oracle's cell rows of the whole set
    ci, cf = O.run(s.arrays, "cell", s.gene_is_mito, len(s.gene_names))
    assert np.array_equal(got["ci"], ci)
    a, b = got["cf"], cf
    assert np.array_equal(np.isnan(a), np.isnan(b))
    assert (np.isnan(a) | (np.abs(a - b) <= 1e-9 * np.maximum(np.abs(a), np.abs(b)))).all()


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
