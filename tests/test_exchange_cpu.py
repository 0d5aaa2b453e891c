"""The cell-bin exchange for unsorted input (sctools_amd/distributed.exchange_records) on CPU with
gloo, world_size 2 and 3.

The reference's route for an unsorted BAM is SplitBam (barcode -> bin, bam.py:439-448; the pieces
of a bin merged, 454-480) + TagSortBam per chunk (platform.py:55-97) + Calculate*Metrics.  Here
rank r holds the r-th contiguous part of a shuffled record set, bins it by cell (contiguous
barcode-rank ranges: ``bin_of`` below restates sct_bin_records' rule, which the GPU tests check
against the kernel), and the ranks swap bins.  The test requires:

* every rank receives exactly the records of its cells, in global file order (the stable bins
  received in rank order);
* sorting them by (CB, UB, GE, query name) and running the oracle per rank, then concatenating the
  ranks' cell rows, gives the oracle's cell rows of the whole set sorted once -- integers AND
  Welford floats bit for bit (the order inside every cell is the single-process order).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle as O
from sctools_amd import _native as N
from sctools_amd import distributed as D
from sctools_amd import synth


def bin_of(cell: np.ndarray, n_bins: int, n_cell_ids: int) -> np.ndarray:
    """sct_bin_records' default bins: contiguous cell-id ranges, cell * n_bins / n_cell_ids."""
    return (cell.astype(np.int64) * n_bins) // n_cell_ids


def shuffled_set(seed=5, n=60_000):
    cfg = synth.SynthConfig(n_reads=n, n_cells=37, n_genes=400, seed=seed, p_secondary=0.1, p_nh1=0.7, p_dup=0.4,
                            p_none_cell_reads=0.01)
    d = synth.generate(cfg, device="cpu")
    perm = np.random.default_rng(seed).permutation(n)
    cols = {c: t.numpy()[perm] for c, t in d.cols.items()}
    for c in ("gq_sum", "gq_len", "gq_gt30"):
        cols[c] = cols[c].view(np.uint16)
    qname = d.extra["qname"].numpy()[perm]
    return cols, qname, d


def sort_tag_order(cols, qname):
    order = np.lexsort((qname, cols["gene"], cols["umi"], cols["cell"]))  # stable, as sorted()
    return {c: a[order] for c, a in cols.items()}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, balanced=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cols, qname, d = shuffled_set()
        n = cols["cell"].shape[0]
        lo, hi = n * rank // world, n * (rank + 1) // world
        part = {c: a[lo:hi] for c, a in cols.items()}
        if balanced:  # record-balanced barcode ranges (multigpu.sorted_cell_and_gene_rows' table)
            table = D.balanced_cell_bins(np.bincount(cols["cell"], minlength=d.n_cell_ids), world)
            bin_of_w = (lambda c, nb, nc: table[c].astype(np.int64))  # noqa: E731
        else:
            bin_of_w = bin_of
        b = bin_of_w(part["cell"], world, d.n_cell_ids)
        order = np.argsort(b, kind="stable")
        binned = {c: torch.from_numpy(np.ascontiguousarray(a[order].view(np.int16) if a.dtype == np.uint16
                                                            else a[order])) for c, a in part.items()}
        tie = torch.from_numpy(np.ascontiguousarray(qname[lo:hi][order]))
        counts = torch.from_numpy(np.bincount(b, minlength=world).astype(np.int64))
        calls = []
        a2a = dist.all_to_all_single

        def counted(*a, **k):
            calls.append(1)
            return a2a(*a, **k)

        dist.all_to_all_single = counted
        try:
            got, gtie, recv = D.exchange_records(binned, tie, counts)
        finally:
            dist.all_to_all_single = a2a
        assert len(calls) == 2, "one collective for the counts, ONE for the packed records"
        mine = {c: (t.numpy().view(np.uint16) if t.dtype == torch.int16 else t.numpy()) for c, t in got.items()}
        # every record of this rank's cells, in global file order
        want = bin_of_w(cols["cell"], world, d.n_cell_ids) == rank
        for c in cols:
            assert np.array_equal(mine[c], cols[c][want]), c
        assert np.array_equal(gtie.numpy(), qname[want])
        assert sum(recv) == int(want.sum())
        # the rank's cells sorted and measured: rows of the whole set, in rank order
        srt = sort_tag_order(mine, gtie.numpy())
        ints, floats = O.run(srt, "cell", d.gene_is_mito, d.n_gene_ids)
        q.put((rank, ints, floats))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,balanced", [(2, False), (3, False), (3, True)])
def test_exchange_then_sort_equals_one_process(world, balanced):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, balanced)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    import queue
    import time

    deadline = time.monotonic() + 240
    while len(got) < world:
        try:
            r, ints, floats = q.get(timeout=1)
            got[r] = (ints, floats)
        except queue.Empty:
            assert not any(p.exitcode not in (None, 0) for p in procs), "a rank failed"
            assert time.monotonic() < deadline, "timed out"
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    cols, qname, d = shuffled_set()
    wi, wf = O.run(sort_tag_order(cols, qname), "cell", d.gene_is_mito, d.n_gene_ids)
    gi = np.concatenate([got[r][0] for r in range(world)])
    gf = np.concatenate([got[r][1] for r in range(world)])
    assert gi.shape == wi.shape
    cols_i = [i for i in range(N.SCT_NI) if i != N.I_ENTITY]  # (first-record index: per rank)
    assert np.array_equal(gi[:, cols_i], wi[:, cols_i])
    assert np.array_equal(np.nan_to_num(gf, nan=-1.0), np.nan_to_num(wf, nan=-1.0))


def test_exchange_one_rank_is_identity():
    binned = {"cell": torch.arange(5, dtype=torch.int32)}
    got, tie, recv = D.exchange_records(binned, None, torch.tensor([5]))
    assert got["cell"] is binned["cell"] and tie is None and recv == [5]


def test_pack_rows_round_trip():
    """The exchange's packed rows: the 32-byte record (+ 4-byte tiebreak) per row, unpacked bit for bit."""
    cols, qname, _ = shuffled_set(n=5000)
    t = {c: torch.from_numpy(np.ascontiguousarray(a.view(np.int16) if a.dtype == np.uint16 else a))
         for c, a in cols.items()}
    tie = torch.from_numpy(np.ascontiguousarray(qname))
    rows, layout = D.pack_rows(t, tie)
    assert rows.dtype == torch.int32 and tuple(rows.shape) == (5000, 9)
    got, gtie = D.unpack_rows(rows, layout)
    assert list(got) == list(t)
    for c in t:
        assert got[c].dtype == t[c].dtype and torch.equal(got[c], t[c]), c
    assert torch.equal(gtie, tie)
    rows, layout = D.pack_rows(t, None)
    assert tuple(rows.shape) == (5000, 8)
    got, gtie = D.unpack_rows(rows, layout)
    assert gtie is None and all(torch.equal(got[c], t[c]) for c in t)


def test_balanced_cell_bins():
    """Record-balanced barcode ranges: non-decreasing in the cell id (rank order = barcode order), every
    bin used when the counts allow, and far better balanced than equal id ranges on skewed cells."""
    rng = np.random.default_rng(3)
    counts = np.sort(rng.lognormal(0, 2.0, 5000)).astype(np.int64)[::-1].copy()  # big cells first
    counts[0] = 0  # (the missing-CB id may be empty)
    for world in (1, 2, 3, 8, 64):
        b = D.balanced_cell_bins(counts, world)
        assert b.dtype == np.uint8 and b.shape == counts.shape
        assert np.all(np.diff(b.astype(int)) >= 0) and b.max() < world
        load = np.bincount(b, weights=counts, minlength=world)
        ideal = counts.sum() / world
        assert load.max() <= ideal + counts.max(), (world, load.max(), ideal)
        if world > 1:
            naive = np.bincount((np.arange(counts.size) * world) // counts.size, weights=counts, minlength=world)
            assert load.max() < naive.max()
    assert D.balanced_cell_bins(np.zeros(4, np.int64), 4).tolist() == [0, 0, 0, 0]
