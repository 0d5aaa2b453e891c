"""
Multi-GPU cell + gene metrics: one process per GPU, cells sharded across ranks.

The reference scales this path by splitting the BAM into cell-disjoint chunks
(``SplitBam``, ``/root/reference/src/sctools/bam.py:361-488``), running the
gatherer on each chunk and merging the CSVs (``MergeCellMetrics`` concatenates,
``metrics/merge.py:59-71``; ``MergeGeneMetrics`` folds, ``metrics/merge.py:74-191``).  Here the same
invariant -- no cell spans two shards -- gives:

* cell rows: each rank's rows are final; rank order = record order, so the
  rows are gathered to one rank and concatenated (the MergeCellMetrics step);
* gene rows: each rank produces additive per-gene partial rows (int64 counters
  and exact-sum lanes, ``include/sctools_gpu.h`` SCT_NP layout).  Because
  molecules, fragments and cells of a gene are keyed by cell, distinct counts
  of disjoint cell sets add; so ONE all-reduce(SUM) of the [n_gene_ids, 64]
  int64 block followed by the finalize kernel gives exactly the unsharded gene
  rows (the MergeGeneMetrics step, without its weighted-mean approximation).

The all-reduce is the only data-path collective (RCCL over xGMI with the
``nccl`` backend; the CPU tests drive the same code with ``gloo``).
"""

from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

from sctools_amd import _native as N


def shard_bounds(entity, world: int) -> List[Tuple[int, int]]:
    """Split records [0, n) into ``world`` contiguous ranges, balanced by record count,
    cutting only at entity-run boundaries (a run never spans two ranges)."""
    if world < 1:
        raise ValueError("world must be >= 1")
    e = entity if isinstance(entity, torch.Tensor) else torch.as_tensor(np.asarray(entity))
    n = int(e.numel())
    if n == 0:
        return [(0, 0)] * world
    heads = (torch.nonzero(e[1:] != e[:-1]).flatten() + 1).cpu()
    cuts = [0]
    for r in range(1, world):
        t = (n * r + world - 1) // world
        j = int(torch.searchsorted(heads, torch.tensor([t], dtype=heads.dtype)).item())
        c = int(heads[j].item()) if j < heads.numel() else n
        cuts.append(max(c, cuts[-1]))
    cuts.append(n)
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def balanced_cell_bins(cell_counts, world: int) -> np.ndarray:
    """Cell id -> bin (uint8) for the cell-bin exchange: contiguous cell-id (barcode) ranges balanced
    by record count, so bin order is barcode order and a few large cells cannot land together in
    one bin of an equal-id-range split.  A cell goes to the bin that holds the midpoint of its
    records in the cumulative count (non-decreasing in the cell id)."""
    if not 1 <= world <= 256:
        raise ValueError("world must be in [1, 256]")
    c = np.asarray(cell_counts, dtype=np.int64)
    total = int(c.sum())
    if total == 0 or world == 1:
        return np.zeros(max(1, c.shape[0]), np.uint8)
    mid2 = 2 * (np.cumsum(c) - c) + c  # twice the midpoint of each cell's records
    b = (mid2 * world) // (2 * total)
    return np.minimum(b, world - 1).astype(np.uint8)


def shard(cols, lo: int, hi: int):
    """The record range [lo, hi) of every column (contiguous views)."""
    return {k: v[lo:hi] for k, v in cols.items()}


def allreduce_partials(partials: torch.Tensor, group=None) -> torch.Tensor:
    """Sum the per-gene partial rows of every rank in place (int64: exact, order-free)."""
    if partials.dtype != torch.int64:
        raise TypeError("partials must be int64")
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(partials, op=dist.ReduceOp.SUM, group=group)
    return partials


def pack_rows(cols: dict, tiebreak: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, list]:
    """Records as one row-major int32 buffer [n, W / 4]: every column's bytes side by side (the 32-byte
    record of SURVEY.md 8(d), + 4 bytes of tiebreak), so a bin moves in ONE collective.  Returns the
    buffer and the layout (name, dtype, byte offset, bytes) for unpack_rows."""
    names = list(cols) + (["_tie"] if tiebreak is not None else [])
    ts = [cols[c] for c in cols] + ([tiebreak] if tiebreak is not None else [])
    n = int(ts[0].numel()) if ts else 0
    layout, parts, off = [], [], 0
    for name, t in zip(names, ts):
        w = t.element_size()
        parts.append(t.contiguous().view(torch.uint8).view(n, w))
        layout.append((name, t.dtype, off, w))
        off += w
    pad = (-off) % 4
    if pad:
        parts.append(torch.zeros((n, pad), dtype=torch.uint8, device=ts[0].device))
    rows = torch.cat(parts, dim=1) if parts else torch.zeros((0, 4), dtype=torch.uint8)
    return rows.view(torch.int32), layout


def unpack_rows(rows: torch.Tensor, layout) -> Tuple[dict, Optional[torch.Tensor]]:
    """pack_rows' inverse: (columns, tiebreak or None), each a fresh contiguous tensor."""
    n = int(rows.shape[0])
    b = rows.contiguous().view(torch.uint8).view(n, -1)
    cols, tie = {}, None
    for name, dt, off, w in layout:
        t = b[:, off:off + w].contiguous().view(dt).view(n)
        if name == "_tie":
            tie = t
        else:
            cols[name] = t
    return cols, tie


def exchange_records(binned: dict, tiebreak: Optional[torch.Tensor], counts: torch.Tensor,
                     group=None) -> Tuple[dict, Optional[torch.Tensor], List[int]]:
    """The cell-bin swap between ranks (SplitBam's bins, bam.py:439-480, as a collective): bin p of
    this rank's ``binned`` columns (``counts[p]`` records, bins consecutive in bin order, as
    ``Engine.bin_records`` lays them out) goes to rank p; this rank receives rank 0's bin for it,
    then rank 1's, ... -- file order when rank r holds the r-th part of the file.  One all_to_all of
    the counts, then ONE of the records packed as rows (pack_rows: the 32-byte record + the 4-byte
    tiebreak; RCCL with the ``nccl`` backend, gloo on CPU).
    Returns (columns, tiebreak or None, received counts per source rank)."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if counts.numel() != world:
        raise ValueError("%d bin counts for %d ranks" % (counts.numel(), world))
    if world == 1:
        return dict(binned), tiebreak, [int(counts[0].item())]
    # gloo moves host tensors only: device columns travel through host memory there
    host = dist.get_backend(group) == "gloo" and counts.device.type != "cpu"
    dev = counts.device

    def io(t):
        return t.cpu() if host else t

    send = io(counts.to(torch.int64))
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send, group=group)
    send_l, recv_l = send.tolist(), recv.tolist()
    total = int(sum(recv_l))
    rows, layout = pack_rows(binned, tiebreak)
    src = io(rows)
    out = torch.empty((total, src.shape[1]), dtype=src.dtype, device=src.device)
    dist.all_to_all_single(out, src, output_split_sizes=recv_l, input_split_sizes=send_l, group=group)
    del rows, src
    cols, tie = unpack_rows(out.to(dev) if host else out, layout)
    return cols, tie, [int(x) for x in recv_l]


def gather_rows(tensors: Sequence[torch.Tensor], dst: int = 0, group=None) -> Optional[List[torch.Tensor]]:
    """Concatenate each [rows_r, k] tensor over ranks in rank order; result on ``dst`` only."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return list(tensors)
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = tensors[0].device
    cnt = torch.tensor([tensors[0].shape[0]], dtype=torch.int64, device=dev)
    counts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(counts, cnt, group=group)
    counts = [int(c.item()) for c in counts]
    top = max(max(counts), 1)
    out = []
    for t in tensors:
        pad = torch.zeros((top,) + tuple(t.shape[1:]), dtype=t.dtype, device=dev)
        pad[: t.shape[0]] = t
        bufs = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(bufs, pad, group=group)
        out.append(torch.cat([b[:c] for b, c in zip(bufs, counts)]) if rank == dst else None)
    return out if rank == dst else None


class ShardedCellGeneMetrics:
    """Cell rows + grouped gene rows of a cell-sharded record set.

    ``backend`` is the engine (``sctools_amd.engine.Engine``): it provides
    ``cell_and_gene(cols, dims, mito, n_entities=None, partials=None)`` and
    ``finalize_partials(partials)``.  Each rank calls :meth:`run` on its shard.
    """

    def __init__(self, backend, group=None, dst: int = 0):
        self.backend = backend
        self.group = group
        self.dst = dst

    def run(self, shard_cols, dims, gene_is_mito, record_offset: int = 0, partials=None):
        ci, cf, part = self.backend.cell_and_gene(shard_cols, dims, gene_is_mito, partials=partials)
        allreduce_partials(part, self.group)
        gi, gf = self.backend.finalize_partials(part)
        ci = ci.clone()
        ci[:, N.I_ENTITY] += record_offset  # first-record index in the whole record set
        cells = gather_rows([ci, cf], self.dst, self.group)
        return (cells[0], cells[1]) if cells is not None else (None, None), (gi, gf)
