"""
Several GPUs behind the ``sctools.metrics`` drop-in: one host thread per device.

The reference scales the metric path by splitting a BAM into cell-disjoint chunks
(``SplitBam``, ``/root/reference/src/sctools/bam.py:361-488``; CLI ``platform.py:153-223``),
running ``Calculate*Metrics`` on each chunk and merging the CSVs (``MergeCellMetrics``
concatenates, ``MergeGeneMetrics`` folds, ``metrics/merge.py:59-191``).  Here the file is
decoded once on the host -- so the cell / gene / umi dictionaries are global -- and:

* RUN-mode rows (``GatherCellMetrics`` on a cell-sorted file, ``GatherGeneMetrics`` on a
  gene-sorted one): the records are cut at entity-run boundaries into contiguous ranges
  balanced by record count (``distributed.shard_bounds``); each device computes the rows of
  its range; rows are concatenated in range order, which is file order.  No collective is
  needed: an entity never spans two ranges.
* Gene rows of a cell-sorted file (what ``TagSortBam`` by (GE, CB, UB) followed by
  ``GatherGeneMetrics`` gives, or SplitBam + per-chunk gene metrics + ``MergeGeneMetrics``):
  each device turns its cell range into additive per-gene partial rows, ONE in-place
  RCCL all-reduce over xGMI (``sct_allreduce_gene_partials`` on communicators from
  ``sct_comm_init_all``) sums them, and the finalize kernel turns the sum into gene rows --
  exactly the rows of the unsharded file (exact-sum floats).

The threads only issue work: H2D copies, C-ABI calls and the collective all release the GIL.
"""

import ctypes
import os
import threading
import time
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np
import torch

from sctools_amd import _native as N
from sctools_amd import columnar
from sctools_amd import distributed as D

# bound on the wait for the other ranks at the collective and for its completion (seconds)
COLLECTIVE_TIMEOUT_S = float(os.environ.get("SCT_COLLECTIVE_TIMEOUT_S", "600"))


def parse_devices(devices) -> List[int]:
    """``devices``: an int N (devices 0..N-1) or a sequence of device indices, one per shard (a
    device may be listed more than once: several shards on one device)."""
    if isinstance(devices, int):
        if devices < 1:
            raise ValueError("devices must be >= 1")
        return list(range(devices))
    out = [int(d) for d in devices]
    if not out or min(out) < 0:
        raise ValueError("devices must be device indices")
    return out


class GroupAborted(RuntimeError):
    """Raised in a rank whose peers failed: the collective was skipped or cancelled."""


class GroupRun:
    """One call of ``fn(rank)`` on every rank, each in its own thread, with a failure protocol for the
    one collective of the call (the gene-partial all-reduce):

    * ``before_collective(rank)``: every rank waits here until all ranks arrive (bounded by
      ``timeout``).  If a rank failed before arriving, the others raise :class:`GroupAborted`
      instead of issuing a collective whose peers never come;
    * ``wait(rank, done)``: polls ``done()`` (the collective's completion) until it is true, a rank
      failed (:class:`GroupAborted`) or the timeout passes (``TimeoutError``);
    * a failing rank calls ``abort_fn`` once (``ncclCommAbort`` on every communicator), which
      cancels collectives already in flight on the device.

    ``run`` re-raises the first rank's own error; the :class:`GroupAborted` of its peers only if no
    rank has another error."""

    def __init__(self, size: int, abort_fn: Optional[Callable[[], None]] = None,
                 timeout: float = COLLECTIVE_TIMEOUT_S):
        self.size = size
        self.timeout = timeout
        self._abort_fn = abort_fn
        self._barrier = threading.Barrier(size)
        self._failed = threading.Event()
        self._lock = threading.Lock()
        self.aborted = False

    def fail(self) -> None:
        with self._lock:
            if self._failed.is_set():
                return
            self._failed.set()
            self._barrier.abort()
            if self._abort_fn is not None:
                self._abort_fn()
                self.aborted = True

    def before_collective(self, rank: int) -> None:
        if self._failed.is_set():
            raise GroupAborted("rank %d: another rank failed before the collective" % rank)
        try:
            self._barrier.wait(self.timeout)
        except threading.BrokenBarrierError:
            if self._failed.is_set():
                raise GroupAborted("rank %d: another rank failed before the collective" % rank) from None
            self.fail()
            raise TimeoutError("rank %d: the other ranks did not reach the collective within %.0f s"
                               % (rank, self.timeout)) from None

    def wait(self, rank: int, done: Callable[[], bool]) -> None:
        deadline = time.monotonic() + self.timeout
        while not done():
            if self._failed.is_set():
                raise GroupAborted("rank %d: another rank failed during the collective" % rank)
            if time.monotonic() > deadline:
                self.fail()
                raise TimeoutError("rank %d: the collective did not complete within %.0f s" % (rank, self.timeout))
            time.sleep(0.0005)

    def run(self, fn: Callable[[int], object], setup: Optional[Callable[[int], object]] = None) -> List[object]:
        out: List[object] = [None] * self.size
        errs: List[Optional[BaseException]] = [None] * self.size

        def work(r):
            try:
                if setup is not None:
                    with setup(r):
                        out[r] = fn(r)
                else:
                    out[r] = fn(r)
            except BaseException as e:  # re-raised on the caller's thread
                errs[r] = e
                self.fail()

        threads = [threading.Thread(target=work, args=(r,)) for r in range(self.size)]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
        first = next((e for e in errs if e is not None and not isinstance(e, GroupAborted)), None)
        if first is None:
            first = next((e for e in errs if e is not None), None)
        if first is not None:
            raise first
        return out


class DeviceGroup:
    """Engines on several devices, one worker thread per shard, RCCL communicators on demand.

    Shards listed on one device (``devices=[0, 0]``) share its engine and sum their partials in
    device memory instead of over RCCL (an RCCL communicator holds one rank per device)."""

    def __init__(self, devices):
        from sctools_amd import engine as E

        self.devices = parse_devices(devices)
        if not torch.cuda.is_available():
            raise RuntimeError("sctools_amd needs ROCm GPUs; there is no CPU fallback")
        if max(self.devices) >= torch.cuda.device_count():
            raise ValueError("device %d requested, %d visible" % (max(self.devices), torch.cuda.device_count()))
        self.shared = len(set(self.devices)) != len(self.devices)
        # shards sharing a device get an engine (a workspace) each: their threads run concurrently
        self.engines = [E.Engine(torch.device("cuda", d)) if self.shared else E.get_engine(torch.device("cuda", d))
                        for d in self.devices]
        self.lib = N.load()
        self._comms: Optional[ctypes.Array] = None
        self._aborted = False  # communicators aborted: never re-created (a late rank would hang on them)
        self._run: Optional[GroupRun] = None
        self._slots: List[Optional[torch.Tensor]] = [None] * len(self.devices)

    @property
    def size(self) -> int:
        return len(self.devices)

    def run(self, fn: Callable[[int], object]) -> List[object]:
        """fn(rank) on every rank, each in its own thread with its device current.  If a rank raises,
        the group's collective is skipped (or aborted) on every rank and the error is re-raised here."""
        self._run = GroupRun(self.size, abort_fn=self.abort)
        self._slots = [None] * self.size
        self._xslots = [None] * self.size
        try:
            return self._run.run(fn, setup=lambda r: torch.cuda.device(self.devices[r]))
        finally:
            self._run = None

    def comms(self) -> Optional[ctypes.Array]:
        """The group's communicators (ncclCommInitAll; none for shards sharing a device); create them
        on the caller's thread before the ranks' threads use them."""
        if self.shared:
            return None
        if self._aborted:
            raise GroupAborted("the group's communicators were aborted after a rank failed")
        if self._comms is None:
            comms = (ctypes.c_void_p * self.size)()
            devs = (ctypes.c_int * self.size)(*self.devices)
            N.check(self.lib.sct_comm_init_all(comms, self.size, devs))
            self._comms = comms
        return self._comms

    def _rank_comm(self, rank: int) -> int:
        """A rank thread's communicator: created beforehand on the caller's thread (comms()); never
        created here, so a rank that arrives after an abort raises instead of re-initialising."""
        comms = self._comms
        if comms is None:
            if self._aborted:
                raise GroupAborted("the group's communicators were aborted after a rank failed")
            raise RuntimeError("DeviceGroup.comms() must be called before the ranks run")
        return comms[rank]

    def allreduce_partials(self, rank: int, partials: torch.Tensor) -> None:
        """In-place sum of every rank's [rows, SCT_NP] int64 partials (call from every rank's thread,
        inside run()).  Returns once the sum is complete on this rank's stream."""
        if partials.dtype != torch.int64 or not partials.is_contiguous():
            raise TypeError("partials must be contiguous int64")
        g = self._run
        if g is None:
            raise RuntimeError("allreduce_partials is called from the ranks of DeviceGroup.run")
        g.before_collective(rank)
        stream = torch.cuda.current_stream(partials.device)
        if self.shared:
            self._local_sum(rank, partials)
            return
        N.check(self.lib.sct_allreduce_gene_partials(ctypes.c_void_p(partials.data_ptr()), int(partials.shape[0]),
                                                     ctypes.c_void_p(self._rank_comm(rank)),
                                                     ctypes.c_void_p(stream.cuda_stream)))
        done = torch.cuda.Event()
        done.record(stream)
        g.wait(rank, done.query)

    def _local_sum(self, rank: int, partials: torch.Tensor) -> None:
        """Shards on shared devices: every rank's partials become the sum of all (device memory)."""
        g = self._run
        torch.cuda.current_stream(partials.device).synchronize()
        self._slots[rank] = partials
        g.before_collective(rank)  # every slot filled
        if rank == 0:
            tot = self._slots[0].clone()
            for t in self._slots[1:]:
                tot += t.to(tot.device)
            torch.cuda.current_stream(tot.device).synchronize()
            self._slots = [tot] + [None] * (self.size - 1)
        g.before_collective(rank)  # the sum is ready
        partials.copy_(self._slots[0].to(partials.device))
        torch.cuda.current_stream(partials.device).synchronize()
        g.before_collective(rank)  # every rank has copied it
        if rank == 0:
            self._slots = [None] * self.size

    def exchange(self, rank: int, binned: dict, tiebreak: Optional[torch.Tensor], counts: torch.Tensor):
        """The cell-bin swap (call from every rank's thread, inside run()): bin p of every rank's
        ``binned`` records (``counts``: device int64 [size], Engine.bin_records) goes to rank p; each rank
        receives its bin of rank 0, then of rank 1, ... -- file order when rank r holds the r-th part of
        the file.  RCCL send / recv (sct_exchange_records); shards sharing a device copy in device
        memory.  Returns (columns, tiebreak or None) on the rank's device."""
        g = self._run
        if g is None:
            raise RuntimeError("exchange is called from the ranks of DeviceGroup.run")
        if counts.numel() != self.size:
            raise ValueError("%d bin counts for %d ranks" % (counts.numel(), self.size))
        g.before_collective(rank)
        eng = self.engines[rank]
        stream = torch.cuda.current_stream(eng.device)
        if self.shared:
            return self._local_exchange(rank, binned, tiebreak, counts)
        comm = self._rank_comm(rank)
        recv = eng.exchange_counts(counts, comm)
        done = torch.cuda.Event()
        done.record(stream)
        g.wait(rank, done.query)  # (a peer that failed never sends: no blocking read before this)
        send_h, recv_h = counts.cpu().tolist(), recv.cpu().tolist()
        out = eng.exchange_records(binned, tiebreak, send_h, recv_h, comm)
        done = torch.cuda.Event()
        done.record(stream)
        g.wait(rank, done.query)
        return out

    def _local_exchange(self, rank: int, binned: dict, tiebreak, counts):
        """Shards on shared devices: the same swap by device copies."""
        g = self._run
        dev = self.engines[rank].device
        torch.cuda.current_stream(dev).synchronize()
        self._xslots[rank] = (binned, tiebreak, counts.cpu().tolist())
        g.before_collective(rank)  # every rank's bins are ready
        cols, ties = {c: [] for c in binned}, []
        for p in range(self.size):
            b, t, cnt = self._xslots[p]
            lo = int(sum(cnt[:rank]))
            hi = lo + int(cnt[rank])
            for c in cols:
                cols[c].append(b[c][lo:hi].to(dev))
            if t is not None:
                ties.append(t[lo:hi].to(dev))
        out = {c: torch.cat(v) for c, v in cols.items()}
        tie = torch.cat(ties) if tiebreak is not None else None
        torch.cuda.current_stream(dev).synchronize()
        g.before_collective(rank)  # every rank has its pieces
        self._xslots[rank] = None  # (its binned copy is freed once the caller drops it)
        return out, tie

    def abort(self) -> None:
        """A rank failed: cancel the collective on every communicator (ncclCommAbort).  The group
        stays aborted: a rank that reaches comms() afterwards raises GroupAborted instead of
        initialising fresh communicators whose peers never come."""
        self._aborted = True
        if self._comms is not None:
            comms, self._comms = self._comms, None
            for c in comms:
                self.lib.sct_comm_abort(ctypes.c_void_p(c))

    def close(self) -> None:
        if self._comms is not None:
            for c in self._comms:
                self.lib.sct_comm_destroy(ctypes.c_void_p(c))
            self._comms = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def _bounds(cols, key, size: int):
    """Each rank's record range [lo, hi): the decoded shards as they are (ShardedColumns), or
    run-aligned, record-balanced cuts of one column set."""
    if isinstance(cols, columnar.ShardedColumns):
        off = cols.offsets
        if len(off) - 1 != size:
            raise ValueError("%d decoded shards for %d devices" % (len(off) - 1, size))
        return [(off[r], off[r + 1]) for r in range(size)]
    return D.shard_bounds(cols.arrays[key], size)


def _rank_cols(cols, r: int, lo: int, hi: int, device) -> dict:
    """Rank r's columns on its device: its decoded shard, or records [lo, hi) copied there."""
    if isinstance(cols, columnar.ShardedColumns):
        sh = cols.shards[r]
        if sh["cell"].device != device:
            sh = {c: t.to(device) for c, t in sh.items()}
        return sh
    return _shard_to(cols, lo, hi, device)


def _cells_twice(cols) -> bool:
    """A cell barcode forming two runs (the records are not cell-sorted)."""
    if isinstance(cols, columnar.ShardedColumns):
        hv = []
        for sh in cols.shards:
            c = sh["cell"]
            if c.shape[0]:
                hv.append(c[torch.cat((torch.zeros(1, dtype=torch.long, device=c.device),
                                       torch.nonzero(c[1:] != c[:-1]).flatten() + 1))].cpu().numpy())
        if not hv:
            return False
        heads = np.concatenate(hv)
        keep = np.concatenate(([True], heads[1:] != heads[:-1]))  # (shards are cut at runs)
        return np.bincount(heads[keep]).max() > 1
    cell = cols.arrays["cell"]
    if not cell.shape[0]:
        return False
    if cols.on_device:
        heads = cell[torch.cat((torch.zeros(1, dtype=torch.long, device=cell.device),
                                torch.nonzero(cell[1:] != cell[:-1]).flatten() + 1))]
        return int(torch.bincount(heads.long()).max().item()) > 1
    heads = cell[np.concatenate(([0], np.flatnonzero(cell[1:] != cell[:-1]) + 1))]
    return np.bincount(heads).max() > 1


def cell_record_counts(cols, n_cell_ids: int) -> np.ndarray:
    """Records per cell id over the whole record set (host or device columns, or decoded shards)."""
    if isinstance(cols, columnar.ShardedColumns):
        tot = np.zeros(max(1, n_cell_ids), np.int64)
        for sh in cols.shards:
            c = sh["cell"]
            if c.shape[0]:
                tot += torch.bincount(c.long(), minlength=tot.shape[0]).cpu().numpy()[: tot.shape[0]]
        return tot
    cell = cols.arrays["cell"]
    if isinstance(cell, torch.Tensor):
        return torch.bincount(cell.long(), minlength=max(1, n_cell_ids)).cpu().numpy().astype(np.int64)
    return np.bincount(np.asarray(cell), minlength=max(1, n_cell_ids)).astype(np.int64)


def cells_twice(cols) -> bool:
    """True when a cell barcode forms two runs: the records are not cell-sorted."""
    return _cells_twice(cols)


def _shard_to(cols: columnar.Columns, lo: int, hi: int, device) -> dict:
    """Records [lo, hi) of every column on ``device``: host columns are copied up; device columns
    (decoded on the GPU, ``gbam``) are sliced in place and copied device to device (over xGMI when
    the shard's device is another GPU)."""
    from sctools_amd import engine as E

    if not cols.on_device:
        return E.to_device({c: np.ascontiguousarray(a[lo:hi]) for c, a in cols.arrays.items()}, device)
    return {c: t[lo:hi].to(device, copy=True) for c, t in cols.arrays.items()}  # (fresh, aligned buffers)


def _dims(cols: columnar.Columns):
    from sctools_amd import engine as E

    return E.Dims(len(cols.cells), len(cols.genes), len(cols.umis))


def compute_rows(cols: columnar.Columns, mode: str, mitochondrial_gene_ids=frozenset(), float_mode: str = "welford",
                 devices=1) -> Tuple[np.ndarray, np.ndarray]:
    """RUN-mode rows of every entity run, the runs spread over ``devices``; the same rows, in the
    same order, as one device computes (``metrics.gatherer.compute_rows``)."""
    from sctools_amd import engine as E

    key = "cell" if mode == "cell" else "gene"
    mito, multi = cols.gene_flags(mitochondrial_gene_ids)
    dims = _dims(cols)
    with DeviceGroup(devices) as g:
        bounds = _bounds(cols, key, g.size)

        def rank_rows(r):
            lo, hi = bounds[r]
            if hi == lo:
                return np.zeros((0, N.SCT_NI), np.int64), np.zeros((0, N.SCT_NF), np.float64)
            eng = g.engines[r]
            dev_cols = _rank_cols(cols, r, lo, hi, eng.device)
            gm = torch.from_numpy(mito).to(eng.device)
            gx = torch.from_numpy(multi).to(eng.device)
            ints, floats = eng.compute(dev_cols, mode, dims, gm, gx, float_mode=float_mode)
            ints, floats = ints.cpu().numpy(), floats.cpu().numpy()
            ints[:, N.I_ENTITY] += lo  # first-record index in the whole file
            return ints, floats

        parts = g.run(rank_rows)
    return np.concatenate([p[0] for p in parts]), np.concatenate([p[1] for p in parts])


def compute_cell_and_gene_rows(cols: columnar.Columns, mitochondrial_gene_ids=frozenset(),
                               float_mode: str = "exact", devices=1):
    """Cell rows of a cell-sorted record set and its grouped gene rows (every record of a gene
    id, as after TagSortBam by (GE, CB, UB)), cell ranges spread over ``devices``, gene partials
    summed by the RCCL all-reduce.  Returns ((cell ints, cell floats), (gene ints, gene floats));
    gene rows are indexed by gene id (zero-read ids included; the writer skips them)."""
    from sctools_amd import engine as E

    # grouped gene rows need every cell in ONE run (the cell-sharding invariant)
    if _cells_twice(cols):
        raise ValueError("gene rows of a record set need cell-sorted records (a cell barcode forms two runs)")
    mito, multi = cols.gene_flags(mitochondrial_gene_ids)
    dims = _dims(cols)
    with DeviceGroup(devices) as g:
        bounds = _bounds(cols, "cell", g.size)
        g.comms()

        def rank_rows(r):
            lo, hi = bounds[r]
            eng = g.engines[r]
            dev_cols = _rank_cols(cols, r, lo, hi, eng.device)
            gm = torch.from_numpy(mito).to(eng.device)
            gx = torch.from_numpy(multi).to(eng.device)
            if hi == lo:
                part = torch.zeros((max(1, dims.n_gene_ids), N.SCT_NP), dtype=torch.int64, device=eng.device)
                ci = np.zeros((0, N.SCT_NI), np.int64)
                cf = np.zeros((0, N.SCT_NF), np.float64)
            elif float_mode == "exact":  # one pass: cell rows and gene partials share the cell-view work
                ci, cf, part = eng.cell_and_gene(dev_cols, dims, gm)
                ci, cf = ci.cpu().numpy(), cf.cpu().numpy()
            else:  # Welford cell rows (record order), exact-sum gene partials
                ci, cf = eng.compute(dev_cols, "cell", dims, gm, gx, float_mode=float_mode)
                ci, cf = ci.cpu().numpy(), cf.cpu().numpy()
                part = eng.gene_partials(dev_cols, dims)
            if ci.shape[0]:
                ci[:, N.I_ENTITY] += lo
            g.allreduce_partials(r, part)  # RCCL over xGMI: every rank now holds the sums
            gene = None
            if r == 0:
                gi, gf = eng.finalize_partials(part)
                gene = (gi.cpu().numpy(), gf.cpu().numpy())
            return ci, cf, gene

        parts = g.run(rank_rows)
    cell = (np.concatenate([p[0] for p in parts]), np.concatenate([p[1] for p in parts]))
    return cell, parts[0][2]


def sorted_cell_and_gene_rows(cols, mitochondrial_gene_ids=frozenset(), float_mode: str = "exact", devices=1,
                              tiebreak: Optional[np.ndarray] = None, n_tiebreak_ids: int = 0):
    """Cell rows and grouped gene rows of records in ANY order: the cell rows TagSortBam by
    (CB, UB, GE[, query name]) followed by GatherCellMetrics writes, the gene rows those of
    TagSortBam by (GE, CB, UB) + GatherGeneMetrics -- the reference's SplitBam + TagSortBam +
    Calculate*Metrics + Merge*Metrics route for an unsorted BAM (bam.py:361-488, platform.py:55-97,
    merge.py:59-191) on the devices:

    * rank r takes the r-th part of the records (its decoded shard, or a contiguous range) and bins
      them by cell: contiguous ranges of barcode ranks, one per rank (sct_bin_records);
    * the ranks swap bins over RCCL (sct_exchange_records): rank r then holds every record of its
      cells, in file order;
    * each rank sorts them (sct_tag_sort, the query-name rank ``tiebreak`` as the last field if
      given, ties in input order as sorted() keeps them) and computes its cells' rows and gene
      partials; ONE all-reduce sums the partials; rank 0 finalizes the gene rows.

    Rank r's cells are the r-th barcode range, so rank order is barcode order: the concatenated
    cell rows are in TagSortBam's order.  Returns ((ints, floats, cell ids), (gene ints, gene floats))."""
    from sctools_amd import engine as E

    mito, _ = cols.gene_flags(mitochondrial_gene_ids)
    dims = _dims(cols)
    if tiebreak is not None:
        tiebreak = np.ascontiguousarray(tiebreak, dtype=np.int32)
        n_all = cols.offsets[-1] if isinstance(cols, columnar.ShardedColumns) else int(cols.arrays["cell"].shape[0])
        if tiebreak.shape[0] != n_all:
            raise ValueError("tiebreak has %d entries for %d records" % (tiebreak.shape[0], n_all))
        if n_tiebreak_ids <= 0:
            raise ValueError("n_tiebreak_ids must be positive with a tiebreak")
    with DeviceGroup(devices) as g:
        bounds = _bounds(cols, "cell", g.size)
        if g.size > N.SCT_MAX_BINS:
            raise ValueError("at most %d devices" % N.SCT_MAX_BINS)
        # bins = contiguous barcode ranges balanced by record count (rank order stays barcode order)
        table = D.balanced_cell_bins(cell_record_counts(cols, dims.n_cell_ids), g.size)
        g.comms()

        def rank_rows(r):
            lo, hi = bounds[r]
            eng = g.engines[r]
            part = _rank_cols(cols, r, lo, hi, eng.device)
            tie = torch.from_numpy(tiebreak[lo:hi]).to(eng.device) if tiebreak is not None else None
            bin_of_cell = torch.from_numpy(table).to(eng.device)
            binned, btie, counts = eng.bin_records(part, dims, g.size, tie, bin_of_cell=bin_of_cell)
            del part, tie
            mine, mtie = g.exchange(r, binned, btie, counts)
            del binned, btie
            n = int(mine["cell"].shape[0])
            srt = eng.tag_sort(mine, dims, "cell_umi_gene", mtie, n_tiebreak_ids if mtie is not None else 0) \
                if n else mine
            del mine, mtie
            gm = torch.from_numpy(mito).to(eng.device)
            if n == 0:
                part = torch.zeros((max(1, dims.n_gene_ids), N.SCT_NP), dtype=torch.int64, device=eng.device)
                ci = np.zeros((0, N.SCT_NI), np.int64)
                cf = np.zeros((0, N.SCT_NF), np.float64)
                ids = np.zeros(0, np.int64)
            else:
                if float_mode == "exact":
                    ci, cf, part = eng.cell_and_gene(srt, dims, gm)
                else:
                    gx = torch.zeros_like(gm)
                    ci, cf = eng.compute(srt, "cell", dims, gm, gx, float_mode=float_mode)
                    part = eng.gene_partials(srt, dims)
                ids = srt["cell"][ci[:, N.I_ENTITY]].to(torch.int64).cpu().numpy()
                ci, cf = ci.cpu().numpy(), cf.cpu().numpy()
            g.allreduce_partials(r, part)
            gene = None
            if r == 0:
                gi, gf = eng.finalize_partials(part)
                gene = (gi.cpu().numpy(), gf.cpu().numpy())
            return ci, cf, ids, gene

        parts = g.run(rank_rows)
    cell = tuple(np.concatenate([p[k] for p in parts]) for k in range(3))
    return cell, parts[0][3]
