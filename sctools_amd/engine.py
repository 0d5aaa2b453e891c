"""
Device-side driver of the HIP metric engine.

Owns the plumbing around the C-ABI of ``include/sctools_gpu.h``: device
buffers (torch CUDA tensors on ROCm), the workspace, and the stream.  All
metric arithmetic happens in the HIP kernels of ``sctools_amd/csrc``; this
module never computes a metric itself and has no CPU fallback: without a GPU
or without ``libsctools_gpu.so`` it raises.
"""

import ctypes
from dataclasses import dataclass
from typing import Dict, Optional, Tuple

import numpy as np
import torch

from sctools_amd import _native as N

_TORCH_DTYPES = {
    "cell": torch.int32, "umi": torch.int32, "gene": torch.int32, "ref": torch.int32, "pos": torch.int32,
    "gq_sum": torch.int16, "gq_len": torch.int16, "gq_gt30": torch.int16,  # uint16 bit patterns
    "bits": torch.uint8, "xf": torch.uint8, "cy_gt30": torch.uint8, "cy_len": torch.uint8,
    "uy_gt30": torch.uint8, "uy_len": torch.uint8,
}

MODES = {"cell": N.MODE_CELL, "gene": N.MODE_GENE, "gene_grouped": N.MODE_GENE_GROUPED}
FLOAT_MODES = {"exact": N.FLOAT_EXACT_SUM, "welford": N.FLOAT_WELFORD}


def _device(device=None) -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError("sctools_amd needs a ROCm GPU (torch.cuda.is_available() is False); "
                           "there is no CPU fallback")
    if device is None:
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device(device)


def to_device(arrays: Dict[str, np.ndarray], device=None) -> Dict[str, torch.Tensor]:
    """Copy host columns (numpy) to device tensors of the engine's dtypes."""
    dev = _device(device)
    out = {}
    for c in N.RECORD_COLUMNS:
        a = np.ascontiguousarray(arrays[c])
        t = _TORCH_DTYPES[c]
        if t == torch.int16:
            a = a.astype(np.uint16, copy=False).view(np.int16)
        out[c] = torch.from_numpy(a).to(dev, non_blocking=False)
    return out


def records_struct(cols: Dict[str, torch.Tensor]) -> N.Records:
    n = int(cols["cell"].numel())
    r = N.Records()
    r.n = n
    for c in N.RECORD_COLUMNS:
        t = cols[c]
        if t.numel() != n:
            raise ValueError("column %s has %d records, expected %d" % (c, t.numel(), n))
        if not t.is_contiguous():
            raise ValueError("column %s is not contiguous" % c)
        if t.element_size() != torch.empty((), dtype=_TORCH_DTYPES[c]).element_size():
            raise ValueError("column %s has element size %d" % (c, t.element_size()))
        setattr(r, c, t.data_ptr() if n else None)
    return r


@dataclass
class Dims:
    n_cell_ids: int
    n_gene_ids: int
    n_umi_ids: int


class Engine:
    """One engine per device; calls are issued on torch's current stream."""

    def __init__(self, device=None):
        self.lib = N.load()
        self.device = _device(device)
        self._ws: Optional[torch.Tensor] = None

    # ---- helpers ----
    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _plan(self, n, mode, float_mode, dims: Dims, max_entities=0, flags=0) -> N.Plan:
        p = N.Plan()
        p.flags = int(flags)
        p.n_records = int(n)
        p.max_entities = int(max_entities)
        p.mode = MODES[mode]
        p.float_mode = FLOAT_MODES[float_mode]
        p.n_cell_ids = max(1, int(dims.n_cell_ids))
        p.n_gene_ids = max(1, int(dims.n_gene_ids))
        p.n_umi_ids = max(1, int(dims.n_umi_ids))
        return p

    def workspace(self, plan: N.Plan) -> torch.Tensor:
        nbytes = ctypes.c_size_t(0)
        N.check(self.lib.sct_workspace_size(ctypes.byref(plan), ctypes.byref(nbytes)))
        need = int(nbytes.value)
        if self._ws is None or self._ws.numel() < need:
            self._ws = None
            self._ws = torch.empty(need, dtype=torch.uint8, device=self.device)
        return self._ws

    def release(self):
        self._ws = None

    # ---- entry points ----
    def count_entities(self, cols, mode: str, dims: Dims) -> int:
        rec = records_struct(cols)
        plan = self._plan(rec.n, mode, "exact", dims, max_entities=1)
        ws = self.workspace(plan)
        out = ctypes.c_int64(0)
        N.check(self.lib.sct_count_entities(ctypes.byref(plan), ctypes.byref(rec), ctypes.c_void_p(ws.data_ptr()),
                                            ws.numel(), ctypes.byref(out), self._stream()))
        return int(out.value)

    def compute(self, cols, mode: str, dims: Dims, gene_is_mito: torch.Tensor, gene_is_multi: torch.Tensor,
                float_mode: str = "exact", n_entities: Optional[int] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        """RUN-mode rows: (ints [rows, 24] int64, floats [rows, 12] float64) on the device."""
        if mode not in ("cell", "gene"):
            raise ValueError("compute() handles RUN modes 'cell' and 'gene'")
        rec = records_struct(cols)
        if n_entities is None:
            n_entities = self.count_entities(cols, mode, dims)
        cap = max(1, int(n_entities))
        plan = self._plan(rec.n, mode, float_mode, dims, max_entities=cap)
        ws = self.workspace(plan)
        ints = torch.empty((cap, N.SCT_NI), dtype=torch.int64, device=self.device)
        floats = torch.empty((cap, N.SCT_NF), dtype=torch.float64, device=self.device)
        rows = ctypes.c_int64(0)
        N.check(self.lib.sct_compute_metrics(
            ctypes.byref(plan), ctypes.byref(rec), ctypes.c_void_p(gene_is_mito.data_ptr()),
            ctypes.c_void_p(gene_is_multi.data_ptr()), ctypes.c_void_p(ws.data_ptr()), ws.numel(),
            ctypes.c_void_p(ints.data_ptr()), ctypes.c_void_p(floats.data_ptr()), cap, ctypes.byref(rows),
            self._stream()))
        r = int(rows.value)
        return ints[:r], floats[:r]

    def gene_partials(self, cols, dims: Dims, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """GROUPED per-gene additive partials int64 [n_gene_ids, 64] (device)."""
        rec = records_struct(cols)
        plan = self._plan(rec.n, "gene_grouped", "exact", dims)
        ws = self.workspace(plan)
        if out is None:
            out = torch.empty((max(1, dims.n_gene_ids), N.SCT_NP), dtype=torch.int64, device=self.device)
        N.check(self.lib.sct_gene_partials(ctypes.byref(plan), ctypes.byref(rec), ctypes.c_void_p(ws.data_ptr()),
                                           ws.numel(), ctypes.c_void_p(out.data_ptr()), self._stream()))
        return out

    def cell_and_gene(self, cols, dims: Dims, gene_is_mito: torch.Tensor, n_entities: Optional[int] = None,
                      partials: Optional[torch.Tensor] = None):
        """Cell rows (exact-sum floats) and grouped gene partials from one pass over cell-sorted records."""
        rec = records_struct(cols)
        if n_entities is None:
            n_entities = self.count_entities(cols, "cell", dims)
        cap = max(1, int(n_entities))
        plan = self._plan(rec.n, "cell", "exact", dims, max_entities=cap, flags=N.PLAN_GENE_PARTIALS)
        ws = self.workspace(plan)
        ints = torch.empty((cap, N.SCT_NI), dtype=torch.int64, device=self.device)
        floats = torch.empty((cap, N.SCT_NF), dtype=torch.float64, device=self.device)
        if partials is None:
            partials = torch.empty((max(1, dims.n_gene_ids), N.SCT_NP), dtype=torch.int64, device=self.device)
        rows = ctypes.c_int64(0)
        N.check(self.lib.sct_cell_metrics_gene_partials(
            ctypes.byref(plan), ctypes.byref(rec), ctypes.c_void_p(gene_is_mito.data_ptr()),
            ctypes.c_void_p(ws.data_ptr()), ws.numel(), ctypes.c_void_p(ints.data_ptr()),
            ctypes.c_void_p(floats.data_ptr()), cap, ctypes.byref(rows), ctypes.c_void_p(partials.data_ptr()),
            self._stream()))
        r = int(rows.value)
        return ints[:r], floats[:r], partials

    def finalize_partials(self, partials: torch.Tensor, mode: str = "gene_grouped"):
        rows = int(partials.shape[0])
        ints = torch.empty((max(1, rows), N.SCT_NI), dtype=torch.int64, device=self.device)
        floats = torch.empty((max(1, rows), N.SCT_NF), dtype=torch.float64, device=self.device)
        N.check(self.lib.sct_finalize_partials(MODES[mode], ctypes.c_void_p(partials.data_ptr()), rows,
                                               ctypes.c_void_p(ints.data_ptr()), ctypes.c_void_p(floats.data_ptr()),
                                               self._stream()))
        return ints[:rows], floats[:rows]

    # ---- tag sort (TagSortBam / bam.sort_by_tags_and_queryname, bam.py:638-709) ----
    def _sort_ws(self, plan: N.Plan) -> torch.Tensor:
        nbytes = ctypes.c_size_t(0)
        N.check(self.lib.sct_tag_sort_workspace_size(ctypes.byref(plan), ctypes.byref(nbytes)))
        need = int(nbytes.value)
        if self._ws is None or self._ws.numel() < need:
            self._ws = None
            self._ws = torch.empty(need, dtype=torch.uint8, device=self.device)
        return self._ws

    def tag_sort(self, cols, dims: Dims, order: str = "cell_umi_gene", tiebreak: Optional[torch.Tensor] = None,
                 n_tiebreak_ids: int = 0) -> Dict[str, torch.Tensor]:
        """Stably sorted copy of the columns by `order` ('cell', 'cell_umi_gene', 'gene_cell_umi'), then by
        `tiebreak` ids (the query-name rank) if given; ties keep input order, as sorted() does."""
        rec = records_struct(cols)
        out = {c: torch.empty_like(cols[c]) for c in N.RECORD_COLUMNS}
        orec = records_struct(out)
        plan = self._plan(rec.n, "cell", "exact", dims)
        ws = self._sort_ws(plan)
        tb = ctypes.c_void_p(tiebreak.data_ptr()) if tiebreak is not None else None
        N.check(self.lib.sct_tag_sort(ctypes.byref(plan), ctypes.byref(rec), tb, int(n_tiebreak_ids), ORDERS[order],
                                      ctypes.byref(orec), ctypes.c_void_p(ws.data_ptr()), ws.numel(), self._stream()))
        return out

    def verify_sort(self, cols, dims: Dims, order: str = "cell_umi_gene",
                    tiebreak: Optional[torch.Tensor] = None) -> int:
        """verify_sort (bam.py:712-724): -1 if sorted, else the first out-of-order record index."""
        rec = records_struct(cols)
        plan = self._plan(rec.n, "cell", "exact", dims)
        ws = self._sort_ws(plan)
        tb = ctypes.c_void_p(tiebreak.data_ptr()) if tiebreak is not None else None
        out = ctypes.c_int64(0)
        N.check(self.lib.sct_verify_sort(ctypes.byref(plan), ctypes.byref(rec), tb, ORDERS[order],
                                         ctypes.c_void_p(ws.data_ptr()), ws.numel(), ctypes.byref(out),
                                         self._stream()))
        return int(out.value)

    # ---- cell bins exchanged between devices (SplitBam's bins, bam.py:439-480; exchange.h) ----
    def bin_records(self, cols, dims: Dims, n_bins: int, tiebreak: Optional[torch.Tensor] = None,
                    bin_of_cell: Optional[torch.Tensor] = None):
        """Records grouped by the bin of their cell, input order kept inside a bin (sct_bin_records):
        (binned columns, the tiebreak carried along or None, device int64 [n_bins] records per bin).
        Bins are contiguous cell-id ranges unless ``bin_of_cell`` (device uint8 per cell id) is given."""
        if not 1 <= int(n_bins) <= N.SCT_MAX_BINS:
            raise ValueError("n_bins must be in [1, %d]" % N.SCT_MAX_BINS)
        rec = records_struct(cols)
        out = {c: torch.empty_like(cols[c]) for c in N.RECORD_COLUMNS}
        orec = records_struct(out)
        tie_out = torch.empty_like(tiebreak) if tiebreak is not None else None
        plan = self._plan(rec.n, "cell", "exact", dims)
        nbytes = ctypes.c_size_t(0)
        N.check(self.lib.sct_bin_workspace_size(ctypes.byref(plan), int(n_bins), ctypes.byref(nbytes)))
        ws = torch.empty(max(1, int(nbytes.value)), dtype=torch.uint8, device=self.device)
        counts = torch.empty(int(n_bins), dtype=torch.int64, device=self.device)
        ptr = (lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None)
        N.check(self.lib.sct_bin_records(ctypes.byref(plan), ctypes.byref(rec), ptr(tiebreak), ptr(bin_of_cell),
                                         int(n_bins), ctypes.byref(orec), ptr(tie_out), ptr(counts),
                                         ctypes.c_void_p(ws.data_ptr()), ws.numel(), self._stream()))
        return out, tie_out, counts

    def exchange_counts(self, counts: torch.Tensor, comm) -> torch.Tensor:
        """Every rank's bin counts swapped over the communicator (sct_exchange_counts): device int64
        [n_ranks], entry p = the records rank p sends here."""
        recv = torch.empty_like(counts)
        N.check(self.lib.sct_exchange_counts(ctypes.c_void_p(counts.data_ptr()), ctypes.c_void_p(recv.data_ptr()),
                                             int(counts.numel()), ctypes.c_void_p(comm), self._stream()))
        return recv

    def exchange_records(self, binned, tiebreak, send_counts, recv_counts, comm):
        """Bin p of this rank to rank p, rank p's bin for this rank received in rank order
        (sct_exchange_records over RCCL); send / recv counts are host sequences.  Returns (columns,
        tiebreak or None)."""
        n_ranks = len(send_counts)
        total = int(sum(int(c) for c in recv_counts))
        out = {c: torch.empty(total, dtype=_TORCH_DTYPES[c], device=self.device) for c in N.RECORD_COLUMNS}
        tie_out = torch.empty(total, dtype=torch.int32, device=self.device) if tiebreak is not None else None
        rec, orec = records_struct(binned), records_struct(out)
        sc = (ctypes.c_int64 * n_ranks)(*[int(c) for c in send_counts])
        rc = (ctypes.c_int64 * n_ranks)(*[int(c) for c in recv_counts])
        N.check(self.lib.sct_exchange_records(
            ctypes.byref(rec), ctypes.c_void_p(tiebreak.data_ptr()) if tiebreak is not None else None, sc, rc, n_ranks,
            ctypes.byref(orec), ctypes.c_void_p(tie_out.data_ptr()) if tie_out is not None else None,
            ctypes.c_void_p(comm), self._stream()))
        return out, tie_out

    # ---- count matrix (CountMatrix.from_sorted_tagged_bam, count.py:134-328) ----
    def count_matrix(self, cell: torch.Tensor, umi: torch.Tensor, gene: torch.Tensor, xf: torch.Tensor,
                     qhead: torch.Tensor, gene_col: torch.Tensor, n_cell_ids: int, n_umi_ids: int, cell_none: int,
                     umi_none: int, n_cols: int):
        """CSR of the molecule counts: (row_cell, indptr, indices, data) device tensors and the first
        record index of a counted molecule whose gene is outside the annotation (-1 if none; the
        matrix is then not built).  Columns are int32 ids / uint8 codes on this engine's device."""
        n = int(cell.numel())
        for t in (umi, gene, xf, qhead):
            if int(t.numel()) != n:
                raise ValueError("record columns differ in length")
        ci = N.CountInput()
        ci.n = n
        ci.cell, ci.umi, ci.gene = cell.data_ptr(), umi.data_ptr(), gene.data_ptr()
        ci.xf, ci.qhead = xf.data_ptr(), qhead.data_ptr()
        ci.n_cell_ids, ci.n_umi_ids, ci.n_gene_ids = int(n_cell_ids), int(n_umi_ids), int(gene_col.numel())
        ci.cell_none, ci.umi_none = int(cell_none), int(umi_none)
        ci.gene_col, ci.n_cols = gene_col.data_ptr(), int(n_cols)
        nbytes = ctypes.c_size_t(0)
        N.check(self.lib.sct_count_matrix_workspace_size(ctypes.byref(ci), ctypes.byref(nbytes)))
        ws = torch.empty(int(nbytes.value), dtype=torch.uint8, device=self.device)
        nc = max(1, int(n_cell_ids))
        row_cell = torch.empty(nc, dtype=torch.int32, device=self.device)
        indptr = torch.empty(nc + 1, dtype=torch.int32, device=self.device)
        indices = torch.empty(max(1, n), dtype=torch.int32, device=self.device)
        data = torch.empty(max(1, n), dtype=torch.int32, device=self.device)  # uint32 counts (< 2^31)
        co = N.CountOutput()
        co.row_cell, co.indptr, co.indices, co.data = (row_cell.data_ptr(), indptr.data_ptr(), indices.data_ptr(),
                                                       data.data_ptr())
        N.check(self.lib.sct_count_matrix(ctypes.byref(ci), ctypes.byref(co), ctypes.c_void_p(ws.data_ptr()),
                                          ws.numel(), self._stream()))
        del ws
        self.count_stats = {"sorted": int(co.n_sorted), "rows": int(co.n_rows), "nnz": int(co.nnz)}
        if co.unknown_record >= 0:
            return None, int(co.unknown_record)
        r, z = int(co.n_rows), int(co.nnz)
        return (row_cell[:r], indptr[:r + 1], indices[:z], data[:z]), -1

    # ---- profiling (HIP events inside the library) ----
    def profile_enable(self, on: bool = True):
        self.lib.sct_profile_enable(1 if on else 0)

    def profile_only(self, kernel: str = ""):
        """Time only the launches of `kernel` ("" = all) while profiling is enabled."""
        self.lib.sct_profile_only(kernel.encode())

    def profile_read(self) -> Dict[str, Tuple[float, int]]:
        return {k: v[:2] for k, v in self.profile_read_items().items()}

    def profile_read_items(self) -> Dict[str, Tuple[float, int, int]]:
        """{kernel: (total ms, launches, items processed over those launches or -1)}; resets."""
        cap = 64
        names = (ctypes.c_char_p * cap)()
        ms = (ctypes.c_double * cap)()
        launches = (ctypes.c_int64 * cap)()
        items = (ctypes.c_int64 * cap)()
        if hasattr(self.lib, "sct_profile_read_items"):
            k = self.lib.sct_profile_read_items(names, ms, launches, items, cap)
        else:  # an older engine (SCT_LIB_PATH, A/B runs): no item counts
            k = self.lib.sct_profile_read(names, ms, launches, cap)
            for i in range(cap):
                items[i] = -1
        return {names[i].decode(): (float(ms[i]), int(launches[i]), int(items[i])) for i in range(min(k, cap))}


ORDERS = {"cell": N.ORDER_CELL, "cell_umi_gene": N.ORDER_CELL_UMI_GENE, "gene_cell_umi": N.ORDER_GENE_CELL_UMI}

_engines: Dict[str, Engine] = {}


def get_engine(device=None) -> Engine:
    dev = _device(device)
    key = str(dev)
    if key not in _engines:
        _engines[key] = Engine(dev)
    return _engines[key]
