"""
ctypes binding of ``libsct_gbam.so`` (``include/sct_gbam.h``): BAM -> columns decoded on the GPU.

The compressed file goes to HBM once; BGZF members inflate one wavefront each, record starts are
found and proven on the device, every record is parsed by one lane and CB / UB / GE are interned
in device hash tables.  The columns stay in HBM as the engine's input tensors; only the distinct
dictionary strings visit the host (to be ranked in Python's ``sorted()`` order).

It stands in for the same reference reads as ``bamnative`` (the per-record pysam loop of
``MetricAggregator.parse_molecule``, ``aggregator.py:251-334``, and
``CellMetrics.parse_extra_fields``, ``aggregator.py:507-530``).  A file the device path does not
reproduce exactly (a record the reference rejects, typed dictionary tags, non-ASCII dictionary
bytes, a malformed deflate stream, an empty file) returns ``None``: the caller decodes it with
``bamnative``, whose error is the reference's exception for the first offending record.
"""
import ctypes
import os
from typing import Optional

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SCT_GBAM_LIB_PATH") or os.path.join(HERE, "libsct_gbam.so")  # override: experiments only

OK, HOST = 0, 1
_MODES = {"cell": 0, "gene": 1}
EXPORTED = ("sct_gbam_open", "sct_gbam_open_part", "sct_gbam_part_bounds", "sct_gbam_merge_dictionaries",
            "sct_gbam_remap", "sct_gbam_parse", "sct_gbam_parse_count", "sct_gbam_dictionary", "sct_gbam_read_inflated",
            "sct_gbam_timing", "sct_gbam_windows", "sct_gbam_close", "sct_gbam_last_error")
STAGES = ("map_scan", "h2d", "inflate", "record_starts", "parse_intern", "dictionaries", "members",
          "start_rounds")

_lib: Optional[ctypes.CDLL] = None


def available() -> bool:
    return os.path.exists(LIB_PATH)


def load() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not available():
        raise RuntimeError("%s is missing: run __graft_entry__.build() (or make)" % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, i64, u64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64
    L.sct_gbam_open.restype = ctypes.c_int
    L.sct_gbam_open.argtypes = [ctypes.c_char_p, i32, vp, ctypes.POINTER(vp), ctypes.POINTER(i64)]
    L.sct_gbam_open_part.restype = ctypes.c_int
    L.sct_gbam_open_part.argtypes = [ctypes.c_char_p, i32, i32, i64, i32, vp, ctypes.POINTER(vp), ctypes.POINTER(i64)]
    L.sct_gbam_part_bounds.restype = ctypes.c_int
    L.sct_gbam_part_bounds.argtypes = [vp, ctypes.POINTER(i64), ctypes.POINTER(i64)]
    L.sct_gbam_merge_dictionaries.restype = ctypes.c_int
    L.sct_gbam_merge_dictionaries.argtypes = [ctypes.POINTER(vp), i32, i32, ctypes.POINTER(ctypes.POINTER(i32))]
    L.sct_gbam_remap.restype = ctypes.c_int
    L.sct_gbam_remap.argtypes = [vp, ctypes.POINTER(i32), i64, vp, i64]
    L.sct_gbam_parse.restype = ctypes.c_int
    L.sct_gbam_parse.argtypes = [vp, i32, ctypes.POINTER(vp)]
    L.sct_gbam_parse_count.restype = ctypes.c_int
    L.sct_gbam_parse_count.argtypes = [vp, ctypes.c_char_p, ctypes.POINTER(vp)]
    L.sct_gbam_dictionary.restype = ctypes.c_int
    L.sct_gbam_dictionary.argtypes = [vp, i32, ctypes.POINTER(i64), ctypes.POINTER(vp), ctypes.POINTER(vp),
                                      ctypes.POINTER(i32)]
    L.sct_gbam_read_inflated.restype = ctypes.c_int
    L.sct_gbam_read_inflated.argtypes = [vp, u64, u64, vp, ctypes.POINTER(u64)]
    L.sct_gbam_timing.restype = ctypes.c_int
    L.sct_gbam_timing.argtypes = [vp, ctypes.POINTER(ctypes.c_double)]
    L.sct_gbam_windows.restype = ctypes.c_int64
    L.sct_gbam_windows.argtypes = [vp]
    L.sct_gbam_close.restype = None
    L.sct_gbam_close.argtypes = [vp]
    L.sct_gbam_last_error.restype = ctypes.c_char_p
    L.sct_gbam_last_error.argtypes = []
    _lib = L
    return L


def last_error() -> str:
    return load().sct_gbam_last_error().decode("utf-8", "replace")


def _device(device):
    import torch

    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    if dev.index is None:  # "cuda": the current device, for the library and the stream alike
        dev = torch.device("cuda", torch.cuda.current_device())
    return dev


class _Handle:
    def __init__(self, path: str, device, part: int = 0, n_parts: int = 1, first_start: int = -1):
        import torch

        self.L = load()
        self.dev = _device(device)
        self.stream = torch.cuda.current_stream(self.dev)
        self.h = ctypes.c_void_p()
        n = ctypes.c_int64(0)
        self.rc = self.L.sct_gbam_open_part(os.fsencode(path), int(part), int(n_parts), int(first_start),
                                            int(self.dev.index), ctypes.c_void_p(self.stream.cuda_stream),
                                            ctypes.byref(self.h), ctypes.byref(n))
        self.err = last_error()  # (thread-local in the library: read on the calling thread)
        self.n = int(n.value)

    def bounds(self):
        a, b = ctypes.c_int64(), ctypes.c_int64()
        _check(self.L.sct_gbam_part_bounds(self.h, ctypes.byref(a), ctypes.byref(b)))
        return int(a.value), int(b.value)

    def dictionary_size(self, which: int) -> int:
        """Entries of dictionary ``which`` (the count alone: no copy of its strings)."""
        cnt, by, off, hn = ctypes.c_int64(), ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_int32()
        self.L.sct_gbam_dictionary(self.h, which, ctypes.byref(cnt), ctypes.byref(by), ctypes.byref(off),
                                   ctypes.byref(hn))
        return int(cnt.value)

    def dictionary(self, which: int, lazy: bool = True):
        cnt, by, off, hn = ctypes.c_int64(), ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_int32()
        self.L.sct_gbam_dictionary(self.h, which, ctypes.byref(cnt), ctypes.byref(by), ctypes.byref(off),
                                   ctypes.byref(hn))
        k = int(cnt.value)
        if k == 0 or not off.value:
            offs = np.zeros(1, dtype=np.int64)
        else:
            offs = np.frombuffer((ctypes.c_int64 * (k + 1)).from_address(off.value), dtype=np.int64).copy()
        total = int(offs[-1])
        raw = ctypes.string_at(by.value, total) if total else b""
        if lazy:
            from sctools_amd.columnar import PackedDictionary

            return PackedDictionary(raw, offs, bool(hn.value))
        lst = [raw[offs[i]:offs[i + 1]].decode("utf-8") for i in range(k)]
        if hn.value:
            lst[0] = None
        return lst

    def close(self):
        if self.h:
            self.L.sct_gbam_close(self.h)
            self.h = ctypes.c_void_p()

    def timing(self):
        t = (ctypes.c_double * 8)()
        self.L.sct_gbam_timing(self.h, t)
        out = dict(zip(STAGES, list(t)))
        out["windows"] = int(self.L.sct_gbam_windows(self.h))
        return out


def _check(rc: int):
    if rc not in (OK, HOST):
        raise OSError("device BAM decode failed (%d): %s" % (rc, last_error()))


COUNT_COLUMNS = ("cell", "umi", "gene", "xf", "qhead")


def decode(path: str, metric_mode: str = "cell", device=None, timings: Optional[dict] = None,
           lazy: bool = False, tags=None):
    """(device column tensors, [cell names, umi names, gene names]) -- or None when the file needs
    the host decoder.  Names in id order, None first when a record lacks the tag; with ``lazy``
    each dictionary is a ``columnar.PackedDictionary`` (strings decoded only when asked for).

    ``metric_mode`` "count": the count-matrix columns ``COUNT_COLUMNS`` of the three tags named by
    ``tags`` (cell, molecule, gene), as ``bamnative.decode(path, "count", tags=tags)``."""
    import torch

    from sctools_amd import _native as N
    from sctools_amd.engine import _TORCH_DTYPES

    H = _Handle(path, device)
    try:
        _check(H.rc)
        if H.rc == HOST:
            return None
        if metric_mode == "count" and (tags is None or len(tags) != 3 or any(len(t) != 2 for t in tags)):
            raise ValueError("count mode needs three 2-character tag names")
        names_ = COUNT_COLUMNS if metric_mode == "count" else N.RECORD_COLUMNS
        try:  # columns that do not fit the device: the host decoder takes the file
            if metric_mode == "count":
                cols = {c: torch.empty(H.n, dtype=torch.int32 if c in ("cell", "umi", "gene") else torch.uint8,
                                       device=H.dev) for c in COUNT_COLUMNS}
            else:
                cols = {c: torch.empty(H.n, dtype=_TORCH_DTYPES[c], device=H.dev) for c in N.RECORD_COLUMNS}
        except torch.cuda.OutOfMemoryError:
            return None
        ptrs = (ctypes.c_void_p * len(names_))(*[cols[c].data_ptr() for c in names_])
        if metric_mode == "count":
            rc = H.L.sct_gbam_parse_count(H.h, "".join(tags).encode("ascii"), ptrs)
        else:
            rc = H.L.sct_gbam_parse(H.h, _MODES[metric_mode], ptrs)
        _check(rc)
        if rc == HOST:
            return None
        names = [H.dictionary(which, lazy) for which in range(3)]
        if timings is not None:
            timings.update(H.timing())
        return cols, names
    finally:
        H.close()


def inflate(path: str, device=None) -> Optional[bytes]:
    """The concatenated BGZF payload as the device inflated it (tests compare it with zlib), or
    None when the device path declines the file."""
    H = _Handle(path, device)
    try:
        _check(H.rc)
        if H.rc == HOST:
            return None
        total = ctypes.c_uint64(0)
        H.L.sct_gbam_read_inflated(H.h, 0, 0, None, ctypes.byref(total))
        buf = ctypes.create_string_buffer(int(total.value))
        rc = H.L.sct_gbam_read_inflated(H.h, 0, int(total.value), buf, None)
        _check(rc)
        return buf.raw
    finally:
        H.close()


def decode_parts(path: str, metric_mode: str, devices, timings: Optional[dict] = None):
    """One file decoded by several devices together (``GatherCellMetrics(devices=N)``): part p of
    len(devices) -- a byte-balanced range of BGZF members and the records starting in them -- is
    inflated, parsed and interned on devices[p] (``sct_gbam_open_part``), so no device holds the
    whole file.  The parts' record starts are checked against each other (part p's first record is
    the landing of part p-1's walk; a part that guessed wrong is reopened there), their dictionaries
    merged into the global ranked ones and every part's ids renumbered on its device.

    Returns (per-part column dicts on their devices, [cells, umis, genes] ``PackedDictionary``) --
    records in file order, part after part -- or None when the file needs the host decoder."""
    import threading

    import torch

    from sctools_amd import _native as N
    from sctools_amd.engine import _TORCH_DTYPES

    if metric_mode not in _MODES:
        raise ValueError("decode_parts reads the cell and gene metric modes")
    devs = [_device(d) for d in devices]
    P = len(devs)
    hs: list = [None] * P
    errs: list = [None] * P

    def each(fn):
        def work(p):
            try:
                with torch.cuda.device(devs[p]):
                    fn(p)
            except BaseException as e:  # noqa: BLE001 -- re-raised below
                errs[p] = e

        th = [threading.Thread(target=work, args=(p,)) for p in range(P)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        for e in errs:
            if e is not None:
                raise e

    def close_all():
        for h in hs:
            if h is not None:
                h.close()

    try:
        def open_one(p):
            hs[p] = _Handle(path, devs[p], p, P)

        each(open_one)
        for h in hs:
            if h.rc not in (OK, HOST):
                raise OSError("device BAM decode failed (%d): %s" % (h.rc, h.err))
        if hs[0].rc == HOST:
            return None
        # part p starts where part p-1's walk lands: a part whose own guess disagrees (or failed
        # from a wrong guess) is reopened there
        for p in range(1, P):
            land = hs[p - 1].bounds()[1]
            if hs[p].rc == HOST or hs[p].bounds()[0] != land:
                hs[p].close()
                with torch.cuda.device(devs[p]):
                    hs[p] = _Handle(path, devs[p], p, P, first_start=land)
                if hs[p].rc not in (OK, HOST):
                    raise OSError("device BAM decode failed (%d): %s" % (hs[p].rc, hs[p].err))
                if hs[p].rc == HOST:
                    return None
        cols: list = [None] * P
        rcs = [OK] * P
        msgs = [""] * P

        def parse_one(p):
            h = hs[p]
            try:
                cols[p] = {c: torch.empty(h.n, dtype=_TORCH_DTYPES[c], device=h.dev) for c in N.RECORD_COLUMNS}
            except torch.cuda.OutOfMemoryError:
                rcs[p] = HOST
                return
            if h.n:
                ptrs = (ctypes.c_void_p * len(N.RECORD_COLUMNS))(*[cols[p][c].data_ptr() for c in N.RECORD_COLUMNS])
                rcs[p] = h.L.sct_gbam_parse(h.h, _MODES[metric_mode], ptrs)
                msgs[p] = last_error()

        each(parse_one)
        for rc, msg in zip(rcs, msgs):
            if rc not in (OK, HOST):
                raise OSError("device BAM decode failed (%d): %s" % (rc, msg))
        if any(rc == HOST for rc in rcs):
            return None
        L = load()
        remaps = []
        for which in range(3):
            sizes = [hs[p].dictionary_size(which) for p in range(P)]
            arrs = [np.zeros(max(1, k), dtype=np.int32) for k in sizes]
            ptrs = (ctypes.POINTER(ctypes.c_int32) * P)(
                *[a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)) for a in arrs])
            handles = (ctypes.c_void_p * P)(*[h.h.value for h in hs])
            _check(L.sct_gbam_merge_dictionaries(handles, P, which, ptrs))
            remaps.append((arrs, sizes))

        def remap_one(p):
            h = hs[p]
            if not h.n:
                return
            for which, col in enumerate(("cell", "umi", "gene")):
                arrs, sizes = remaps[which]
                a = arrs[p]
                _check(h.L.sct_gbam_remap(h.h, a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), sizes[p],
                                          ctypes.c_void_p(cols[p][col].data_ptr()), h.n))

        each(remap_one)
        names = [hs[0].dictionary(which) for which in range(3)]
        if timings is not None:
            timings.update(hs[0].timing())
            timings["parts"] = [h.n for h in hs]
        return cols, names
    finally:
        close_all()
