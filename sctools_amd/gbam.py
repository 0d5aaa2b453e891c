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
EXPORTED = ("sct_gbam_open", "sct_gbam_parse", "sct_gbam_parse_count", "sct_gbam_dictionary", "sct_gbam_read_inflated", "sct_gbam_timing",
            "sct_gbam_close", "sct_gbam_last_error")
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
    L.sct_gbam_close.restype = None
    L.sct_gbam_close.argtypes = [vp]
    L.sct_gbam_last_error.restype = ctypes.c_char_p
    L.sct_gbam_last_error.argtypes = []
    _lib = L
    return L


def last_error() -> str:
    return load().sct_gbam_last_error().decode("utf-8", "replace")


class _Handle:
    def __init__(self, path: str, device):
        import torch

        self.L = load()
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        if dev.index is None:  # "cuda": the current device, for the library and the stream alike
            dev = torch.device("cuda", torch.cuda.current_device())
        self.dev = dev
        self.stream = torch.cuda.current_stream(self.dev)
        self.h = ctypes.c_void_p()
        n = ctypes.c_int64(0)
        self.rc = self.L.sct_gbam_open(os.fsencode(path), int(self.dev.index),
                                       ctypes.c_void_p(self.stream.cuda_stream), ctypes.byref(self.h), ctypes.byref(n))
        self.n = int(n.value)

    def close(self):
        if self.h:
            self.L.sct_gbam_close(self.h)
            self.h = ctypes.c_void_p()

    def timing(self):
        t = (ctypes.c_double * 8)()
        self.L.sct_gbam_timing(self.h, t)
        return dict(zip(STAGES, list(t)))


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
        names = []
        for which in range(3):
            cnt, by, off, hn = ctypes.c_int64(), ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_int32()
            H.L.sct_gbam_dictionary(H.h, which, ctypes.byref(cnt), ctypes.byref(by), ctypes.byref(off),
                                    ctypes.byref(hn))
            k = int(cnt.value)
            offs = np.frombuffer((ctypes.c_int64 * (k + 1)).from_address(off.value), dtype=np.int64).copy()
            total = int(offs[-1])
            raw = ctypes.string_at(by.value, total) if total else b""
            if lazy:
                from sctools_amd.columnar import PackedDictionary

                names.append(PackedDictionary(raw, offs, bool(hn.value)))
                continue
            lst = [raw[offs[i]:offs[i + 1]].decode("utf-8") for i in range(k)]
            if hn.value:
                lst[0] = None
            names.append(lst)
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
