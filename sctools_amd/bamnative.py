"""
ctypes binding of ``libsct_bam.so`` (``include/sct_bam.h``): the native BAM -> columns decoder.

It replaces the per-record pysam reads of the reference's aggregation loop
(``aggregator.py:251-334, 507-530``) for ``GatherCellMetrics`` /
``GatherGeneMetrics`` on BAM input: BGZF blocks inflate and records parse on all
cores, and CB / UB / GE are dictionary-encoded natively.  Validation and the
exception classes are those of :func:`sctools_amd.columnar.columnarize` (the
first offending record in file order decides), which the tests check against
the pure-Python decoder on every fixture.
"""
import ctypes
import os
from typing import Optional

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libsct_bam.so")

OK, EIO, EFORMAT = 0, -1, -2
KEYERROR, TYPEERROR, ZERODIV, VALUEERROR, EMPTY, MISSING_TAG, ETYPED = -10, -11, -12, -13, -14, -15, -16


class TypedTagValue(Exception):
    """A dictionary tag holds a float or array value (or, for the sort keys, an integer): the native
    decoder cannot key it as the Python reader does, so the caller decodes with the Python reader
    (include/sct_bam.h SCT_BAM_ETYPED)."""
CELL_METRICS, GENE_METRICS, COUNT_MATRIX, SORT_KEYS = 0, 1, 2, 3
_MODES = {"cell": CELL_METRICS, "gene": GENE_METRICS, "count": COUNT_MATRIX, "sortkeys": SORT_KEYS}
EXPORTED = ("sct_bam_decode", "sct_bam_decode_tags", "sct_bam_last_error", "sct_bam_n", "sct_bam_column", "sct_bam_dictionary",
            "sct_bam_close", "sct_bam_split", "sct_bam_write_order")

_lib: Optional[ctypes.CDLL] = None


def load() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError("%s is missing: run __graft_entry__.build() (or make)" % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    vp = ctypes.c_void_p
    L.sct_bam_decode.restype = ctypes.c_int
    L.sct_bam_decode.argtypes = [ctypes.c_char_p, ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(vp),
                                 ctypes.POINTER(ctypes.c_int64)]
    L.sct_bam_decode_tags.restype = ctypes.c_int
    L.sct_bam_decode_tags.argtypes = [ctypes.c_char_p, ctypes.c_int32, ctypes.c_char_p, ctypes.c_int32,
                                      ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_int64)]
    L.sct_bam_last_error.restype = ctypes.c_char_p
    L.sct_bam_last_error.argtypes = []
    L.sct_bam_n.restype = ctypes.c_int64
    L.sct_bam_n.argtypes = [vp]
    L.sct_bam_column.restype = vp
    L.sct_bam_column.argtypes = [vp, ctypes.c_char_p]
    L.sct_bam_dictionary.restype = ctypes.c_int
    L.sct_bam_dictionary.argtypes = [vp, ctypes.c_int32, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(vp),
                                     ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_int32)]
    L.sct_bam_close.restype = None
    L.sct_bam_close.argtypes = [vp]
    i32 = ctypes.c_int32
    L.sct_bam_split.restype = ctypes.c_int
    L.sct_bam_split.argtypes = [ctypes.POINTER(ctypes.c_char_p), i32, ctypes.c_char_p, ctypes.c_char_p, i32, i32, i32,
                                i32, i32, ctypes.POINTER(i32), ctypes.POINTER(ctypes.c_int64)]
    L.sct_bam_write_order.restype = ctypes.c_int
    L.sct_bam_write_order.argtypes = [ctypes.c_char_p, ctypes.c_char_p, vp, ctypes.c_int64, i32, i32]
    _lib = L
    return L


def available() -> bool:
    return os.path.exists(LIB_PATH)


_EXC = {KEYERROR: KeyError, TYPEERROR: TypeError, ZERODIV: ZeroDivisionError, VALUEERROR: ValueError,
        EMPTY: RuntimeError, EFORMAT: ValueError, EIO: OSError, MISSING_TAG: RuntimeError, ETYPED: TypedTagValue}


def decode(path: str, metric_mode: str = "cell", threads: int = 0, tags=("CB", "UB", "GE")):
    """(arrays, [cell names, umi names, gene names]) -- names in id order, None first if present.

    metric_mode "count" (CountMatrix): only cell / umi / gene / xf are meaningful, the three
    dictionary tags are ``tags``, nothing is validated, and ``arrays["qhead"]`` marks the first
    record of each run of equal query names.

    metric_mode "sortkeys" (TagSortBam / VerifyBamSort): cell / umi / gene are the ranks of the
    three ``tags`` (a missing tag and an empty value both rank first, as "" does),
    ``arrays["qname"]`` the rank of the query name, and a fourth name list holds the query
    names in rank order."""
    from sctools_amd.columnar import COLUMNS

    L = load()
    h = ctypes.c_void_p()
    bad = ctypes.c_int64(-1)
    tag_bytes = "".join(tags).encode()
    if len(tag_bytes) != 6 or any(len(t) != 2 for t in tags):
        raise ValueError("tags must be three two-character BAM tag names: %r" % (tags,))
    rc = L.sct_bam_decode_tags(os.fsencode(path), _MODES[metric_mode], tag_bytes, int(threads), ctypes.byref(h),
                               ctypes.byref(bad))
    if rc != OK:
        msg = L.sct_bam_last_error().decode("utf-8", "replace")
        raise _EXC.get(rc, RuntimeError)(msg)
    try:
        n = int(L.sct_bam_n(h))
        arrays = {}
        extra = {"count": [("qhead", np.uint8)], "sortkeys": [("qname", np.int32)]}
        cols = list(COLUMNS) + extra.get(metric_mode, [])
        for name, dt in cols:
            ptr = L.sct_bam_column(h, name.encode())
            buf = (ctypes.c_char * (n * np.dtype(dt).itemsize)).from_address(ptr) if n else b""
            arrays[name] = np.frombuffer(buf, dtype=dt, count=n).copy()
        names = []
        for which in range(4 if metric_mode == "sortkeys" else 3):
            cnt, by, off, hn = ctypes.c_int64(), ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_int32()
            L.sct_bam_dictionary(h, which, ctypes.byref(cnt), ctypes.byref(by), ctypes.byref(off), ctypes.byref(hn))
            k = int(cnt.value)
            offs = np.frombuffer((ctypes.c_int64 * (k + 1)).from_address(off.value), dtype=np.int64).copy()
            total = int(offs[-1])
            raw = ctypes.string_at(by.value, total) if total else b""
            lst = [raw[offs[i]:offs[i + 1]].decode("utf-8") for i in range(k)]
            if hn.value:
                lst[0] = None
            names.append(lst)
        return arrays, names
    finally:
        L.sct_bam_close(h)


def split(in_paths, out_prefix: str, tags, n_subfiles: int, raise_missing: bool = True, level: int = 6,
          threads: int = 0) -> int:
    """sct_bam_split: chunk files ``<out_prefix>_<k>.bam``; returns the number written."""
    L = load()
    for t in tags:
        if len(t) != 2:
            raise ValueError("tags must be two-character BAM tag names: %r" % (tags,))
    arr = (ctypes.c_char_p * len(in_paths))(*[os.fsencode(p) for p in in_paths])
    n_out = ctypes.c_int32(0)
    bad = ctypes.c_int64(-1)
    rc = L.sct_bam_split(arr, len(in_paths), os.fsencode(out_prefix), "".join(tags).encode(), len(tags),
                         int(n_subfiles), 1 if raise_missing else 0, int(level), int(threads), ctypes.byref(n_out),
                         ctypes.byref(bad))
    if rc != OK:
        raise _EXC.get(rc, RuntimeError)(L.sct_bam_last_error().decode("utf-8", "replace"))
    return int(n_out.value)


def write_order(in_path: str, out_path: str, perm, level: int = 6, threads: int = 0) -> None:
    """sct_bam_write_order: the records of ``in_path`` in the order ``perm`` (output record k is
    input record perm[k]) under the input's header."""
    L = load()
    p = np.ascontiguousarray(perm, dtype=np.int64)
    rc = L.sct_bam_write_order(os.fsencode(in_path), os.fsencode(out_path), p.ctypes.data if p.size else None,
                               int(p.size), int(level), int(threads))
    if rc != OK:
        raise _EXC.get(rc, RuntimeError)(L.sct_bam_last_error().decode("utf-8", "replace"))
