"""
ctypes binding of ``libsct_csv.so`` (``include/sct_csv.h``): metric CSV rows formatted natively
(Python ``str`` / ``float.__repr__`` text, byte for byte) and gzip in parallel members.

The reference formats every value with ``str`` in Python and compresses with one
``gzip.open(..., "wt")`` stream (``writer.py:55-61, 84-103``); at 500k cell rows that is
~13 s of formatting and ~34 s of gzip level 9 on one core.
"""
import ctypes
import os
from typing import Optional, Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libsct_csv.so")
EXPORTED = ("sct_csv_repr_double", "sct_csv_format_rows", "sct_csv_gzip", "sct_csv_free")
INT, FLOAT = 0, 1

_lib: Optional[ctypes.CDLL] = None


def available() -> bool:
    return os.path.exists(LIB_PATH)


def load() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not available():
            raise RuntimeError("%s is missing: run __graft_entry__.build() (or make)" % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        vp, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
        L.sct_csv_repr_double.restype = i32
        L.sct_csv_repr_double.argtypes = [ctypes.c_double, ctypes.c_char_p, i32]
        L.sct_csv_format_rows.restype = ctypes.c_int
        L.sct_csv_format_rows.argtypes = [i64, vp, vp, i32, vp, vp, vp, i32, vp, i32, i32, ctypes.POINTER(vp),
                                          ctypes.POINTER(i64)]
        L.sct_csv_gzip.restype = ctypes.c_int
        L.sct_csv_gzip.argtypes = [vp, i64, i32, i64, i32, ctypes.POINTER(vp), ctypes.POINTER(i64)]
        L.sct_csv_free.restype = None
        L.sct_csv_free.argtypes = [vp]
        _lib = L
    return _lib


def repr_double(x: float) -> str:
    buf = ctypes.create_string_buffer(40)
    n = load().sct_csv_repr_double(float(x), buf, 40)
    return buf.raw[:n].decode()


def _take(ptr, n) -> bytes:
    L = load()
    try:
        return ctypes.string_at(ptr, n) if n else b""
    finally:
        L.sct_csv_free(ptr)


def format_rows(names: Sequence[str], kinds: Sequence[int], slots: Sequence[int], ints: np.ndarray,
                floats: np.ndarray, threads: int = 0) -> bytes:
    """CSV lines for every row (names already rendered, e.g. 'None' for a missing barcode)."""
    L = load()
    enc = [s.encode("utf-8") for s in names]
    off = np.zeros(len(enc) + 1, dtype=np.int64)
    if enc:
        off[1:] = np.cumsum([len(b) for b in enc])
    blob = b"".join(enc)
    ints = np.ascontiguousarray(ints, dtype=np.int64)
    floats = np.ascontiguousarray(floats, dtype=np.float64)
    kind = np.asarray(kinds, dtype=np.int32)
    slot = np.asarray(slots, dtype=np.int32)
    out, n = ctypes.c_void_p(), ctypes.c_int64()
    rc = L.sct_csv_format_rows(len(enc), blob, off.ctypes.data, len(kind), kind.ctypes.data, slot.ctypes.data,
                               ints.ctypes.data, ints.shape[1] if ints.ndim == 2 else 0, floats.ctypes.data,
                               floats.shape[1] if floats.ndim == 2 else 0, int(threads), ctypes.byref(out),
                               ctypes.byref(n))
    if rc:
        raise RuntimeError("sct_csv_format_rows failed")
    return _take(out, n.value)


def gzip(data: bytes, level: int = 9, chunk: int = 1 << 18, threads: int = 0) -> bytes:
    """gzip members of `chunk` input bytes compressed in parallel (concatenated members are one
    valid gzip stream); 256 KB members spread even a few-thousand-row CSV over the cores."""
    L = load()
    out, n = ctypes.c_void_p(), ctypes.c_int64()
    if L.sct_csv_gzip(data, len(data), int(level), int(chunk), int(threads), ctypes.byref(out), ctypes.byref(n)):
        raise RuntimeError("sct_csv_gzip failed")
    return _take(out, n.value)
