"""ctypes binding of oracle/liboracle.so (TEST INFRASTRUCTURE ONLY; see oracle/__init__.py).

``run(arrays, mode, gene_is_mito, n_gene_ids, threads)`` returns the same
(ints, floats) row arrays as the HIP engine's C-ABI, computed by the C
restatement of the reference (``oracle/sct_oracle.c``).
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

SCT_NI, SCT_NF = 24, 12
MODES = {"cell": 0, "gene": 1, "gene_grouped": 2}


class Records(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int64)] + [
        (c, ctypes.c_void_p)
        for c in ("cell", "umi", "gene", "ref", "pos", "gq_sum", "gq_len", "gq_gt30", "bits", "xf",
                  "cy_gt30", "cy_len", "uy_gt30", "uy_len")
    ]


_DTYPES = {"cell": np.int32, "umi": np.int32, "gene": np.int32, "ref": np.int32, "pos": np.int32,
           "gq_sum": np.uint16, "gq_len": np.uint16, "gq_gt30": np.uint16, "bits": np.uint8,
           "xf": np.uint8, "cy_gt30": np.uint8, "cy_len": np.uint8, "uy_gt30": np.uint8,
           "uy_len": np.uint8}

_lib = None


def build():
    import subprocess

    subprocess.run(["make", "-s", "-C", HERE, "liboracle.so"], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.orc_metrics.restype = ctypes.c_int64
        L.orc_metrics.argtypes = [ctypes.POINTER(Records), ctypes.c_int, ctypes.c_void_p, ctypes.c_int32,
                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int]
        L.orc_count_entities.restype = ctypes.c_int64
        L.orc_count_entities.argtypes = [ctypes.POINTER(Records), ctypes.c_int, ctypes.c_int32]
        _lib = L
    return _lib


def _records(arrays):
    keep = {}
    n = int(arrays["cell"].shape[0])
    r = Records()
    r.n = n
    for c, dt in _DTYPES.items():
        a = np.ascontiguousarray(np.asarray(arrays[c]).view(dt) if np.asarray(arrays[c]).dtype.itemsize
                                 == np.dtype(dt).itemsize else np.asarray(arrays[c], dtype=dt))
        keep[c] = a
        setattr(r, c, a.ctypes.data)
    return r, keep


def run(arrays, mode, gene_is_mito, n_gene_ids, threads=1):
    """Run the oracle on host numpy columns. Returns (ints [rows, 24], floats [rows, 12])."""
    L = lib()
    m = MODES[mode] if isinstance(mode, str) else int(mode)
    r, keep = _records(arrays)
    rows = L.orc_count_entities(ctypes.byref(r), m, int(n_gene_ids))
    ints = np.zeros((max(rows, 1), SCT_NI), dtype=np.int64)
    floats = np.zeros((max(rows, 1), SCT_NF), dtype=np.float64)
    mito = np.ascontiguousarray(np.asarray(gene_is_mito, dtype=np.uint8))
    got = L.orc_metrics(ctypes.byref(r), m, mito.ctypes.data, int(n_gene_ids), ints.ctypes.data,
                        floats.ctypes.data, ints.shape[0], int(threads))
    if got < 0:
        raise RuntimeError("oracle capacity error")
    del keep
    return ints[:got], floats[:got]
