"""
ctypes binding of ``libsctools_gpu.so`` (declared in ``include/sctools_gpu.h``).

The library is built in-tree by ``__graft_entry__.build()`` (hipcc,
``--offload-arch=gfx950``).  There is no CPU fallback: if the shared library
is missing, importing the engine raises immediately.
"""

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SCT_LIB_PATH") or os.path.join(HERE, "libsctools_gpu.so")  # override: experiments only

SCT_ABI_VERSION = 2
SCT_NI, SCT_NF, SCT_NP = 24, 12, 64
SCT_P_FLOAT_BASE, SCT_P_STREAM_LANES = 24, 8

MODE_CELL, MODE_GENE, MODE_GENE_GROUPED = 0, 1, 2
FLOAT_EXACT_SUM, FLOAT_WELFORD = 0, 1

# output int columns
I_N_READS, I_NOISE_READS, I_PERFECT_UMI, I_EXONIC, I_INTRONIC, I_UTR = 0, 1, 2, 3, 4, 5
I_UNIQUE, I_MULTIPLE, I_DUP, I_SPLICED, I_ANTISENSE = 6, 7, 8, 9, 10
I_N_MOL, I_N_FRAG, I_FRAG_SINGLE, I_MOL_SINGLE = 11, 12, 13, 14
I_PERFECT_CB, I_INTERGENIC, I_UNMAPPED, I_TOO_MANY_LOCI = 15, 16, 17, 18
I_N_K1, I_K1_MULTI, I_MITO_GENES, I_MITO_READS, I_ENTITY = 19, 20, 21, 22, 23
# output float columns
F_UY_MEAN, F_UY_VAR, F_GQF_MEAN, F_GQF_VAR, F_GQ_MEAN, F_GQ_VAR = 0, 1, 2, 3, 4, 5
F_RPM, F_RPF, F_FPM, F_CY_VAR, F_CY_MEAN, F_PCT_MITO = 6, 7, 8, 9, 10, 11

RECORD_COLUMNS = ("cell", "umi", "gene", "ref", "pos", "gq_sum", "gq_len", "gq_gt30", "bits", "xf",
                  "cy_gt30", "cy_len", "uy_gt30", "uy_len")

EXPORTED = ("sct_abi_version", "sct_last_error", "sct_workspace_size", "sct_count_entities",
            "sct_compute_metrics", "sct_gene_partials", "sct_cell_metrics_gene_partials",
            "sct_finalize_partials", "sct_profile_enable", "sct_profile_only", "sct_profile_read",
            "sct_profile_read_items",
            "sct_tag_sort_workspace_size", "sct_tag_sort", "sct_verify_sort", "sct_count_matrix_workspace_size", "sct_count_matrix",
            "sct_allreduce_gene_partials", "sct_comm_unique_id", "sct_comm_init_rank", "sct_comm_init_all",
            "sct_comm_destroy", "sct_comm_abort", "sct_bin_workspace_size", "sct_bin_records", "sct_exchange_counts",
            "sct_exchange_records")
SCT_MAX_BINS = 256
ORDER_CELL, ORDER_CELL_UMI_GENE, ORDER_GENE_CELL_UMI = 0, 1, 2
PLAN_GENE_PARTIALS = 0x1


class Records(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int64)] + [(c, ctypes.c_void_p) for c in RECORD_COLUMNS]


class Plan(ctypes.Structure):
    _fields_ = [
        ("n_records", ctypes.c_int64),
        ("max_entities", ctypes.c_int64),
        ("mode", ctypes.c_int32),
        ("float_mode", ctypes.c_int32),
        ("n_cell_ids", ctypes.c_int32),
        ("n_gene_ids", ctypes.c_int32),
        ("n_umi_ids", ctypes.c_int32),
        ("flags", ctypes.c_int32),
    ]


COUNT_SKIP, COUNT_UNKNOWN = -1, -2


class CountInput(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_int64),
        ("cell", ctypes.c_void_p),
        ("umi", ctypes.c_void_p),
        ("gene", ctypes.c_void_p),
        ("xf", ctypes.c_void_p),
        ("qhead", ctypes.c_void_p),
        ("n_cell_ids", ctypes.c_int32),
        ("n_umi_ids", ctypes.c_int32),
        ("n_gene_ids", ctypes.c_int32),
        ("cell_none", ctypes.c_int32),
        ("umi_none", ctypes.c_int32),
        ("gene_col", ctypes.c_void_p),
        ("n_cols", ctypes.c_int32),
    ]


class CountOutput(ctypes.Structure):
    _fields_ = [
        ("row_cell", ctypes.c_void_p),
        ("indptr", ctypes.c_void_p),
        ("indices", ctypes.c_void_p),
        ("data", ctypes.c_void_p),
        ("n_rows", ctypes.c_int64),
        ("nnz", ctypes.c_int64),
        ("unknown_record", ctypes.c_int64),
        ("n_sorted", ctypes.c_int64),
    ]


class EngineError(RuntimeError):
    """A C-ABI call returned an error code (message from sct_last_error)."""


_lib = None


def load() -> ctypes.CDLL:
    """Load the HIP engine; raise loudly if it was not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            "sctools_amd HIP engine not built (%s missing); run `python -c "
            "'import __graft_entry__ as g; g.build()'`" % LIB_PATH
        )
    L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    vp, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32
    L.sct_abi_version.restype = ctypes.c_int
    L.sct_abi_version.argtypes = []
    L.sct_last_error.restype = ctypes.c_char_p
    L.sct_last_error.argtypes = []
    L.sct_workspace_size.restype = ctypes.c_int
    L.sct_workspace_size.argtypes = [ctypes.POINTER(Plan), ctypes.POINTER(ctypes.c_size_t)]
    L.sct_count_entities.restype = ctypes.c_int
    L.sct_count_entities.argtypes = [ctypes.POINTER(Plan), ctypes.POINTER(Records), vp, ctypes.c_size_t,
                                     ctypes.POINTER(i64), vp]
    L.sct_compute_metrics.restype = ctypes.c_int
    L.sct_compute_metrics.argtypes = [ctypes.POINTER(Plan), ctypes.POINTER(Records), vp, vp, vp,
                                      ctypes.c_size_t, vp, vp, i64, ctypes.POINTER(i64), vp]
    L.sct_gene_partials.restype = ctypes.c_int
    L.sct_gene_partials.argtypes = [ctypes.POINTER(Plan), ctypes.POINTER(Records), vp, ctypes.c_size_t, vp, vp]
    L.sct_cell_metrics_gene_partials.restype = ctypes.c_int
    L.sct_cell_metrics_gene_partials.argtypes = [ctypes.POINTER(Plan), ctypes.POINTER(Records), vp, vp,
                                                 ctypes.c_size_t, vp, vp, i64, ctypes.POINTER(i64), vp, vp]
    L.sct_finalize_partials.restype = ctypes.c_int
    L.sct_finalize_partials.argtypes = [i32, vp, i64, vp, vp, vp]
    L.sct_tag_sort_workspace_size.restype = ctypes.c_int
    L.sct_tag_sort_workspace_size.argtypes = [ctypes.POINTER(Plan), ctypes.POINTER(ctypes.c_size_t)]
    L.sct_tag_sort.restype = ctypes.c_int
    L.sct_tag_sort.argtypes = [ctypes.POINTER(Plan), ctypes.POINTER(Records), vp, i32, i32, ctypes.POINTER(Records),
                               vp, ctypes.c_size_t, vp]
    L.sct_verify_sort.restype = ctypes.c_int
    L.sct_verify_sort.argtypes = [ctypes.POINTER(Plan), ctypes.POINTER(Records), vp, i32, vp, ctypes.c_size_t,
                                  ctypes.POINTER(ctypes.c_int64), vp]
    L.sct_count_matrix_workspace_size.restype = ctypes.c_int
    L.sct_count_matrix_workspace_size.argtypes = [ctypes.POINTER(CountInput), ctypes.POINTER(ctypes.c_size_t)]
    L.sct_count_matrix.restype = ctypes.c_int
    L.sct_count_matrix.argtypes = [ctypes.POINTER(CountInput), ctypes.POINTER(CountOutput), vp, ctypes.c_size_t, vp]
    L.sct_allreduce_gene_partials.restype = ctypes.c_int
    L.sct_allreduce_gene_partials.argtypes = [vp, i64, vp, vp]
    L.sct_comm_unique_id.restype = ctypes.c_int
    L.sct_comm_unique_id.argtypes = [vp, ctypes.c_size_t]
    L.sct_comm_init_rank.restype = ctypes.c_int
    L.sct_comm_init_rank.argtypes = [ctypes.POINTER(vp), ctypes.c_int, vp, ctypes.c_size_t, ctypes.c_int, ctypes.c_int]
    L.sct_comm_init_all.restype = ctypes.c_int
    L.sct_comm_init_all.argtypes = [ctypes.POINTER(vp), ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    L.sct_comm_destroy.restype = ctypes.c_int
    L.sct_comm_destroy.argtypes = [vp]
    if hasattr(L, "sct_comm_abort"):
        L.sct_comm_abort.restype = ctypes.c_int
        L.sct_comm_abort.argtypes = [vp]
    if hasattr(L, "sct_bin_records"):  # (an older engine given by SCT_LIB_PATH for an A/B lacks them)
        L.sct_bin_workspace_size.restype = ctypes.c_int
        L.sct_bin_workspace_size.argtypes = [ctypes.POINTER(Plan), i32, ctypes.POINTER(ctypes.c_size_t)]
        L.sct_bin_records.restype = ctypes.c_int
        L.sct_bin_records.argtypes = [ctypes.POINTER(Plan), ctypes.POINTER(Records), vp, vp, i32,
                                      ctypes.POINTER(Records), vp, vp, vp, ctypes.c_size_t, vp]
        L.sct_exchange_counts.restype = ctypes.c_int
        L.sct_exchange_counts.argtypes = [vp, vp, i32, vp, vp]
        L.sct_exchange_records.restype = ctypes.c_int
        L.sct_exchange_records.argtypes = [ctypes.POINTER(Records), vp, ctypes.POINTER(i64), ctypes.POINTER(i64), i32,
                                           ctypes.POINTER(Records), vp, vp, vp]
    L.sct_profile_enable.restype = ctypes.c_int
    L.sct_profile_enable.argtypes = [ctypes.c_int]
    L.sct_profile_only.restype = ctypes.c_int
    L.sct_profile_only.argtypes = [ctypes.c_char_p]
    L.sct_profile_read.restype = ctypes.c_int
    L.sct_profile_read.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_double),
                                   ctypes.POINTER(i64), ctypes.c_int]
    if hasattr(L, "sct_profile_read_items"):  # (an older engine given by SCT_LIB_PATH for an A/B lacks it)
        L.sct_profile_read_items.restype = ctypes.c_int
        L.sct_profile_read_items.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_double),
                                             ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64),
                                             ctypes.c_int]
    if L.sct_abi_version() != SCT_ABI_VERSION:
        raise ImportError("libsctools_gpu.so ABI %d != %d" % (L.sct_abi_version(), SCT_ABI_VERSION))
    _lib = L
    return L


def check(rc: int) -> None:
    if rc != 0:
        msg = load().sct_last_error().decode("utf-8", "replace")
        raise EngineError("sctools_gpu error %d: %s" % (rc, msg))
