"""The C-ABI library loads and exports what include/sctools_gpu.h declares (no GPU needed)."""
import ctypes
import os
import re

import pytest

from sctools_amd import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    text = open(os.path.join(ROOT, "include", "sctools_gpu.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(sct_\w+)\(", text, flags=re.M)))


def test_every_declared_symbol_is_exported():
    lib = N.load()
    names = declared_functions()
    assert len(names) >= 9
    for name in names:
        assert hasattr(lib, name), name
    assert set(names) == set(N.EXPORTED)


def test_abi_version_and_workspace_query():
    lib = N.load()
    assert lib.sct_abi_version() == N.SCT_ABI_VERSION
    p = N.Plan(n_records=1_000_000, max_entities=1000, mode=N.MODE_CELL, float_mode=N.FLOAT_EXACT_SUM,
               n_cell_ids=1000, n_gene_ids=30001, n_umi_ids=1 << 20)
    nbytes = ctypes.c_size_t(0)
    assert lib.sct_workspace_size(ctypes.byref(p), ctypes.byref(nbytes)) == 0
    # two key/value buffer pairs dominate: >= 24 B per record
    assert nbytes.value >= 24 * 1_000_000


def test_invalid_plans_are_rejected_with_messages():
    lib = N.load()
    nbytes = ctypes.c_size_t(0)
    p = N.Plan(n_records=10, mode=7, float_mode=0, n_cell_ids=1, n_gene_ids=1, n_umi_ids=1)
    assert lib.sct_workspace_size(ctypes.byref(p), ctypes.byref(nbytes)) == -1
    assert b"mode" in lib.sct_last_error()
    p = N.Plan(n_records=10, mode=N.MODE_GENE_GROUPED, float_mode=N.FLOAT_WELFORD, n_cell_ids=1, n_gene_ids=1,
               n_umi_ids=1)
    assert lib.sct_workspace_size(ctypes.byref(p), ctypes.byref(nbytes)) == -1
    with pytest.raises(N.EngineError):
        N.check(lib.sct_workspace_size(ctypes.byref(p), ctypes.byref(nbytes)))


def test_struct_layout_matches_header():
    # sct_records_t: int64 n + 14 pointers; sct_plan_t: 2 x int64 + 6 x int32
    assert ctypes.sizeof(N.Records) == 8 + 14 * 8
    assert ctypes.sizeof(N.Plan) == 16 + 6 * 4
