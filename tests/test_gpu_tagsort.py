"""On-GPU tag sort (sct_tag_sort / sct_verify_sort) against the reference's sort semantics.

The reference sorts with Python's stable sorted() by tag values then query name
(bam.sort_by_tags_and_queryname, bam.py:638-709) and checks with verify_sort
(bam.py:712-724).  Pinned by the reference's own fixtures: its
`cell-gene-umi-queryname-sorted.bam` is exactly `unsorted.bam` in (CB, UB, GE,
query name) order (checked by test_fixture_order_is_lexsort on CPU), so tag-sorting
`unsorted.bam` on the GPU must reproduce that file's records and, through the
Welford pipeline, the reference's metric CSVs byte for byte.
"""
import os

import numpy as np
import pytest
import torch

import helpers as H
from sctools_amd import _native as N
from sctools_amd import bam as B

ORDERS = {"cell": ("cell",), "cell_umi_gene": ("cell", "umi", "gene"), "gene_cell_umi": ("gene", "cell", "umi")}


def qname_ranks(name):
    q = [r.query_name for r in B.open_alignments(os.path.join(H.GOLDEN, "bam", name + ".bam"), "rb")]
    rank = {v: i for i, v in enumerate(sorted(set(q)))}
    return np.array([rank[v] for v in q], dtype=np.int32), len(rank)


def np_order(arrays, order, tie=None):
    keys = [arrays[f] for f in reversed(ORDERS[order])]
    if tie is not None:
        keys = [tie] + keys
    return np.lexsort(keys)  # stable: ties keep input order, as sorted() does


def test_fixture_order_is_lexsort():
    """CPU: the reference's sorted fixture is lexsort(CB, UB, GE, query name) of unsorted.bam."""
    u = H.bam_columns("unsorted", "cell")
    s = H.bam_columns("cell-gene-umi-queryname-sorted", "cell")
    tie, _ = qname_ranks("unsorted")
    order = np_order(u.arrays, "cell_umi_gene", tie)
    for c in N.RECORD_COLUMNS:
        assert np.array_equal(u.arrays[c][order], s.arrays[c]), c


def test_invalid_order_is_rejected_without_a_gpu():
    import ctypes

    lib = N.load()
    plan = N.Plan(n_records=0, n_cell_ids=1, n_gene_ids=1, n_umi_ids=1)
    rec = N.Records(n=0)
    rc = lib.sct_tag_sort(ctypes.byref(plan), ctypes.byref(rec), None, 0, 9, ctypes.byref(rec), None, 0, None)
    assert rc == -1 and b"order" in lib.sct_last_error()
    nbytes = ctypes.c_size_t(0)
    plan.n_records = 1000
    assert lib.sct_tag_sort_workspace_size(ctypes.byref(plan), ctypes.byref(nbytes)) == 0
    assert nbytes.value >= 56 * 1000  # packed record + two key/value buffer pairs


@pytest.fixture(scope="module")
def eng():
    from sctools_amd import engine as E

    return E.get_engine("cuda:0")


def to_dev(eng, arrays):
    from sctools_amd import engine as E

    return E.to_device(arrays, eng.device)


def to_host(cols):
    out = {c: t.cpu().numpy() for c, t in cols.items()}
    for c in ("gq_sum", "gq_len", "gq_gt30"):
        out[c] = out[c].view(np.uint16)
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["cell", "gene"])
def test_unsorted_bam_tag_sorted_on_gpu_matches_reference(eng, mode):
    from sctools_amd import engine as E

    u = H.bam_columns("unsorted", mode)
    tie, n_tie = qname_ranks("unsorted")
    d = E.Dims(len(u.cells), len(u.genes), len(u.umis))
    cols = eng.tag_sort(to_dev(eng, u.arrays), d, "cell_umi_gene", torch.from_numpy(tie).to(eng.device), n_tie)
    host = to_host(cols)
    ref = H.bam_columns("cell-gene-umi-queryname-sorted", mode)
    for c in N.RECORD_COLUMNS:
        assert np.array_equal(host[c], ref.arrays[c]), c
    assert eng.verify_sort(cols, d, "cell_umi_gene", torch.from_numpy(tie[np_order(u.arrays, "cell_umi_gene", tie)])
                           .to(eng.device)) == -1
    # and the metrics of the sorted records are the reference's, byte for byte (Welford)
    mito, _ = u.gene_flags()
    gm = torch.from_numpy(np.ascontiguousarray(mito, dtype=np.uint8)).to(eng.device)
    gi, gf = eng.compute(cols, mode, d, gm, gm, float_mode="welford")
    got = H.render(mode, gi.cpu().numpy(), gf.cpu().numpy(), host, u.cells.names, u.genes.names)
    assert got == H.golden_text("cell-gene-umi-queryname-sorted", mode)


def shuffled_synth(n, seed, n_cells=300):
    from sctools_amd import synth

    d = synth.generate(synth.SynthConfig(n_reads=n, n_cells=n_cells, n_genes=2000, seed=seed), device="cpu")
    arrays = to_host(d.cols)
    perm = np.random.default_rng(seed).permutation(n)
    return d, arrays, {c: np.ascontiguousarray(a[perm]) for c, a in arrays.items()}


@pytest.mark.gpu
@pytest.mark.parametrize("order", list(ORDERS))
@pytest.mark.parametrize("with_tie", [False, True])
def test_tag_sort_matches_numpy_lexsort(eng, order, with_tie):
    from sctools_amd import engine as E

    d, _, arrays = shuffled_synth(200_000, 5)
    n = arrays["cell"].shape[0]
    tie = np.random.default_rng(1).integers(0, 1000, n).astype(np.int32) if with_tie else None
    dims = E.Dims(d.n_cell_ids, d.n_gene_ids, d.n_umi_ids)
    out = eng.tag_sort(to_dev(eng, arrays), dims, order, None if tie is None else torch.from_numpy(tie).to(eng.device),
                       1000)
    host = to_host(out)
    idx = np_order(arrays, order, tie)
    for c in N.RECORD_COLUMNS:
        assert np.array_equal(host[c], arrays[c][idx]), c


@pytest.mark.gpu
def test_tag_sort_with_keys_wider_than_64_bits(eng):
    """Inflated dictionary sizes: the fields need two 64-bit rounds ([gene | tie], then [cell | umi])."""
    from sctools_amd import engine as E

    d, _, arrays = shuffled_synth(100_000, 6)
    n = arrays["cell"].shape[0]
    tie = np.random.default_rng(2).integers(0, 1 << 20, n).astype(np.int32)
    dims = E.Dims(1 << 28, 1 << 30, 1 << 30)
    out = eng.tag_sort(to_dev(eng, arrays), dims, "cell_umi_gene", torch.from_numpy(tie).to(eng.device), 1 << 20)
    host = to_host(out)
    idx = np_order(arrays, "cell_umi_gene", tie)
    for c in N.RECORD_COLUMNS:
        assert np.array_equal(host[c], arrays[c][idx]), c


@pytest.mark.gpu
def test_tag_sort_small_radix_tiles():
    """The engine built with 1024-item radix tiles (tests/native/libsct_engine_si4.so) sorts like
    numpy.  Round 3's tag-sort layout sized the digit counts by the 2048-record row tile, so this
    tiling overflowed them (an illegal memory access in config 5's sort); the counts
    now cover both tilings and radix_sort checks its capacity.  Runs in a child process (one
    engine library per process)."""
    import subprocess
    import sys

    lib = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native", "libsct_engine_si4.so")
    assert os.path.exists(lib), "build it first: make tests/native/libsct_engine_si4.so"
    env = dict(os.environ, SCT_LIB_PATH=lib)
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(lib), "..", "si4_check.py"), "2000000"], env=env,
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert r.stdout.count("equal numpy's lexsort") == 2, r.stdout


def test_tag_sort_workspace_covers_every_radix_tiling():
    """CPU: the tag-sort workspace holds the digit counts of radix_sort's tiles (kSortTile), not
    only the row passes' (kRowTile).  The si4 engine (1024-item tiles) needs 256 counts per 1024
    records in each of `counts` and `offsets` on top of the 56 B/record of rows and key buffers
    (since round 6 the shipped engine reserves as much for the group sort's 9-bit MSD pass)."""
    import ctypes

    lib_path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native", "libsct_engine_si4.so")
    if not os.path.exists(lib_path):
        pytest.skip("tests/native/libsct_engine_si4.so not built")
    lib = ctypes.CDLL(lib_path)
    n = 1 << 20
    plan = N.Plan(n_records=n, n_cell_ids=1, n_gene_ids=1, n_umi_ids=1)
    a, b = ctypes.c_size_t(0), ctypes.c_size_t(0)
    assert N.load().sct_tag_sort_workspace_size(ctypes.byref(plan), ctypes.byref(a)) == 0
    assert lib.sct_tag_sort_workspace_size(ctypes.byref(plan), ctypes.byref(b)) == 0
    # 2 x 4 B x 256 counts per 1024-record tile in the si4 build (its radix tiles); the shipped build
    # needs as many for the group sort's MSD pass (512 digits per 2048-record tile)
    assert b.value >= a.value
    assert b.value >= 56 * n + 2 * 4 * 256 * (n // 1024)


@pytest.mark.gpu
def test_verify_sort_finds_the_first_violation(eng):
    from sctools_amd import engine as E

    d, sorted_arrays, arrays = shuffled_synth(50_000, 7)
    dims = E.Dims(d.n_cell_ids, d.n_gene_ids, d.n_umi_ids)
    assert eng.verify_sort(to_dev(eng, sorted_arrays), dims, "cell") == -1
    c = arrays["cell"]
    first = int(np.argmax(c[1:] < c[:-1])) + 1
    assert eng.verify_sort(to_dev(eng, arrays), dims, "cell") == first
    key = np.lexsort((arrays["gene"], arrays["umi"], arrays["cell"]))
    s = {k: v[key] for k, v in arrays.items()}
    assert eng.verify_sort(to_dev(eng, s), dims, "cell_umi_gene") == -1
    assert eng.verify_sort(to_dev(eng, s), dims, "gene_cell_umi") > 0


@pytest.mark.gpu
def test_unsorted_input_cell_metrics_after_gpu_sort(eng):
    """Config 5 shape: globally shuffled records, GPU sort by cell, then the exact-sum cell and
    grouped gene metrics equal those of the cell-sorted original (integers and floats exactly)."""
    from sctools_amd import engine as E
    from sctools_amd import synth

    data = synth.generate(synth.SynthConfig(n_reads=4_000_000, n_cells=400, n_genes=5000, seed=9), device=eng.device)
    dims = E.Dims(data.n_cell_ids, data.n_gene_ids, data.n_umi_ids)
    mito = torch.from_numpy(data.gene_is_mito).to(eng.device)
    perm = torch.randperm(data.cols["cell"].numel(), generator=torch.Generator().manual_seed(3)).to(eng.device)
    shuffled = {c: t[perm].contiguous() for c, t in data.cols.items()}
    assert eng.verify_sort(shuffled, dims, "cell") > 0
    regrouped = eng.tag_sort(shuffled, dims, "cell")
    assert eng.verify_sort(regrouped, dims, "cell") == -1
    ci0, cf0, p0 = eng.cell_and_gene(data.cols, dims, mito)
    ci0, cf0, p0 = ci0.cpu().numpy(), cf0.cpu().numpy(), p0.clone()
    ci1, cf1, p1 = eng.cell_and_gene(regrouped, dims, mito)
    ci1, cf1 = ci1.cpu().numpy(), cf1.cpu().numpy()
    ent = N.I_ENTITY
    keep = [i for i in range(ci0.shape[1]) if i != ent]  # first-record index differs; the rest must not
    assert np.array_equal(ci0[:, keep], ci1[:, keep])
    assert np.array_equal(np.nan_to_num(cf0, nan=-7.0), np.nan_to_num(cf1, nan=-7.0))
    assert torch.equal(p0, p1)


@pytest.mark.gpu
@pytest.mark.parametrize("n_cell_ids", [200, 1 << 12, 1 << 20])
def test_cell_order_row_passes(eng, n_cell_ids):
    """Cell order without a tiebreak moves whole rows through 1, 2 or 3 LSD passes."""
    from sctools_amd import engine as E

    d, _, arrays = shuffled_synth(300_000, 8, n_cells=150)
    dims = E.Dims(max(n_cell_ids, d.n_cell_ids), d.n_gene_ids, d.n_umi_ids)
    out = to_host(eng.tag_sort(to_dev(eng, arrays), dims, "cell"))
    idx = np_order(arrays, "cell")
    for c in N.RECORD_COLUMNS:
        assert np.array_equal(out[c], arrays[c][idx]), c


@pytest.mark.gpu
def test_tie_runs_of_every_length(eng):
    """(CB, UB, GE) runs of 1 .. 5000 equal records with random query names: the short runs are
    ordered by the in-register network, the long ones (> 16) by the compact (run, name) sort --
    both must give numpy's stable lexsort, ties of equal names in input order."""
    from sctools_amd import engine as E

    d, _, arrays = shuffled_synth(60_000, 11, n_cells=50)
    arrays = {c: a.copy() for c, a in arrays.items()}
    rng = np.random.default_rng(4)
    start = 0
    for L in [2, 3, 4, 5, 8, 9, 15, 16, 17, 31, 64, 300, 5000]:
        idx = rng.choice(arrays["cell"].shape[0], size=L, replace=False)
        for c in ("cell", "umi", "gene"):
            arrays[c][idx] = arrays[c][idx[0]]
        start += L
    n = arrays["cell"].shape[0]
    tie = rng.integers(0, 40, n).astype(np.int32)  # few names: equal names inside runs too
    dims = E.Dims(d.n_cell_ids, d.n_gene_ids, d.n_umi_ids)
    out = to_host(eng.tag_sort(to_dev(eng, arrays), dims, "cell_umi_gene", torch.from_numpy(tie).to(eng.device), 40))
    idx = np_order(arrays, "cell_umi_gene", tie)
    for c in N.RECORD_COLUMNS:
        assert np.array_equal(out[c], arrays[c][idx]), c


@pytest.mark.gpu
@pytest.mark.parametrize("with_tie", [False, True])
def test_group_sort_long_groups(eng, with_tie):
    """Round 6 group sort (tagsort.h): groups of equal (cell, top umi bits) longer than a wave go to the
    one-block-per-group LDS sort (65 .. 2048 records), the rest to the 64-lane networks -- all must give
    numpy's stable lexsort by (CB, UB, GE[, query name]), ties in input order."""
    from sctools_amd import engine as E

    d, _, arrays = shuffled_synth(120_000, 12, n_cells=40)
    arrays = {c: a.copy() for c, a in arrays.items()}
    rng = np.random.default_rng(5)
    n = arrays["cell"].shape[0]
    for L in [63, 64, 65, 66, 100, 127, 128, 129, 300, 1000, 2048]:
        idx = rng.choice(n, size=L, replace=False)
        arrays["cell"][idx] = arrays["cell"][idx[0]]
        arrays["umi"][idx] = arrays["umi"][idx[0]]  # genes stay random: sorted inside the group
    tie = rng.integers(0, 50, n).astype(np.int32) if with_tie else None
    dims = E.Dims(d.n_cell_ids, d.n_gene_ids, d.n_umi_ids)
    out = to_host(eng.tag_sort(to_dev(eng, arrays), dims, "cell_umi_gene",
                               None if tie is None else torch.from_numpy(tie).to(eng.device), 50))
    idx = np_order(arrays, "cell_umi_gene", tie)
    for c in N.RECORD_COLUMNS:
        assert np.array_equal(out[c], arrays[c][idx]), c


@pytest.mark.gpu
@pytest.mark.parametrize("n_cell_ids,n_umi_ids,n_gene_ids,n_tie", [
    (32, 1 << 12, 1 << 16, 1 << 28),         # K1 of 9 bits: the MSD digit is all of it (no segmented pass)
    (512, 1 << 12, 1 << 16, 1 << 28),        # 17 bits: one segmented pass
    (1 << 14, 1 << 20, 1 << 16, 1 << 28),    # 32 bits: the top digit at bit 23, three segmented passes
])
def test_group_sort_key_widths(eng, n_cell_ids, n_umi_ids, n_gene_ids, n_tie):
    """The group sort's 9-bit MSD digit with 0, 1 and 3 segmented 8-bit passes below it (sct_tag_sort
    picks the group key's width from the dictionary sizes: tests/test_group_sort_cpu.py) gives numpy's
    stable lexsort by (CB, UB, GE, query name)."""
    from sctools_amd import engine as E

    _, _, arrays = shuffled_synth(150_000, 14, n_cells=min(300, n_cell_ids - 2))
    arrays = {c: a.copy() for c, a in arrays.items()}
    arrays["umi"] %= min(n_umi_ids, 64)  # few umis: long groups and equal keys
    n = arrays["cell"].shape[0]
    tie = np.random.default_rng(6).integers(0, 1000, n).astype(np.int32)
    dims = E.Dims(n_cell_ids, n_gene_ids, n_umi_ids)
    out = to_host(eng.tag_sort(to_dev(eng, arrays), dims, "cell_umi_gene", torch.from_numpy(tie).to(eng.device), n_tie))
    idx = np_order(arrays, "cell_umi_gene", tie)
    for c in N.RECORD_COLUMNS:
        assert np.array_equal(out[c], arrays[c][idx]), c


@pytest.mark.gpu
def test_group_sort_equals_general_path(eng, monkeypatch):
    """The group sort and the general path (7 LSD passes + run fix-up; SCT_TAG_GROUP_SORT=0) give the same
    records on a config-5-shaped shuffled set, and fall back to the general path for a cell id the group
    key cannot hold."""
    from sctools_amd import engine as E
    from sctools_amd import synth

    cfg = synth.SynthConfig(n_reads=2_000_000, n_cells=200, n_genes=30_000, seed=13, p_secondary=0.1, p_nh1=0.7,
                            p_dup=0.4)
    data = synth.generate(cfg, device=eng.device)
    perm = torch.randperm(cfg.n_reads, generator=torch.Generator().manual_seed(4)).to(eng.device)
    cols = {c: t[perm].contiguous() for c, t in data.cols.items()}
    tie = data.extra["qname"][perm].contiguous()
    dims = E.Dims(data.n_cell_ids, data.n_gene_ids, data.n_umi_ids)
    nq = data.extra["n_qnames"]
    got = to_host(eng.tag_sort(cols, dims, "cell_umi_gene", tie, nq))
    monkeypatch.setenv("SCT_TAG_GROUP_MSD", "0")  # the group sort without its MSD pass (LSD over all of K1)
    got_lsd = to_host(eng.tag_sort(cols, dims, "cell_umi_gene", tie, nq))
    monkeypatch.delenv("SCT_TAG_GROUP_MSD")
    monkeypatch.setenv("SCT_TAG_GROUP_SORT", "0")
    want = to_host(eng.tag_sort(cols, dims, "cell_umi_gene", tie, nq))
    monkeypatch.delenv("SCT_TAG_GROUP_SORT")
    for c in N.RECORD_COLUMNS:
        assert np.array_equal(got[c], want[c]), c
        assert np.array_equal(got_lsd[c], want[c]), c
    # a cell id >= 2^bits(n_cell_ids): the general path's result (which keeps the id in its row)
    bad = {c: t.clone() for c, t in cols.items()}
    bad["cell"][17] = 1 << 20
    got = to_host(eng.tag_sort(bad, dims, "cell_umi_gene", tie, nq))
    monkeypatch.setenv("SCT_TAG_GROUP_SORT", "0")
    want = to_host(eng.tag_sort(bad, dims, "cell_umi_gene", tie, nq))
    for c in N.RECORD_COLUMNS:
        assert np.array_equal(got[c], want[c]), c
