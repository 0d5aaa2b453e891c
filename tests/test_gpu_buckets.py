"""Edge cases of the bucket path (sctools_amd/csrc/bucket.h) against the oracle.

Records are crafted so that every branch of the MSD partition runs:
* a k1 value (gene of a cell) with > 3071 reads, split over sibling buckets (k1 split flags);
* a molecule with > 3071 reads over many positions, split on fragment-hash bits (molecule flags);
* a molecule with > 3071 reads at ONE fragment: a giant bucket (whole key fixed);
* a giant holding two different fragments whose hashes collide in the key's hash bits,
  plus unmapped records (the exact fragment loop);
* big buckets (1024-3071 records) from level 0 and from a level-1 child;
* thousands of tiny entities (many buckets per tile);
both with narrow dictionaries (the k1 boundary inside the first digit) and wide ones.
The global-sort path (SCT_FORCE_GLOBAL_SORT=1) must give identical rows.
"""
import os

import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu

REL = 1e-9
M32 = 0xFFFFFFFF


def frag_hash(ref, pos, strand):
    """util.h frag_hash, for crafting top-bit collisions."""
    h = ((ref * 0x9E3779B1) ^ (pos * 0x85EBCA77) ^ (strand * 0xC2B2AE3D)) & M32
    h ^= h >> 15
    h = (h * 0x2C1B3C6D) & M32
    h ^= h >> 12
    h = (h * 0x297A2D39) & M32
    h ^= h >> 15
    return h


def bitlen(v):
    return 0 if v <= 1 else int(v - 1).bit_length()


def colliding_pos(ref, pos, hbits, start=5000):
    want = frag_hash(ref & M32, pos, 0) >> (32 - hbits)
    p = start
    while True:
        if p != pos and frag_hash(ref & M32, p, 0) >> (32 - hbits) == want:
            return p
        p += 1


def craft(n_gene_ids, n_umi_ids, seed):
    rng = np.random.default_rng(seed)
    hbits = min(8, 47 - bitlen(n_gene_ids) - bitlen(n_umi_ids))  # bucket.h kMaxKeyBits
    rows = []  # (cell, gene, umi, ref, pos, unmapped)

    def add(cell, gene, umi, ref, pos, unmapped=False, k=1):
        for _ in range(k):
            rows.append((cell, gene, umi, ref, pos, unmapped))

    g_heavy = n_gene_ids - 3
    # cell 0: background + a giant molecule at one fragment + a colliding-hash giant + unmapped reads
    # (giants: > kBigCap = 3071 records under one fixed key')
    for _ in range(2000):
        add(0, int(rng.integers(1, n_gene_ids)), int(rng.integers(0, n_umi_ids)), int(rng.integers(0, 25)),
            int(rng.integers(0, 1 << 20)))
    add(0, g_heavy, 5, 1, 1000, k=4000)
    p2 = colliding_pos(3, 777, hbits)
    add(0, g_heavy, 6, 3, 777, k=2000)
    add(0, g_heavy, 6, 3, p2, k=1800)
    add(0, g_heavy, 6, 3, 777, k=1)
    add(0, g_heavy, 6, -1, -1, unmapped=True, k=40)
    # cell 1: one gene with 9000 reads over 12 UMIs (k1 split across sibling buckets)
    for _ in range(9000):
        add(1, 7 % n_gene_ids, int(rng.integers(0, 12)), 2, int(rng.integers(0, 1 << 16)))
    # cell 2: one molecule with 5000 reads over 400 positions (molecule split on hash bits)
    for _ in range(5000):
        add(2, 9 % n_gene_ids, 3, 4, int(rng.integers(0, 400)) * 10)
    # cell 3: 2500 reads of one gene over 30 UMIs: a big bucket straight from level 0
    for _ in range(2500):
        add(3, 11 % n_gene_ids, int(rng.integers(0, min(30, n_umi_ids))), 5, int(rng.integers(0, 1 << 18)))
    # cell 4: background + 2800 reads of one gene: a big bucket from a level-1 child
    for _ in range(2000):
        add(4, int(rng.integers(1, n_gene_ids)), int(rng.integers(0, n_umi_ids)), int(rng.integers(0, 25)),
            int(rng.integers(0, 1 << 20)))
    for _ in range(2800):
        add(4, 13 % n_gene_ids, int(rng.integers(0, min(200, n_umi_ids))), 6, int(rng.integers(0, 1 << 18)))
    # cells 5..: thousands of tiny cells (1-4 reads)
    c = 5
    for _ in range(4000):
        for _ in range(int(rng.integers(1, 5))):
            add(c, int(rng.integers(0, n_gene_ids)), int(rng.integers(0, n_umi_ids)), int(rng.integers(0, 25)),
                int(rng.integers(0, 1 << 20)), unmapped=bool(rng.random() < 0.05))
        c += 1
    a = np.array(rows, dtype=np.int64)
    # shuffle within cells (input order inside an entity is arbitrary)
    order = np.lexsort((rng.random(len(a)), a[:, 0]))
    a = a[order]
    n = len(a)
    unm = a[:, 5].astype(bool)
    bits = np.where(unm, 1, 0) | np.where(rng.random(n) < 0.5, 2, 0)
    bits[(a[:, 0] == 0) & (a[:, 1] == g_heavy)] &= ~2  # giants on the + strand (crafted positions)
    bits |= np.where(~unm & (rng.random(n) < 0.3), 4, 0) | np.where(~unm & (rng.random(n) < 0.1), 8, 0)
    bits |= np.where(~unm & (rng.random(n) < 0.8), 16, 0) | np.where(rng.random(n) < 0.9, 32, 0)
    bits |= 64 | np.where(rng.random(n) < 0.95, 128, 0)
    glen = rng.integers(30, 99, n)
    arrays = {
        "cell": a[:, 0].astype(np.int32), "umi": a[:, 2].astype(np.int32), "gene": a[:, 1].astype(np.int32),
        "ref": np.where(unm, -1, a[:, 3]).astype(np.int32), "pos": np.where(unm, -1, a[:, 4]).astype(np.int32),
        "gq_len": glen.astype(np.uint16), "gq_sum": (glen * rng.integers(20, 40, n)).astype(np.uint16),
        "gq_gt30": rng.integers(0, glen + 1).astype(np.uint16), "bits": bits.astype(np.uint8),
        "xf": np.where(unm, 0, rng.integers(1, 5, n)).astype(np.uint8),
        "cy_len": np.full(n, 16, np.uint8), "cy_gt30": rng.integers(0, 17, n).astype(np.uint8),
        "uy_len": np.full(n, 10, np.uint8), "uy_gt30": rng.integers(0, 11, n).astype(np.uint8),
    }
    mito = np.zeros(n_gene_ids, np.uint8)
    mito[[7 % n_gene_ids, g_heavy]] = 1
    return arrays, mito, int(a[:, 0].max()) + 1


@pytest.fixture(scope="module")
def eng():
    from sctools_amd import engine as E

    return E.get_engine("cuda:0")


def compare(gi, gf, oi, of, exact):
    assert gi.shape == oi.shape
    assert np.array_equal(gi, oi), np.argwhere(gi != oi)[:10]
    ng, no = np.isnan(gf), np.isnan(of)
    assert np.array_equal(ng, no)
    if exact:
        assert np.array_equal(gf[~ng], of[~no])
    else:
        x, y = gf[~ng], of[~no]
        rel = np.abs(x - y) / np.maximum(np.maximum(np.abs(x), np.abs(y)), 1e-300)
        assert (rel <= REL).all(), rel.max()


def run_all(eng, arrays, mito, n_cells, n_gene_ids, n_umi_ids):
    from sctools_amd import engine as E

    dims = E.Dims(n_cells, n_gene_ids, n_umi_ids)
    cols = E.to_device(arrays, eng.device)
    gm = torch.from_numpy(mito).to(eng.device)
    out = {}
    for mode in ("cell", "gene"):
        for fm in ("welford", "exact"):
            gi, gf = eng.compute(cols, mode, dims, gm, gm, float_mode=fm)
            out[(mode, fm)] = (gi.cpu().numpy(), gf.cpu().numpy())
    ci, cf, part = eng.cell_and_gene(cols, dims, gm)
    gi, gf = eng.finalize_partials(part)
    out["combined_cell"] = (ci.cpu().numpy(), cf.cpu().numpy())
    out["grouped"] = (gi.cpu().numpy(), gf.cpu().numpy())
    return out


@pytest.mark.parametrize("n_gene_ids,n_umi_ids,seed", [(50, 100, 1), (30_000, 1 << 20, 2),
                                                       (120_000, 1 << 24, 5)])  # 10x v3: 12-bp UMIs
def test_bucket_edge_cases_match_oracle(eng, n_gene_ids, n_umi_ids, seed):
    arrays, mito, n_cells = craft(n_gene_ids, n_umi_ids, seed)
    got = run_all(eng, arrays, mito, n_cells, n_gene_ids, n_umi_ids)
    for mode in ("cell", "gene"):
        oi, of = O.run(arrays, mode, mito, n_gene_ids, threads=8)
        compare(*got[(mode, "welford")], oi, of, exact=True)
        compare(*got[(mode, "exact")], oi, of, exact=False)
        if mode == "cell":
            compare(*got["combined_cell"], oi, of, exact=False)
    oi, of = O.run(arrays, "gene_grouped", mito, n_gene_ids, threads=8)
    gi, gf = got["grouped"]
    live = oi[:, 0] > 0
    assert np.array_equal(gi[:, 0] > 0, live)
    compare(gi[live], gf[live], oi[live], of[live], exact=False)


def test_global_sort_path_agrees(eng, monkeypatch):
    arrays, mito, n_cells = craft(300, 4096, 3)
    a = run_all(eng, arrays, mito, n_cells, 300, 4096)
    monkeypatch.setenv("SCT_FORCE_GLOBAL_SORT", "1")
    b = run_all(eng, arrays, mito, n_cells, 300, 4096)
    for k in a:
        assert np.array_equal(a[k][0], b[k][0]), k
        assert np.array_equal(np.nan_to_num(a[k][1], nan=7.0), np.nan_to_num(b[k][1], nan=7.0)), k


@pytest.mark.parametrize("column", ["gene", "umi", "cell"])
def test_ids_outside_the_dictionaries_are_rejected(eng, column):
    """Invalid input fails loudly (SCT_EINVAL) instead of corrupting keys or indexing tables."""
    from sctools_amd import _native as N
    from sctools_amd import engine as E

    arrays, mito, n_cells = craft(300, 4096, 4)
    arrays = {k: v.copy() for k, v in arrays.items()}
    limit = {"gene": 300, "umi": 4096, "cell": n_cells}[column]
    arrays[column][len(arrays[column]) // 2] = limit + 5
    dims = E.Dims(n_cells, 300, 4096)
    cols = E.to_device(arrays, eng.device)
    gm = torch.from_numpy(mito).to(eng.device)
    if column == "cell":  # the cell id indexes the grouped-partials duplicate check
        with pytest.raises(N.EngineError, match="outside"):
            eng.cell_and_gene(cols, dims, gm)
    else:
        with pytest.raises(N.EngineError, match="outside"):
            eng.compute(cols, "cell", dims, gm, gm, float_mode="exact")
        with pytest.raises(N.EngineError, match="outside"):
            eng.cell_and_gene(cols, dims, gm)


@pytest.mark.parametrize("n", [1, 5, 4099, 1_000_003, 20_000_002])
def test_run_count_aligned_and_misaligned_columns(eng, n):
    """Entity-run counting (k_heads4 on 16-byte aligned columns, k_heads otherwise) and the
    chunked tile-count scan (> 4096 tiles at 20M records) against numpy on the same runs."""
    from sctools_amd import _native as N
    from sctools_amd import engine as E

    rng = np.random.default_rng(n)
    lens = rng.geometric(1.0 / 37, size=n)
    cell = np.repeat(np.arange(lens.size, dtype=np.int32), lens)[:n]
    cell = (cell * 7919 % 1_000_003).astype(np.int32)  # runs of distinct, unsorted values
    want = 1 + int(np.count_nonzero(cell[1:] != cell[:-1]))
    dims = E.Dims(1_000_003, 1, 1)
    for shift in (0, 1):  # shift 1: the cell column starts 4 bytes past a 16-byte boundary
        buf = torch.zeros(n + 1, dtype=torch.int32, device=eng.device)
        buf[shift:shift + n] = torch.from_numpy(cell).to(eng.device)
        cols = {c: torch.zeros(n, dtype=E._TORCH_DTYPES[c], device=eng.device) for c in N.RECORD_COLUMNS}
        cols["cell"] = buf[shift:shift + n]
        assert (cols["cell"].data_ptr() % 16 == 0) == (shift == 0)
        assert eng.count_entities(cols, "cell", dims) == want, shift


def kernels_run(eng, fn):
    eng.profile_only("")
    eng.profile_enable(True)
    try:
        fn()
        torch.cuda.synchronize()
    finally:
        eng.profile_enable(False)
    return set(eng.profile_read())


def test_10x_v3_shard_stays_on_the_bucket_path(eng):
    """k1 + k2 = 17 + 24 bits (2^24 UMI ids, 120k gene ids) fits the 47-bit bucket key: no
    device-wide LSD sort runs, and the rows match the oracle."""
    from sctools_amd import engine as E
    from sctools_amd import synth

    d = synth.generate(synth.SynthConfig(n_reads=2_000_000, n_cells=300, n_genes=60_000, seed=12, umi_bits=24),
                       device=eng.device)
    assert d.n_umi_ids == 1 << 24 and d.n_gene_ids > 1 << 16
    dims = E.Dims(d.n_cell_ids, d.n_gene_ids, d.n_umi_ids)
    mito = torch.from_numpy(d.gene_is_mito).to(eng.device)
    out = {}
    ran = kernels_run(eng, lambda: out.update(zip(("ci", "cf", "p"), eng.cell_and_gene(d.cols, dims, mito))))
    assert "hash_tile" in ran and not any(k.startswith("radix") for k in ran), ran
    h = {c: t.cpu().numpy() for c, t in d.cols.items()}
    for c in ("gq_sum", "gq_len", "gq_gt30"):
        h[c] = h[c].view(np.uint16)
    oi, of = O.run(h, "cell", d.gene_is_mito, d.n_gene_ids, threads=8)
    compare(out["ci"].cpu().numpy(), out["cf"].cpu().numpy(), oi, of, exact=False)
    gi, gf = eng.finalize_partials(out["p"])
    oi, of = O.run(h, "gene_grouped", d.gene_is_mito, d.n_gene_ids, threads=8)
    live = oi[:, 0] > 0
    compare(gi.cpu().numpy()[live], gf.cpu().numpy()[live], oi[live], of[live], exact=False)


def test_reference_ids_beyond_the_payload_fall_back_to_the_global_sort(eng):
    """A mapped ref id >= 2^14 does not fit the bucket payload: the call reruns on the LSD-sort
    path and the rows still match the oracle."""
    from sctools_amd import engine as E

    arrays, mito, n_cells = craft(300, 4096, 6)
    arrays = {k: v.copy() for k, v in arrays.items()}
    mapped = arrays["ref"] >= 0
    arrays["ref"][mapped] += 20_000
    dims = E.Dims(n_cells, 300, 4096)
    cols = E.to_device(arrays, eng.device)
    gm = torch.from_numpy(mito).to(eng.device)
    out = {}
    ran = kernels_run(eng, lambda: out.update(zip(("i", "f"), eng.compute(cols, "cell", dims, gm, gm,
                                                                           float_mode="welford"))))
    assert any(k.startswith("radix") for k in ran), ran
    oi, of = O.run(arrays, "cell", mito, 300, threads=8)
    compare(out["i"].cpu().numpy(), out["f"].cpu().numpy(), oi, of, exact=True)


# Round 6: the side stream after the key pass (big buckets beside the partition levels, the gene
# view's plan, the cell rows' finalize) and the bucket-descriptor fill behind the entity count only
# reorder work between streams: every switch must leave the rows bit-identical.
SIDE_SWITCHES = [
    {"SCT_NO_SIDE": "1", "SCT_NO_PREFILL": "1"},
    {"SCT_NO_LEVEL_BIG": "1"},
    {"SCT_NO_EARLY_BIG": "1"},
    {"SCT_NO_SIDE_FIN": "1"},
    {"SCT_BIG_BESIDE_HASH": "1"},
]


def _same_rows(a, b):
    for k in a:
        assert np.array_equal(a[k][0], b[k][0]), k
        assert np.array_equal(np.nan_to_num(a[k][1], nan=7.0).view(np.int64),
                              np.nan_to_num(b[k][1], nan=7.0).view(np.int64)), k


@pytest.mark.parametrize("switches", SIDE_SWITCHES, ids=lambda d: ",".join(d))
def test_side_stream_switches_leave_rows_identical(eng, monkeypatch, switches):
    arrays, mito, n_cells = craft(30_000, 1 << 20, 6)
    a = run_all(eng, arrays, mito, n_cells, 30_000, 1 << 20)
    for k, v in switches.items():
        monkeypatch.setenv(k, v)
    b = run_all(eng, arrays, mito, n_cells, 30_000, 1 << 20)
    _same_rows(a, b)


def test_side_stream_switches_on_a_config2_shaped_shard(eng, monkeypatch):
    """4M config-2-shaped records (Zipf genes, ~10k-record cells): partition levels 2-3, big buckets
    from several levels, so the side stream carries work at every level."""
    from sctools_amd import engine as E
    from sctools_amd import synth

    d = synth.generate(synth.SynthConfig(n_reads=4_000_000, n_cells=400, n_genes=30_000, seed=11),
                       device=eng.device, chunk=16_000_000)
    dims = E.Dims(d.n_cell_ids, d.n_gene_ids, d.n_umi_ids)
    mito = torch.from_numpy(d.gene_is_mito).to(eng.device)

    def rows():
        ci, cf, part = eng.cell_and_gene(d.cols, dims, mito)
        gi, gf = eng.finalize_partials(part)
        return {"cell": (ci.cpu().numpy(), cf.cpu().numpy()), "gene": (gi.cpu().numpy(), gf.cpu().numpy())}

    a = rows()
    monkeypatch.setenv("SCT_NO_SIDE", "1")
    monkeypatch.setenv("SCT_NO_PREFILL", "1")
    b = rows()
    _same_rows(a, b)
