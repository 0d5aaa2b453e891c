"""HIP engine parity: the GPU path against the reference's outputs and the oracle.

* bundled BAMs and synthetic fixture sets: SCT_FLOAT_WELFORD output must be
  byte-identical to the reference CSVs; SCT_FLOAT_EXACT_SUM must match every
  integer and every float within 1e-9 relative (north-star tolerance);
* larger synthetic sets generated on the GPU: ints identical to the oracle,
  Welford floats bit-identical, exact-sum floats within 1e-9;
* size-independent properties at multi-million records.
"""
import numpy as np
import pytest
import torch

import helpers as H
from oracle import oracle as O

pytestmark = pytest.mark.gpu

REL = 1e-9


@pytest.fixture(scope="module")
def eng():
    from sctools_amd import engine as E

    return E.get_engine("cuda:0")


def dims_of(n_cells, n_genes, n_umis):
    from sctools_amd import engine as E

    return E.Dims(n_cells, n_genes, n_umis)


def run_gpu(eng, arrays, mode, dims, mito, float_mode):
    from sctools_amd import engine as E

    cols = E.to_device(arrays, eng.device)
    gm = torch.from_numpy(np.ascontiguousarray(mito, dtype=np.uint8)).to(eng.device)
    if mode == "gene_grouped":
        part = eng.gene_partials(cols, dims)
        gi, gf = eng.finalize_partials(part)
    else:
        gi, gf = eng.compute(cols, mode, dims, gm, gm, float_mode=float_mode)
    return gi.cpu().numpy(), gf.cpu().numpy()


@pytest.mark.parametrize("bam", H.BAMS)
@pytest.mark.parametrize("mode", ["cell", "gene"])
def test_bundled_bams_welford_byte_identical(eng, bam, mode):
    cols = H.bam_columns(bam, mode)
    mito, _ = cols.gene_flags()
    d = dims_of(len(cols.cells), len(cols.genes), len(cols.umis))
    gi, gf = run_gpu(eng, cols.arrays, mode, d, mito, "welford")
    got = H.render(mode, gi, gf, cols.arrays, cols.cells.names, cols.genes.names)
    assert got == H.golden_text(bam, mode)


@pytest.mark.parametrize("bam", H.BAMS)
@pytest.mark.parametrize("mode", ["cell", "gene"])
def test_bundled_bams_exact_sum_within_tolerance(eng, bam, mode):
    cols = H.bam_columns(bam, mode)
    mito, _ = cols.gene_flags()
    d = dims_of(len(cols.cells), len(cols.genes), len(cols.umis))
    gi, gf = run_gpu(eng, cols.arrays, mode, d, mito, "exact")
    got = H.render(mode, gi, gf, cols.arrays, cols.cells.names, cols.genes.names)
    H.assert_csv_close(got, H.golden_text(bam, mode), rel=REL)


@pytest.mark.parametrize("name", H.SYNTH)
@pytest.mark.parametrize("mode,kind", [("cell", "cell"), ("gene", "gene_run")])
@pytest.mark.parametrize("float_mode", ["welford", "exact"])
def test_synthetic_fixtures(eng, name, mode, kind, float_mode):
    s = H.synth(name)
    gi, gf = run_gpu(eng, s.arrays, mode, dims_of(*s.dims), s.gene_is_mito, float_mode)
    got = H.render(mode, gi, gf, s.arrays, s.cell_names, s.gene_names)
    if float_mode == "welford":
        assert got == H.synth_text(name, kind)
    else:
        H.assert_csv_close(got, H.synth_text(name, kind), rel=REL)


@pytest.mark.parametrize("name", H.SYNTH)
def test_synthetic_grouped_gene(eng, name):
    s = H.synth(name)
    gi, gf = run_gpu(eng, s.arrays, "gene_grouped", dims_of(*s.dims), s.gene_is_mito, "exact")
    got = H.render("gene_grouped", gi, gf, s.arrays, s.cell_names, s.gene_names)
    H.assert_csv_close(got, H.synth_text(name, "gene_grouped"), rel=REL)


def gpu_synth(n, cells, genes, seed, sigma=1.0, **kw):
    from sctools_amd import synth

    return synth.generate(synth.SynthConfig(n_reads=n, n_cells=cells, n_genes=genes, seed=seed, sigma=sigma,
                                            **kw), device="cuda:0")


def host_cols(d):
    h = {c: t.cpu().numpy() for c, t in d.cols.items()}
    for c in ("gq_sum", "gq_len", "gq_gt30"):
        h[c] = h[c].view(np.uint16)
    return h


def compare(gi, gf, oi, of, exact_floats):
    assert gi.shape == oi.shape
    assert np.array_equal(gi, oi)
    nan_g, nan_o = np.isnan(gf), np.isnan(of)
    assert np.array_equal(nan_g, nan_o)
    if exact_floats:
        assert np.array_equal(gf[~nan_g], of[~nan_o])
    else:
        a, b = gf[~nan_g], of[~nan_o]
        rel = np.abs(a - b) / np.maximum(np.maximum(np.abs(a), np.abs(b)), 1e-300)
        assert (rel <= REL).all(), rel.max()


@pytest.mark.parametrize("seed,n,cells,genes,sigma", [
    (21, 300_000, 60, 3_000, 1.0),
    (22, 2_000_000, 200, 30_000, 1.0),
    (23, 1_500_000, 2_000, 5_000, 2.0),
    (24, 8_000_000, 100, 30_000, 2.0),  # heavy tail: cells of 10^5-10^6 reads, several partition levels
    (25, 1_000_000, 300, 100_000, 1.0),  # 200,001 gene ids: more gene buckets than 2048 (dynamic LDS)
])
def test_gpu_generated_against_oracle(eng, seed, n, cells, genes, sigma):
    from sctools_amd import engine as E

    d = gpu_synth(n, cells, genes, seed, sigma=sigma, p_none_cell_reads=0.005)
    h = host_cols(d)
    dims = E.Dims(d.n_cell_ids, d.n_gene_ids, d.n_umi_ids)
    mito = torch.from_numpy(d.gene_is_mito).to(eng.device)
    for mode in ("cell", "gene"):
        oi, of = O.run(h, mode, d.gene_is_mito, d.n_gene_ids, threads=8)
        for fm in ("welford", "exact"):
            gi, gf = eng.compute(d.cols, mode, dims, mito, mito, float_mode=fm)
            compare(gi.cpu().numpy(), gf.cpu().numpy(), oi, of, exact_floats=(fm == "welford"))
    oi, of = O.run(h, "gene_grouped", d.gene_is_mito, d.n_gene_ids, threads=8)
    gi, gf = eng.finalize_partials(eng.gene_partials(d.cols, dims))
    gi, gf = gi.cpu().numpy(), gf.cpu().numpy()
    live = oi[:, 0] > 0
    assert np.array_equal(gi[:, 0] > 0, live)
    compare(gi[live], gf[live], oi[live], of[live], exact_floats=False)


@pytest.mark.parametrize("layout", ["boundaries", "head_65", "one_giant"])
def test_welford_head_entities(eng, layout):
    """The Welford drop-in's entity classes against the oracle, bit for bit (finalize.h): lanes of
    one entity (< 48 records), the head kernel (k_welford_head2: the 64 largest entities, 16 per
    block, 16-record chunks, a 224-record LDS ring) and the other chains (k_welford_chains).  Entity
    lengths sit on the class boundary (47 / 48 / 49), on and beside chunk and ring multiples, one
    past a full head group (65 big entities), and a 300k-record entity beside short ones."""
    from sctools_amd import engine as E

    if layout == "boundaries":
        sizes = [47, 48, 49, 1, 2, 15, 16, 17, 223, 224, 225, 239, 240, 241, 4096, 4097, 5000]
    elif layout == "head_65":
        sizes = [3000 + 37 * i for i in range(65)] + [48] * 5 + [30] * 20
    else:
        sizes = [300_000, 60, 49, 48, 47, 3] + [700] * 10
    n = int(sum(sizes))
    d = gpu_synth(n, 50, 3_000, 91 + len(sizes))
    cell = np.repeat(np.arange(len(sizes), dtype=np.int32), np.asarray(sizes))
    d.cols["cell"] = torch.from_numpy(cell).to(eng.device)
    h = host_cols(d)
    dims = E.Dims(max(d.n_cell_ids, len(sizes)), d.n_gene_ids, d.n_umi_ids)
    mito = torch.from_numpy(d.gene_is_mito).to(eng.device)
    oi, of = O.run(h, "cell", d.gene_is_mito, d.n_gene_ids, threads=8)
    gi, gf = eng.compute(d.cols, "cell", dims, mito, mito, float_mode="welford")
    compare(gi.cpu().numpy(), gf.cpu().numpy(), oi, of, exact_floats=True)


def test_welford_head_entities_gene_mode(eng):
    """The same kernels in the gene view's three-stream form (GatherGeneMetrics' entities are
    genes): gene runs of boundary lengths, 70 big genes and one 200k-record gene."""
    from sctools_amd import engine as E

    sizes = [200_000, 47, 48, 49, 224, 225] + [2000 + 29 * i for i in range(70)] + [5] * 30
    n = int(sum(sizes))
    d = gpu_synth(n, 300, 3_000, 97)
    gene = np.repeat(np.arange(len(sizes), dtype=np.int32), np.asarray(sizes))
    d.cols["gene"] = torch.from_numpy(gene).to(eng.device)
    h = host_cols(d)
    n_genes = max(d.n_gene_ids, len(sizes))
    mito_np = np.zeros(n_genes, dtype=np.uint8)
    mito_np[: d.gene_is_mito.shape[0]] = d.gene_is_mito
    dims = E.Dims(d.n_cell_ids, n_genes, d.n_umi_ids)
    mito = torch.from_numpy(mito_np).to(eng.device)
    oi, of = O.run(h, "gene", mito_np, n_genes, threads=8)
    gi, gf = eng.compute(d.cols, "gene", dims, mito, mito, float_mode="welford")
    compare(gi.cpu().numpy(), gf.cpu().numpy(), oi, of, exact_floats=True)


def test_properties_at_scale(eng):
    """Size-independent invariants on 20M records (the oracle would take too long)."""
    from sctools_amd import engine as E
    from sctools_amd import _native as N

    d = gpu_synth(20_000_000, 2_000, 30_000, 31)
    dims = E.Dims(d.n_cell_ids, d.n_gene_ids, d.n_umi_ids)
    mito = torch.from_numpy(d.gene_is_mito).to(eng.device)
    ci, cf = eng.compute(d.cols, "cell", dims, mito, mito, float_mode="exact")
    ci2, cf2 = eng.compute(d.cols, "cell", dims, mito, mito, float_mode="exact")
    assert torch.equal(ci, ci2) and torch.equal(torch.nan_to_num(cf, 7.0), torch.nan_to_num(cf2, 7.0))
    gi, gf = eng.finalize_partials(eng.gene_partials(d.cols, dims))
    n = d.cols["cell"].numel()
    assert int(ci[:, N.I_N_READS].sum()) == n
    assert int(gi[:, N.I_N_READS].sum()) == n
    # every molecule / fragment is counted once from the cell side and once from the gene side
    for col in (N.I_N_MOL, N.I_N_FRAG, N.I_MOL_SINGLE, N.I_FRAG_SINGLE, N.I_DUP, N.I_SPLICED):
        assert int(ci[:, col].sum()) == int(gi[:, col].sum())
    # (cell, gene) pairs: sum of n_genes over cells == sum of cells_expressing over genes
    assert int(ci[:, N.I_N_K1].sum()) == int(gi[:, N.I_N_K1].sum())
    assert int(ci[:, N.I_K1_MULTI].sum()) == int(gi[:, N.I_K1_MULTI].sum())
    # Welford and exact-sum agree within tolerance at this size
    wi, wf = eng.compute(d.cols, "cell", dims, mito, mito, float_mode="welford")
    assert torch.equal(wi, ci)
    a, b = wf.cpu().numpy(), cf.cpu().numpy()
    ok = np.isclose(a, b, rtol=REL, atol=0) | (np.isnan(a) & np.isnan(b))
    assert ok.all()


def test_combined_cell_and_gene_pass(eng):
    """sct_cell_metrics_gene_partials == separate cell rows + grouped gene partials."""
    from sctools_amd import engine as E

    d = gpu_synth(1_000_000, 150, 8_000, 41, p_none_cell_reads=0.01)
    dims = E.Dims(d.n_cell_ids, d.n_gene_ids, d.n_umi_ids)
    mito = torch.from_numpy(d.gene_is_mito).to(eng.device)
    ci, cf, part = eng.cell_and_gene(d.cols, dims, mito)
    ci2, cf2 = eng.compute(d.cols, "cell", dims, mito, mito, float_mode="exact")
    part2 = eng.gene_partials(d.cols, dims)
    assert torch.equal(ci, ci2)
    assert torch.equal(torch.nan_to_num(cf, 3.0), torch.nan_to_num(cf2, 3.0))
    assert torch.equal(part, part2)
    h = host_cols(d)
    oi, of = O.run(h, "gene_grouped", d.gene_is_mito, d.n_gene_ids, threads=8)
    gi, gf = eng.finalize_partials(part)
    gi, gf = gi.cpu().numpy(), gf.cpu().numpy()
    live = oi[:, 0] > 0
    compare(gi[live], gf[live], oi[live], of[live], exact_floats=False)


@pytest.mark.parametrize("case", ["at_limits", "over_limits"])
def test_gene_payload_formats(eng, case):
    """Grouped gene partials use the 8-byte payload when every stream operand fits its field
    (uy <= 31, gq <= 511, gq_sum <= 32767: gene.h gene_payload8) and the 16-byte one otherwise;
    the rows equal the oracle's either way, and the one-pass partials equal the gene-only pass's
    (which always uses the 16-byte payload)."""
    from sctools_amd import engine as E

    d = gpu_synth(400_000, 80, 4_000, 26)
    cols = {c: t.clone() for c, t in d.cols.items()}
    n = cols["cell"].numel()
    gen = torch.Generator().manual_seed(9)
    idx = torch.randperm(n, generator=gen)[: n // 40].to(eng.device)
    k = idx.numel()
    uy, gq, gs = (31, 511, 32767) if case == "at_limits" else (40, 600, 40000)
    rnd = torch.rand(k, generator=gen).to(eng.device)
    cols["uy_len"][idx] = uy
    cols["uy_gt30"][idx] = (rnd * (uy + 1)).to(torch.uint8).clamp(max=uy)
    cols["gq_len"][idx] = gq
    cols["gq_gt30"][idx] = (rnd * (gq + 1)).to(torch.int32).clamp(max=gq).to(torch.int16)
    cols["gq_sum"][idx] = torch.tensor(gs, dtype=torch.int32).to(torch.int16).item()  # uint16 bits
    dims = E.Dims(d.n_cell_ids, d.n_gene_ids, d.n_umi_ids)
    mito = torch.from_numpy(d.gene_is_mito).to(eng.device)
    ci, cf, part = eng.cell_and_gene(cols, dims, mito)
    assert torch.equal(part, eng.gene_partials(cols, dims))
    h = {c: t.cpu().numpy() for c, t in cols.items()}
    for c in ("gq_sum", "gq_len", "gq_gt30"):
        h[c] = h[c].view(np.uint16)
    assert int(h["gq_sum"].max()) == gs and int(h["uy_len"].max()) == uy
    oi, of = O.run(h, "gene_grouped", d.gene_is_mito, d.n_gene_ids, threads=8)
    gi, gf = eng.finalize_partials(part)
    gi, gf = gi.cpu().numpy(), gf.cpu().numpy()
    live = oi[:, 0] > 0
    compare(gi[live], gf[live], oi[live], of[live], exact_floats=False)
    oi, of = O.run(h, "cell", d.gene_is_mito, d.n_gene_ids, threads=8)
    compare(ci.cpu().numpy(), cf.cpu().numpy(), oi, of, exact_floats=False)


def test_grouped_needs_cell_sorted_input(eng):
    from sctools_amd import _native as N

    cols = H.bam_columns("unsorted", "cell")
    d = dims_of(len(cols.cells), len(cols.genes), len(cols.umis))
    from sctools_amd import engine as E

    dev = E.to_device(cols.arrays, eng.device)
    with pytest.raises(N.EngineError, match="cell-sorted"):
        eng.gene_partials(dev, d)


@pytest.mark.parametrize("name", ["s0", "s1", "s2"])
def test_sharded_partials_add_up(eng, name):
    """Cell-sharded partial rows summed (what the RCCL all-reduce does) finalize to exactly the
    unsharded gene rows -- floats included, since exact-sum lanes are order-free integers."""
    from sctools_amd import distributed as D
    from sctools_amd import engine as E

    s = H.synth(name)
    d = dims_of(*s.dims)
    cols = E.to_device(s.arrays, eng.device)
    gm = torch.from_numpy(s.gene_is_mito).to(eng.device)
    ci, cf, whole = eng.cell_and_gene(cols, d, gm)
    wi, wf = eng.finalize_partials(whole.clone())
    acc = torch.zeros_like(whole)
    rows_i, rows_f = [], []
    for lo, hi in D.shard_bounds(cols["cell"], 3):
        si, sf, p = eng.cell_and_gene(D.shard(cols, lo, hi), d, gm)
        si = si.clone()
        si[:, 23] += lo
        rows_i.append(si)
        rows_f.append(sf.clone())
        acc += p
    gi, gf = eng.finalize_partials(acc)
    assert torch.equal(gi, wi)
    assert torch.equal(gf.view(torch.int64), wf.view(torch.int64))
    assert torch.equal(torch.cat(rows_i), ci)
    assert torch.equal(torch.cat(rows_f).view(torch.int64), cf.view(torch.int64))
