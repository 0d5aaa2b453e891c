"""BASELINE.json configs 2-5 at their own sizes: the HIP path against the oracle.

Each config is generated on the GPU with the SURVEY.md 8(d) recipe at the size BASELINE.json
names, run through the C-ABI, copied back and checked against the C restatement of the
reference (oracle/sct_oracle.c, 16 OpenMP threads):

* config 2: 100M cell-sorted records, 10k cells (lognormal sigma 1), 30k genes -- cell rows
  (Welford bit-identical, exact-sum within 1e-9) and grouped gene rows;
* config 3: the config-2 shard cut into 8 cell-disjoint ranges (distributed.shard_bounds): the
  summed per-shard gene partials (what the RCCL all-reduce adds) equal the unsharded ones bit
  for bit, and the concatenated cell rows equal the unsharded rows;
* config 4: one GPU's shard of the 1B-read atlas -- 125M records over 62.5k cells with
  lognormal(0, 2) reads per cell (cells of ~10^6 reads);
* config 5: 100M globally shuffled records (30 % NH > 1, 40 % duplicates, secondary
  alignments sharing a query name) sorted on the GPU in the order of
  bam.sort_by_tags_and_queryname (bam.py:698-709): (CB, UB, GE) then query name, stable.  The
  sort is checked as THE stable sort (a record-identity column rides along), then the cell
  metrics of the (CB, UB, GE) order and the gene metrics of the (GE, CB, UB) order are checked
  against the oracle on the same records.

Pass criteria: integers bit-exact, Welford floats bit-exact, exact-sum floats within 1e-9
relative, nan positions identical.  Each test stays well under the 3-minute silence limit.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(600)]

REL = 1e-9
THREADS = 16


@pytest.fixture(scope="module")
def eng():
    from sctools_amd import engine as E

    return E.get_engine("cuda:0")


def generate(n, cells, genes, sigma, seed, **kw):
    from sctools_amd import synth

    cfg = synth.SynthConfig(n_reads=n, n_cells=cells, n_genes=genes, sigma=sigma, seed=seed, **kw)
    return synth.generate(cfg, device="cuda:0", chunk=16_000_000)


def host(cols):
    h = {c: t.cpu().numpy() for c, t in cols.items()}
    for c in ("gq_sum", "gq_len", "gq_gt30"):
        h[c] = h[c].view(np.uint16)
    return h


def dims_of(d):
    from sctools_amd import engine as E

    return E.Dims(d.n_cell_ids, d.n_gene_ids, d.n_umi_ids)


def compare(gi, gf, oi, of, exact_floats):
    assert gi.shape == oi.shape, (gi.shape, oi.shape)
    assert np.array_equal(gi, oi)
    nan_g, nan_o = np.isnan(gf), np.isnan(of)
    assert np.array_equal(nan_g, nan_o)
    if exact_floats:
        assert np.array_equal(gf[~nan_g].view(np.int64), of[~nan_o].view(np.int64))
    else:
        a, b = gf[~nan_g], of[~nan_o]
        rel = np.abs(a - b) / np.maximum(np.maximum(np.abs(a), np.abs(b)), 1e-300)
        assert (rel <= REL).all(), rel.max()


def check_cell_rows(eng, d, cols, h):
    dims = dims_of(d)
    mito = torch.from_numpy(d.gene_is_mito).to(eng.device)
    oi, of = O.run(h, "cell", d.gene_is_mito, d.n_gene_ids, threads=THREADS)
    for fm in ("welford", "exact"):
        gi, gf = eng.compute(cols, "cell", dims, mito, mito, float_mode=fm)
        compare(gi.cpu().numpy(), gf.cpu().numpy(), oi, of, exact_floats=(fm == "welford"))
    return oi


def check_grouped_gene_rows(eng, d, cols, h):
    dims = dims_of(d)
    mito = torch.from_numpy(d.gene_is_mito).to(eng.device)
    ci, cf, part = eng.cell_and_gene(cols, dims, mito)
    gi, gf = eng.finalize_partials(part)
    gi, gf = gi.cpu().numpy(), gf.cpu().numpy()
    oi, of = O.run(h, "gene_grouped", d.gene_is_mito, d.n_gene_ids, threads=THREADS)
    live = oi[:, 0] > 0
    assert np.array_equal(gi[:, 0] > 0, live)
    compare(gi[live], gf[live], oi[live], of[live], exact_floats=False)
    return ci, cf, part


# ---------------- config 2 (and config 3's arithmetic on the same shard) ----------------
@pytest.fixture(scope="module")
def cfg2():
    d = generate(100_000_000, 10_000, 30_000, 1.0, seed=0)
    return d, host(d.cols)


def test_config2_cell_rows_100M(eng, cfg2):
    d, h = cfg2
    oi = check_cell_rows(eng, d, d.cols, h)
    assert oi.shape[0] == 10_000 and int(oi[:, 0].sum()) == 100_000_000


def test_config2_grouped_gene_rows_100M(eng, cfg2):
    d, h = cfg2
    ci, _, _ = check_grouped_gene_rows(eng, d, d.cols, h)
    assert int(ci[:, 0].sum()) == 100_000_000


def test_config3_eight_shards_add_up_100M(eng, cfg2):
    """8 cell-disjoint shards of the config-2 shard: summed partials == unsharded, bit for bit."""
    from sctools_amd import distributed as D

    d, _ = cfg2
    dims = dims_of(d)
    mito = torch.from_numpy(d.gene_is_mito).to(eng.device)
    ci, cf, whole = eng.cell_and_gene(d.cols, dims, mito)
    ci, cf, whole = ci.clone(), cf.clone(), whole.clone()
    bounds = D.shard_bounds(d.cols["cell"], 8)
    assert bounds[0][0] == 0 and bounds[-1][1] == 100_000_000
    sizes = [hi - lo for lo, hi in bounds]
    assert min(sizes) > 0.8 * 100_000_000 / 8  # balanced by records
    acc = torch.zeros_like(whole)
    rows_i, rows_f = [], []
    for lo, hi in bounds:
        si, sf, p = eng.cell_and_gene(D.shard(d.cols, lo, hi), dims, mito)
        si = si.clone()
        si[:, 23] += lo
        rows_i.append(si)
        rows_f.append(sf.clone())
        acc += p
    assert torch.equal(acc, whole)
    wi, wf = eng.finalize_partials(whole)
    gi, gf = eng.finalize_partials(acc)
    assert torch.equal(gi, wi)
    assert torch.equal(gf.view(torch.int64), wf.view(torch.int64))
    assert torch.equal(torch.cat(rows_i), ci)
    assert torch.equal(torch.cat(rows_f).view(torch.int64), cf.view(torch.int64))


# ---------------- config 4: one GPU's 125M-record shard of the 1B-read atlas ----------------
@pytest.fixture(scope="module")
def cfg4():
    d = generate(125_000_000, 62_500, 30_000, 2.0, seed=4)
    return d, host(d.cols)


def test_config4_shard_cell_rows_125M(eng, cfg4):
    d, h = cfg4
    oi = check_cell_rows(eng, d, d.cols, h)
    assert oi[:, 0].max() > 500_000  # the heavy tail is really there


def test_config4_shard_grouped_gene_rows_125M(eng, cfg4):
    d, h = cfg4
    check_grouped_gene_rows(eng, d, d.cols, h)


# ---------------- config 5: shuffled, TagSortBam order on the GPU ----------------
@pytest.fixture(scope="module")
def cfg5(eng):
    d = generate(100_000_000, 10_000, 30_000, 1.0, seed=5, p_nh1=0.70, p_dup=0.40, p_secondary=0.10)
    n = d.cols["cell"].numel()
    g = torch.Generator(device=eng.device)
    g.manual_seed(1)
    perm = torch.randperm(n, generator=g, device=eng.device)
    cols = {c: t[perm].contiguous() for c, t in d.cols.items()}
    tie = d.extra["qname"][perm].contiguous()
    d.cols = None
    del perm
    return d, cols, tie, int(d.extra["n_qnames"])


def test_config5_gpu_sort_is_the_reference_stable_sort_100M(eng, cfg5):
    d, cols, tie, nq = cfg5
    dims = dims_of(d)
    n = cols["cell"].numel()
    assert nq < n  # secondary alignments share query names
    probe = dict(cols)
    probe["pos"] = torch.arange(n, dtype=torch.int32, device=eng.device)  # record identity
    out = eng.tag_sort(probe, dims, "cell_umi_gene", tie, nq)
    p = out["pos"].long()
    seen = torch.zeros(n, dtype=torch.bool, device=eng.device)
    seen[p] = True
    assert bool(seen.all())  # a permutation
    for c in cols:
        if c != "pos":
            assert torch.equal(out[c], cols[c][p]), c
    # (CB, UB, GE) then query name, ties in input order: the sort sorted() performs
    k = (out["cell"].long() << 37) | (out["umi"].long() << 17) | out["gene"].long()
    assert int(out["gene"].max()) < (1 << 17) and int(out["umi"].max()) < (1 << 20)
    t = tie[p]
    gt, eq = k[1:] > k[:-1], k[1:] == k[:-1]
    ok = gt | (eq & ((t[1:] > t[:-1]) | ((t[1:] == t[:-1]) & (p[1:] > p[:-1]))))
    assert bool(ok.all())
    assert bool((eq & (t[1:] == t[:-1])).any())  # the tiebreak ties really occur
    assert eng.verify_sort(out, dims, "cell_umi_gene", t.to(torch.int32).contiguous()) == -1


def test_config5_cell_metrics_after_gpu_sort_100M(eng, cfg5):
    d, cols, tie, nq = cfg5
    srt = eng.tag_sort(cols, dims_of(d), "cell_umi_gene", tie, nq)
    check_cell_rows(eng, d, srt, host(srt))


def test_config5_gene_metrics_after_gpu_sort_100M(eng, cfg5):
    d, cols, tie, nq = cfg5
    dims = dims_of(d)
    srt = eng.tag_sort(cols, dims, "gene_cell_umi", tie, nq)
    h = host(srt)
    mito = torch.from_numpy(d.gene_is_mito).to(eng.device)
    oi, of = O.run(h, "gene", d.gene_is_mito, d.n_gene_ids, threads=THREADS)
    for fm in ("welford", "exact"):
        gi, gf = eng.compute(srt, "gene", dims, mito, mito, float_mode=fm)
        compare(gi.cpu().numpy(), gf.cpu().numpy(), oi, of, exact_floats=(fm == "welford"))
