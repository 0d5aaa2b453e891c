"""Multi-GPU for unsorted input: cell bins swapped between devices, then sorted and measured.

The reference's route for an unsorted BAM is SplitBam (every barcode gets a bin, bam.py:439-448;
each input written bin by bin and the pieces of a bin merged, 454-480), TagSortBam on every
chunk (platform.py:55-97) and Calculate*Metrics + Merge*Metrics.  Here (include/sctools_gpu.h):
sct_bin_records (stable partition by the cell's bin) -> sct_exchange_counts /
sct_exchange_records (RCCL) -> sct_tag_sort -> the metrics -> the gene-partial all-reduce.

* the bin kernel against numpy's stable partition (bins of 1..256, a caller table, the tiebreak
  carried along, ragged and empty inputs);
* the C-ABI exchange on a one-rank communicator (the box has one GPU: a self copy through the
  same entry points);
* ``multigpu.sorted_cell_and_gene_rows`` with three shards on one device (bins swapped by device
  copies) and with one device (the RCCL entry points) against one device sorting everything;
* ``GatherCellAndGeneMetrics`` on the reference's ``unsorted.bam``: the cell CSV byte for byte the
  reference's CSV of the same reads TagSortBam-ed (``cell-gene-umi-queryname-sorted``), the gene
  CSV the reference's gene-sorted CSV within 1e-9.
"""
import ctypes
import os

import numpy as np
import pytest
import torch

import helpers as H
from sctools_amd import _native as N

pytestmark = pytest.mark.gpu

BAM_DIR = os.path.join(H.GOLDEN, "bam")


@pytest.fixture(scope="module")
def eng():
    from sctools_amd import engine as E

    return E.get_engine(torch.device("cuda", 0))


def _shuffled(n, seed, n_cells=57, device="cuda:0"):
    from sctools_amd import synth

    cfg = synth.SynthConfig(n_reads=n, n_cells=n_cells, n_genes=700, seed=seed, p_secondary=0.1, p_nh1=0.7,
                            p_dup=0.4, p_none_cell_reads=0.01)
    d = synth.generate(cfg, device=device)
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    perm = torch.randperm(n, generator=g, device=device)
    cols = {c: t[perm].contiguous() for c, t in d.cols.items()}
    return d, cols, d.extra["qname"][perm].contiguous()


def _dims(d):
    from sctools_amd import engine as E

    return E.Dims(d.n_cell_ids, d.n_gene_ids, d.n_umi_ids)


@pytest.mark.parametrize("n,n_bins,table,tie", [(300_000, 3, False, True), (300_000, 8, False, False),
                                                (1000, 1, False, True), (777, 256, False, True),
                                                (123_457, 5, True, True), (1, 2, False, True)])
def test_bin_records_is_a_stable_partition(eng, n, n_bins, table, tie):
    d, cols, qname = _shuffled(max(n, 1000), seed=3 + n_bins)
    cols = {c: t[:n].contiguous() for c, t in cols.items()}
    qname = qname[:n].contiguous()
    cell = cols["cell"].cpu().numpy().astype(np.int64)
    tab = None
    if table:
        rng = np.random.default_rng(n_bins)
        tab_np = rng.integers(0, n_bins + 2, size=d.n_cell_ids).astype(np.uint8)  # >= n_bins: the last bin
        tab = torch.from_numpy(tab_np).to(eng.device)
        b = np.minimum(tab_np[cell], n_bins - 1)
    else:
        b = cell * n_bins // d.n_cell_ids
    out, tout, counts = eng.bin_records(cols, _dims(d), n_bins, qname if tie else None, tab)
    order = np.argsort(b, kind="stable")
    for c in N.RECORD_COLUMNS:
        assert np.array_equal(out[c].cpu().numpy(), cols[c].cpu().numpy()[order]), c
    if tie:
        assert np.array_equal(tout.cpu().numpy(), qname.cpu().numpy()[order])
    else:
        assert tout is None
    assert np.array_equal(counts.cpu().numpy(), np.bincount(b, minlength=n_bins))


def test_bin_records_rejects_bad_arguments(eng):
    from sctools_amd import engine as E

    d, cols, _ = _shuffled(1000, seed=1)
    with pytest.raises(ValueError):
        eng.bin_records(cols, _dims(d), 0)
    with pytest.raises(ValueError):
        eng.bin_records(cols, _dims(d), 257)
    empty = {c: t[:0].contiguous() for c, t in cols.items()}
    out, _, counts = eng.bin_records(empty, _dims(d), 4)
    assert counts.cpu().tolist() == [0, 0, 0, 0] and out["cell"].numel() == 0
    lib = N.load()
    plan = N.Plan(n_records=10, n_cell_ids=5, n_gene_ids=5, n_umi_ids=5)
    rec = N.Records(n=10)
    assert lib.sct_bin_records(ctypes.byref(plan), ctypes.byref(rec), None, None, 4, ctypes.byref(N.Records(n=9)),
                               None, None, None, 0, None) == -1


def test_exchange_c_abi_one_rank(eng):
    """sct_exchange_counts / sct_exchange_records on a one-rank communicator: the rank's own bin is
    copied through; bad counts are refused."""
    lib = N.load()
    uid = (ctypes.c_uint8 * 128)()
    N.check(lib.sct_comm_unique_id(uid, 128))
    comm = ctypes.c_void_p()
    N.check(lib.sct_comm_init_rank(ctypes.byref(comm), 1, uid, 128, 0, 0))
    try:
        d, cols, qname = _shuffled(50_000, seed=9)
        binned, btie, counts = eng.bin_records(cols, _dims(d), 1, qname)
        recv = eng.exchange_counts(counts, comm.value)
        assert recv.cpu().tolist() == [50_000]
        out, tout = eng.exchange_records(binned, btie, [50_000], [50_000], comm.value)
        torch.cuda.synchronize()
        for c in N.RECORD_COLUMNS:
            assert torch.equal(out[c], binned[c]), c
        assert torch.equal(tout, btie)
        with pytest.raises(N.EngineError, match="send counts"):
            eng.exchange_records(binned, btie, [49_999], [49_999], comm.value)
        with pytest.raises(N.EngineError, match="n_ranks"):
            eng.exchange_records(binned, btie, [25_000, 25_000], [25_000, 25_000], comm.value)
    finally:
        N.check(lib.sct_comm_destroy(comm))


def _one_device_rows(eng, d, cols, qname, float_mode, tie):
    """Everything on one device: the tag sort of all records, then the rows (the reference)."""
    dims = _dims(d)
    srt = eng.tag_sort(cols, dims, "cell_umi_gene", qname if tie else None, d.extra["n_qnames"] if tie else 0)
    gm = torch.from_numpy(d.gene_is_mito).to(eng.device)
    if float_mode == "exact":
        ci, cf, part = eng.cell_and_gene(srt, dims, gm)
    else:
        ci, cf = eng.compute(srt, "cell", dims, gm, torch.zeros_like(gm), float_mode="welford")
        part = eng.gene_partials(srt, dims)
    ids = srt["cell"][ci[:, N.I_ENTITY]].to(torch.int64).cpu().numpy()
    gi, gf = eng.finalize_partials(part)
    return (ci.cpu().numpy(), cf.cpu().numpy(), ids), (gi.cpu().numpy(), gf.cpu().numpy())


def _as_columns(d, cols):
    """The synthetic set as the gatherers' Columns (dictionary sizes only; mito / multi flags)."""
    from sctools_amd import columnar

    class SynthColumns(columnar.Columns):
        def gene_flags(self, mitochondrial_gene_ids=frozenset()):
            return d.gene_is_mito, d.gene_is_multi

    return SynthColumns(cols, list(range(d.n_cell_ids)), list(range(d.n_umi_ids)), list(range(d.n_gene_ids)))


@pytest.mark.parametrize("devices", [[0, 0, 0], [0]])
@pytest.mark.parametrize("float_mode,tie", [("exact", False), ("welford", True)])
def test_sorted_rows_over_devices_equal_one_device(eng, devices, float_mode, tie):
    from sctools_amd import multigpu

    d, cols, qname = _shuffled(2_000_000, seed=21)
    want_cell, want_gene = _one_device_rows(eng, d, cols, qname, float_mode, tie)
    c = _as_columns(d, cols)
    assert multigpu.cells_twice(c)
    got_cell, got_gene = multigpu.sorted_cell_and_gene_rows(
        c, float_mode=float_mode, devices=devices, tiebreak=qname.cpu().numpy() if tie else None,
        n_tiebreak_ids=d.extra["n_qnames"] if tie else 0)
    ent = [i for i in range(N.SCT_NI) if i != N.I_ENTITY]  # (first-record index: per shard)
    assert np.array_equal(got_cell[0][:, ent], want_cell[0][:, ent])
    assert np.array_equal(np.nan_to_num(got_cell[1], nan=-1.0), np.nan_to_num(want_cell[1], nan=-1.0))
    assert np.array_equal(got_cell[2], want_cell[2])
    assert np.array_equal(got_cell[2], np.sort(got_cell[2]))  # barcode order, as TagSortBam writes
    assert np.array_equal(got_gene[0], want_gene[0])
    assert np.array_equal(np.nan_to_num(got_gene[1], nan=-1.0), np.nan_to_num(want_gene[1], nan=-1.0))


@pytest.mark.parametrize("float_mode,tie", [("exact", False), ("welford", True)])
def test_sorted_rows_over_two_gpus_equal_one_device(eng, float_mode, tie):
    """the multi-device exchange over RCCL (sct_exchange_counts / sct_exchange_records with
    two ranks on two GPUs: the per-peer send / recv groups, the non-shared-device path) against one
    device sorting everything.  Skipped on a one-GPU box -- the case the round-end driver runs on an
    8-GPU node."""
    from sctools_amd import multigpu

    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs")
    d, cols, qname = _shuffled(2_000_000, seed=22)
    want_cell, want_gene = _one_device_rows(eng, d, cols, qname, float_mode, tie)
    got_cell, got_gene = multigpu.sorted_cell_and_gene_rows(
        _as_columns(d, cols), float_mode=float_mode, devices=[0, 1], tiebreak=qname.cpu().numpy() if tie else None,
        n_tiebreak_ids=d.extra["n_qnames"] if tie else 0)
    ent = [i for i in range(N.SCT_NI) if i != N.I_ENTITY]
    assert np.array_equal(got_cell[0][:, ent], want_cell[0][:, ent])
    assert np.array_equal(np.nan_to_num(got_cell[1], nan=-1.0), np.nan_to_num(want_cell[1], nan=-1.0))
    assert np.array_equal(got_cell[2], want_cell[2])
    assert np.array_equal(got_gene[0], want_gene[0])
    assert np.array_equal(np.nan_to_num(got_gene[1], nan=-1.0), np.nan_to_num(want_gene[1], nan=-1.0))


@pytest.mark.parametrize("devices", [1, [0, 0, 0]])
def test_unsorted_bam_cell_and_gene_csvs_equal_the_reference(tmp_path, devices):
    """GatherCellAndGeneMetrics on the reference's unsorted.bam: the cell CSV is, byte for byte,
    what the reference writes for the same reads TagSortBam-ed by (CB, UB, GE, query name)
    (its cell-gene-umi-queryname-sorted.bam fixture); the gene CSV is its CSV of the reads sorted by
    gene (small-gene-sorted.bam), integers exact and floats within 1e-9."""
    from sctools_amd.metrics import GatherCellAndGeneMetrics

    cstem, gstem = str(tmp_path / "c"), str(tmp_path / "g")
    GatherCellAndGeneMetrics(os.path.join(BAM_DIR, "unsorted.bam"), cstem, gstem, compress=False,
                             devices=devices).extract_metrics()
    assert open(cstem + ".csv").read() == H.golden_text("cell-gene-umi-queryname-sorted", "cell")
    H.assert_csv_close(open(gstem + ".csv").read(), H.golden_text("small-gene-sorted", "gene"), rel=1e-9)
