"""End-to-end drop-in API on the GPU: gatherers, CLI entry points, aggregator protocol.

Every output is compared with the reference's own output on the same BAM
(``tests/golden/ref``, made by ``tests/golden/make_golden.py``): byte-identical
in the default Welford mode, within 1e-9 relative in exact-sum mode.
"""
import gzip
import os

import pytest

import helpers as H

pytestmark = pytest.mark.gpu

BAM_DIR = os.path.join(H.GOLDEN, "bam")


def _read(path):
    return gzip.open(path, "rt").read() if path.endswith(".gz") else open(path).read()


@pytest.mark.parametrize("bam", H.BAMS)
@pytest.mark.parametrize("kind", ["cell", "gene"])
@pytest.mark.parametrize("compress", [False, True])
def test_gatherers_match_reference(tmp_path, bam, kind, compress):
    from sctools_amd.metrics import GatherCellMetrics, GatherGeneMetrics

    cls = GatherCellMetrics if kind == "cell" else GatherGeneMetrics
    stem = str(tmp_path / "out")
    cls(os.path.join(BAM_DIR, bam + ".bam"), stem, compress=compress).extract_metrics()
    got = _read(stem + (".csv.gz" if compress else ".csv"))
    assert got == H.golden_text(bam, kind)


@pytest.mark.parametrize("kind", ["cell", "gene"])
def test_gatherers_exact_mode_within_tolerance(tmp_path, kind):
    from sctools_amd.metrics import GatherCellMetrics, GatherGeneMetrics

    cls = GatherCellMetrics if kind == "cell" else GatherGeneMetrics
    stem = str(tmp_path / "out")
    cls(os.path.join(BAM_DIR, "cell-sorted-missing-cb.bam"), stem, compress=False,
        float_mode="exact").extract_metrics()
    H.assert_csv_close(_read(stem + ".csv"), H.golden_text("cell-sorted-missing-cb", kind), rel=1e-9)


def test_cli_commands(tmp_path):
    from sctools_amd.platform import GenericPlatform

    stem = str(tmp_path / "c")
    assert GenericPlatform.calculate_cell_metrics(
        ["-i", os.path.join(BAM_DIR, "small-cell-sorted.bam"), "-o", stem]) == 0
    assert _read(stem + ".csv.gz") == H.golden_text("small-cell-sorted", "cell")
    stem = str(tmp_path / "g")
    assert GenericPlatform.calculate_gene_metrics(
        ["-i", os.path.join(BAM_DIR, "small-gene-sorted.bam"), "-o", stem]) == 0
    assert _read(stem + ".csv.gz") == H.golden_text("small-gene-sorted", "gene")
    # the mito annotation reaches the cell rows (reference computes it from the GTF gene ids)
    gtf = tmp_path / "m.gtf"
    gtf.write_text('chrM\tx\tgene\t1\t10\t.\t+\t.\tgene_id "%s"; gene_name "MT-A";\n' % _some_gene())
    stem = str(tmp_path / "m")
    assert GenericPlatform.calculate_cell_metrics(
        ["-i", os.path.join(BAM_DIR, "small-cell-sorted.bam"), "-o", stem, "-a", str(gtf)]) == 0
    header, rows = H.parse_csv(_read(stem + ".csv.gz"))
    j = header.index("n_mitochondrial_genes")
    assert any(r[j] == "1" for r in rows)


def _some_gene():
    cols = H.bam_columns("small-cell-sorted", "cell")
    return next(g for g in cols.genes.names if g is not None and "," not in g)


def _tag(rec, k):
    return rec.get_tag(k) if rec.has_tag(k) else None


@pytest.mark.parametrize("kind", ["cell", "gene"])
def test_aggregator_protocol(kind):
    """parse_molecule / finalize per entity (gatherer.py:120-159, 195-232) reproduces each row."""
    from sctools_amd.bam import open_alignments
    from sctools_amd.metrics import CellMetrics, GeneMetrics
    from sctools_amd.metrics import rows as R

    bam = "small-cell-sorted" if kind == "cell" else "small-gene-sorted"
    recs = list(open_alignments(os.path.join(BAM_DIR, bam + ".bam"), "rb"))
    keys = ("CB", "UB", "GE") if kind == "cell" else ("GE", "CB", "UB")
    groups = []
    for r in recs:
        t = tuple(_tag(r, k) for k in keys)
        if groups and groups[-1][0] == t[0]:
            groups[-1][1].append((t, r))
        else:
            groups.append((t[0], [(t, r)]))
    header, body = H.parse_csv(H.golden_text(bam, kind))
    want = {r[0]: dict(zip(header[1:], r[1:])) for r in body}
    checked = 0
    for name, items in groups[:8]:
        if kind == "gene" and (name is None or "," in name):
            continue
        agg = CellMetrics() if kind == "cell" else GeneMetrics()
        for t, r in items:
            agg.parse_molecule(tags=t, records=[r])
        agg.finalize()
        row = want[str(name)]
        for col, k, _ in R.columns_for(kind):
            v = getattr(agg, col)
            assert str(v) == row[col], (name, col)
        checked += 1
    assert checked >= 4


@pytest.mark.parametrize("bam", H.BAMS)
@pytest.mark.parametrize("kind", ["cell", "gene"])
def test_gatherers_multi_device_path_matches_reference(tmp_path, bam, kind):
    """devices=N (every visible GPU; N=1 on a one-GPU box): the sharded, threaded path gives the
    reference's CSV byte for byte."""
    import torch

    from sctools_amd.metrics import GatherCellMetrics, GatherGeneMetrics

    cls = GatherCellMetrics if kind == "cell" else GatherGeneMetrics
    stem = str(tmp_path / "out")
    cls(os.path.join(BAM_DIR, bam + ".bam"), stem, compress=False,
        devices=torch.cuda.device_count()).extract_metrics()
    assert _read(stem + ".csv") == H.golden_text(bam, kind)


def test_cli_devices_flag(tmp_path):
    from sctools_amd.platform import GenericPlatform

    stem = str(tmp_path / "c")
    assert GenericPlatform.calculate_cell_metrics(
        ["-i", os.path.join(BAM_DIR, "small-cell-sorted.bam"), "-o", stem, "--devices", "1"]) == 0
    assert _read(stem + ".csv.gz") == H.golden_text("small-cell-sorted", "cell")
    stem = str(tmp_path / "g")
    assert GenericPlatform.calculate_gene_metrics(
        ["-i", os.path.join(BAM_DIR, "small-gene-sorted.bam"), "-o", stem, "--devices", "1"]) == 0
    assert _read(stem + ".csv.gz") == H.golden_text("small-gene-sorted", "gene")


@pytest.mark.parametrize("float_mode", ["welford", "exact"])
def test_cell_and_gene_rows_from_one_cell_sorted_pass(tmp_path, float_mode):
    """CalculateCellMetrics --gene-output-filestem on the reference's cell-sorted fixture: the cell
    CSV is the reference's (byte for byte in Welford mode); the gene CSV is what the reference
    writes for the SAME reads sorted by gene (small-gene-sorted.bam): integers and row order
    exact, floats within 1e-9 (exact sums vs the reference's Welford in its file order).  The
    gene partials pass through sct_allreduce_gene_partials (RCCL) even on one device."""
    from sctools_amd.platform import GenericPlatform

    cstem, gstem = str(tmp_path / "c"), str(tmp_path / "g")
    assert GenericPlatform.calculate_cell_metrics(
        ["-i", os.path.join(BAM_DIR, "cell-gene-umi-queryname-sorted.bam"), "-o", cstem,
         "--gene-output-filestem", gstem, "--float-mode", float_mode, "--devices", "1"]) == 0
    cell_want = H.golden_text("cell-gene-umi-queryname-sorted", "cell")
    if float_mode == "welford":
        assert _read(cstem + ".csv.gz") == cell_want
    else:
        H.assert_csv_close(_read(cstem + ".csv.gz"), cell_want, rel=1e-9)
    H.assert_csv_close(_read(gstem + ".csv.gz"), H.golden_text("small-gene-sorted", "gene"), rel=1e-9)


def test_cell_sorted_pass_refuses_unsorted_input():
    """The one-pass route (no sort) needs every cell in one run; GatherCellAndGeneMetrics sends an
    unsorted file through the bin exchange + tag sort instead (tests/test_gpu_exchange.py)."""
    from sctools_amd import columnar, multigpu

    cols = columnar.columnarize(os.path.join(BAM_DIR, "unsorted.bam"), "rb", "cell")
    with pytest.raises(ValueError, match="cell-sorted"):
        multigpu.compute_cell_and_gene_rows(cols, float_mode="exact", devices=[0])


def test_allreduce_c_abi_with_own_communicator():
    """The torch-free route: sct_comm_unique_id + sct_comm_init_rank + sct_allreduce_gene_partials
    on a one-rank communicator leaves the partials unchanged (the sum over one rank)."""
    import ctypes

    import torch

    from sctools_amd import _native as N

    lib = N.load()
    uid = (ctypes.c_uint8 * 128)()
    N.check(lib.sct_comm_unique_id(uid, 128))
    comm = ctypes.c_void_p()
    N.check(lib.sct_comm_init_rank(ctypes.byref(comm), 1, uid, 128, 0, 0))
    try:
        part = torch.randint(-2**40, 2**40, (777, N.SCT_NP), dtype=torch.int64, device="cuda:0")
        want = part.clone()
        s = ctypes.c_void_p(torch.cuda.current_stream(part.device).cuda_stream)
        N.check(lib.sct_allreduce_gene_partials(ctypes.c_void_p(part.data_ptr()), 777, comm, s))
        torch.cuda.synchronize()
        assert torch.equal(part, want)
        assert lib.sct_allreduce_gene_partials(None, 5, comm, s) == -1
    finally:
        N.check(lib.sct_comm_destroy(comm))


def test_aggregator_protocol_golden_finalize():
    """The protocol golden's undamaged (and damaged-but-not-raising) cases finalized on the GPU:
    every public attribute equals the reference aggregator's (tests/golden/protocol)."""
    import math

    import test_protocol_cpu as P

    done = 0
    for case in P.CASES:
        if case["final"] is None:
            continue
        agg, _, raised = P.replay(case)
        assert raised is None
        agg.finalize()
        got = {k: v for k, v in vars(agg).items() if not k.startswith("_")}
        assert list(got) == list(case["final"])
        for k, v in got.items():
            w = case["final"][k]
            if w == "nan":
                assert isinstance(v, float) and math.isnan(v), (case["entity_name"], k)
            else:
                assert str(v) == w, (case["entity_name"], case["damage"], k, v, w)
        done += 1
    assert done >= 8


# damaged records whose partial state the aggregator reproduces -- all of them since round 6: CY
# missing (nothing consumed yet), CR missing (its CY sample only), UY missing (the molecule
# histogram), no / empty aligned qualities (and the UY sample), a mapped read without XF / NH (up to
# its fragment and genomic streams)
EXACT_AFTER_ERROR = ("drop:CY", "drop:CR", "drop:UY", "noqual", "emptyqual", "drop:XF", "drop:NH")


def _same_final(got, want, label):
    import math

    assert list(got) == list(want), label
    for k, v in got.items():
        w = want[k]
        if w == "nan":
            assert isinstance(v, float) and math.isnan(v), (label, k)
        else:
            assert str(v) == w, (label, k, v, w)


def test_finalize_after_a_caught_error_matches_reference():
    """a caller catches the damaged record's exception and calls finalize() at once
    (final_after_error) or after parsing the entity's remaining records (final_continued); every
    public attribute equals the reference's (tests/golden/protocol, make_protocol_golden.py)."""
    import copy

    import test_protocol_cpu as P

    done = 0
    for case in P.CASES:
        if case["raised"] is None or case["damage"] not in EXACT_AFTER_ERROR:
            continue
        agg, steps, raised = P.replay(case)
        assert raised == case["raised"]
        label = (case["kind"], case["bam"], case["entity"], case["damage"])
        after = copy.deepcopy(agg)
        after.finalize()
        _same_final({k: v for k, v in vars(after).items() if not k.startswith("_")}, case["final_after_error"], label)
        _, items = P.entity_records(case["kind"], case["bam"], case["entity"])
        for t, r in items[len(steps):]:
            agg.parse_molecule(tags=t, records=[r])
        agg.finalize()
        _same_final({k: v for k, v in vars(agg).items() if not k.startswith("_")}, case["final_continued"], label)
        done += 1
    assert done >= 17


@pytest.mark.parametrize("bam", H.BAMS)
@pytest.mark.parametrize("kind", ["cell", "gene"])
def test_gatherers_three_shards_on_one_device(tmp_path, bam, kind):
    """devices=[0, 0, 0]: the file cut into three entity-aligned shards (record offsets > 0), each
    on its own thread and engine of device 0, rows concatenated: the reference's CSV byte for byte."""
    from sctools_amd.metrics import GatherCellMetrics, GatherGeneMetrics

    cls = GatherCellMetrics if kind == "cell" else GatherGeneMetrics
    stem = str(tmp_path / "out")
    cls(os.path.join(BAM_DIR, bam + ".bam"), stem, compress=False, devices=[0, 0, 0]).extract_metrics()
    assert _read(stem + ".csv") == H.golden_text(bam, kind)


@pytest.mark.parametrize("float_mode", ["exact", "welford"])
def test_shards_with_an_empty_shard_equal_one_device(float_mode):
    """A record set whose first cell holds most records: three shards cut at cell boundaries leave
    the middle one empty (zero partials, no rows).  Cell rows, first-record offsets and the summed
    gene partials equal the one-device result exactly."""
    import numpy as np

    from sctools_amd import columnar, distributed as D, multigpu

    full = columnar.columnarize(os.path.join(BAM_DIR, "cell-sorted-missing-cb.bam"), "rb", "cell")
    cols = columnar.Columns({c: a[:216] for c, a in full.arrays.items()}, full.cells, full.umis, full.genes)
    bounds = D.shard_bounds(cols.arrays["cell"], 3)
    assert any(lo == hi for lo, hi in bounds), bounds
    one = multigpu.compute_cell_and_gene_rows(cols, float_mode=float_mode, devices=[0])
    three = multigpu.compute_cell_and_gene_rows(cols, float_mode=float_mode, devices=[0, 0, 0])
    for a, b in zip(one[0] + one[1], three[0] + three[1]):
        assert np.array_equal(np.nan_to_num(a, nan=-7.0), np.nan_to_num(b, nan=-7.0))
    r1 = multigpu.compute_rows(cols, "cell", float_mode=float_mode, devices=[0])
    r3 = multigpu.compute_rows(cols, "cell", float_mode=float_mode, devices=[0, 0, 0])
    for a, b in zip(r1, r3):
        assert np.array_equal(np.nan_to_num(a, nan=-7.0), np.nan_to_num(b, nan=-7.0))


def test_shard_failure_raises_without_hanging(monkeypatch):
    """One shard's engine call fails (injected) while the others wait at the gene-partial collective:
    the group raises that error promptly instead of blocking in the all-reduce."""
    import time

    from sctools_amd import columnar, engine as E, multigpu

    cols = columnar.columnarize(os.path.join(BAM_DIR, "small-cell-sorted.bam"), "rb", "cell")
    real = E.Engine.cell_and_gene
    calls = []

    def flaky(self, *a, **k):
        calls.append(1)
        if len(calls) == 2:
            raise MemoryError("injected: shard engine out of memory")
        return real(self, *a, **k)

    monkeypatch.setattr(E.Engine, "cell_and_gene", flaky)
    t0 = time.monotonic()
    with pytest.raises(MemoryError, match="injected"):
        multigpu.compute_cell_and_gene_rows(cols, float_mode="exact", devices=[0, 0, 0])
    assert time.monotonic() - t0 < 60
