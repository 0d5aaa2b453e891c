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
