"""Host-side API pieces that need no GPU: merges, GTF mito ids, column layout, BAM reader."""
import gzip
import os

import numpy as np
import pandas as pd
import pytest

import helpers as H
from sctools_amd import columnar, gtf
from sctools_amd.metrics import CellMetrics, GeneMetrics, MetricCSVWriter
from sctools_amd.metrics.merge import MergeCellMetrics, MergeGeneMetrics
from sctools_amd.metrics import rows as R

MERGE = os.path.join(H.GOLDEN, "merge")


def _read(path):
    return pd.read_csv(path, index_col=0)


@pytest.mark.parametrize("kind,merger", [("cell", MergeCellMetrics), ("gene", MergeGeneMetrics)])
def test_merges_match_reference(tmp_path, kind, merger):
    parts = [os.path.join(MERGE, "%s_part%d.csv" % (kind, k)) for k in (1, 2)]
    out = str(tmp_path / "merged")
    merger(parts, out).execute()
    got = _read(out + ".csv.gz")
    want = _read(os.path.join(MERGE, "%s_merged.csv" % kind))
    assert list(got.columns) == list(want.columns)
    assert list(got.index) == list(want.index)
    np.testing.assert_allclose(got.to_numpy(dtype=float), want.to_numpy(dtype=float), rtol=1e-9, equal_nan=True)


def test_gene_merge_drops_none_rows_like_reference(tmp_path):
    """Gene CSVs carry a `None` row for reads without GE; the reference's groupby drops it
    (fixture: tests/golden/make_merge_none.py), and raises when no row is left."""
    none = os.path.join(H.GOLDEN, "ref", "cell-sorted-missing-cb.gene.csv")
    small = os.path.join(H.GOLDEN, "ref", "small-gene-sorted.gene.csv")
    out = str(tmp_path / "m")
    MergeGeneMetrics([none, small, none], out).execute()
    got = _read(out + ".csv.gz")
    want = _read(os.path.join(MERGE, "gene_none_merged.csv"))
    assert list(got.columns) == list(want.columns)
    assert list(got.index) == list(want.index)
    np.testing.assert_allclose(got.to_numpy(dtype=float), want.to_numpy(dtype=float), rtol=1e-9, equal_nan=True)
    with pytest.raises(ValueError):
        MergeGeneMetrics([none, none], str(tmp_path / "n")).execute()


def test_gene_merge_zero_weights_raise(tmp_path):
    """np.average(..., weights=n_reads) raises ZeroDivisionError when a gene's weights sum to 0."""
    src = os.path.join(MERGE, "gene_part1.csv")
    df = _read(src)
    df["n_reads"] = 0
    p = str(tmp_path / "z.csv")
    df.to_csv(p)
    with pytest.raises(ZeroDivisionError):
        MergeGeneMetrics([p, p], str(tmp_path / "zz")).execute()


def test_header_from_aggregators():
    assert R.header_line("cell").rstrip("\n") == H.golden_text("small-cell-sorted", "cell").split("\n")[0]
    assert R.header_line("gene").rstrip("\n") == H.golden_text("small-gene-sorted", "gene").split("\n")[0]
    assert [k for k in vars(CellMetrics()) if not k.startswith("_")][-1] == "pct_mitochondrial_molecules"
    assert [k for k in vars(GeneMetrics()) if not k.startswith("_")][-1] == "number_cells_expressing"


def test_writer_compress_roundtrip(tmp_path):
    for compress in (True, False):
        w = MetricCSVWriter(str(tmp_path / ("x%d" % compress)), compress)
        w.write_header(vars(GeneMetrics()))
        rec = {k: 1.5 for k in vars(GeneMetrics())}
        w.write(None, rec)
        w.write("G1", rec)
        w.close()
        fn = w.filename
        assert fn.endswith(".csv.gz" if compress else ".csv")
        text = gzip.open(fn, "rt").read() if compress else open(fn).read()
        lines = text.splitlines()
        assert lines[1].startswith("None,1.5,") and lines[2].startswith("G1,")


def test_mito_gene_ids_from_gtf(tmp_path):
    p = tmp_path / "a.gtf"
    p.write_text(
        "#hdr\n"
        'chrM\tx\tgene\t1\t10\t.\t+\t.\tgene_id "ENSG1"; gene_name "MT-CO1";\n'
        'chrM\tx\tgene\t1\t10\t.\t+\t.\tgene_id "ENSG2"; gene_name "mt-Nd1";\n'
        'chr1\tx\tgene\t1\t10\t.\t+\t.\tgene_id "ENSG3"; gene_name "ACTB";\n'
        'chr1\tx\texon\t1\t10\t.\t+\t.\tgene_id "ENSG4"; gene_name "MT-X";\n')
    assert gtf.get_mitochondrial_gene_names(str(p)) == {"ENSG1", "ENSG2"}
    bad = tmp_path / "b.gtf"
    bad.write_text('chr1\tx\tgene\t1\t10\t.\t+\t.\tgene_id "ENSG3";\n')
    with pytest.raises(ValueError):
        gtf.get_mitochondrial_gene_names(str(bad))


def test_columnar_layout_is_32_bytes():
    assert columnar.BYTES_PER_RECORD == 32


def test_bam_reader_counts_match_fixture_facts():
    """records, runs and tag presence of the bundled BAMs."""
    c = H.bam_columns("small-cell-sorted", "cell")
    assert c.n == 656 and len(c.cells) == 58
    a = c.arrays
    assert int((a["xf"] == columnar.XF_CODING).sum()) == 609
    assert int((a["bits"] & columnar.B_SPLICED > 0).sum()) == 2
    m = H.bam_columns("cell-sorted-missing-cb", "cell")
    assert m.n == 13236
    assert int((m.arrays["bits"] & columnar.B_UNMAPPED > 0).sum()) == 10238
    assert m.cells.names[0] is None and int((m.arrays["cell"] == 0).sum()) == 210


def test_sam_and_bam_agree(tmp_path):
    """mode='r' (SAM text) decodes to the same columns as the BAM of the same reads."""
    from sctools_amd.bam import open_alignments
    bam = os.path.join(H.GOLDEN, "bam", "small-gene-sorted.bam")
    recs = list(open_alignments(bam, "rb"))
    lines = ["@HD\tVN:1.4"]
    for r in recs:
        tags = []
        for k, v in r._tags.items():
            tags.append("%s:%s:%s" % (k, "i" if isinstance(v, int) else "Z", v))
        cig = "".join("%d%s" % (n, "MIDNSHP=X"[op]) for op, n in r.cigar) or "*"
        qual = "".join(chr(q + 33) for q in r._qual)
        lines.append("\t".join([r.query_name, str(r.flag), "chr%d" % r.reference_id if r.reference_id >= 0 else "*",
                                str(r.pos + 1), str(r.mapq), cig, "*", "0", "0", "N" * r.l_seq, qual] + tags))
    refs = sorted({r.reference_id for r in recs if r.reference_id >= 0})
    hdr = ["@SQ\tSN:chr%d\tLN:1000000000" % i for i in range(max(refs) + 1)]
    sam = tmp_path / "x.sam"
    sam.write_text("\n".join(lines[:1] + hdr + lines[1:]) + "\n")
    a = columnar.columnarize(bam, "rb", "gene").arrays
    b = columnar.columnarize(str(sam), "r", "gene").arrays
    for k in a:
        assert np.array_equal(a[k], b[k]), k


@pytest.mark.parametrize("mode", ["cell", "gene"])
def test_errors_like_reference(tmp_path, mode):
    """Missing required tags raise the reference's exception types before any launch."""
    from sctools_amd.bam import open_alignments
    bam = os.path.join(H.GOLDEN, "bam", "small-cell-sorted.bam")
    recs = list(open_alignments(bam, "rb"))

    class Fake:
        def __init__(self, rec, drop):
            self.__dict__.update({s: getattr(rec, s) for s in rec.__slots__})
            self._tags = {k: v for k, v in rec._tags.items() if k != drop}
            self._rec = rec

        query_alignment_qualities = property(lambda self: self._rec.query_alignment_qualities)
        flag = property(lambda self: self._rec.flag)

        def get_tag(self, k):
            return self._tags[k]

        def has_tag(self, k):
            return k in self._tags

        def n_skip_length(self):
            return self._rec.n_skip_length()

    mapped = next(r for r in recs if not r.flag & 4)
    with pytest.raises(KeyError):
        columnar.record_fields(Fake(mapped, "UY"), mapped._tags.get("CB"), mode == "cell", True)
    with pytest.raises(KeyError):
        columnar.record_fields(Fake(mapped, "XF"), mapped._tags.get("CB"), mode == "cell", True)
    with pytest.raises(KeyError):
        columnar.record_fields(Fake(mapped, "NH"), mapped._tags.get("CB"), mode == "cell", True)
    if mode == "cell":
        with pytest.raises(KeyError):
            columnar.record_fields(Fake(mapped, "CY"), mapped._tags.get("CB"), True, True)
    else:  # gene metrics never read CY
        columnar.record_fields(Fake(mapped, "CY"), mapped._tags.get("CB"), False, True)


def test_empty_bam_raises_runtime_error(tmp_path):
    sam = tmp_path / "empty.sam"
    sam.write_text("@HD\tVN:1.4\n")
    with pytest.raises(RuntimeError):
        columnar.columnarize(str(sam), "r", "cell")
