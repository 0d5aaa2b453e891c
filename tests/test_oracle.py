"""The CPU oracle (oracle/sct_oracle.c) against the reference's own outputs.

Golden CSVs were produced by the unmodified reference gatherer in the build
container (tests/golden/make_golden.py).  The oracle must reproduce them
byte-for-byte: integers, row order, and Welford floats in Python repr.
"""
import pytest

import helpers as H
from oracle import oracle as O


@pytest.mark.parametrize("bam", H.BAMS)
@pytest.mark.parametrize("mode", ["cell", "gene"])
def test_oracle_matches_reference_on_bundled_bams(bam, mode):
    cols = H.bam_columns(bam, mode)
    mito, _ = cols.gene_flags()
    ints, floats = O.run(cols.arrays, mode, mito, len(cols.genes))
    got = H.render(mode, ints, floats, cols.arrays, cols.cells.names, cols.genes.names)
    assert got == H.golden_text(bam, mode)


def test_oracle_reproduces_notebook_golden():
    """The reference's only full-precision golden vector (gene notebook cell 42)."""
    cols = H.bam_columns("small-gene-sorted", "gene")
    mito, _ = cols.gene_flags()
    ints, floats = O.run(cols.arrays, "gene", mito, len(cols.genes))
    got = H.render("gene", ints, floats, cols.arrays, cols.cells.names, cols.genes.names)
    nb = open(H.GOLDEN + "/ref/notebook_gene_metrics.csv").read()
    assert got == nb


@pytest.mark.parametrize("name", H.SYNTH)
@pytest.mark.parametrize("mode,kind", [("cell", "cell"), ("gene", "gene_run"),
                                       ("gene_grouped", "gene_grouped")])
def test_oracle_matches_reference_on_synthetic(name, mode, kind):
    s = H.synth(name)
    ints, floats = O.run(s.arrays, mode, s.gene_is_mito, len(s.gene_names))
    got = H.render(mode, ints, floats, s.arrays, s.cell_names, s.gene_names)
    assert got == H.synth_text(name, kind)


def test_oracle_threads_do_not_change_results():
    s = H.synth("s1")
    a = O.run(s.arrays, "cell", s.gene_is_mito, len(s.gene_names), threads=1)
    b = O.run(s.arrays, "cell", s.gene_is_mito, len(s.gene_names), threads=4)
    assert (a[0] == b[0]).all()
    assert ((a[1] == b[1]) | ((a[1] != a[1]) & (b[1] != b[1]))).all()


def test_reference_assertions_hold_on_oracle():
    """Known-answer totals of the reference's test_metrics.py (lines 90-258, 792-809)."""
    g = H.bam_columns("small-gene-sorted", "gene")
    gi, _ = O.run(g.arrays, "gene", g.gene_flags()[0], len(g.genes))
    c = H.bam_columns("small-cell-sorted", "cell")
    ci, _ = O.run(c.arrays, "cell", c.gene_flags()[0], len(c.genes))
    m = H.bam_columns("cell-sorted-missing-cb", "cell")
    mi, _ = O.run(m.arrays, "cell", m.gene_flags()[0], len(m.genes))
    from sctools_amd import _native as N
    assert gi[:, N.I_N_READS].sum() == 300 and ci[:, N.I_N_READS].sum() == 656
    assert gi.shape[0] == 8
    assert abs(ci[:, N.I_N_K1].mean() - 1.9827) < 1e-4
    assert gi[:, N.I_N_MOL].sum() == 88 and ci[:, N.I_N_MOL].sum() == 249
    assert gi[:, N.I_N_FRAG].sum() == 217 and ci[:, N.I_N_FRAG].sum() == 499
    assert gi[:, N.I_N_READS].max() == 245 and ci[:, N.I_N_READS].max() == 94
    assert gi[:, N.I_PERFECT_UMI].sum() == 300 and ci[:, N.I_PERFECT_UMI].sum() == 655
    assert ci[:, N.I_PERFECT_CB].sum() == 650 and mi[:, N.I_PERFECT_CB].sum() == 12861
    assert gi[:, N.I_EXONIC].sum() == 300 and ci[:, N.I_EXONIC].sum() == 609
    assert gi[:, N.I_INTRONIC].sum() == 0 and ci[:, N.I_INTRONIC].sum() == 28
    assert gi[:, N.I_UTR].sum() == 0 and ci[:, N.I_UTR].sum() == 19
    assert gi[:, N.I_UNIQUE].sum() == 300 and ci[:, N.I_UNIQUE].sum() == 656
    assert gi[:, N.I_DUP].sum() == 90 and ci[:, N.I_DUP].sum() == 107
    assert gi[:, N.I_SPLICED].sum() == 29 and ci[:, N.I_SPLICED].sum() == 2
    assert gi[:, N.I_FRAG_SINGLE].sum() == 155 and gi[:, N.I_MOL_SINGLE].sum() == 42
