"""Count matrix on the CPU: the oracle against the reference's own outputs (tests/golden/count,
made by tests/golden/make_count_golden.py from the unmodified reference) and against the
matrix known by construction; the native count-mode decode; GTF gene names; save / load /
merge and the MergeCountMatrices CLI (no GPU needed for those)."""
import itertools
import json
import os

import numpy as np
import pytest
import scipy.sparse as sp

import countgen
import helpers as H
from oracle import count_oracle as O
from sctools_amd import bam, bamnative, gtf
from sctools_amd import count as C

GOLD = os.path.join(H.GOLDEN, "count")
CASES = sorted(f[:-4] for f in os.listdir(GOLD) if f.endswith(".npz"))


def case_input(case):
    for ext, mode in ((".bam", "rb"), (".sam", "r")):
        p = os.path.join(GOLD, case + ext)
        if os.path.exists(p):
            return p, mode
    b = case[len("fixture_"):]
    if b.endswith("_gtf"):
        b = b[:-4]
    return os.path.join(H.GOLDEN, "bam", b + ".bam"), "rb"


def case_genes(case):
    return json.load(open(os.path.join(GOLD, case + ".genes.json")))


def golden(case):
    return np.load(os.path.join(GOLD, case + ".npz"), allow_pickle=False)


def assert_matches_golden(case, matrix, row_index, col_index):
    g = golden(case)
    assert "error" not in g.files
    csr = matrix.tocsr() if not sp.isspmatrix_csr(matrix) else matrix
    assert tuple(csr.shape) == tuple(g["shape"])
    assert csr.data.dtype == g["data"].dtype == np.uint32
    assert np.array_equal(csr.indptr, g["indptr"])
    assert np.array_equal(csr.indices, g["indices"])
    assert np.array_equal(csr.data, g["data"])
    assert row_index.dtype == g["row_index"].dtype and np.array_equal(row_index, g["row_index"])
    assert col_index.dtype == g["col_index"].dtype and np.array_equal(col_index, g["col_index"])


def check_case(case, fn):
    g = golden(case)
    if "error" in g.files:
        with pytest.raises(KeyError) as e:
            fn()
        assert "KeyError: " + str(e.value.args[0]) == str(g["error"])
    else:
        assert_matches_golden(case, *fn())


@pytest.mark.parametrize("case", CASES)
def test_oracle_matches_reference_outputs(case):
    path, mode = case_input(case)
    check_case(case, lambda: O.count_alignments(bam.open_alignments(path, mode), case_genes(case)))


@pytest.mark.parametrize("case", [c for c in CASES if not c.endswith("sam")])
def test_native_count_decode_and_column_oracle(case):
    """Count-mode columns: qhead = itertools.groupby heads, ids = sorted-name ranks; the column
    restatement of the oracle gives the reference's matrix from them."""
    path, _ = case_input(case)
    arrays, (cells, umis, genes) = bamnative.decode(path, "count")
    recs = list(bam.open_alignments(path, "rb"))
    assert arrays["cell"].shape[0] == len(recs)
    heads = [1 if i == 0 or recs[i].query_name != recs[i - 1].query_name else 0 for i in range(len(recs))]
    assert arrays["qhead"].tolist() == heads
    for i, r in enumerate(recs):
        assert cells[arrays["cell"][i]] == (str(r._tags["CB"]) if "CB" in r._tags else None)
        assert genes[arrays["gene"][i]] == (str(r._tags["GE"]) if "GE" in r._tags else None)
    check_case(case, lambda: O.count_columns(arrays, cells, umis, genes, case_genes(case)))


def test_python_columns_match_native_decode():
    path = os.path.join(GOLD, "synth_b_tags.bam")
    a, names = bamnative.decode(path, "count")
    b, names_py = C._python_columns(path, "rb", ("CB", "UB", "GE"))
    assert names == names_py
    for c in ("cell", "umi", "gene", "qhead"):
        assert np.array_equal(a[c], b[c]), c
    counted = lambda x: np.isin(x, (0, 4))  # noqa: E731 -- absent / INTERGENIC
    assert np.array_equal(counted(a["xf"]), counted(b["xf"]))


def test_custom_tags_decode():
    path = os.path.join(GOLD, "synth_a_qname.bam")
    a, (cells, umis, genes) = bamnative.decode(path, "count", tags=("UB", "CB", "GE"))
    b, (cells2, umis2, _) = bamnative.decode(path, "count")
    assert cells == umis2 and umis == cells2
    assert np.array_equal(a["cell"], b["umi"])
    with pytest.raises(ValueError):
        bamnative.decode(path, "count", tags=("C", "UB", "GE"))
    with pytest.raises(OSError):
        bamnative.decode(path, "cell", tags=("UB", "CB", "GE"))  # metric modes read CB / UB / GE


def test_empty_bam_decodes_to_zero_records_in_count_mode():
    a, names = bamnative.decode(os.path.join(GOLD, "empty.bam"), "count")
    assert a["cell"].shape[0] == 0 and a["qhead"].shape[0] == 0
    with pytest.raises(RuntimeError):
        bamnative.decode(os.path.join(GOLD, "empty.bam"), "cell")


def test_oracle_matches_matrix_by_construction():
    """The reference test's check (test_count.py:755-842): rows / cols sorted by name, equal counts."""
    names = json.load(open(os.path.join(GOLD, "chr1.30k_gene_names.json")))
    for seed in (777, 11, 3):
        recs, expected, rows, cols = countgen.generate(names, seed=seed, n_extra=15)
        csr, row_index, col_index = O.count_alignments(recs, names)
        r = np.argsort(row_index)
        c = np.argsort(col_index)
        assert np.array_equal(row_index[r], np.sort(rows))
        assert np.array_equal(col_index[c], np.sort(cols))
        er, ec = np.argsort(rows), np.argsort(cols)
        assert np.array_equal(csr.toarray()[r][:, c], expected[er][:, ec])


def test_extract_gene_names_matches_reference():
    names = gtf.extract_gene_names(os.path.join(GOLD, "chr1.30k_genes.gtf.gz"))
    ref = json.load(open(os.path.join(GOLD, "chr1.30k_gene_names.json")))
    assert list(names.items()) == list(ref.items())


def test_gene_columns():
    col = C.gene_columns([None, "A", "A,B", "Z", "B"], {"B": 0, "A": 1})
    assert col.tolist() == [-1, 1, -1, -2, 0]


def _matrix(seed, n_rows, n_cols=7):
    rng = np.random.default_rng(seed)
    m = sp.random(n_rows, n_cols, density=0.4, random_state=seed, dtype=np.float64)
    m.data = rng.integers(1, 9, m.nnz).astype(np.float64)
    return sp.csr_matrix(m.astype(np.uint32))


def test_save_load_merge_and_cli(tmp_path):
    """MergeCountMatrices: vstack of the chunks, first chunk's columns (test_entrypoints.py:289-310)."""
    from sctools_amd import platform

    col = np.asarray(["g%d" % i for i in range(7)])
    prefixes = []
    for k, n in enumerate((5, 0, 3)):
        cm = C.CountMatrix(_matrix(k, n), np.asarray(["c%d_%d" % (k, i) for i in range(n)]), col)
        p = str(tmp_path / ("chunk%d" % k))
        cm.save(p)
        back = C.CountMatrix.load(p)
        assert (back.matrix != cm.matrix).nnz == 0 and np.array_equal(back.row_index, cm.row_index)
        prefixes.append(p)
    out = str(tmp_path / "merged")
    assert platform.GenericPlatform.merge_count_matrices(["-i"] + prefixes + ["-o", out]) == 0
    m = C.CountMatrix.load(out)
    want = sp.vstack([C.CountMatrix.load(p).matrix for p in prefixes], format="csr")
    assert (m.matrix != want).nnz == 0 and m.matrix.shape == (8, 7)
    assert list(m.row_index) == list(itertools.chain(*(C.CountMatrix.load(p).row_index for p in prefixes)))
    assert np.array_equal(m.col_index, col)
