"""CountMatrix on the GPU (sct_count_matrix through the C-ABI) against the reference's own
outputs (tests/golden/count: matrix, row order, indices and dtypes equal) and, at sizes the
golden files do not reach, against the oracle's column restatement and a vectorized
restatement for single-alignment groups."""
import os

import numpy as np
import pytest
import scipy.sparse as sp
import torch

import test_count_cpu as T
from oracle import count_oracle as O
from sctools_amd import count as C

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from sctools_amd import engine as E

    return E.get_engine("cuda:0")


@pytest.mark.parametrize("case", T.CASES)
def test_count_matrix_matches_reference(eng, case):
    path, mode = T.case_input(case)

    def run():
        m = C.CountMatrix.from_sorted_tagged_bam(path, T.case_genes(case), open_mode=mode, device=eng.device)
        return m.matrix, m.row_index, m.col_index

    T.check_case(case, run)


def test_create_count_matrix_cli(tmp_path):
    from sctools_amd import platform

    out = str(tmp_path / "counts")
    bam = os.path.join(T.GOLD, "synth_b_qname.bam")
    gtf = os.path.join(T.GOLD, "chr1.30k_genes.gtf.gz")
    assert platform.GenericPlatform.bam_to_count_matrix(["-b", bam, "-o", out, "-a", gtf]) == 0
    m = C.CountMatrix.load(out)
    T.assert_matches_golden("synth_b_qname", m.matrix, m.row_index, m.col_index)
    # -c / -m / -g: swapped barcode tags give the matrix of the swapped roles (oracle)
    assert platform.GenericPlatform.bam_to_count_matrix(["-b", bam, "-o", out + "2", "-a", gtf, "-c", "UB", "-m",
                                                         "CB"]) == 0
    from sctools_amd import bam as B

    names = T.case_genes("synth_b_qname")
    csr, rows, cols = O.count_alignments(B.open_alignments(bam, "rb"), names, cell_tag="UB", molecule_tag="CB")
    m2 = C.CountMatrix.load(out + "2")
    assert np.array_equal(m2.matrix.indptr, csr.indptr) and np.array_equal(m2.matrix.indices, csr.indices)
    assert np.array_equal(m2.matrix.data, csr.data) and np.array_equal(m2.row_index, rows)


def synthetic_columns(n, seed, n_cells=3000, n_umis=50000, n_genes=4000, group_p=0.3):
    rng = np.random.default_rng(seed)
    qhead = (rng.random(n) > group_p).astype(np.uint8)
    qhead[0] = 1
    cell = rng.integers(0, n_cells, n).astype(np.int32)
    umi = rng.integers(0, n_umis, n).astype(np.int32)
    gene = rng.integers(0, n_genes, n).astype(np.int32)
    xf = rng.choice(np.array([0, 1, 2, 3, 4, 5], np.uint8), n, p=[0.05, 0.5, 0.15, 0.1, 0.1, 0.1])
    cells = [None] + ["C%05d" % i for i in range(1, n_cells)]
    umis = [None] + ["U%06d" % i for i in range(1, n_umis)]
    genes = [None] + ["G%05d" % i for i in range(1, n_genes)]
    for g in range(1, n_genes, 97):  # multi-gene values
        genes[g] = genes[g] + ",X"
    names = {"G%05d" % i: j for j, i in enumerate(rng.permutation(np.arange(1, n_genes)))}
    arrays = dict(cell=cell, umi=umi, gene=gene, xf=xf, qhead=qhead)
    return arrays, cells, umis, genes, names


def gpu_count(eng, arrays, cells, umis, genes, names):
    dev = eng.device
    gc = torch.from_numpy(C.gene_columns(genes, names)).to(dev)
    cols = [torch.from_numpy(arrays[c]).to(dev) for c in ("cell", "umi", "gene", "xf", "qhead")]
    res, unknown = eng.count_matrix(*cols, gc, len(cells), len(umis), 0, 0, len(names))
    assert unknown == -1
    return [t.cpu().numpy() for t in res]


@pytest.mark.parametrize("n,seed,group_p", [(300_000, 1, 0.3), (1_000_000, 2, 0.3), (200_000, 5, 0.97)])
def test_count_matrix_matches_column_oracle(eng, n, seed, group_p):
    """group_p 0.97: query-name groups of ~33 alignments, many spanning wave boundaries (the
    count-groups kernel resolves in-wave groups by ballots and walks the rest)."""
    arrays, cells, umis, genes, names = synthetic_columns(n, seed, group_p=group_p)
    row_cell, indptr, indices, data = gpu_count(eng, arrays, cells, umis, genes, names)
    csr, row_index, _ = O.count_columns(arrays, cells, umis, genes, names)
    assert np.array_equal(indptr, csr.indptr) and np.array_equal(indices, csr.indices)
    assert np.array_equal(data.view(np.uint32), csr.data)
    assert [cells[c] for c in row_cell] == list(row_index)


def test_count_matrix_single_alignment_groups_at_scale(eng):
    """30M one-alignment groups: the matrix from a vectorized restatement (np.unique of the
    kept triples; rows by first counted record)."""
    n = 30_000_000
    arrays, cells, umis, genes, names = synthetic_columns(n, 3, n_cells=20000, n_umis=1 << 16, n_genes=30000,
                                                          group_p=0.0)
    row_cell, indptr, indices, data = gpu_count(eng, arrays, cells, umis, genes, names)
    col = C.gene_columns(genes, names)
    a = arrays
    keep = (a["cell"] != 0) & (a["umi"] != 0) & (a["xf"] != 0) & (a["xf"] != 4) & (col[a["gene"]] >= 0)
    idx = np.nonzero(keep)[0]
    c, u, g = a["cell"][idx].astype(np.int64), a["umi"][idx].astype(np.int64), col[a["gene"][idx]].astype(np.int64)
    triple = (c << 40) | (g << 20) | u
    _, first = np.unique(triple, return_index=True)
    pair = (c[first] << 20) | g[first]
    pairs, counts = np.unique(pair, return_counts=True)
    pc, pg = pairs >> 20, pairs & ((1 << 20) - 1)
    first_rec = np.full(len(cells), np.iinfo(np.int64).max)
    np.minimum.at(first_rec, c, idx)
    order = np.argsort(first_rec[first_rec < np.iinfo(np.int64).max], kind="stable")
    counted_cells = np.nonzero(first_rec < np.iinfo(np.int64).max)[0][order]
    assert np.array_equal(row_cell, counted_cells)
    want = sp.csr_matrix((counts.astype(np.uint32), (pc, pg)), shape=(len(cells), len(names)))[counted_cells]
    assert np.array_equal(indptr, want.indptr) and np.array_equal(indices, want.indices)
    assert np.array_equal(data.view(np.uint32), want.data)


def test_count_matrix_rejects_keys_wider_than_63_bits(eng):
    from sctools_amd import _native as N

    arrays, cells, umis, genes, names = synthetic_columns(1000, 4)
    dev = eng.device
    gc = torch.from_numpy(C.gene_columns(genes, names)).to(dev)
    cols = [torch.from_numpy(arrays[c]).to(dev) for c in ("cell", "umi", "gene", "xf", "qhead")]
    with pytest.raises(N.EngineError, match="exceed 63"):
        eng.count_matrix(*cols, gc, 1 << 30, 1 << 30, 0, 0, len(names))
    bad = dict(arrays, cell=np.full(1000, 5000, np.int32))
    cols = [torch.from_numpy(bad[c]).to(dev) for c in ("cell", "umi", "gene", "xf", "qhead")]
    with pytest.raises(N.EngineError, match="outside"):
        eng.count_matrix(*cols, gc, len(cells), len(umis), 0, 0, len(names))


def test_count_matrix_gene_id_outside_dictionary_in_a_group_tail(eng):
    """A gene id outside the dictionary on a non-first alignment of a counted group is rejected,
    also when the group continues past a wave of 64 lanes; in a group whose first alignment has
    no cell barcode it is never looked at (the reference skips the group before its genes)."""
    from sctools_amd import _native as N

    arrays, cells, umis, genes, names = synthetic_columns(4096, 6, group_p=0.0)
    dev = eng.device
    gc = torch.from_numpy(C.gene_columns(genes, names)).to(dev)
    for start, length, bad_at in ((100, 5, 103), (60, 10, 68), (30, 200, 220)):
        a = {k: v.copy() for k, v in arrays.items()}
        a["qhead"][start + 1:start + length] = 0
        a["cell"][start], a["umi"][start] = 7, 9
        a["gene"][bad_at] = len(genes) + 3
        cols = [torch.from_numpy(a[c]).to(dev) for c in ("cell", "umi", "gene", "xf", "qhead")]
        with pytest.raises(N.EngineError, match="outside"):
            eng.count_matrix(*cols, gc, len(cells), len(umis), 0, 0, len(names))
        a["cell"][start] = 0  # cell None: the group is skipped, its genes unread
        cols = [torch.from_numpy(a[c]).to(dev) for c in ("cell", "umi", "gene", "xf", "qhead")]
        res, unknown = eng.count_matrix(*cols, gc, len(cells), len(umis), 0, 0, len(names))
        assert unknown == -1
