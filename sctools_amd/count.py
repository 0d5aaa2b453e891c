"""
Count matrices -- same interface as the reference's ``sctools.count.CountMatrix``
(``/root/reference/src/sctools/count.py:36-390``), built on the GPU.

``from_sorted_tagged_bam`` decodes the BAM on the GPU (``libsct_gbam.so``; a file it declines
natively on the host, ``libsct_bam.so``), count-matrix mode: the three dictionary tags, XF and a
query-name group flag per record, and counts on the
device (``sct_count_matrix``, ``csrc/countmat.h``): one molecule key per query-name group,
an LSD sort, distinct (cell, molecule, gene) triples summed per (cell, gene), rows ordered
by each cell's first counted molecule -- the matrix, row index and column index of the
reference's set-and-COO loop (count.py:222-328), not a reordering of them.

``save`` / ``load`` / ``merge_matrices`` / ``from_mtx`` keep the reference's file layout
(``<prefix>.npz`` via scipy.sparse.save_npz, ``<prefix>_row_index.npy``,
``<prefix>_col_index.npy``).
"""

import operator
from typing import Dict, List, Optional, Sequence

import numpy as np
import scipy.sparse as sp
from scipy.io import mmread

from sctools_amd import consts

XF_ABSENT, XF_INTERGENIC = 0, 4


def _python_columns(path: str, open_mode: str, tags):
    """SAM (or any ``open_mode`` the native decoder does not read) through the pure-Python reader:
    the same columns and dictionaries as ``bamnative.decode(..., "count")``."""
    from sctools_amd import bam
    from sctools_amd.columnar import Dictionary

    cells: List = []
    umis: List = []
    genes: List = []
    xf: List[int] = []
    qhead: List[int] = []
    prev = object()
    for r in bam.open_alignments(path, open_mode):
        t = r._tags
        cells.append(None if tags[0] not in t else str(t[tags[0]]))
        umis.append(None if tags[1] not in t else str(t[tags[1]]))
        genes.append(None if tags[2] not in t else str(t[tags[2]]))
        x = t.get("XF", None)
        xf.append(XF_ABSENT if "XF" not in t else (XF_INTERGENIC if x == "INTERGENIC" else 5))
        qhead.append(1 if r.query_name != prev else 0)
        prev = r.query_name
    dicts = [Dictionary(v) for v in (cells, umis, genes)]
    arrays = {
        "cell": dicts[0].encode(cells), "umi": dicts[1].encode(umis), "gene": dicts[2].encode(genes),
        "xf": np.asarray(xf, dtype=np.uint8), "qhead": np.asarray(qhead, dtype=np.uint8),
    }
    return arrays, [d.names for d in dicts]


def _device_columns(path: str, open_mode: str, tags, dev):
    """The count columns decoded on `dev` by libsct_gbam.so, or None (SAM, no device decoder, tag
    names it cannot take, or a file it declines: typed tag values, non-ASCII strings ...)."""
    from sctools_amd import gbam

    if open_mode != "rb" or dev.type != "cuda" or not gbam.available():
        return None
    if any(len(t) != 2 or not t.isascii() or "\0" in t for t in tags):
        return None
    return gbam.decode(path, "count", device=dev, tags=tags)


def gene_columns(gene_names: Sequence[Optional[str]], gene_name_to_index: Dict[str, int]) -> np.ndarray:
    """Per gene-dictionary id: its matrix column, SKIP (-1: no tag, or a multi-gene "a,b" value --
    count.py:248-263 never counts those) or UNKNOWN (-2: the gene_name_to_index KeyError)."""
    col = np.empty(len(gene_names), dtype=np.int32)
    for g, name in enumerate(gene_names):
        if name is None or "," in name:
            col[g] = -1
        else:
            col[g] = gene_name_to_index.get(name, -2)
    return col


def _unknown_gene(arrays, gene_names, gene_col, i: int) -> str:
    """The implicated gene name of the group starting at record i (its gene is UNKNOWN)."""
    n = arrays["cell"].shape[0]
    j = i
    while j < n and (j == i or not arrays["qhead"][j]):
        g = int(arrays["gene"][j])
        x = int(arrays["xf"][j])
        if x not in (XF_ABSENT, XF_INTERGENIC) and gene_col[g] != -1:
            return gene_names[g]
        j += 1
    raise AssertionError("record %d does not start a counted group" % i)


class CountMatrix:
    def __init__(self, matrix: sp.csr_matrix, row_index: np.ndarray, col_index: np.ndarray):
        self._matrix = matrix
        self._row_index = row_index
        self._col_index = col_index

    @property
    def matrix(self):
        return self._matrix

    @property
    def row_index(self):
        return self._row_index

    @property
    def col_index(self):
        return self._col_index

    @classmethod
    def from_sorted_tagged_bam(
        cls,
        bam_file: str,
        gene_name_to_index: Dict[str, int],
        chromosomes_gene_locations_extended: Dict[str, List[tuple]] = None,
        cell_barcode_tag: str = consts.CELL_BARCODE_TAG_KEY,
        molecule_barcode_tag: str = consts.MOLECULE_BARCODE_TAG_KEY,
        gene_name_tag: str = consts.GENE_NAME_TAG_KEY,
        open_mode: str = "rb",
        device=None,
        gpu_decode: bool = True,
    ) -> "CountMatrix":
        """Cells x genes molecule counts of a query-name-grouped tagged BAM (count.py:134-328).

        ``chromosomes_gene_locations_extended`` is accepted and, as in the reference, unused.
        A BAM is inflated and parsed on the counting device (``gbam``, count mode) unless
        ``gpu_decode`` is False or the device decoder declines the file (then ``bamnative``)."""
        import torch

        from sctools_amd import bamnative, engine

        tags = (cell_barcode_tag or consts.CELL_BARCODE_TAG_KEY,
                molecule_barcode_tag or consts.MOLECULE_BARCODE_TAG_KEY,
                gene_name_tag or consts.GENE_NAME_TAG_KEY)
        eng = engine.get_engine(device)
        dev = eng.device
        got = _device_columns(bam_file, open_mode, tags, dev) if gpu_decode else None
        if got is not None:  # decoded on the device: the columns are already in HBM
            arrays, (cells, umis, genes) = got
        else:
            try:
                if open_mode != "rb":
                    raise bamnative.TypedTagValue("not BAM")
                arrays, (cells, umis, genes) = bamnative.decode(bam_file, "count", tags=tags)
            except bamnative.TypedTagValue:  # SAM, or float / array tag values: the Python reader
                arrays, (cells, umis, genes) = _python_columns(bam_file, open_mode, tags)
        gene_col = gene_columns(genes, gene_name_to_index)

        def put(a):
            if isinstance(a, torch.Tensor):
                return a
            return torch.from_numpy(np.ascontiguousarray(a)).to(dev)

        n = int(arrays["cell"].shape[0])
        if n:
            cols = [put(arrays[c]) for c in ("cell", "umi", "gene", "xf", "qhead")]
        else:
            cols = [torch.empty(0, dtype=torch.int32, device=dev) for _ in range(3)]
            cols += [torch.empty(0, dtype=torch.uint8, device=dev) for _ in range(2)]
        res, unknown = eng.count_matrix(
            *cols, put(gene_col if len(gene_col) else np.full(1, -1, np.int32)), max(1, len(cells)),
            max(1, len(umis)), 0 if cells and cells[0] is None else -1, 0 if umis and umis[0] is None else -1,
            len(gene_name_to_index))
        if unknown >= 0:
            host = {c: (v.cpu().numpy() if isinstance(v, torch.Tensor) else v) for c, v in arrays.items()}
            raise KeyError(_unknown_gene(host, genes, gene_col, unknown))
        row_cell, indptr, indices, data = (t.cpu().numpy() for t in res)
        n_rows = int(row_cell.shape[0])
        matrix = sp.csr_matrix((data.view(np.uint32), indices, indptr), shape=(n_rows, len(gene_name_to_index)))
        col_index = np.asarray([k for k, v in sorted(gene_name_to_index.items(), key=operator.itemgetter(1))])
        row_index = np.asarray([cells[c] for c in row_cell.tolist()])
        return cls(matrix, row_index, col_index)

    def save(self, prefix: str) -> None:
        sp.save_npz(prefix + ".npz", self._matrix, compressed=True)
        np.save(prefix + "_row_index.npy", self._row_index)
        np.save(prefix + "_col_index.npy", self._col_index)

    @classmethod
    def load(cls, prefix: str) -> "CountMatrix":
        matrix = sp.load_npz(prefix + ".npz")
        row_index = np.load(prefix + "_row_index.npy")
        col_index = np.load(prefix + "_col_index.npy")
        return cls(matrix, row_index, col_index)

    @classmethod
    def merge_matrices(cls, input_prefixes) -> "CountMatrix":
        """vstack of per-chunk matrices (chunks hold disjoint cells); the first chunk's columns."""
        col_indices = [np.load(p + "_col_index.npy") for p in input_prefixes]
        row_indices = [np.load(p + "_row_index.npy") for p in input_prefixes]
        matrices = [sp.load_npz(p + ".npz") for p in input_prefixes]
        matrix = sp.vstack(matrices, format="csr")
        return cls(matrix, np.concatenate(row_indices), col_indices[0])

    @classmethod
    def from_mtx(cls, matrix_mtx: str, row_index_file: str, col_index_file: str) -> "CountMatrix":
        matrix = mmread(matrix_mtx).tocsr()
        with open(row_index_file, "r") as fin:
            row_index = np.array(fin.readlines())
        with open(col_index_file, "r") as fin:
            col_index = np.array(fin.readlines())
        return cls(matrix, row_index, col_index)
