"""CPU restatement of CountMatrix.from_sorted_tagged_bam -- TEST INFRASTRUCTURE ONLY
(see oracle/__init__.py): the checker for sct_count_matrix, never the product path.

Follows /root/reference/src/sctools/count.py line by line:
  count.py:83-96    groups = itertools.groupby(records, query_name); cell / molecule barcode
                    of the group's first alignment (None when the tag is missing)
  count.py:240-245  groups without a cell or molecule barcode are skipped
  count.py:247-259  one alignment: counted when it has the gene tag and an XF tag other than
                    INTERGENIC and the gene value holds no ','
  count.py:260-274  several alignments: the set of single-name gene values of alignments with
                    a gene tag and a non-INTERGENIC XF must have exactly one element
  count.py:279-287  a (cell, molecule, gene) triple counts once
  count.py:289-306  gene_name_to_index[gene] (KeyError for an unknown gene); cells numbered in
                    order of their first counted molecule; one COO entry per molecule
  count.py:308-328  coo_matrix(..., dtype=uint32).tocsr(); row / col index arrays

Parity pinning: the reference's own count test builds its expected matrix by construction
from a synthetic BAM (test/test_count.py:151-420); tests/countgen.py restates that generator
and tests/test_count_cpu.py checks this oracle against the constructed matrix.
"""
import itertools
import operator
from typing import Dict, Iterable, List, Optional

import numpy as np
import scipy.sparse as sp

XF_ABSENT, XF_INTERGENIC = 0, 4


def _finish(data_cells: List[int], data_genes: List[int], cell_to_index: Dict, gene_name_to_index: Dict[str, int]):
    n_cells = len(cell_to_index)
    coo = sp.coo_matrix((np.ones(len(data_cells), dtype=np.uint32), (data_cells, data_genes)),
                        shape=(n_cells, len(gene_name_to_index)), dtype=np.uint32)
    col_index = np.asarray([k for k, v in sorted(gene_name_to_index.items(), key=operator.itemgetter(1))])
    row_index = np.asarray([k for k, v in sorted(cell_to_index.items(), key=operator.itemgetter(1))])
    return coo.tocsr(), row_index, col_index


def count_alignments(alignments: Iterable, gene_name_to_index: Dict[str, int], cell_tag: str = "CB",
                     molecule_tag: str = "UB", gene_tag: str = "GE"):
    """(csr, row_index, col_index) from records with .query_name / .has_tag / .get_tag
    (sctools_amd.bam.BamRecord), in file order."""
    seen = set()
    cells: List[int] = []
    genes: List[int] = []
    cell_to_index: Dict[str, int] = {}

    def tag(r, t) -> Optional[str]:
        return r.get_tag(t) if r.has_tag(t) else None

    def candidate(r):
        return r.has_tag(gene_tag) and r.has_tag("XF") and r.get_tag("XF") != "INTERGENIC"

    for _, grouper in itertools.groupby(alignments, key=lambda r: r.query_name):
        group = list(grouper)
        cell, molecule = tag(group[0], cell_tag), tag(group[0], molecule_tag)
        if cell is None or molecule is None:
            continue
        if len(group) == 1:
            r = group[0]
            if not candidate(r):
                continue
            gene = r.get_tag(gene_tag)
            if len(gene.split(",")) != 1:
                continue
        else:
            implicated = set()
            for r in group:
                if candidate(r) and len(r.get_tag(gene_tag).split(",")) == 1:
                    implicated.add(r.get_tag(gene_tag))
            if len(implicated) != 1:
                continue
            gene = next(iter(implicated))
        if (cell, molecule, gene) in seen:
            continue
        seen.add((cell, molecule, gene))
        col = gene_name_to_index[gene]
        if cell not in cell_to_index:
            cell_to_index[cell] = len(cell_to_index)
        cells.append(cell_to_index[cell])
        genes.append(col)
    return _finish(cells, genes, cell_to_index, gene_name_to_index)


def count_columns(arrays: Dict[str, np.ndarray], cell_names: List, umi_names: List, gene_names: List,
                  gene_name_to_index: Dict[str, int]):
    """The same loop over dictionary-id columns (cell, umi, gene, xf, qhead) -- for the larger
    synthetic parity cases.  Raises KeyError(gene name) as the reference does."""
    cell, umi, gene = arrays["cell"].tolist(), arrays["umi"].tolist(), arrays["gene"].tolist()
    xf, qhead = arrays["xf"].tolist(), arrays["qhead"].tolist()
    n = len(cell)
    single = [name is not None and "," not in name for name in gene_names]
    seen = set()
    cells: List[int] = []
    genes: List[int] = []
    cell_to_index: Dict[str, int] = {}
    i = 0
    while i < n:
        j = i + 1
        while j < n and not qhead[j]:
            j += 1
        c, u = cell_names[cell[i]], umi_names[umi[i]]
        if c is not None and u is not None:
            implicated = set()
            for k in range(i, j):
                if gene_names[gene[k]] is not None and xf[k] not in (XF_ABSENT, XF_INTERGENIC) and single[gene[k]]:
                    implicated.add(gene[k])
            if len(implicated) == 1:
                g = next(iter(implicated))
                if (c, u, g) not in seen:
                    seen.add((c, u, g))
                    col = gene_name_to_index[gene_names[g]]
                    if c not in cell_to_index:
                        cell_to_index[c] = len(cell_to_index)
                    cells.append(cell_to_index[c])
                    genes.append(col)
        i = j
    return _finish(cells, genes, cell_to_index, gene_name_to_index)
