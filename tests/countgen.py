"""Synthetic tagged alignments with a count matrix known by construction (count-matrix tests).

Same recipe as the reference's count test generator (test/test_count.py:151-420):
`max_genes` annotated genes get Poisson(rate) molecules per cell, one "necessary" query per
molecule (distinct molecule barcodes); then duplicate queries of necessary molecules,
queries missing a tag (or XF INTERGENIC / absent), and multi-alignment queries implicating
several genes -- none of which may change the matrix.  Extra cases the reference's loop
decides (count.py:247-287), each with its effect on the expected matrix:
  * multi-alignment queries implicating one gene (counted once);
  * a query whose INTERGENIC alignment names another gene (the other alignment counts);
  * "A,B" gene values (never implicated; "A,B" + "A" counts A);
  * a group whose first alignment has no cell barcode (dropped, whatever the others carry).
"""
import operator
from typing import Dict, List

import numpy as np

from sctools_amd.bam import BamRecord

XF_COUNTED = ("CODING", "UTR", "INTRONIC", "EXONIC")


def _barcodes(rng, n, length, taken=None):
    taken = set() if taken is None else taken
    out = []
    while len(out) < n:
        b = "".join(rng.choice(list("ACGT"), length))
        if b not in taken:
            taken.add(b)
            out.append(b)
    return out


def record(qname, tags, pos=0):
    return BamRecord(qname, 0, 0, pos, 255, [(0, 10)], 10, bytes([30] * 10), dict(tags))


def generate(gene_name_to_index: Dict[str, int], n_cells=50, max_genes=20, rate=5.0, n_duplicates=20,
             n_missing=20, n_multi=20, max_hits=5, n_extra=10, seed=777):
    """(records in query-name order, dense expected counts, row names, col names)."""
    rng = np.random.RandomState(seed)
    genes = [k for k, _ in sorted(gene_name_to_index.items(), key=operator.itemgetter(1))]
    used = rng.choice(len(genes), size=max_genes, replace=False)
    counts = np.zeros((n_cells, len(genes)), dtype=np.int64)
    counts[:, used] = rng.poisson(rate, size=(n_cells, max_genes))
    cells = _barcodes(rng, n_cells, 16)
    umis_taken = set()
    queries: List[List[dict]] = []  # one list of alignment tag dicts per query
    necessary = []
    for ci in range(n_cells):
        for gi in used:
            for ub in _barcodes(rng, int(counts[ci, gi]), 10, umis_taken):
                t = {"CB": cells[ci], "UB": ub, "GE": genes[gi], "XF": XF_COUNTED[rng.randint(4)]}
                necessary.append(t)
                queries.append([t])
    for k in rng.randint(0, len(necessary), size=n_duplicates):
        queries.append([dict(necessary[k], XF=XF_COUNTED[rng.randint(4)])])
    for _ in range(n_missing):
        t = {"CB": cells[rng.randint(n_cells)], "UB": _barcodes(rng, 1, 10, umis_taken)[0],
             "GE": genes[used[rng.randint(max_genes)]], "XF": "CODING"}
        defect = rng.randint(5)
        if defect < 3:
            del t[("CB", "UB", "GE")[defect]]
        elif defect == 3:
            t["XF"] = "INTERGENIC"
        else:
            del t["XF"]
        queries.append([t])
    for _ in range(n_multi):
        hits = rng.choice(used, size=rng.randint(2, max_hits + 1), replace=False)
        cb, ub = cells[rng.randint(n_cells)], _barcodes(rng, 1, 10, umis_taken)[0]
        queries.append([{"CB": cb, "UB": ub, "GE": genes[g], "XF": "CODING"} for g in hits])
    for _ in range(n_extra):
        ci = rng.randint(n_cells)
        cb = cells[ci]
        g1, g2 = (int(x) for x in rng.choice(used, size=2, replace=False))
        ub = _barcodes(rng, 4, 10, umis_taken)
        # one gene over 2-3 alignments: counted once
        queries.append([{"CB": cb, "UB": ub[0], "GE": genes[g1], "XF": "CODING"}] * rng.randint(2, 4))
        counts[ci, g1] += 1
        # INTERGENIC alignment of g1 + coding alignment of g2: g2 counts
        queries.append([{"CB": cb, "UB": ub[1], "GE": genes[g1], "XF": "INTERGENIC"},
                        {"CB": cb, "UB": ub[1], "GE": genes[g2], "XF": "UTR"}])
        counts[ci, g2] += 1
        # "g1,g2" alone: dropped; "g1,g2" + "g1": g1 counts
        queries.append([{"CB": cb, "UB": ub[2], "GE": genes[g1] + "," + genes[g2], "XF": "CODING"}])
        queries.append([{"CB": cb, "UB": ub[3], "GE": genes[g1] + "," + genes[g2], "XF": "CODING"},
                        {"CB": cb, "UB": ub[3], "GE": genes[g1], "XF": "CODING"}])
        counts[ci, g1] += 1
        # first alignment without CB: dropped
        ub4 = _barcodes(rng, 1, 10, umis_taken)[0]
        queries.append([{"UB": ub4, "GE": genes[g2], "XF": "CODING"},
                        {"CB": cb, "UB": ub4, "GE": genes[g2], "XF": "CODING"}])
    order = rng.permutation(len(queries))
    records = []
    for qi, q in enumerate(order):
        name = "QUERY_%07d" % qi
        for a, tags in enumerate(queries[q]):
            records.append(record(name, tags, pos=100 * qi + a))
    keep = counts.sum(axis=1) > 0
    return records, counts[keep], np.asarray(cells)[keep], np.asarray(genes)


def tag_sorted(records):
    """(CB, UB, GE, query name) order with "N" for a missing tag (the reference test's
    CellMoleculeGeneQueryNameSortOrder, test_count.py:115-148); multi-alignment queries may
    split into several groups -- the reference groups only consecutive equal names."""
    def key(r):
        t = r._tags
        return (str(t.get("CB", "N")), str(t.get("UB", "N")), str(t.get("GE", "N")), r.query_name)

    return sorted(records, key=key)
