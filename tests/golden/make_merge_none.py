"""
Reference MergeGeneMetrics on gene CSVs that carry a ``None`` row (reads without GE),
as the gatherer writes them (``/root/reference/src/sctools/metrics/merge.py:74-191``).

Run here only (the reference never leaves this container):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_merge_none.py

Inputs are the committed reference outputs ``ref/cell-sorted-missing-cb.gene.csv`` (one
``None`` row) and ``ref/small-gene-sorted.gene.csv``; writes ``merge/gene_none_merged.csv``
(the reference's merge of [missing-cb, small-gene, missing-cb]: the ``None`` rows are
dropped by pandas' ``groupby(level=0)``).  Merging missing-cb with itself leaves no row and
the reference raises ``ValueError``; the script prints that instead of writing a file.
"""
import gzip
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REF_SRC = "/root/reference/src"
sys.dont_write_bytecode = True
sys.path.insert(0, os.path.join(HERE, "stubs"))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, REF_SRC)

from sctools.metrics.merge import MergeGeneMetrics  # noqa: E402


def run(parts, name):
    out = os.path.join(HERE, "merge", name)
    MergeGeneMetrics(parts, out).execute()
    with gzip.open(out + ".csv.gz", "rt") as f:
        text = f.read()
    os.remove(out + ".csv.gz")
    with open(out + ".csv", "w") as f:
        f.write(text)
    print(name, len(text.splitlines()) - 1, "rows")


def main():
    none = os.path.join(HERE, "ref", "cell-sorted-missing-cb.gene.csv")
    small = os.path.join(HERE, "ref", "small-gene-sorted.gene.csv")
    run([none, small, none], "gene_none_merged")
    try:  # every row has a NaN index: the reference's groupby drops them all and pandas raises
        run([none, none], "gene_none_self_merged")
    except ValueError as e:
        print("gene_none_self_merged: ValueError:", e)


if __name__ == "__main__":
    main()
