"""
Generate the count-matrix golden fixtures under tests/golden/count/ by running the UNMODIFIED
reference ``CountMatrix.from_sorted_tagged_bam`` (/root/reference/src/sctools/count.py) and
``gtf.extract_gene_names`` in the build container, through the same stand-in pysam as
make_golden.py (tests/golden/stubs).  Run here only:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_count_golden.py

Writes (data only):
* ``chr1.30k_genes.gtf.gz``  the ``gene`` records of the reference's chr1.30k_records.gtf.gz
  (the only records extract_gene_names reads);
* ``chr1.30k_gene_names.json``  the reference's extract_gene_names of the FULL file;
* ``<case>.bam`` / ``<case>.sam``  synthetic inputs (tests/countgen.py, written with
  tests/bamwriter.py);
* ``<case>.genes.json``  the gene_name_to_index used for a case;
* ``<case>.npz``  the reference's matrix (indptr, indices, data, shape) and row / col index,
  or ``error`` = "KeyError: <message>" when the reference raises.
"""
import gzip
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_SRC = "/root/reference/src"
REF_DATA = os.path.join(REF_SRC, "sctools", "test", "data")
OUT = os.path.join(HERE, "count")

sys.dont_write_bytecode = True
sys.path.insert(0, os.path.join(HERE, "stubs"))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, REF_SRC)

import numpy as np  # noqa: E402

from sctools import gtf as ref_gtf  # noqa: E402
from sctools.count import CountMatrix  # noqa: E402

import bamwriter  # noqa: E402
import countgen  # noqa: E402
from sctools_amd import bam  # noqa: E402

FIXTURE_BAMS = ["small-cell-sorted", "small-gene-sorted", "cell-sorted-missing-cb", "unsorted",
                "cell-gene-umi-queryname-sorted"]


def save_result(case, fn):
    path = os.path.join(OUT, case + ".npz")
    try:
        m = fn()
    except KeyError as e:
        np.savez(path, error=np.asarray("KeyError: " + str(e.args[0])))
        return "KeyError %s" % e.args[0]
    csr = m.matrix
    np.savez(path, indptr=csr.indptr, indices=csr.indices, data=csr.data, shape=np.asarray(csr.shape),
             row_index=m.row_index, col_index=m.col_index)
    return "%dx%d nnz=%d" % (csr.shape[0], csr.shape[1], csr.nnz)


def write_sam(path, records):
    with open(path, "w") as f:
        f.write("@HD\tVN:1.6\n@SQ\tSN:chr0\tLN:1000000000\n")
        for r in records:
            tags = "\t".join("%s:Z:%s" % (k, v) for k, v in r._tags.items())
            f.write("%s\t0\tchr0\t%d\t255\t10M\t*\t0\t0\tACGTACGTAC\tIIIIIIIIII\t%s\n" % (r.query_name, r.pos + 1, tags))


def main():
    os.makedirs(OUT, exist_ok=True)
    gtf_path = os.path.join(REF_DATA, "chr1.30k_records.gtf.gz")
    names = ref_gtf.extract_gene_names(gtf_path)
    json.dump(names, open(os.path.join(OUT, "chr1.30k_gene_names.json"), "w"))
    with gzip.open(gtf_path, "rt") as src, gzip.open(os.path.join(OUT, "chr1.30k_genes.gtf.gz"), "wt") as dst:
        for line in src:
            f = line.split("\t")
            if line.startswith("#") or (len(f) > 2 and f[2] == "gene"):
                dst.write(line)
    print("gtf: %d gene names" % len(names))

    def run(case, path, genes, mode="rb"):
        json.dump(genes, open(os.path.join(OUT, case + ".genes.json"), "w"))
        print(case, save_result(case, lambda: CountMatrix.from_sorted_tagged_bam(path, genes, open_mode=mode)))

    # synthetic cases (reference test recipe, test_count.py:151-420)
    for case, kw in [("synth_a", dict(seed=777)), ("synth_b", dict(seed=11, n_cells=30, max_genes=40, n_multi=60,
                                                                    n_extra=40))]:
        recs, _, _, _ = countgen.generate(names, **kw)
        for order, rs in [("qname", recs), ("tags", countgen.tag_sorted(recs))]:
            p = os.path.join(OUT, "%s_%s.bam" % (case, order))
            bamwriter.write_bam(p, rs)
            run("%s_%s" % (case, order), p, names)
    recs, _, _, _ = countgen.generate(names, seed=5, n_cells=12, max_genes=10)
    p = os.path.join(OUT, "synth_sam.sam")
    write_sam(p, recs)
    run("synth_sam", p, names, mode="r")
    p = os.path.join(OUT, "empty.bam")
    bamwriter.write_bam(p, [])
    run("empty", p, names)
    # the reference's metric BAMs: with the chr1.30k annotation (their genes are not all in
    # it: KeyError) and with an annotation of their own single gene names
    for b in FIXTURE_BAMS:
        p = os.path.join(HERE, "bam", b + ".bam")
        run("fixture_%s_gtf" % b, p, names)
        ge = sorted({str(r._tags["GE"]) for r in bam.open_alignments(p, "rb")
                     if "GE" in r._tags and "," not in str(r._tags["GE"])})
        run("fixture_%s" % b, p, {g: i for i, g in enumerate(["PADDING_GENE"] + ge[::-1])})


if __name__ == "__main__":
    main()
