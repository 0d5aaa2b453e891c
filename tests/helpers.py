"""Shared fixture loaders and CSV rendering for the parity tests."""
import functools
import os

import numpy as np

from sctools_amd import _native as N
from sctools_amd import columnar
from sctools_amd.metrics import rows as R

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
BAMS = ["small-cell-sorted", "small-gene-sorted", "cell-sorted-missing-cb", "unsorted",
        "cell-gene-umi-queryname-sorted"]
SYNTH = ["s0", "s1", "s2", "s3"]


@functools.lru_cache(maxsize=None)
def bam_columns(name: str, metric_mode: str) -> columnar.Columns:
    return columnar.columnarize(os.path.join(GOLDEN, "bam", name + ".bam"), "rb", metric_mode)


def golden_text(name: str, kind: str) -> str:
    return open(os.path.join(GOLDEN, "ref", "%s.%s.csv" % (name, kind))).read()


def synth_text(name: str, kind: str) -> str:
    return open(os.path.join(GOLDEN, "synth", "%s.%s.csv" % (name, kind))).read()


class Synth:
    def __init__(self, name):
        z = np.load(os.path.join(GOLDEN, "synth", name + ".npz"), allow_pickle=False)
        self.arrays = {c: z[c] for c in N.RECORD_COLUMNS}
        self.gene_names = [None if none else str(g) for g, none in zip(z["gene_names"], z["gene_none"])]
        self.cell_names = [None if none else str(c) for c, none in zip(z["cell_names"], z["cell_none"])]
        self.gene_is_mito = z["gene_is_mito"].astype(np.uint8)
        self.gene_is_multi = z["gene_is_multi"].astype(np.uint8)
        self.n_umi_ids = int(z["n_umi_ids"])
        self.n = int(self.arrays["cell"].shape[0])

    @property
    def dims(self):
        return (len(self.cell_names), len(self.gene_names), self.n_umi_ids)


@functools.lru_cache(maxsize=None)
def synth(name: str) -> Synth:
    return Synth(name)


def entity_names(mode, ints, arrays, cell_names, gene_names):
    ent = ints[:, N.I_ENTITY]
    if mode == "cell":
        return [cell_names[arrays["cell"][i]] for i in ent]
    if mode == "gene":
        return [gene_names[arrays["gene"][i]] for i in ent]
    return [gene_names[g] for g in ent]


def render(mode, ints, floats, arrays, cell_names, gene_names) -> str:
    """Full CSV text, as the reference writer would produce it."""
    names = entity_names(mode, ints, arrays, cell_names, gene_names)
    keep, kept_names = R.select_rows(mode, ints, names)
    out_mode = "cell" if mode == "cell" else "gene"
    lines = [R.header_line(out_mode)]
    lines.extend(R.format_rows(out_mode, kept_names, ints[keep], floats[keep]))
    return "".join(lines)


def parse_csv(text):
    """{entity: [field strings]} plus header, for tolerance comparisons."""
    lines = text.rstrip("\n").split("\n")
    header = lines[0].split(",")
    rows = []
    for line in lines[1:]:
        # entity names may contain commas only for multi-gene ids, which are never emitted
        parts = line.split(",")
        rows.append(parts)
    return header, rows


def assert_csv_close(got: str, want: str, rel=1e-9):
    """Integers and row order exact; floats within `rel` (nan positions identical)."""
    hg, rg = parse_csv(got)
    hw, rw = parse_csv(want)
    assert hg == hw
    assert len(rg) == len(rw), (len(rg), len(rw))
    worst = 0.0
    for a, b in zip(rg, rw):
        assert a[0] == b[0]
        for x, y in zip(a[1:], b[1:]):
            if x == y:
                continue
            fx, fy = float(x), float(y)
            if np.isnan(fx) or np.isnan(fy):
                raise AssertionError("nan mismatch %s vs %s in row %s" % (x, y, a[0]))
            if "." not in y and "e" not in y and y != "nan":
                raise AssertionError("integer mismatch %s vs %s in row %s" % (x, y, a[0]))
            d = abs(fx - fy) / max(abs(fx), abs(fy))
            worst = max(worst, d)
            assert d <= rel, "row %s: %s vs %s (rel %.3g)" % (a[0], x, y, d)
    return worst
