"""
Generate tests/golden/protocol/*.json: the reference aggregator's public state after every
``parse_molecule`` call (``/root/reference/src/sctools/metrics/aggregator.py:236-334, 492-530,
580-595``), recorded by running the UNMODIFIED reference ``CellMetrics`` / ``GeneMetrics`` in the
build container through the stand-in pysam (tests/golden/stubs, pinned by make_golden.py).

Run here only (the reference never leaves this container):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_protocol_golden.py

Each case names an entity of a bundled BAM (its records in file order) and, optionally, one
record to damage (a tag dropped, no base qualities, or empty aligned qualities).  Recorded: the integer attributes after
each record, the exception type a record raised (the case stops there), and, for cases without
an error, every public attribute after ``finalize()`` as ``str`` (the CSV text, writer.py:96).  An empty aggregator's
``finalize()`` is recorded too.  For a case whose damaged record raised, two more states (round 5):
``final_after_error`` -- the caller catches the exception and calls ``finalize()`` at once -- and
``final_continued`` -- the caller catches it, parses the entity's remaining records, then
``finalize()`` -- each every public attribute as ``str`` (or the exception ``finalize`` raised).
"""

import copy
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_SRC = "/root/reference/src"

sys.dont_write_bytecode = True
sys.path.insert(0, os.path.join(HERE, "stubs"))
sys.path.insert(0, REPO)
sys.path.insert(0, REF_SRC)

import pysam  # noqa: E402  (the stub)
from sctools.metrics.aggregator import CellMetrics, GeneMetrics  # noqa: E402

from sctools_amd.bam import open_alignments  # noqa: E402

INT_ATTRS = ["n_reads", "noise_reads", "perfect_molecule_barcodes", "reads_mapped_exonic", "reads_mapped_intronic",
             "reads_mapped_utr", "reads_mapped_uniquely", "reads_mapped_multiple", "duplicate_reads",
             "spliced_reads", "antisense_reads", "_plus_strand_reads"]
CELL_INT_ATTRS = ["perfect_cell_barcodes", "reads_mapped_intergenic", "reads_unmapped",
                  "reads_mapped_too_many_loci"]

# (kind, bam, entity index, damaged record index or None, damage)
CASES = [
    ("cell", "small-cell-sorted", 17, None, None),
    ("cell", "small-cell-sorted", 14, None, None),
    ("cell", "cell-sorted-missing-cb", 0, None, None),
    ("cell", "cell-sorted-missing-cb", 28, None, None),
    ("cell", "small-cell-sorted", 17, 40, "drop:UY"),
    ("cell", "small-cell-sorted", 17, 11, "drop:CY"),
    ("cell", "small-cell-sorted", 22, 7, "drop:CR"),
    ("cell", "small-cell-sorted", 22, 9, "drop:XF"),
    ("cell", "small-cell-sorted", 14, 20, "drop:NH"),
    ("cell", "small-cell-sorted", 14, 3, "drop:UR"),
    ("cell", "small-cell-sorted", 14, 12, "drop:UB"),
    ("cell", "small-cell-sorted", 17, 60, "noqual"),
    ("cell", "cell-sorted-missing-cb", 0, 30, "drop:XF"),
    ("cell", "cell-sorted-missing-cb", 0, 100, "drop:NH"),
    ("gene", "small-gene-sorted", 4, None, None),
    ("gene", "small-gene-sorted", 3, None, None),
    ("gene", "small-gene-sorted", 4, 100, "drop:UY"),
    ("gene", "small-gene-sorted", 7, 5, "drop:CY"),
    ("gene", "small-gene-sorted", 3, 20, "drop:NH"),
    ("gene", "small-gene-sorted", 7, 9, "drop:XF"),
    ("gene", "small-gene-sorted", 3, 2, "noqual"),
    # round 6: more partial states -- the first record raising (nothing but a CY sample, or only the
    # molecule histogram, fed), empty aligned qualities (all soft-clipped: ZeroDivisionError at 288)
    ("cell", "small-cell-sorted", 22, 0, "drop:CR"),
    ("cell", "small-cell-sorted", 14, 0, "drop:UY"),
    ("cell", "small-cell-sorted", 17, 5, "emptyqual"),
    ("cell", "small-cell-sorted", 14, 0, "noqual"),
    ("cell", "cell-sorted-missing-cb", 28, 2, "drop:UY"),
    ("gene", "small-gene-sorted", 4, 10, "emptyqual"),
    ("gene", "small-gene-sorted", 3, 0, "drop:UY"),
]


def _tag(r, k):
    return r.get_tag(k) if r.has_tag(k) else None


def entities(kind, bam):
    keys = ("CB", "UB", "GE") if kind == "cell" else ("GE", "CB", "UB")
    groups = []
    for r in open_alignments(os.path.join(HERE, "bam", bam + ".bam"), "rb"):
        t = tuple(_tag(r, k) for k in keys)
        if groups and groups[-1][0] == t[0]:
            groups[-1][1].append((t, r))
        else:
            groups.append((t[0], [(t, r)]))
    return groups


def damaged(rec, damage):
    seg = pysam.AlignedSegment.from_bam(rec)
    if damage is None:
        return seg
    if damage == "noqual":
        seg._aq = None
        return seg
    if damage == "emptyqual":  # every base soft-clipped: query_alignment_qualities is empty
        seg._aq = seg._aq[:0]
        return seg
    tags = dict(seg._tags)
    tags.pop(damage.split(":")[1], None)
    seg._tags = tags
    return seg


def finalized(agg):
    try:
        agg.finalize()
    except Exception as e:  # noqa: BLE001 -- recorded
        return {"raised": type(e).__name__}
    return {k: str(v) for k, v in vars(agg).items() if not k.startswith("_")}


def attrs(kind):
    return INT_ATTRS + (CELL_INT_ATTRS if kind == "cell" else [])


def state(agg, kind):
    return [getattr(agg, a) for a in attrs(kind)]


def main():
    os.makedirs(os.path.join(HERE, "protocol"), exist_ok=True)
    out = []
    for kind, bam, ent, bad, damage in CASES:
        name, items = entities(kind, bam)[ent]
        agg = CellMetrics() if kind == "cell" else GeneMetrics()
        steps, raised = [], None
        for i, (t, r) in enumerate(items):
            seg = damaged(r, damage if i == bad else None)
            try:
                agg.parse_molecule(tags=t, records=[seg])
            except Exception as e:  # noqa: BLE001 -- recorded, the case stops
                raised = type(e).__name__
            steps.append(state(agg, kind))
            if raised:
                break
        final = final_after = final_cont = None
        if raised is None:
            agg.finalize()
            final = {k: str(v) for k, v in vars(agg).items() if not k.startswith("_")}
        else:
            final_after = finalized(copy.deepcopy(agg))
            for t, r in items[len(steps):]:
                agg.parse_molecule(tags=t, records=[damaged(r, None)])
            final_cont = finalized(agg)
        out.append({"kind": kind, "bam": bam, "entity": ent, "entity_name": name, "bad_record": bad,
                    "damage": damage, "attrs": attrs(kind), "steps": steps, "raised": raised, "final": final,
                    "final_after_error": final_after, "final_continued": final_cont})
    empty = {}
    for kind in ("cell", "gene"):
        agg = CellMetrics() if kind == "cell" else GeneMetrics()
        agg.finalize()
        empty[kind] = {k: str(v) for k, v in vars(agg).items() if not k.startswith("_")}
    with open(os.path.join(HERE, "protocol", "aggregator_steps.json"), "w") as f:
        json.dump({"reference": "fredlas/sctools aggregator.py (unmodified), via tests/golden/stubs",
                   "cases": out, "empty_finalize": empty}, f, separators=(",", ":"))
    print("wrote", len(out), "cases")


if __name__ == "__main__":
    main()
