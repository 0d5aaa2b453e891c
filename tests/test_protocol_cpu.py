"""The aggregator protocol record by record (aggregator.py:236-334, 492-530, 580-595).

The golden (tests/golden/protocol/aggregator_steps.json, made by make_protocol_golden.py with the
unmodified reference aggregator) holds the reference's integer attributes after every
parse_molecule call, on entities of the bundled BAMs, with and without one damaged record (a tag
dropped, or no base qualities).  Here the same calls go to sctools_amd.metrics.CellMetrics /
GeneMetrics: the counters must match after every record, the damaged record must raise the same
exception type in the same call, and an empty aggregator's finalize() must give the reference's
values.  finalize() of the parsed entities runs on the GPU (test_api_gpu.py).
"""

import json
import math
import os

import pytest

from sctools_amd.bam import BamRecord, open_alignments
from sctools_amd.metrics import CellMetrics, GeneMetrics

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden", "protocol", "aggregator_steps.json")


def _load():
    with open(GOLDEN) as f:
        return json.load(f)


def _tag(r, k):
    return r.get_tag(k) if r.has_tag(k) else None


def entity_records(kind, bam, ent):
    keys = ("CB", "UB", "GE") if kind == "cell" else ("GE", "CB", "UB")
    groups = []
    for r in open_alignments(os.path.join(HERE, "golden", "bam", bam + ".bam"), "rb"):
        t = tuple(_tag(r, k) for k in keys)
        if groups and groups[-1][0] == t[0]:
            groups[-1][1].append((t, r))
        else:
            groups.append((t[0], [(t, r)]))
    return groups[ent]


def damaged(r: BamRecord, damage):
    if damage is None:
        return r
    tags = dict(r._tags)
    qual = r._qual
    cigar = r.cigar
    if damage == "noqual":
        qual = None
    elif damage == "emptyqual":  # every base soft-clipped: empty aligned qualities
        cigar = [(4, r.l_seq)]
    else:
        tags.pop(damage.split(":")[1], None)
    return BamRecord(r.query_name, r.flag, r.reference_id, r.pos, r.mapq, cigar, r.l_seq, qual, tags)


CASES = _load()["cases"]


def replay(case):
    """Parse the case's records one call each; returns the aggregator, the per-call states and the
    exception type raised (or None)."""
    name, items = entity_records(case["kind"], case["bam"], case["entity"])
    assert name == case["entity_name"]
    agg = CellMetrics() if case["kind"] == "cell" else GeneMetrics()
    steps, raised = [], None
    for i, (t, r) in enumerate(items):
        rec = damaged(r, case["damage"] if i == case["bad_record"] else None)
        try:
            agg.parse_molecule(tags=t, records=[rec])
        except Exception as e:  # noqa: BLE001 -- compared with the reference's
            raised = type(e).__name__
        steps.append([getattr(agg, a) for a in case["attrs"]])
        if raised:
            break
    return agg, steps, raised


@pytest.mark.parametrize("case", CASES, ids=lambda c: "%s-%s-%d-%s" % (c["kind"], c["bam"], c["entity"], c["damage"]))
def test_counters_after_every_record(case):
    _, steps, raised = replay(case)
    assert raised == case["raised"]
    assert len(steps) == len(case["steps"])
    for i, (got, want) in enumerate(zip(steps, case["steps"])):
        assert got == want, (i, dict(zip(case["attrs"], zip(got, want))))


@pytest.mark.parametrize("kind", ["cell", "gene"])
def test_empty_finalize(kind):
    agg = CellMetrics() if kind == "cell" else GeneMetrics()
    agg.finalize()
    want = _load()["empty_finalize"][kind]
    got = {k: v for k, v in vars(agg).items() if not k.startswith("_")}
    assert list(got) == list(want)
    for k, v in got.items():
        w = want[k]
        if w == "nan":
            assert isinstance(v, float) and math.isnan(v), k
        else:
            assert str(v) == w, (k, v, w)


def test_protocol_golden_covers_the_error_paths():
    raised = {c["raised"] for c in CASES}
    assert {"KeyError", "TypeError", "ZeroDivisionError", None} <= raised
    assert any(c["kind"] == "gene" and c["raised"] for c in CASES)


def test_protocol_golden_records_finalize_after_caught_errors():
    """Every raising case carries the reference's finalize() after the caught error, at once and after
    the entity's remaining records (make_protocol_golden.py, round 5)."""
    for c in CASES:
        if c["raised"]:
            assert c["final_after_error"] and c["final_continued"], c["damage"]
            assert "n_molecules" in c["final_after_error"]
