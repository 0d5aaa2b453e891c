"""Tag values that are not strings, through the native decoders (bgzf.h read_tag, bamdec.cpp,
bamsplit.cpp).

The reference reads tag values through pysam as Python objects: integers compare numerically and
an integer never compares with a string (TypeError) in TagSortBam / VerifyBamSort (bam.py:638-724);
float and array values stay distinct keys in SplitBam (bam.py:263-290, 439-448).  The native
sort-key decode therefore reports typed sort-tag values (SCT_BAM_ETYPED) and the host takes the
Python values; the metric and count decoders do the same for float / array dictionary tags; a tag
value running past its record is a malformed record.
"""
import os
import struct

import numpy as np
import pytest

import helpers as H
from sctools_amd import bam as B
from sctools_amd import bamnative as BN
from sctools_amd import columnar
from bamwriter import record_bytes, write_bam

GOLD = os.path.join(H.GOLDEN, "bam")


def _recs(n=40, seed=3, tagger=None):
    """Records of small-cell-sorted.bam with one extra tag per record from tagger(i, rng)."""
    rng = np.random.default_rng(seed)
    out = []
    for i, r in enumerate(B.open_alignments(os.path.join(GOLD, "small-cell-sorted.bam"), "rb")):
        if i >= n:
            break
        tags = dict(r._tags)
        tags.update(tagger(i, rng))
        out.append(B.BamRecord("q%03d" % (n - i), r.flag, r.reference_id, r.pos, r.mapq, r.cigar, r.l_seq, r._qual,
                               tags))
    return out


@pytest.fixture
def int_tag_bam(tmp_path):
    """XN: integer values 0..12 (9 < 10 numerically, "10" < "9" as strings), XS: strings."""
    recs = _recs(tagger=lambda i, rng: {"XN": int(rng.integers(0, 13)), "XS": "s%d" % rng.integers(0, 3)})
    path = str(tmp_path / "int.bam")
    write_bam(path, recs)
    return path


def test_native_sort_keys_report_integer_values(int_tag_bam):
    with pytest.raises(BN.TypedTagValue):
        BN.decode(int_tag_bam, "sortkeys", tags=("XN", "XS", "~0"))
    arrays, _ = BN.decode(int_tag_bam, "sortkeys", tags=("XS", "~0", "~1"))  # strings stay native
    assert arrays["cell"].shape[0] == 40


def test_integer_sort_keys_rank_numerically(int_tag_bam):
    keys, names, qrank, qnames, typed = B._sort_keys(int_tag_bam, ["XN", "XS"])
    assert typed
    vals = [B.get_tag_or_default(r, "XN", "") for r in B.open_alignments(int_tag_bam, "rb")]
    order = sorted(range(len(vals)), key=lambda i: (vals[i], i))
    assert [names[0][keys[0][i]][0] for i in order] == sorted(vals)  # 9 before 10
    assert names[0][keys[0][order[0]]][0] == min(vals)


def test_mixed_int_and_missing_values_raise_type_error(tmp_path):
    recs = _recs(tagger=lambda i, rng: ({"XN": i} if i % 3 else {}))  # missing -> "" against ints
    path = str(tmp_path / "mixed.bam")
    write_bam(path, recs)
    with pytest.raises(TypeError):
        B._sort_keys(path, ["XN"])
    with pytest.raises(TypeError):
        sorted(B.TagSortableRecord.from_aligned_segment(r, ["XN"]) for r in B.open_alignments(path, "rb"))


def test_float_dictionary_tags_decode_through_the_python_reader(tmp_path):
    recs = _recs(tagger=lambda i, rng: {"CB": float(i // 10) + 0.5})
    path = str(tmp_path / "float_cb.bam")
    write_bam(path, recs)
    with pytest.raises(BN.TypedTagValue):
        BN.decode(path, "cell")
    cols = columnar.columnarize(path, "rb", "cell")
    py = columnar.columnarize(path, "rb", "cell", native=False)
    assert cols.cells.names == py.cells.names == [0.5, 1.5, 2.5, 3.5]
    for c in columnar.COLUMN_NAMES:
        assert np.array_equal(cols.arrays[c], py.arrays[c]), c


def test_split_keeps_float_and_array_barcodes_distinct(tmp_path):
    for kind, tagger in (("float", lambda i, rng: {"CB": float(i % 4) + 0.25}),
                         ("array", lambda i, rng: {"CB": [i % 4, 7]})):
        recs = _recs(n=40, tagger=tagger)
        src = str(tmp_path / ("%s.bam" % kind))
        write_bam(src, recs)
        n = BN.split([src], str(tmp_path / kind), ["CB"], 4, True)
        assert n == 4, kind
        per = [[str(r.get_tag("CB")) for r in B.open_alignments(str(tmp_path / ("%s_%d.bam" % (kind, k))), "rb")]
               for k in range(n)]
        assert sum(len(p) for p in per) == 40
        assert all(len(set(p)) == 1 for p in per), (kind, per)  # one barcode per chunk, none merged
        assert len({p[0] for p in per}) == 4


def test_truncated_trailing_tag_is_a_malformed_record(tmp_path):
    recs = _recs(n=5, tagger=lambda i, rng: {})
    raw = [record_bytes(r) for r in recs]
    body = raw[2][4:] + b"XNi\x01\x00"  # an int32 tag with two of its four bytes
    raw[2] = struct.pack("<i", len(body)) + body
    path = str(tmp_path / "trunc.bam")
    import bamwriter

    hdr = b"BAM\x01" + struct.pack("<i", 0) + struct.pack("<i", 32)
    for i in range(32):
        nm = ("chr%d" % i).encode() + b"\x00"
        hdr += struct.pack("<i", len(nm)) + nm + struct.pack("<i", 1 << 30)
    with open(path, "wb") as f:
        f.write(bamwriter._bgzf_block(hdr + b"".join(raw)))
        f.write(bamwriter._EOF)
    with pytest.raises(ValueError, match="truncated"):
        BN.decode(path, "cell")


@pytest.mark.gpu
def test_tag_sort_bam_orders_integer_tags_numerically(int_tag_bam, tmp_path):
    out = str(tmp_path / "s.bam")
    B.tag_sort_bam(int_tag_bam, out, ["XN", "XS"])
    py = list(B.open_alignments(int_tag_bam, "rb"))
    stable = sorted(range(len(py)), key=lambda i: B.TagSortableRecord.from_aligned_segment(py[i], ["XN", "XS"]))
    assert [r.query_name for r in B.open_alignments(out, "rb")] == [py[i].query_name for i in stable]


@pytest.mark.gpu
def test_verify_bam_sort_with_integer_tags_raises_as_the_reference(int_tag_bam):
    """verify_sort starts from a record of "" values: an int first value meets "" -> TypeError."""
    with pytest.raises(TypeError):
        B.verify_bam_sort(int_tag_bam, ["XN"])
    with pytest.raises(TypeError):
        B.verify_sort((B.TagSortableRecord.from_aligned_segment(r, ["XN"])
                       for r in B.open_alignments(int_tag_bam, "rb")), ["XN"])
