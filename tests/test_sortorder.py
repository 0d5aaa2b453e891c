"""TagSortBam / VerifyBamSort order (bam.py:602-728; platform.py:100-143).

CPU: the record-level mirror (TagSortableRecord, verify_sort, sort_by_tags_and_queryname)
on the exhaustive 3-tag value grid the reference's test_bam.py exercises and on the
reference's own BAM fixtures; the native sort-key decode against the Python reader.
GPU: verify_bam_sort (native decode + sct_verify_sort) and the VerifyBamSort CLI give the
same verdict and the same SortError message as the record-level verify_sort, for several
tag lists on sorted and unsorted fixtures.
"""
import itertools
import os

import numpy as np
import pytest

import helpers as H
from sctools_amd import bam as B
from sctools_amd import bamnative as BN

KEYS = ["FOO", "BAR", "BAZ"]
GRID = [(list(v), q) for v in itertools.product("AB", repeat=3) for q in "AB"]  # ascending


def recs(values, keys=KEYS):
    return [B.TagSortableRecord(keys, v, q) for v, q in values]


def bam_path(name):
    return os.path.join(H.GOLDEN, "bam", name + ".bam")


def host_verdict(path, tags):
    """None if sorted, else the SortError text, from the record-level verify_sort."""
    rs = (B.TagSortableRecord.from_aligned_segment(r, tags) for r in B.open_alignments(path, "rb"))
    try:
        B.verify_sort(rs, tags)
    except B.SortError as e:
        return str(e)
    return None


def test_grid_compares_in_order():
    rs = recs(GRID)
    for i, j in itertools.product(range(len(rs)), repeat=2):
        assert (rs[i] < rs[j]) == (i < j) and (rs[i] == rs[j]) == (i == j) and (rs[i] > rs[j]) == (i > j)


def test_different_tag_lists_do_not_compare():
    with pytest.raises(ValueError):
        B.TagSortableRecord(["FOO", "BAR"], ["A", "A"], "A") == B.TagSortableRecord(["BAR", "BAZ"], ["A", "A"], "A")
    assert "['FOO', 'BAR', 'BAZ']" in str(recs(GRID[:1])[0]) and "TagSortableRecord" in str(recs(GRID[:1])[0])


def test_verify_sort_on_the_grid():
    B.verify_sort(recs(GRID), KEYS)
    B.verify_sort(sorted(recs(GRID[::-1])), KEYS)
    shuffled = [GRID[i] for i in np.random.default_rng(3).permutation(len(GRID))]
    with pytest.raises(B.SortError, match="are not in correct order"):
        B.verify_sort(recs(shuffled), KEYS)
    B.verify_sort(sorted(recs([([], q) for _, q in shuffled], [])), [])


@pytest.mark.parametrize("tags", [["UB", "CB", "GE"], []])
def test_sort_by_tags_and_queryname_on_the_fixture(tags):
    out = list(B.sort_by_tags_and_queryname(B.open_alignments(bam_path("unsorted"), "rb"), tags))
    assert len(out) == 300
    B.verify_sort((B.TagSortableRecord.from_aligned_segment(r, tags) for r in out), tags)


def test_missing_tag_value_is_empty_string():
    r = next(iter(B.open_alignments(bam_path("unsorted"), "rb")))
    assert B.TagSortableRecord.from_aligned_segment(r, ["_NOT_REAL_TAG_"]).tag_values == [""]


def test_reference_sorted_fixture_verifies_on_the_host():
    assert host_verdict(bam_path("cell-gene-umi-queryname-sorted"), ["CB", "UB", "GE"]) is None
    assert host_verdict(bam_path("unsorted"), ["CB", "UB", "GE"]) is not None


@pytest.mark.parametrize("name", ["unsorted", "cell-sorted-missing-cb"])
def test_native_sort_keys_match_the_python_reader(name):
    """bamdec sort-key mode: tag and query-name ranks order exactly as the strings do ("" for a
    missing tag), against the Python reader."""
    tags = ("CB", "UB", "GE")
    arrays, names = BN.decode(bam_path(name), "sortkeys", tags=tags)
    rows = [(tuple(str(B.get_tag_or_default(r, t, "")) for t in tags), r.query_name)
            for r in B.open_alignments(bam_path(name), "rb")]
    assert len(rows) == len(arrays["qname"])
    for k, t in enumerate(("cell", "umi", "gene")):
        vals = ["" if v is None else v for v in names[k]]
        assert vals == sorted(vals) and len(set(vals)) == len(vals)
        assert [vals[i] for i in arrays[t]] == [r[0][k] for r in rows]
    assert names[3] == sorted(set(q for _, q in rows))
    assert [names[3][i] for i in arrays["qname"]] == [q for _, q in rows]


TAG_LISTS = [[], ["CB"], ["CB", "UB"], ["CB", "UB", "GE"], ["UB", "CB", "GE"], ["CB", "UB", "GE", "XF"]]


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cell-gene-umi-queryname-sorted", "unsorted", "small-cell-sorted"])
@pytest.mark.parametrize("tags", TAG_LISTS, ids=["-".join(t) or "none" for t in TAG_LISTS])
def test_gpu_verify_matches_the_record_level_verify(name, tags):
    path = bam_path(name)
    want = host_verdict(path, tags)
    if want is None:
        B.verify_bam_sort(path, tags)
    else:
        with pytest.raises(B.SortError) as e:
            B.verify_bam_sort(path, tags)
        assert str(e.value) == want


@pytest.mark.gpu
def test_verify_bam_sort_cli(capsys):
    from sctools_amd import platform

    path = bam_path("cell-gene-umi-queryname-sorted")
    assert platform.GenericPlatform.verify_bam_sort(["-i", path, "-t", "CB", "UB", "-t", "GE"]) == 0
    assert capsys.readouterr().out.strip() == "{0} is correctly sorted by {1} and query name".format(
        path, ["CB", "UB", "GE"])
    with pytest.raises(B.SortError):
        platform.GenericPlatform.verify_bam_sort(["-i", bam_path("unsorted"), "-t", "CB"])


def raw_records(path):
    """The inflated record bytes of a BAM, one bytes object per record, and its header bytes."""
    import gzip
    import struct

    data = gzip.open(path, "rb").read()
    off = 8 + struct.unpack("<i", data[4:8])[0]
    (n_ref,) = struct.unpack("<i", data[off:off + 4])
    off += 4
    for _ in range(n_ref):
        (l_name,) = struct.unpack("<i", data[off:off + 4])
        off += 4 + l_name + 4
    header, recs = data[:off], []
    while off < len(data):
        (bs,) = struct.unpack("<i", data[off:off + 4])
        recs.append(data[off:off + 4 + bs])
        off += 4 + bs
    return header, recs


@pytest.mark.parametrize("order", ["identity", "reverse", "shuffle"])
def test_write_order_rewrites_records_byte_for_byte(tmp_path, order):
    src = bam_path("unsorted")
    header, recs = raw_records(src)
    n = len(recs)
    perm = {"identity": np.arange(n), "reverse": np.arange(n)[::-1],
            "shuffle": np.random.default_rng(1).permutation(n)}[order]
    out = str(tmp_path / "o.bam")
    BN.write_order(src, out, perm)
    h2, r2 = raw_records(out)
    assert h2 == header and r2 == [recs[i] for i in perm]
    names = [r.query_name for r in B.open_alignments(src, "rb")]
    assert [r.query_name for r in B.open_alignments(out, "rb")] == [names[i] for i in perm]


def test_write_order_rejects_a_wrong_length(tmp_path):
    with pytest.raises(OSError, match="records"):
        BN.write_order(bam_path("unsorted"), str(tmp_path / "o.bam"), np.arange(5))


@pytest.mark.gpu
def test_tag_sort_bam_reproduces_the_reference_sorted_fixture(tmp_path):
    """TagSortBam -t CB UB GE of unsorted.bam: record for record the reference's own
    cell-gene-umi-queryname-sorted.bam (the reference's TagSortBam output)."""
    from sctools_amd import platform

    out = str(tmp_path / "sorted.bam")
    assert platform.GenericPlatform.tag_sort_bam(["-i", bam_path("unsorted"), "-o", out, "-t", "CB", "UB", "GE"]) == 0
    _, got = raw_records(out)
    _, want = raw_records(bam_path("cell-gene-umi-queryname-sorted"))
    assert got == want
    B.verify_bam_sort(out, ["CB", "UB", "GE"])


@pytest.mark.gpu
@pytest.mark.parametrize("tags", TAG_LISTS, ids=["-".join(t) or "none" for t in TAG_LISTS])
def test_tag_sort_bam_is_the_stable_sort(tmp_path, tags):
    src = bam_path("small-cell-sorted")
    out = str(tmp_path / "s.bam")
    B.tag_sort_bam(src, out, tags)
    _, raw = raw_records(src)
    py = list(B.open_alignments(src, "rb"))
    stable = sorted(range(len(py)), key=lambda i: B.TagSortableRecord.from_aligned_segment(py[i], tags))
    _, got = raw_records(out)
    assert got == [raw[i] for i in stable]  # sorted() is stable: ties keep input order
    assert host_verdict(out, tags) is None


@pytest.mark.gpu
@pytest.mark.parametrize("tags", [["CB", "UB", "GE"], ["GE", "CB"], []], ids=["CB-UB-GE", "GE-CB", "none"])
def test_tag_sort_bam_on_a_shuffled_13k_record_file(tmp_path, tags):
    """cell-sorted-missing-cb.bam (13,236 records, CB missing on some, secondaries sharing query
    names) shuffled by the native writer, then TagSortBam: the records in exactly the order of
    Python's stable sort of the shuffled file; VerifyBamSort accepts the output and rejects the
    shuffled input."""
    src = bam_path("cell-sorted-missing-cb")
    _, raw = raw_records(src)
    shuffled = str(tmp_path / "shuffled.bam")
    BN.write_order(src, shuffled, np.random.default_rng(7).permutation(len(raw)))
    out = str(tmp_path / "sorted.bam")
    B.tag_sort_bam(shuffled, out, tags)
    _, sraw = raw_records(shuffled)
    py = list(B.open_alignments(shuffled, "rb"))
    stable = sorted(range(len(py)), key=lambda i: B.TagSortableRecord.from_aligned_segment(py[i], tags))
    _, got = raw_records(out)
    assert got == [sraw[i] for i in stable]
    B.verify_bam_sort(out, tags)
    with pytest.raises(B.SortError):
        B.verify_bam_sort(shuffled, tags)
