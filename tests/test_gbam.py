"""Device BAM decode (libsct_gbam.so, include/sct_gbam.h) against zlib and the host decoder.

The inflated payload must equal zlib's byte for byte, and the columns and dictionaries must equal
libsct_bam.so's (itself checked against the pure-Python decoder in test_bam_native.py) for every
bundled BAM, for the same payloads re-blocked with other deflate settings (stored, fixed-code,
Huffman-only and RLE blocks, many blocks per member, members cutting records anywhere), and
for files the device path must decline (records the reference rejects, typed dictionary tags):
there ``decode`` returns None and the host decoder raises as the reference does.
"""
import os
import re
import struct
import zlib

import numpy as np
import pytest

import helpers as H
from sctools_amd import bamnative, gbam

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(H.GOLDEN, "bam")
BAMS = sorted(f[:-4] for f in os.listdir(GOLD) if f.endswith(".bam"))


def test_every_declared_symbol_is_exported():
    text = open(os.path.join(ROOT, "include", "sct_gbam.h")).read()
    names = sorted(set(re.findall(r"^\s*(?:int|int64_t|void|const char\*)\s+(sct_\w+)\(", text, flags=re.M)))
    assert set(names) == set(gbam.EXPORTED)
    lib = gbam.load()
    for name in names:
        assert hasattr(lib, name), name


def members(data: bytes):
    off = 0
    while off < len(data):
        xlen = struct.unpack_from("<H", data, off + 10)[0]
        bsize = struct.unpack_from("<H", data, off + 12 + xlen - 2)[0] + 1
        yield data[off + 12 + xlen: off + bsize - 8]
        off += bsize


def payload(path) -> bytes:
    data = open(path, "rb").read()
    return b"".join(zlib.decompress(m, -15) for m in members(data))


def rebgzf(raw: bytes, path, level=6, strategy=zlib.Z_DEFAULT_STRATEGY, block=65280, mem_level=8):
    """raw payload -> BGZF with the given deflate settings (htslib's layout, then the EOF member)."""
    with open(path, "wb") as f:
        for i in range(0, len(raw), block):
            chunk = raw[i:i + block]
            c = zlib.compressobj(level, zlib.DEFLATED, -15, mem_level, strategy)
            comp = c.compress(chunk) + c.flush()
            head = struct.pack("<BBBBIBBHBBHH", 31, 139, 8, 4, 0, 0, 255, 6, 66, 67, 2, len(comp) + 25)
            f.write(head + comp + struct.pack("<II", zlib.crc32(chunk) & 0xFFFFFFFF, len(chunk)))
        f.write(bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000"))


def host(path, mode):
    try:
        return bamnative.decode(path, mode)
    except Exception as e:  # noqa: BLE001 -- the reference's exception for this file
        return e


def same_as_host(path, mode):
    want = host(path, mode)
    got = gbam.decode(path, mode)
    if isinstance(want, Exception):
        assert got is None, (path, mode, want)
        return None
    assert got is not None, (path, mode, gbam.last_error())
    cols, names = got
    arrays, want_names = want
    assert names == want_names
    for c, a in arrays.items():
        g = cols[c].cpu().numpy().view(a.dtype)
        assert np.array_equal(g, a), (path, mode, c)
    return cols


@pytest.mark.gpu
@pytest.mark.parametrize("bam", BAMS)
def test_inflate_matches_zlib(bam):
    path = os.path.join(GOLD, bam + ".bam")
    got = gbam.inflate(path)
    assert got is not None, gbam.last_error()
    assert got == payload(path)


@pytest.mark.gpu
@pytest.mark.parametrize("bam", BAMS)
@pytest.mark.parametrize("mode", ["cell", "gene"])
def test_columns_match_host_decoder(bam, mode):
    same_as_host(os.path.join(GOLD, bam + ".bam"), mode)


SETTINGS = [
    dict(level=0),  # stored blocks
    dict(level=1),
    dict(level=9),
    dict(level=6, strategy=zlib.Z_FIXED),
    dict(level=6, strategy=zlib.Z_HUFFMAN_ONLY),
    dict(level=6, strategy=zlib.Z_RLE),
    dict(level=6, mem_level=1),  # many small deflate blocks per member
    dict(level=6, block=997),  # members cut records anywhere; many records span members
    dict(level=6, block=65536),
]


@pytest.mark.gpu
@pytest.mark.parametrize("setting", SETTINGS, ids=lambda s: "-".join("%s%s" % kv for kv in s.items()))
def test_reblocked_payloads(tmp_path, setting):
    raw = payload(os.path.join(GOLD, "small-cell-sorted.bam"))
    path = str(tmp_path / "re.bam")
    rebgzf(raw, path, **setting)
    assert gbam.inflate(path) == raw
    same_as_host(path, "cell")
    same_as_host(path, "gene")


@pytest.mark.gpu
def test_many_members_and_records(tmp_path):
    """~60k records over ~300 members: every record start found, every string interned."""
    raw = payload(os.path.join(GOLD, "small-cell-sorted.bam"))
    hdr_end = _header_end(raw)
    body = raw[hdr_end:]
    reps = []
    for r in range(90):  # the first CB character per replica: same lengths, new barcodes
        reps.append(re.sub(rb"CBZ.", b"CBZ" + bytes([65 + r % 26]), body))
    big = raw[:hdr_end] + b"".join(reps)
    path = str(tmp_path / "big.bam")
    rebgzf(big, path, level=6, block=65280)
    assert gbam.inflate(path) == big
    cols = same_as_host(path, "cell")
    assert cols is not None and cols["cell"].numel() > 50000


def _header_end(raw: bytes) -> int:
    off = 8 + struct.unpack_from("<i", raw, 4)[0]
    n_ref = struct.unpack_from("<i", raw, off)[0]
    off += 4
    for _ in range(n_ref):
        off += 4 + struct.unpack_from("<i", raw, off)[0] + 4
    return off


@pytest.mark.gpu
def test_corrupt_member_declines(tmp_path):
    raw = payload(os.path.join(GOLD, "small-cell-sorted.bam"))
    path = str(tmp_path / "bad.bam")
    rebgzf(raw, path, level=6)
    data = bytearray(open(path, "rb").read())
    data[60] ^= 0xFF  # inside the first member's deflate data
    open(path, "wb").write(bytes(data))
    try:
        payload(path)
    except zlib.error:
        assert gbam.decode(path, "cell") is None
        return
    same_as_host(path, "cell")  # the flip left a valid stream: both decoders read the same bytes


@pytest.mark.gpu
def test_repeated_records_converge(tmp_path):
    """Identical consecutive records (each of small-gene-sorted.bam's records 20 times, 240k records,
    ~1600 members): a few members' start guesses land inside a record, and the repair must fix each
    from its agreeing predecessor instead of carrying a wrong landing forward member by member (it
    used to give up after 64 rounds and hand the file to the host decoder)."""
    import sys

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import e2e_bench

    path = str(tmp_path / "rep.bam")
    e2e_bench.make_gene_bam(path, 240_000, 20, procs=4)
    tm = {}
    got = gbam.decode(path, "gene", timings=tm)
    assert got is not None, gbam.last_error()
    assert tm["start_rounds"] < 64
    same_as_host(path, "gene")
    same_as_host(path, "cell")


@pytest.mark.gpu
@pytest.mark.parametrize("cap", [1, 200_000])
def test_device_memory_exhausted_declines(tmp_path, monkeypatch, cap):
    """A device allocation that fails (here: past SCT_GBAM_MAX_DEVICE_BYTES, as hipMalloc fails when
    HBM is exhausted) declines the file instead of raising: ``decode`` returns None and
    the gatherer's CSV, made by the host decoder, is still the reference's."""
    from sctools_amd.metrics import GatherCellMetrics

    path = os.path.join(GOLD, "cell-sorted-missing-cb.bam")
    monkeypatch.setenv("SCT_GBAM_MAX_DEVICE_BYTES", str(cap))
    assert gbam.decode(path, "cell") is None
    assert "device memory" in gbam.last_error()
    stem = str(tmp_path / "out")
    GatherCellMetrics(path, stem, compress=False).extract_metrics()
    assert open(stem + ".csv").read() == H.golden_text("cell-sorted-missing-cb", "cell")
    monkeypatch.delenv("SCT_GBAM_MAX_DEVICE_BYTES")
    same_as_host(path, "cell")  # the cap gone, the device decodes it again


def _windows(path, mode, **kw):
    t = {}
    got = gbam.decode(path, mode, timings=t, **kw)
    return got, t.get("windows")


@pytest.mark.gpu
@pytest.mark.parametrize("window", [40_000, 150_000])
@pytest.mark.parametrize("mode", ["cell", "gene"])
def test_windowed_decode_matches_host(tmp_path, monkeypatch, window, mode):
    """Bounded device memory: with SCT_GBAM_WINDOW_BYTES far below the payload the
    file is decoded in >= 3 windows of whole members -- carried records cut by a window's end,
    tables grown between windows, strings moved to the arena -- and the columns and dictionaries
    still equal the host decoder's.  Members of 997 bytes also cut records in every window."""
    raw = payload(os.path.join(GOLD, "cell-sorted-missing-cb.bam"))
    for name, block in (("big", 65280), ("small", 997)):
        path = str(tmp_path / (name + ".bam"))
        rebgzf(raw, path, level=6, block=block)
        monkeypatch.setenv("SCT_GBAM_WINDOW_BYTES", str(window))
        got, nw = _windows(path, mode)
        assert got is not None, gbam.last_error()
        assert nw >= 3, nw
        want, want_names = host(path, mode)
        cols, names = got
        assert names == want_names
        for c, a in want.items():
            assert np.array_equal(cols[c].cpu().numpy().view(a.dtype), a), (name, mode, c)
        monkeypatch.delenv("SCT_GBAM_WINDOW_BYTES")
        assert gbam.inflate(path) == raw  # one window again: the payload is resident


@pytest.mark.gpu
def test_windowed_count_mode_matches_host(tmp_path, monkeypatch):
    """Count mode across windows: the query-name head of each window's first record compares with
    the previous window's last record (carried with the cut one)."""
    raw = payload(os.path.join(H.GOLDEN, "count", "synth_b_qname.bam"))
    path = str(tmp_path / "q.bam")
    rebgzf(raw, path, level=6, block=997)
    monkeypatch.setenv("SCT_GBAM_WINDOW_BYTES", "6000")
    t = {}
    got = gbam.decode(path, "count", tags=("CB", "UB", "GE"), timings=t)
    assert got is not None, gbam.last_error()
    assert t["windows"] >= 3
    want, want_names = bamnative.decode(path, "count", tags=("CB", "UB", "GE"))
    cols, names = got
    assert names == [list(n) for n in want_names]
    for c in gbam.COUNT_COLUMNS:
        assert np.array_equal(cols[c].cpu().numpy(), want[c]), c


@pytest.mark.gpu
def test_windowed_gatherer_matches_reference(tmp_path, monkeypatch):
    """The drop-in through windows: GatherCellMetrics' CSV is still the reference's."""
    from sctools_amd.metrics import GatherCellMetrics, GatherGeneMetrics

    monkeypatch.setenv("SCT_GBAM_WINDOW_BYTES", "100000")
    for bam in ("cell-sorted-missing-cb", "small-gene-sorted"):
        for cls, kind in ((GatherCellMetrics, "cell"), (GatherGeneMetrics, "gene")):
            stem = str(tmp_path / (bam + kind))
            cls(os.path.join(GOLD, bam + ".bam"), stem, compress=False).extract_metrics()
            assert open(stem + ".csv").read() == H.golden_text(bam, kind), (bam, kind)


@pytest.mark.gpu
@pytest.mark.parametrize("n_parts", [2, 3, 7])
@pytest.mark.parametrize("window", [None, 30_000])
def test_parts_decode_matches_host(tmp_path, monkeypatch, n_parts, window):
    """devices=N decodes part p of the file on device p: byte-balanced member
    ranges, each part's first record proven against the previous part's walk, dictionaries merged
    and ids renumbered.  Concatenated in part order, the parts equal the host decoder's columns; the
    shards re-cut at cell runs keep every cell on one shard.  All parts on device 0 here (one GPU)."""
    from sctools_amd import columnar

    raw = payload(os.path.join(GOLD, "cell-sorted-missing-cb.bam"))
    path = str(tmp_path / "p.bam")
    rebgzf(raw, path, level=6, block=997)
    if window:
        monkeypatch.setenv("SCT_GBAM_WINDOW_BYTES", str(window))
    t = {}
    got = gbam.decode_parts(path, "cell", ["cuda:0"] * n_parts, timings=t)
    assert got is not None, gbam.last_error()
    assert len(t["parts"]) == n_parts and min(t["parts"]) > 0, t["parts"]
    shards, names = got
    want, want_names = host(path, "cell")
    assert [d.names for d in names] == want_names
    for c, a in want.items():
        g = np.concatenate([sh[c].cpu().numpy().view(a.dtype) for sh in shards])
        assert np.array_equal(g, a), c
    sc = columnar.ShardedColumns(columnar.cut_runs(shards, "cell"), *names)
    assert sc.n == want["cell"].shape[0]
    heads = [sh["cell"].cpu().numpy() for sh in sc.shards if sh["cell"].shape[0]]
    for a, b in zip(heads, heads[1:]):
        assert a[-1] != b[0]  # no cell run spans two shards
    assert np.array_equal(sc.host().arrays["cell"], want["cell"])
    idx = np.array([0, 5, sc.n // 2, sc.n - 1])
    assert np.array_equal(sc.column_at("gene", idx), want["gene"][idx])


@pytest.mark.gpu
@pytest.mark.parametrize("n_parts,block", [(7, 65280), (12, 30000), (9, 65280)])
def test_parts_with_empty_parts_match_host(tmp_path, n_parts, block):
    """More parts than record members: some parts own no member and decode no record.
    An empty part starts and lands where the previous part's walk landed (records cross member
    boundaries, so that landing can lie past the empty part's member boundary) -- the next part is
    checked against it -- and the parts still concatenate to the host decoder's columns."""
    raw = payload(os.path.join(GOLD, "small-cell-sorted.bam"))
    path = str(tmp_path / "e.bam")
    rebgzf(raw, path, level=6, block=block)
    t = {}
    got = gbam.decode_parts(path, "cell", ["cuda:0"] * n_parts, timings=t)
    assert got is not None, gbam.last_error()
    assert len(t["parts"]) == n_parts and min(t["parts"]) == 0, t["parts"]
    shards, names = got
    want, want_names = host(path, "cell")
    assert [d.names for d in names] == want_names
    for c, a in want.items():
        g = np.concatenate([sh[c].cpu().numpy().view(a.dtype) for sh in shards])
        assert np.array_equal(g, a), c
