"""Minimal BGZF BAM writer for decoder tests (records shaped like sctools_amd.bam.BamRecord)."""
import struct
import zlib

_EOF = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")


def _bgzf_block(data: bytes) -> bytes:
    c = zlib.compressobj(6, zlib.DEFLATED, -15)
    comp = c.compress(data) + c.flush()
    bsize = len(comp) + 25
    head = struct.pack("<BBBBIBBHBBHH", 31, 139, 8, 4, 0, 0, 255, 6, 66, 67, 2, bsize)
    return head + comp + struct.pack("<II", zlib.crc32(data) & 0xFFFFFFFF, len(data))


def _tag(k, v) -> bytes:
    if isinstance(v, str):
        return k.encode() + b"Z" + v.encode("latin-1") + b"\x00"
    if isinstance(v, int):
        return k.encode() + b"i" + struct.pack("<i", v)
    if isinstance(v, float):
        return k.encode() + b"f" + struct.pack("<f", v)
    if isinstance(v, list):  # B array of int32
        return k.encode() + b"Bi" + struct.pack("<i", len(v)) + b"".join(struct.pack("<i", x) for x in v)
    raise TypeError(v)


def record_bytes(r) -> bytes:
    name = r.query_name.encode() + b"\x00"
    cigar = b"".join(struct.pack("<I", (ln << 4) | op) for op, ln in r.cigar)
    seq = bytes((r.l_seq + 1) // 2)
    qual = r._qual if r._qual is not None else b"\xff" * r.l_seq
    tags = b"".join(_tag(k, v) for k, v in r._tags.items())
    core = struct.pack("<iiBBHHHiiii", r.reference_id, r.pos, len(name), r.mapq, 0, len(r.cigar), r.flag,
                       r.l_seq, -1, -1, 0)
    body = core + name + cigar + seq + qual + tags
    return struct.pack("<i", len(body)) + body


def write_bam(path, records, n_ref=32, block=60000):
    hdr = b"BAM\x01" + struct.pack("<i", 0) + struct.pack("<i", n_ref)
    for i in range(n_ref):
        nm = ("chr%d" % i).encode() + b"\x00"
        hdr += struct.pack("<i", len(nm)) + nm + struct.pack("<i", 1 << 30)
    raw = hdr + b"".join(record_bytes(r) for r in records)
    with open(path, "wb") as f:
        for i in range(0, len(raw), block):
            f.write(_bgzf_block(raw[i:i + block]))
        f.write(_EOF)
