"""End-to-end drop-in timing: GatherCellMetrics on a BAM (decode -> GPU metrics -> CSV.gz).

python tools/e2e_bench.py [--records N] [--bam PATH] [--host-decoder]   (needs a GPU)

The BAM is the reference's small-cell-sorted.bam payload (656 records of 58 cells) replicated
until it holds N records, every group of --replicas-per-cell consecutive replicas given one cell
barcode of its own (CB and CR rewritten in place, same length), so cells hold ~2.6k records as in
a 10x v2 run rather than the fixture's ~11 (UB / UR prefixes vary per replica too).  It is written once (BGZF, zlib level 6, 0xff00-byte
members as htslib writes them, compressed by a process pool).  Prints one JSON line: records,
seconds per stage -- the device decode's own stages (map + scan, copy, inflate, record starts,
parse + intern, dictionaries), GPU metrics, CSV text + gzip -- and records/s end to end, for
``GatherCellMetrics(bam).extract_metrics()`` (the drop-in) timed as one call, plus the same call
with the host decoder when --host-decoder is given.
"""
import argparse
import json
import os
import re
import struct
import sys
import time
import zlib
from multiprocessing import Pool

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
FIXTURE = os.path.join(ROOT, "tests", "golden", "bam", "small-cell-sorted.bam")
GENE_FIXTURE = os.path.join(ROOT, "tests", "golden", "bam", "small-gene-sorted.bam")
EOF_MEMBER = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")
BLOCK = 0xff00


def _payload(path):
    data = open(path, "rb").read()
    out, off = [], 0
    while off < len(data):
        xlen = struct.unpack_from("<H", data, off + 10)[0]
        bsize = struct.unpack_from("<H", data, off + 12 + xlen - 2)[0] + 1
        out.append(zlib.decompress(data[off + 12 + xlen: off + bsize - 8], -15))
        off += bsize
    return b"".join(out)


def _header_end(raw):
    off = 8 + struct.unpack_from("<i", raw, 4)[0]
    n_ref = struct.unpack_from("<i", raw, off)[0]
    off += 4
    for _ in range(n_ref):
        off += 4 + struct.unpack_from("<i", raw, off)[0] + 4
    return off


def _bgzf(raw):
    out = []
    for i in range(0, len(raw), BLOCK):
        chunk = raw[i:i + BLOCK]
        c = zlib.compressobj(6, zlib.DEFLATED, -15)
        comp = c.compress(chunk) + c.flush()
        head = struct.pack("<BBBBIBBHBBHH", 31, 139, 8, 4, 0, 0, 255, 6, 66, 67, 2, len(comp) + 25)
        out.append(head + comp + struct.pack("<II", zlib.crc32(chunk) & 0xFFFFFFFF, len(chunk)))
    return b"".join(out)


_BODY = None


def _init(body):
    global _BODY
    _BODY = body


def _group(args):
    """Compressed members of replicas [lo, hi): replica r's CB / CR values become cell r // k, and
    the first 5 bases of its UB / UR values encode r % 1024 (more molecule barcodes)."""
    lo, hi, k = args
    parts = []
    for r in range(lo, hi):
        bc = b"%016d" % (r // k)
        u = bytes(b"ACGT"[(r % 1024) >> (2 * i) & 3] for i in range(5))
        b = re.sub(rb"CBZ[^\x00]{16}\x00", b"CBZ" + bc + b"\x00", _BODY)
        b = re.sub(rb"CRZ[^\x00]{16}\x00", b"CRZ" + bc + b"\x00", b)
        b = re.sub(rb"UBZ[^\x00]{5}", b"UBZ" + u, b)
        parts.append(re.sub(rb"URZ[^\x00]{5}", b"URZ" + u, b))
    return _bgzf(b"".join(parts))


def _group_gene(args):
    """Gene-sorted replicas [lo, hi): the fixture's records each repeated k times (gene runs k times
    longer), the first 3 characters of every GE value replaced by replica r's code (new genes)."""
    lo, hi, k = args
    parts = []
    for r in range(lo, hi):
        code = bytes(65 + (r // 26 ** i) % 26 for i in range(3))
        parts.append(re.sub(rb"GEZ[^\x00]{3}", b"GEZ" + code, _BODY))
    return _bgzf(b"".join(parts))


def make_gene_bam(path, records, per_run, procs=16):
    """A gene-sorted BAM (small-gene-sorted.bam: 300 records of 8 genes) for GatherGeneMetrics."""
    raw = _payload(GENE_FIXTURE)
    h = _header_end(raw)
    body = raw[h:]
    recs, off = [], 0
    while off < len(body):
        n = 4 + struct.unpack_from("<i", body, off)[0]
        recs.append(body[off:off + n])
        off += n
    body = b"".join(r * per_run for r in recs)
    n_body = len(recs) * per_run
    reps = (records + n_body - 1) // n_body
    if reps > 26 ** 3:
        raise ValueError("too many replicas for 3-letter gene codes")
    jobs = [(lo, min(reps, lo + 16), per_run) for lo in range(0, reps, 16)]
    with open(path + ".tmp", "wb") as f:
        f.write(_bgzf(raw[:h]))
        with Pool(procs, initializer=_init, initargs=(body,)) as pool:
            for blob in pool.imap(_group_gene, jobs):
                f.write(blob)
        f.write(EOF_MEMBER)
    os.replace(path + ".tmp", path)
    return reps * n_body


def make_bam(path, records, per_cell, procs=16):
    raw = _payload(FIXTURE)
    h = _header_end(raw)
    body = raw[h:]
    n_body = body.count(b"CBZ")  # every fixture record carries CB
    reps = (records + n_body - 1) // n_body
    step = 64
    jobs = [(lo, min(reps, lo + step), per_cell) for lo in range(0, reps, step)]
    with open(path + ".tmp", "wb") as f:
        f.write(_bgzf(raw[:h]))
        with Pool(procs, initializer=_init, initargs=(body,)) as pool:
            for blob in pool.imap(_group, jobs):
                f.write(blob)
        f.write(EOF_MEMBER)
    os.replace(path + ".tmp", path)
    return reps * n_body


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=24_000_000)
    ap.add_argument("--replicas-per-cell", type=int, default=4)
    ap.add_argument("--bam", default=None)
    ap.add_argument("--host-decoder", action="store_true")
    ap.add_argument("--float-mode", default="welford")
    ap.add_argument("--gene", action="store_true",
                    help="GatherGeneMetrics on a gene-sorted BAM (small-gene-sorted.bam, each record "
                         "repeated --records-per-run times, gene names renamed per replica) instead")
    ap.add_argument("--records-per-run", type=int, default=20)
    ap.add_argument("--synth", action="store_true",
                    help="a config-2-shaped BAM from tools/synthbam.cpp (random 16-mer cells of ~10k reads, "
                         "30k Zipf genes in random name order, 10-mer UMIs, soft clips, CR != CB) instead of "
                         "the replicated fixture")
    ap.add_argument("--devices", type=int, default=0,
                    help="also time GatherCellMetrics(devices=[0] * N): N parts decoded and computed together")
    ap.add_argument("--count", action="store_true",
                    help="CountMatrix.from_sorted_tagged_bam (CreateCountMatrix) on the cell-sorted BAM instead")
    a = ap.parse_args()
    if a.gene:
        return main_gene(a)
    if a.count:
        return main_count(a)
    bam = a.bam or ("/tmp/sct_synth_%d.bam" if a.synth else "/tmp/sct_e2e_%d.bam") % a.records
    if not os.path.exists(bam) and a.synth:
        t0 = time.time()
        exe = os.path.join(ROOT, "tools", "synthbam")
        import subprocess

        if not os.path.exists(exe):
            subprocess.run(["g++", "-O2", "-fopenmp", "-o", exe, os.path.join(ROOT, "tools", "synthbam.cpp"), "-lz"],
                           check=True)
        subprocess.run([exe, bam, str(a.records)], check=True)
        print("wrote %s (%.0f MB) in %.1fs" % (bam, os.path.getsize(bam) / 1e6, time.time() - t0), file=sys.stderr,
              flush=True)
    if not os.path.exists(bam):
        t0 = time.time()
        n = make_bam(bam, a.records, a.replicas_per_cell)
        print("wrote %s (%d records, %.0f MB) in %.1fs" % (bam, n, os.path.getsize(bam) / 1e6, time.time() - t0),
              file=sys.stderr, flush=True)
    import torch

    from sctools_amd import columnar, gbam
    from sctools_amd.metrics import gatherer as G
    from sctools_amd.metrics.aggregator import CellMetrics
    from sctools_amd.metrics.writer import MetricCSVWriter

    torch.cuda.init()
    dev = torch.device("cuda", 0)
    res = {"bam": bam, "bam_mb": os.path.getsize(bam) / 1e6, "float_mode": a.float_mode}

    def log(what):  # progress on stderr (a long run stays visibly alive)
        print("%s %s" % (what, json.dumps({k: v for k, v in res.items() if not isinstance(v, dict)})),
              file=sys.stderr, flush=True)

    with open(bam, "rb") as f:  # page cache warm: the timed runs read memory, not the disk
        while f.read(1 << 26):
            pass
    G.GatherCellMetrics(bam, "/tmp/sct_e2e_warm", float_mode=a.float_mode).extract_metrics()  # warm-up
    torch.cuda.synchronize()

    # stage breakdown of the device path
    tm = {}
    t0 = time.perf_counter()
    got = gbam.decode(bam, "cell", dev, timings=tm, lazy=True)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if got is None:
        raise SystemExit("the device decoder declined %s: %s" % (bam, gbam.last_error()))
    arrays, (cn, un, gn) = got
    cols = columnar.Columns(arrays, cn, un, gn)
    ints, floats = G.compute_rows(cols, "cell", float_mode=a.float_mode, device=dev)
    t2 = time.perf_counter()
    with MetricCSVWriter("/tmp/sct_e2e_cell", compress=True) as w:
        w.write_header(vars(CellMetrics()))
        G.write_rows(w, "cell", cols, ints, floats)
    t3 = time.perf_counter()
    res.update({"records": cols.n, "cells": int(ints.shape[0]), "umis": len(un), "genes": len(gn),
                "device_decode_s": t1 - t0, "device_decode_stages_s": tm, "gpu_metrics_s": t2 - t1,
                "csv_gz_s": t3 - t2, "total_s": t3 - t0, "records_per_s": cols.n / (t3 - t0)})
    del cols, arrays, got
    torch.cuda.empty_cache()
    log("device path")

    runs = []
    for _ in range(3):
        t0 = time.perf_counter()
        G.GatherCellMetrics(bam, "/tmp/sct_e2e_cell2", float_mode=a.float_mode).extract_metrics()
        runs.append(time.perf_counter() - t0)
    res["GatherCellMetrics_s"] = runs
    res["GatherCellMetrics_records_per_s"] = res["records"] / min(runs)
    log("GatherCellMetrics")
    if a.devices:
        runs = []
        for _ in range(2):
            t0 = time.perf_counter()
            G.GatherCellMetrics(bam, "/tmp/sct_e2e_cell4", float_mode=a.float_mode,
                                devices=[0] * a.devices).extract_metrics()
            runs.append(time.perf_counter() - t0)
        res["GatherCellMetrics_parts_devices"] = [0] * a.devices
        res["GatherCellMetrics_parts_s"] = runs
        import gzip

        res["parts_and_one_device_csv_identical"] = (gzip.open("/tmp/sct_e2e_cell2.csv.gz").read()
                                                     == gzip.open("/tmp/sct_e2e_cell4.csv.gz").read())
        log("devices")
    if a.host_decoder:
        t0 = time.perf_counter()
        G.GatherCellMetrics(bam, "/tmp/sct_e2e_cell3", float_mode=a.float_mode, gpu_decode=False).extract_metrics()
        res["GatherCellMetrics_host_decoder_s"] = time.perf_counter() - t0
        res["GatherCellMetrics_host_decoder_records_per_s"] = res["records"] / res["GatherCellMetrics_host_decoder_s"]
        import gzip

        same = gzip.open("/tmp/sct_e2e_cell2.csv.gz").read() == gzip.open("/tmp/sct_e2e_cell3.csv.gz").read()
        res["device_and_host_decoder_csv_identical"] = same
    print(json.dumps(res))


def main_gene(a):
    bam = a.bam or "/tmp/sct_e2e_gene_%d.bam" % a.records
    if not os.path.exists(bam):
        t0 = time.time()
        n = make_gene_bam(bam, a.records, a.records_per_run)
        print("wrote %s (%d records, %.0f MB) in %.1fs" % (bam, n, os.path.getsize(bam) / 1e6, time.time() - t0),
              file=sys.stderr, flush=True)
    import torch

    from sctools_amd.metrics import gatherer as G

    torch.cuda.init()
    res = {"bam": bam, "bam_mb": os.path.getsize(bam) / 1e6, "float_mode": a.float_mode, "entry": "GatherGeneMetrics"}
    with open(bam, "rb") as f:
        while f.read(1 << 26):
            pass
    G.GatherGeneMetrics(bam, "/tmp/sct_e2e_gene_warm", float_mode=a.float_mode).extract_metrics()
    torch.cuda.synchronize()
    runs = []
    for _ in range(3):
        t0 = time.perf_counter()
        G.GatherGeneMetrics(bam, "/tmp/sct_e2e_gene", float_mode=a.float_mode).extract_metrics()
        runs.append(time.perf_counter() - t0)
    from sctools_amd import bamnative

    n = int(bamnative.decode(bam, "gene")[0]["cell"].shape[0]) if a.host_decoder else None
    res["GatherGeneMetrics_s"] = runs
    if a.host_decoder:
        t0 = time.perf_counter()
        G.GatherGeneMetrics(bam, "/tmp/sct_e2e_gene_host", float_mode=a.float_mode, gpu_decode=False).extract_metrics()
        res["GatherGeneMetrics_host_decoder_s"] = time.perf_counter() - t0
        import gzip

        res["device_and_host_decoder_csv_identical"] = (gzip.open("/tmp/sct_e2e_gene.csv.gz").read() ==
                                                        gzip.open("/tmp/sct_e2e_gene_host.csv.gz").read())
        res["records"] = n
        res["GatherGeneMetrics_records_per_s"] = n / min(runs)
    print(json.dumps(res))


def main_count(a):
    """CountMatrix.from_sorted_tagged_bam end to end: device decode (count mode) + GPU counting,
    against the same call with the host decoder; the gene index is every GE value of the file."""
    bam = a.bam or "/tmp/sct_e2e_%d.bam" % a.records
    if not os.path.exists(bam):
        make_bam(bam, a.records, a.replicas_per_cell)
    import numpy as np
    import torch

    from sctools_amd import bamnative
    from sctools_amd import count as C

    torch.cuda.init()
    with open(bam, "rb") as f:
        while f.read(1 << 26):
            pass
    arrays, (_, _, genes) = bamnative.decode(bam, "count", tags=("CB", "UB", "GE"))
    n = int(arrays["cell"].shape[0])
    names = {g: i for i, g in enumerate(sorted(g for g in genes if g is not None and "," not in g))}
    res = {"bam": bam, "bam_mb": os.path.getsize(bam) / 1e6, "entry": "CountMatrix.from_sorted_tagged_bam",
           "records": n, "genes": len(names)}
    C.CountMatrix.from_sorted_tagged_bam(bam, names, device="cuda:0")  # warm-up
    torch.cuda.synchronize()
    runs = []
    for _ in range(3):
        t0 = time.perf_counter()
        m = C.CountMatrix.from_sorted_tagged_bam(bam, names, device="cuda:0")
        runs.append(time.perf_counter() - t0)
    res["device_decode_s"] = runs
    res["records_per_s"] = n / min(runs)
    res["nnz"] = int(m.matrix.nnz)
    if a.host_decoder:
        t0 = time.perf_counter()
        h = C.CountMatrix.from_sorted_tagged_bam(bam, names, device="cuda:0", gpu_decode=False)
        res["host_decoder_s"] = time.perf_counter() - t0
        res["host_decoder_records_per_s"] = n / res["host_decoder_s"]
        res["device_and_host_decoder_identical"] = bool(
            m.matrix.shape == h.matrix.shape and (m.matrix != h.matrix).nnz == 0
            and np.array_equal(m.row_index, h.row_index))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
