"""End-to-end drop-in timing: GatherCellMetrics / GatherGeneMetrics on a BAM (decode -> GPU -> CSV.gz).

python tools/e2e_bench.py [--replicas R] [--bam PATH]   (needs a GPU)

The BAM is the reference's small-cell-sorted.bam fixture replicated R times, each replica with
its own cell barcodes (CB + '-r'), written once with tests/bamwriter.py.  Prints one JSON line:
records, seconds per stage (native decode, H2D + GPU metrics, CSV text + gzip) and records/s.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def make_bam(path, replicas):
    import bamwriter
    from sctools_amd.bam import open_alignments

    base = list(open_alignments(os.path.join(ROOT, "tests", "golden", "bam", "small-cell-sorted.bam"), "rb"))
    out = []
    for r in range(replicas):
        for rec in base:
            t = dict(rec._tags)
            if "CB" in t:
                t["CB"] = "%s-%d" % (t["CB"], r)
                t["CR"] = t["CB"] if rec._tags.get("CR") == rec._tags.get("CB") else t.get("CR")
            x = type(rec)(rec.query_name, rec.flag, rec.reference_id, rec.pos, rec.mapq, rec.cigar, rec.l_seq,
                          rec._qual, t)
            out.append(x)
    bamwriter.write_bam(path, out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--replicas", type=int, default=3000)
    ap.add_argument("--bam", default="/tmp/sct_e2e.bam")
    a = ap.parse_args()
    if not os.path.exists(a.bam):
        t0 = time.time()
        make_bam(a.bam, a.replicas)
        print("wrote %s in %.1fs" % (a.bam, time.time() - t0), file=sys.stderr, flush=True)
    import torch

    from sctools_amd import columnar
    from sctools_amd.metrics import gatherer as G
    from sctools_amd.metrics.writer import MetricCSVWriter
    from sctools_amd.metrics.aggregator import CellMetrics

    torch.cuda.init()
    res = {"bam": a.bam, "bam_mb": os.path.getsize(a.bam) / 1e6}
    G.compute_rows(columnar.columnarize(a.bam, "rb", "cell"), "cell", float_mode="exact")  # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    cols = columnar.columnarize(a.bam, "rb", "cell")
    t1 = time.perf_counter()
    ints, floats = G.compute_rows(cols, "cell", float_mode="welford")
    t2 = time.perf_counter()
    with MetricCSVWriter("/tmp/sct_e2e_cell", compress=True) as w:
        w.write_header(vars(CellMetrics()))
        G.write_rows(w, "cell", cols, ints, floats)
    t3 = time.perf_counter()
    res.update({"records": cols.n, "cells": int(ints.shape[0]), "decode_s": t1 - t0, "gpu_metrics_s": t2 - t1,
                "csv_gz_s": t3 - t2, "total_s": t3 - t0, "records_per_s": cols.n / (t3 - t0)})
    t0 = time.perf_counter()
    G.GatherCellMetrics(a.bam, "/tmp/sct_e2e_cell2").extract_metrics()
    res["GatherCellMetrics_s"] = time.perf_counter() - t0
    print(json.dumps(res))


if __name__ == "__main__":
    main()
