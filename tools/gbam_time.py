"""Device BAM decode timing (experiments): stages of gbam.decode on one BAM, best of --reps.

python tools/gbam_time.py BAM [--reps 3]   (SCT_GBAM_LIB_PATH selects an experimental library)
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("bam")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--mode", default="cell", choices=["cell", "gene"])
    a = ap.parse_args()
    import torch

    from sctools_amd import gbam

    dev = torch.device("cuda", 0)
    torch.cuda.init()
    best = None
    for _ in range(a.reps + 1):
        tm = {}
        t0 = time.perf_counter()
        got = gbam.decode(a.bam, a.mode, dev, timings=tm, lazy=True)
        torch.cuda.synchronize()
        t = time.perf_counter() - t0
        if got is None:
            raise SystemExit("declined: %s" % gbam.last_error())
        n = got[0]["cell"].numel()
        del got
        if best is None or t < best[0]:
            best = (t, tm, n)
    t, tm, n = best
    print(json.dumps({"lib": gbam.LIB_PATH, "records": n, "decode_s": t, "records_per_s": n / t, "stages_s": tm}))


if __name__ == "__main__":
    main()
