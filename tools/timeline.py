"""Timeline of one engine step from a rocprofv3 --kernel-trace CSV: every kernel of the LAST step
(from the last k_heads4 / k_heads launch to the end), its duration, and the idle gap before it --
where the device waits for the host (readbacks, launch latency) inside a step.

  python tools/timeline.py <dir with *kernel_trace.csv>
"""
import csv
import glob
import sys


def main():
    paths = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)
    rows = []
    for p in paths:
        with open(p) as f:
            for r in csv.DictReader(f):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if "k_heads" in r[2]]
    if not starts:
        sys.exit("no k_heads launch")
    first = starts[-2] if len(starts) > 1 else starts[-1]  # the last complete step
    last = starts[-1]
    step = rows[first:last] if last > first else rows[first:]
    t0 = step[0][0]
    busy = 0
    gap_tot = 0
    prev_end = step[0][0]
    print("%9s %9s %8s  %s" % ("start_us", "dur_us", "gap_us", "kernel"))
    for s, e, k in step:
        gap = max(0, s - prev_end)
        gap_tot += gap
        busy += e - s
        print("%9.1f %9.1f %8.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, gap / 1e3, k.split("(")[0][:90]))
        prev_end = max(prev_end, e)
    span = prev_end - t0
    print("span %.3f ms, kernel busy %.3f ms, idle gaps %.3f ms, kernels %d" % (span / 1e6, busy / 1e6, gap_tot / 1e6,
                                                                              len(step)))


if __name__ == "__main__":
    main()
