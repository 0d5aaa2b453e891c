"""Summarize a rocprofv3 --stats kernel_stats.csv: the sct:: kernels, average and total time."""
import csv
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    print("%-28s %6s %12s %12s %7s" % ("kernel", "calls", "avg_us", "total_ms", "pct"))
    for r in rows:
        name = r["Name"]
        if "sct::" not in name:
            continue
        short = name.split("(")[0].replace("void ", "").replace("sct::", "")
        print("%-28s %6s %12.1f %12.3f %7s" % (short, r["Calls"], float(r["AverageNs"]) / 1e3,
                                               float(r["TotalDurationNs"]) / 1e6, r["Percentage"]))


if __name__ == "__main__":
    main(sys.argv[1])
