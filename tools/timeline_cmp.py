"""Per-kernel comparison of several timeline.py tables (tools/gpu_tl_ab.sh): total ms per kernel name."""
import collections
import sys


def load(path):
    tot = collections.OrderedDict()
    span = None
    for line in open(path):
        parts = line.split()
        if line.startswith("span"):
            span = float(parts[1])
            continue
        if len(parts) < 4 or parts[0] == "start_us":
            continue
        name = " ".join(parts[3:]).replace("void ", "").split("<")[0].replace("sct::", "")
        tot[name] = tot.get(name, 0.0) + float(parts[1]) / 1e3
    return tot, span


def main():
    d = sys.argv[1]
    names = [a.split("=")[0] for a in sys.argv[2:]]
    tabs = {n: load("%s/%s.timeline.txt" % (d, n)) for n in names}
    keys = []
    for n in names:
        for k in tabs[n][0]:
            if k not in keys:
                keys.append(k)
    print("%-28s" % "kernel (ms)" + "".join("%12s" % n for n in names))
    for k in keys:
        print("%-28s" % k[:28] + "".join("%12.4f" % tabs[n][0].get(k, 0.0) for n in names))
    print("%-28s" % "span" + "".join("%12.4f" % tabs[n][1] for n in names))


if __name__ == "__main__":
    main()
