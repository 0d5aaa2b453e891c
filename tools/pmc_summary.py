"""Per-kernel HBM traffic from rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE, TCC_EA0_*REQ).

Reads <dir>/{fetch,write,req}_counter_collection.csv written by tools/pmc_passes.sh
and prints, per sct:: kernel, the average per dispatch of each counter, plus the
calibration clone (the last copy kernel of tools/pmc_probe.py: 1 GiB read + 1 GiB
written) so units can be checked.  FETCH_SIZE / WRITE_SIZE are in KiB.
"""
import csv
import json
import sys
from collections import defaultdict


def load(path):
    out = defaultdict(lambda: defaultdict(list))
    order = []
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        short = name.split("(")[0].replace("void ", "")
        if "sct::" in short:
            short = short.replace("sct::", "")
        elif "copy" in name.lower() or "elementwise" in name.lower():
            short = "torch:" + short.split("<")[0].split("::")[-1]
        else:
            continue
        out[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
        order.append((int(r["Dispatch_Id"]), short, r["Counter_Name"], float(r["Counter_Value"])))
    return out, order


def main(d):
    res = defaultdict(dict)
    calib = {}
    for tag in ("fetch", "write", "req"):
        try:
            data, order = load("%s/%s_counter_collection.csv" % (d, tag))
        except FileNotFoundError:
            continue
        for k, ctrs in data.items():
            if k.startswith("torch:"):
                continue
            for c, vals in ctrs.items():
                res[k][c] = sum(vals) / len(vals)
        # calibration: the last torch copy-like dispatch
        torch_rows = [o for o in order if o[1].startswith("torch:")]
        if torch_rows:
            last = max(o[0] for o in torch_rows)
            for o in torch_rows:
                if o[0] == last:
                    calib[o[2]] = o[3]
    print(json.dumps({"per_dispatch_avg": res, "calibration_1GiB_clone": calib}, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1])
