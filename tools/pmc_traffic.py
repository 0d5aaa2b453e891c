"""Per-launch HBM traffic of every engine kernel from rocprofv3 --pmc passes -> a JSON that
bench.py reads for its roofline "traffic" field (MI355X_MICROARCH.md, HBM section).

  tools/pmc_passes.sh writes <dir>/{fetch,write}_counter_collection.csv (one counter per pass);
  python tools/pmc_traffic.py <dir> > profiles/<round>/pmc_traffic.json

FETCH_SIZE and WRITE_SIZE are KiB per dispatch.  gfx950 FETCH_SIZE counts exactly half the bytes
of a wide coalesced read (the guide; checked here on the calibration clone of tools/pmc_probe.py:
1 GiB read + 1 GiB written), so HBM bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024.  The
engine's source hash is recorded: bench.py uses the figures only for the same kernels' source.
"""
import csv
import hashlib
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# the device BAM decoder's and host decoders' sources are not part of the engine library the PMC
# passes measure (libsctools_gpu.so: sct_engine.hip and the headers it includes)
NOT_ENGINE = ("gbam.hip", "inflate.h", "bgzf.h")


def source_hash(root=ROOT):
    d = os.path.join(root, "sctools_amd", "csrc")
    h = hashlib.sha256()
    for f in sorted(os.listdir(d)):
        if f.endswith((".h", ".hip")) and f not in NOT_ENGINE:
            h.update(f.encode())
            h.update(open(os.path.join(d, f), "rb").read())
    return h.hexdigest()


def load(path):
    per = defaultdict(list)
    torch_last = None
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        v = float(r["Counter_Value"])
        if name.startswith("sct::k_"):
            per[name[len("sct::k_"):].split("<")[0]].append(v)
        elif "copy" in name.lower() or "elementwise" in name.lower():
            did = int(r["Dispatch_Id"])
            if torch_last is None or did > torch_last[0]:
                torch_last = (did, v)
    return {k: (sum(v) / len(v), len(v)) for k, v in per.items()}, (torch_last[1] if torch_last else None)


def main(d, extra=()):
    fetch, cf = load(os.path.join(d, "fetch_counter_collection.csv"))
    write, cw = load(os.path.join(d, "write_counter_collection.csv"))
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        f, nf = fetch.get(k, (0.0, 0))
        w, nw = write.get(k, (0.0, 0))
        kernels[k] = {"FETCH_SIZE_KiB": f, "WRITE_SIZE_KiB": w, "hbm_bytes_per_launch": 2 * f * 1024 + w * 1024,
                      "dispatches": max(nf, nw)}  # in the probe run: weights kernels sharing a profile name
    out = {
        "source_sha256": source_hash(),
        "workload": "tools/pmc_probe.py %s: %s, cell + grouped gene" % (" ".join(extra) or "--config 2", {
            "2": "config-2 shard (100M records, 10k cells, 30k genes)",
            "4": "config-4 shard (125M records, 62.5k lognormal(0, 2) cells, 30k genes)",
            "5": "config-5 shard (100M shuffled records sorted by (CB, UB, GE, query name) in the step)"}[
                extra[extra.index("--config") + 1] if "--config" in extra else "2"]),
        "calibration_1GiB_clone": {"FETCH_SIZE_KiB": cf, "WRITE_SIZE_KiB": cw,
                                   "expected_KiB": 1 << 20, "fetch_correction": 2},
        "kernels": kernels,
    }
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
