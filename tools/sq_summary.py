"""Per-kernel SQ counter summary (sum over dispatches) from rocprofv3 --pmc csv files."""
import csv
import sys
from collections import defaultdict


def main(paths):
    agg = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(set)
    for p in paths:
        for r in csv.DictReader(open(p)):
            name = r["Kernel_Name"]
            if "sct::" not in name:
                continue
            short = name.split("(")[0].replace("void ", "").replace("sct::", "")
            agg[short][r["Counter_Name"]] += float(r["Counter_Value"])
            calls[short].add(r["Dispatch_Id"])
    for k, c in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        print("%-34s waves=%-9d busy=%-10d" % (k, c.get("SQ_WAVES", 0), c.get("SQ_BUSY_CYCLES", 0)))
        print("    wait_any %.2f  wait_inst %.2f  active %.2f | valu_act %.2f lds_act %.2f | VALU/wave %.0f LDS/wave %.0f"
              " SALU/wave %.0f VMRD/wave %.0f VMWR/wave %.0f | lds_conf/lds_active %.2f wait_inst_lds %.3f" % (
                  c.get("SQ_WAIT_ANY", 0) / wc, c.get("SQ_WAIT_INST_ANY", 0) / wc, c.get("SQ_ACTIVE_INST_ANY", 0) / wc,
                  c.get("SQ_ACTIVE_INST_VALU", 0) / wc, c.get("SQ_ACTIVE_INST_LDS", 0) / wc,
                  c.get("SQ_INSTS_VALU", 0) / max(1, c.get("SQ_WAVES", 1)),
                  c.get("SQ_INSTS_LDS", 0) / max(1, c.get("SQ_WAVES", 1)),
                  c.get("SQ_INSTS_SALU", 0) / max(1, c.get("SQ_WAVES", 1)),
                  c.get("SQ_INSTS_VMEM_RD", 0) / max(1, c.get("SQ_WAVES", 1)),
                  c.get("SQ_INSTS_VMEM_WR", 0) / max(1, c.get("SQ_WAVES", 1)),
                  c.get("SQ_LDS_BANK_CONFLICT", 0) / max(1, c.get("SQ_LDS_IDX_ACTIVE", 1)),
                  c.get("SQ_WAIT_INST_LDS", 0) / wc))


if __name__ == "__main__":
    main(sys.argv[1:])
