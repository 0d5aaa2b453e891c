"""Instruction mix of k_welford_chains<true> per record (VERDICT r3 Next #7: "count the issued
instructions per record in the ISA before and after").

Usage: python tools/welford_isa_count.py <engine.s> [<engine.s> ...]
where engine.s is `hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off
--offload-device-only -S` of sctools_amd/csrc/sct_engine.hip (of any revision).  The chain's batch
body is the basic blocks that hold its f64 updates (one block per unrolled batch of kWfBatch
records); each is reported with its instruction mix, and per record = block / kWfBatch.
"""
import re
import sys

K_BATCH = 32


def blocks_of(lines, fn_prefix):
    i = next(k for k, l in enumerate(lines) if l.startswith(fn_prefix))
    j = i
    while not lines[j].startswith(".Lfunc_end"):
        j += 1
    out, cur = [], ("entry", [])
    for l in lines[i:j]:
        m = re.match(r"^(\.LBB\d+_\d+):", l)
        if m:
            out.append(cur)
            cur = (m.group(1), [])
            continue
        s = l.strip()
        if s and not s.startswith((";", ".")) and not s.endswith(":"):
            cur[1].append(s)
    out.append(cur)
    return out


def main():
    for path in sys.argv[1:]:
        lines = open(path).read().split("\n")
        print(path)
        for name, ins in blocks_of(lines, "_ZN3sct16k_welford_chainsILb1EEE"):
            ops = [x.split()[0] for x in ins]
            f64 = sum("_f64" in o for o in ops)
            if f64 < 4 * K_BATCH:  # not a batch body
                continue
            mix = {
                "all": len(ops),
                "valu": sum(o.startswith("v_") for o in ops),
                "f64": f64,
                "readlane": sum(o.startswith(("v_readlane", "v_readfirstlane")) for o in ops),
                "dpp": sum("row_newbcast" in x or "row_bcast" in x for x in ins),
                "salu": sum(o.startswith("s_") and not o.startswith(("s_waitcnt", "s_nop", "s_cbranch", "s_branch")) for o in ops),
                "waitcnt+nop": sum(o.startswith(("s_waitcnt", "s_nop")) for o in ops),
                "vmem": sum(o.startswith(("global_", "buffer_", "flat_")) for o in ops),
                "lds": sum(o.startswith("ds_") for o in ops),
            }
            per = {k: round(v / K_BATCH, 2) for k, v in mix.items()}
            print("  %-10s per record: %s" % (name, per))


if __name__ == "__main__":
    main()
