"""Which kernels differ between two device-assembly builds of the engine (experiments, PMC restamps).

hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off --cuda-device-only -S -o A.s sctools_amd/csrc/sct_engine.hip
python tools/isa_same.py A.s B.s    # prints the kernels whose instructions differ
"""
import re
import sys


def kernels(path):
    out, cur, buf = {}, None, []
    for line in open(path):
        m = re.match(r"^(_Z\w+):", line)
        if m:
            cur, buf = m.group(1), []
            continue
        if cur and line.startswith(".Lfunc_end"):
            out[cur] = "\n".join(buf)
            cur = None
            continue
        if cur and line.startswith("\t") and not line.strip().startswith(";"):
            buf.append(line.rstrip())
    return out


if __name__ == "__main__":
    a, b = kernels(sys.argv[1]), kernels(sys.argv[2])
    diff = sorted(k for k in set(a) | set(b) if a.get(k) != b.get(k))
    print("%d / %d kernels; differing: %s" % (len(a), len(b), diff))
