import sys
p = sys.argv[1] + "/segment.h"
s = open(p).read()
old = """      vbt[u] = r.bits[p];
      vxf[u] = r.xf[p];"""
assert old in s
s = s.replace(old, """      vbt[u] = (uint8_t)(0x10 | (vk1[u] & 0x20));  // (ablation: no byte-column loads)
      vxf[u] = 1;""")
open(p, "w").write(s)
