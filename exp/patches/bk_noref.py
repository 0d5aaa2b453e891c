import sys
p = sys.argv[1] + "/segment.h"
s = open(p).read()
old = """      vref[u] = r.ref[p];
      vpos[u] = r.pos[p];"""
assert old in s
s = s.replace(old, """      vref[u] = vk2[u] & 1023;  // (ablation: no ref / pos loads)
      vpos[u] = vk1[u] ^ vk2[u];""")
open(p, "w").write(s)
