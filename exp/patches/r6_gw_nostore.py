# Ablation (wrong results, timing only): the group sort's gather-and-write stores only the cell and
# umi columns -- what the 14 narrow SoA column stores cost k_group_wave.
import sys
p = sys.argv[1] + "/tagsort.h"
s = open(p).read()
old = "  const_cast<int32_t*>(out.gene)[j] = (int32_t)a.z;\n"
i = s.index(old)
e = s.index("}\n", i)
s = s[:i] + "  if (a.z == 0xdeadbeefu && b.x == 0xdeadbeefu) const_cast<int32_t*>(out.gene)[j] = (int32_t)(b.y ^ b.z ^ b.w ^ a.w);  // ABLATION\n" + s[e:]
open(p, "w").write(s)
