import sys
p = sys.argv[1] + "/gene.h"
s = open(p).read()
old = "        if (cur >= 0) acc.flush<k8>(&s_cbin[cur * kGeneCntPad], &s_lbin[cur * 3 * kStreamLanes]);"
assert old in s
s = s.replace(old, "        if (cur == -7) acc.flush<k8>(&s_cbin[cur * kGeneCntPad], &s_lbin[cur * 3 * kStreamLanes]);  // (ablation)")
open(p, "w").write(s)
