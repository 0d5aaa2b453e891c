import sys
p = sys.argv[1] + "/gene.h"
s = open(p).read()
old = """    const double yq = rcp_of(g.qb, s_rcp);  // the two gq quotients share the reciprocal
    fx_accumulate(l + 1 * kStreamLanes, ratio_y(g.qa, g.qb, yq));
    fx_accumulate(l + 2 * kStreamLanes, ratio_y(g.qs, g.qb, yq));"""
assert old in s
s = s.replace(old, """    l[8] += g.qa; l[16] += g.qs; l[9] += g.qb;""")
open(p, "w").write(s)
