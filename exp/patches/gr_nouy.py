import sys
p = sys.argv[1] + "/gene.h"
s = open(p).read()
old = """    if (g.ub == uy_b && g.ua <= uy_b) {
      const uint4 i0 = uy_tab[2 * g.ua], i1 = uy_tab[2 * g.ua + 1];
      l[0] += i0.x, l[1] += i0.y, l[2] += i0.z, l[3] += i0.w;
      l[4] += i1.x, l[5] += i1.y, l[6] += i1.z, l[7] += i1.w;
    } else {
      fx_accumulate(l + 0 * kStreamLanes, ratio_rcp(g.ua, g.ub, s_rcp));
    }
    const double yq = rcp_of(g.qb, s_rcp);  // the two gq quotients share the reciprocal
    fx_accumulate(l + 1 * kStreamLanes, ratio_y(g.qa, g.qb, yq));
    fx_accumulate(l + 2 * kStreamLanes, ratio_y(g.qs, g.qb, yq));"""
assert old in s
s = s.replace(old, """    l[0] += g.ua; l[1] += g.ub; l[8] += g.qa; l[16] += g.qs; l[9] += g.qb;""")
open(p, "w").write(s)
