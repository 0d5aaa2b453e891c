import sys
p = sys.argv[1] + "/gene.h"
s = open(p).read()
old = """    for (int k = 0; k < my_n; k++) {
      const GeneItem g = F::item(s_sorted[F::slot(j0 + k)], g0);
      if ((int)g.lg != cur) {  // a gene boundary inside the thread's payloads: its own bin, no conflict
        if (cur >= 0) acc.flush<k8>(&s_cbin[cur * kGeneCntPad], &s_lbin[cur * 3 * kStreamLanes]);
        acc.clear();
        cur = (int)g.lg;
      }
      acc.add(g, s_rcp, s_uytab, uy_b);
    }"""
assert old in s
s = s.replace(old, """    for (int k = 0; k < my_n; k++) {
      const GeneItem g = F::item(s_sorted[F::slot(j0 + k)], g0);
      acc.n += g.lg ^ g.f ^ g.qs;
    }""")
s = s.replace("""  // the threads' open runs, combined across each wave
  gene_wave_flush<k8>(acc, cur, s_cbin, s_lbin);""", """  if (acc.n == 0x7fffffff) s_cbin[0] = 1;""")
open(p, "w").write(s)
