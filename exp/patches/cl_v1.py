import sys
p = sys.argv[1] + "/bucket.h"
s = open(p).read()
a = s.index("  // big buckets (a few per segment: the hot genes of a cell) reserved once per wave")
b = s.index("  const uint32_t nw = push ? (c + kChunk - 1) / kChunk : 0u;")
s = s[:a] + """  if (big) {
    bigs[atomicAdd(&ctl->n_big, 1u)] = Seg{start, c, sg.ent, fl | par};
    atomicAdd(&ctl->n_big_rec, c);
  }
""" + s[b:]
open(p, "w").write(s)
