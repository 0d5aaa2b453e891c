# diagnostic: k_bucket_classify without the n_big_rec / n_rec counters (profiling items only)
import sys
p = sys.argv[1] + "/bucket.h"
s = open(p).read()
a = "    atomicAdd(&ctl->n_big_rec, c);\n"
b = "  if (push) atomicAdd(&ctl->n_rec, c);  // the new segments' records (a few per block)\n"
assert a in s and b in s
s = s.replace(a, "").replace(b, "")
open(p, "w").write(s)
