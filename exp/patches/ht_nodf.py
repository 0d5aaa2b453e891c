import sys
p = sys.argv[1] + "/bucket.h"
s = open(p).read()
old = "      dflags[x1 >> 32] = f;"
assert old in s
s = s.replace(old, "      if (f == 0xffff) dflags[x1 >> 32] = f;", 1)
open(p, "w").write(s)
