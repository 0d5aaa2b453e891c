import sys
p = sys.argv[1] + "/segment.h"
s = open(p).read()
old = "          reinterpret_cast<Pay*>(keys)[p] = x;  // (the bucket path's keys are payload buffer A)"
assert old in s
s = s.replace(old, "          if (x.w0 == 0x123456789abcdefull) reinterpret_cast<Pay*>(keys)[p] = x;")
open(p, "w").write(s)
