import sys
p = sys.argv[1] + "/finalize.h"
s = open(p).read()
old = "constexpr int kWfBatch = 32;"
assert old in s
s = s.replace(old, "constexpr int kWfBatch = 16;")
open(p, "w").write(s)
