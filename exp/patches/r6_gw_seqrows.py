# Ablation (wrong results, timing only): k_group_wave reads the row at its own position instead of
# the sorted position's source row -- what the random row gather costs.
import sys
p = sys.argv[1] + "/tagsort.h"
s = open(p).read()
for old, new in (("    a = rows[2 * (int64_t)idx];\n    b = rows[2 * (int64_t)idx + 1];\n",
                  "    a = rows[2 * (int64_t)p + (idx & 0)];\n    b = rows[2 * (int64_t)p + 1];\n"),
                 ("    a2 = rows[2 * (int64_t)idx2];\n    b2 = rows[2 * (int64_t)idx2 + 1];\n",
                  "    a2 = rows[2 * (g0 + lane) + (idx2 & 0)];\n    b2 = rows[2 * (g0 + lane) + 1];\n")):
    assert old in s
    s = s.replace(old, new)
open(p, "w").write(s)
