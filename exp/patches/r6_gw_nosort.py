# Ablation (wrong results, timing only): k_group_wave skips the in-wave bitonic network.
import sys
p = sys.argv[1] + "/tagsort.h"
s = open(p).read()
old = "  if (__ballot(need)) {\n    // (group start lane | W | lane)"
assert old in s
s = s.replace(old, "  if (__ballot(need) && gb.c > 99) {\n    // (group start lane | W | lane)")
open(p, "w").write(s)
