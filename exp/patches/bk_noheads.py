import sys
p = sys.argv[1] + "/segment.h"
s = open(p).read()
old = "    if (SCT_KEY_FASTPATH && tile_n == kKTile) {  // block-uniform"
assert old in s
s = s.replace(old, "    if (SCT_KEY_FASTPATH) {  // (ablation: every batch one run)")
s = s.replace("      one_run = elo == ehi;", "      one_run = true;")
open(p, "w").write(s)
