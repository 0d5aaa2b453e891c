# Ablation (wrong results, timing only): the gene emit does not write bucket 0's payloads (the Zipf
# head) -- the HBM write cost a fused head-bucket reduction would save in the emit.
import sys
p = sys.argv[1] + "/gene.h"
s = open(p).read()
old = "      pay[(uint64_t)s_off[b] + (uint32_t)(q - (int)s_loc[b])] = s_pay[q];\n"
assert old in s
s = s.replace(old, "      if (b != 0) pay[(uint64_t)s_off[b] + (uint32_t)(q - (int)s_loc[b])] = s_pay[q];  // ABLATION\n")
open(p, "w").write(s)
