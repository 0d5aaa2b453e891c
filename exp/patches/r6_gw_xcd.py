# Candidate: k_group_wave's blocks mapped to positions XCD by XCD (xcd_tile), so that each XCD's L2
# serves the row gathers of one contiguous range of sorted positions.
import sys
p = sys.argv[1] + "/tagsort.h"
s = open(p).read()
i = s.index("k_group_wave(const uint32_t*")
old = "  const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;\n"
j = s.index(old, i)
s = s[:j] + "  const int64_t p = (int64_t)xcd_tile(blockIdx.x, gridDim.x) * kBlock + threadIdx.x;\n" + s[j + len(old):]
open(p, "w").write(s)
