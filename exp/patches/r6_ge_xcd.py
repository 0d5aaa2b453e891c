# Candidate: the gene emit's tiles mapped XCD by XCD (xcd_tile): consecutive tiles' ranges in a gene
# bucket (reserved in tile order by the key pass) are written from one L2.
import sys
p = sys.argv[1] + "/gene.h"
s = open(p).read()
old = "  const int64_t base = (int64_t)blockIdx.x * kEmitTile;\n  const uint32_t* toff = gtoff + (size_t)blockIdx.x * n_buckets;\n"
assert s.count(old) == 1
s = s.replace(old, "  const unsigned tile = xcd_tile(blockIdx.x, gridDim.x);\n  const int64_t base = (int64_t)tile * kEmitTile;\n  const uint32_t* toff = gtoff + (size_t)tile * n_buckets;\n")
open(p, "w").write(s)
