# Candidate: the key pass's tiles mapped XCD by XCD (xcd_tile), so that consecutive tiles -- the two or
# three tiles of one cell, whose ranges in each level-1 child are adjacent -- share an L2 and merge the
# partial lines at their range boundaries there.
import sys
p = sys.argv[1] + "/segment.h"
s = open(p).read()
i = s.index("k_build_keys_run(KeyCols c, RecCols r")
j = s.index("}  // namespace sct", i)
body = s[i:j]
old = "  const int64_t base = (int64_t)blockIdx.x * kKTile;\n"
assert body.count(old) == 1
body = body.replace(old, "  const unsigned tile = xcd_tile(blockIdx.x, gridDim.x);\n  const int64_t base = (int64_t)tile * kKTile;\n")
for a, b in (("tile_off[(size_t)blockIdx.x * kKTilesPerBlock]", "tile_off[(size_t)tile * kKTilesPerBlock]"),
             ("l1.tslot[blockIdx.x]", "l1.tslot[tile]"),
             ("l1.toff[((size_t)blockIdx.x * kL1Slots + k)", "l1.toff[((size_t)tile * kL1Slots + k)"),
             ("gtoff[(size_t)blockIdx.x * n_buckets + i]", "gtoff[(size_t)tile * n_buckets + i]")):
    assert body.count(a) == 1, a
    body = body.replace(a, b)
assert "blockIdx" not in body.replace("xcd_tile(blockIdx.x, gridDim.x)", "")
s = s[:i] + body + s[j:]
open(p, "w").write(s)
