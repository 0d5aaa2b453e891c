# hash tile 2-window pipeline without the 8-waves-per-SIMD launch bound (no spills, 3 blocks per CU)
import sys
p = sys.argv[1] + "/bucket.h"
s = open(p).read()
s = s.replace("__launch_bounds__(kHBlock, 8) k_hash_tile2(", "__launch_bounds__(kHBlock) k_hash_tile2(")
open(p, "w").write(s)
