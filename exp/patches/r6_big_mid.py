# Experiment: big buckets of <= 1535 records on 512-thread blocks with 2048-slot tables (40 KB of LDS,
# 4 blocks per CU), the larger ones as before (1024 threads, 4096 slots, 80 KB); two launches over the
# one list, each block leaving the other class's buckets.
import sys
d = sys.argv[1]
p = d + "/bucket.h"
s = open(p).read()
a = s.index("template <bool kCell, bool kGene, bool kWideK1>\n__global__ void __launch_bounds__(kBigBlock) k_big_bucket(")
b = s.index("// A bucket whose whole key' is fixed and still holds > kBCap records")
k = s[a:b]
k = k.replace("template <bool kCell, bool kGene, bool kWideK1>\n__global__ void __launch_bounds__(kBigBlock) k_big_bucket(",
              "template <bool kCell, bool kGene, bool kWideK1, int kBlk, int kSlotsMax, int kClass>\n__global__ void __launch_bounds__(kBlk) k_big_bucket(")
k = k.replace("kBigSlots", "kSlotsMax").replace("kBigBlock", "kBlk")
old = "  const Seg g = bigs[blockIdx.x];\n"
assert old in k
k = k.replace(old, old + "  if (kClass == 1 && g.cnt > 3u * kSlotsMax / 4u - 1u) return;  // block-uniform\n"
                         "  if (kClass == 2 && g.cnt <= 1535u) return;\n")
s = s[:a] + k + s[b:]
open(p, "w").write(s)
p = d + "/sct_engine.hip"
s = open(p).read()
old = '''  LAUNCH("big_bucket", (k_big_bucket<C, G, W>), bgrid, dim3(kBigBlock), st, bg, pa, pb, b, partials, dflags)'''
assert old in s
s = s.replace(old, '''  LAUNCH("big_bucket", (k_big_bucket<C, G, W, 512, 2048, 1>), bgrid, dim3(512), st, bg, pa, pb, b, partials, dflags); \\
  LAUNCH("big_bucket", (k_big_bucket<C, G, W, kBigBlock, kBigSlots, 2>), bgrid, dim3(kBigBlock), st, bg, pa, pb, b, partials, dflags)''')
open(p, "w").write(s)
