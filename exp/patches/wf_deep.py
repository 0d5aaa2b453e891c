import sys
p = sys.argv[1] + "/finalize.h"
s = open(p).read()
def rep(a, b):
    global s
    assert a in s, a
    s = s.replace(a, b, 1)
rep("constexpr int kWfBatch = 32;", "constexpr int kWfBatch = 16;\nconstexpr int kWfBufs = 4;  // batches in flight: loads issued kWfBufs - 1 batches ahead")
rep("    double xq[2][kWfBatch];", "    double xq[kWfBufs][kWfBatch];")
rep("""    for (int q = 0; q < kWfBatch; q++) xq[0][q] = X[4 * (q < lastx ? q : lastx)];""",
    """    for (int bb = 0; bb < kWfBufs - 1; bb++)
#pragma unroll
      for (int q = 0; q < kWfBatch; q++) {
        const int64_t kq = bb * kWfBatch + q;
        xq[bb][q] = X[4 * (kq < lastx ? kq : lastx)];
      }""")
rep("          const int64_t nb = c + kWfBatch;", "          const int64_t nb = c + (kWfBufs - 1) * kWfBatch;")
rep("            for (int q = 0; q < kWfBatch; q++) xq[hb ^ 1][q] = B[4 * q];", "            for (int q = 0; q < kWfBatch; q++) xq[(hb + kWfBufs - 1) % kWfBufs][q] = B[4 * q];")
rep("              xq[hb ^ 1][q] = X[4 * (kq < lastx ? kq : lastx)];", "              xq[(hb + kWfBufs - 1) % kWfBufs][q] = X[4 * (kq < lastx ? kq : lastx)];")
rep("          const double x = xq[hb][q];", "          const double x = xq[hb % kWfBufs][q];")
open(p, "w").write(s)
