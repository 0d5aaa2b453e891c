// Microbenchmark (experiments only): k_welford_chains (one wave) against k_welford_head2 (finalize.h,
// three waves) on ONE entity of n records, ns per record, and whether their result bits agree.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include -I sctools_amd/csrc -o w2 tools/debug/welford_head2_micro.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include "finalize.h"

using namespace sct;

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 272000;
  const int threads = argc > 2 ? atoi(argv[2]) : kW2Waves * kWave;
  std::vector<double> hx(4 * (size_t)(n + kWfPad));
  unsigned long long s = 88172645463325252ull;
  for (auto& v : hx) {
    s ^= s << 13, s ^= s >> 7, s ^= s << 17;
    v = (double)(s % 99) / 98.0;
  }
  double *xs, *out;
  int64_t* es;
  uint32_t* ord;
  WelfordCtl* ctl;
  hipMalloc(&xs, hx.size() * 8);
  hipMalloc(&out, SCT_NF * 8);
  hipMalloc(&es, 8);
  hipMalloc(&ord, 4);
  hipMalloc(&ctl, sizeof(WelfordCtl));
  hipMemcpy(xs, hx.data(), hx.size() * 8, hipMemcpyHostToDevice);
  int64_t zero = 0;
  uint32_t z32 = 0;
  hipMemcpy(es, &zero, 8, hipMemcpyHostToDevice);
  hipMemcpy(ord, &z32, 4, hipMemcpyHostToDevice);
  WelfordCtl hc;
  memset(&hc, 0, sizeof(hc));
  hc.n_big = 1;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  unsigned long long hash[2] = {0, 0};
  for (int which = 0; which < 2; which++) {
    float best = 1e30f;
    for (int rep = 0; rep < 5; rep++) {
      hipMemcpy(ctl, &hc, sizeof(hc), hipMemcpyHostToDevice);
      hipMemset(out, 0, SCT_NF * 8);
      hipEventRecord(a);
      if (which == 0)
        hipLaunchKernelGGL(k_welford_chains<true>, dim3(kWfBlocks), dim3(kBlock), 0, 0, (const int64_t*)es, (int64_t)1,
                           n, (const uint32_t*)ord, ctl, (const double*)xs, out);
      else
        hipLaunchKernelGGL(k_welford_head2<true>, dim3(1), dim3(threads), 0, 0, (const int64_t*)es, (int64_t)1, n,
                           (const uint32_t*)ord, (const WelfordCtl*)ctl, (const double*)xs, out);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      if (ms < best) best = ms;
    }
    double ho[SCT_NF];
    hipMemcpy(ho, out, sizeof(ho), hipMemcpyDeviceToHost);
    for (int i = 0; i < 6; i++) {  // the mean / variance slots of the UY and genomic streams
      unsigned long long u;
      memcpy(&u, &ho[i], 8);
      hash[which] = hash[which] * 1000003ull ^ u;
    }
#ifdef SCT_W2_PROF
    if (which) {
      unsigned long long pr[8];
      hipMemcpyFromSymbol(pr, HIP_SYMBOL(sct_w2_prof), sizeof(pr));
      for (int w = 0; w < 3; w++)
        printf("  wave %d: %llu ticks in barriers of %llu (wall clock ticks, 100 MHz)\n", w, pr[2 * w], pr[2 * w + 1]);
    }
#endif
    printf("%s n %lld  best %.3f ms  %.2f ns/record  result %016llx\n", which ? "head2 " : "chains", (long long)n,
           best, best * 1e6 / n, hash[which]);
  }
  printf(hash[0] == hash[1] ? "bits agree\n" : "BITS DIFFER\n");
  return 0;
}
