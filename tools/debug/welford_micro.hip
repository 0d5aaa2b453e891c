// Microbenchmark (experiments only): the engine's own k_welford_chains (finalize.h) on ONE entity of
// n records (one wave, the 4 stream chains of that entity), ns per record, and the same build's
// result bits (to compare variants).  Build variants with -D (SCT_WF_PAIRS, ...):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include -I sctools_amd/csrc -o wm tools/debug/welford_micro.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include "finalize.h"

using namespace sct;

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 272000;
  std::vector<double> hx(4 * (size_t)(n + kWfPad));
  unsigned long long s = 88172645463325252ull;
  for (auto& v : hx) {
    s ^= s << 13, s ^= s >> 7, s ^= s << 17;
    v = (double)(s % 99) / 98.0;  // RN(a / 98)-like values
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
  float best = 1e30f;
  for (int rep = 0; rep < 5; rep++) {
    hipMemcpy(ctl, &hc, sizeof(hc), hipMemcpyHostToDevice);
    hipEventRecord(a);
    hipLaunchKernelGGL(k_welford_chains<true>, dim3(kWfBlocks), dim3(kBlock), 0, 0, (const int64_t*)es, (int64_t)1, n,
                       (const uint32_t*)ord, ctl, (const double*)xs, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    if (ms < best) best = ms;
  }
  double ho[SCT_NF];
  hipMemcpy(ho, out, sizeof(ho), hipMemcpyDeviceToHost);
  unsigned long long h = 0;
  for (int i = 0; i < SCT_NF; i++) {
    unsigned long long u;
    memcpy(&u, &ho[i], 8);
    h = h * 1000003ull ^ u;
  }
  printf("n %lld  best %.3f ms  %.2f ns/record  result %016llx\n", (long long)n, best, best * 1e6 / n, h);
  return 0;
}
