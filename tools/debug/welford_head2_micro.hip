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

// background load for the "in the pipeline" case (argv[3]): 1 = HBM copy passes, 2 = FP64 FMA chains
// on every SIMD, 0 = none
__global__ void k_hog_copy(const int4* __restrict__ src, int4* __restrict__ dst, size_t n, int passes) {
  for (int p = 0; p < passes; p++)
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
      int4 v = src[i];
      v.x += p;
      dst[i] = v;
    }
}
__global__ void k_hog_fp64(double* out, int iters) {
  double a = threadIdx.x * 1e-3, b = 1.0000001, c = 0.5;
  for (int i = 0; i < iters; i++) {
    a = __fma_rn(a, b, c);
    c = __fma_rn(c, b, a);
  }
  if (a == 12345.0) out[0] = a + c;
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 272000;
  const int threads = argc > 2 ? atoi(argv[2]) : kW2Waves * kWave;
  const int hog = argc > 3 ? atoi(argv[3]) : 0;
  const size_t hog_n = (size_t)1 << 26;  // 1 GiB of int4
  int4 *hs = nullptr, *hd = nullptr;
  if (hog == 1) {
    hipMalloc(&hs, hog_n * 16);
    hipMalloc(&hd, hog_n * 16);
    hipMemset(hs, 1, hog_n * 16);
  }
  hipStream_t s1;
  hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
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
      if (hog == 1) hipLaunchKernelGGL(k_hog_copy, dim3(4096), dim3(256), 0, s1, (const int4*)hs, hd, hog_n, 40);
      if (hog == 2) hipLaunchKernelGGL(k_hog_fp64, dim3(2048), dim3(256), 0, s1, (double*)hd, 400000);
      hipEventRecord(a);
      if (which == 0)
        hipLaunchKernelGGL(k_welford_chains<true>, dim3(kWfBlocks), dim3(kBlock), 0, 0, (const int64_t*)es, (int64_t)1,
                           n, (const uint32_t*)ord, ctl, (const double*)xs, out);
      else
        hipLaunchKernelGGL(k_welford_head2<true>, dim3(1), dim3(threads), 0, 0, (const int64_t*)es, (int64_t)1, n,
                           (const uint32_t*)ord, ctl, (const double*)xs, out);
      hipEventRecord(b);
      hipEventSynchronize(b);
      hipDeviceSynchronize();
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
      unsigned long long pr[10];
      hipMemcpyFromSymbol(pr, HIP_SYMBOL(sct_w2_prof), sizeof(pr));
      for (int w = 0; w < 4; w++)
        printf("  wave %d: %llu ticks in barriers of %llu (wall clock ticks, 100 MHz)\n", w, pr[2 * w], pr[2 * w + 1]);
      printf("  shader clock: %.0f MHz\n", pr[1] ? 100.0 * (double)pr[8] / (double)pr[1] : 0.0);
    }
#endif
    printf("%s n %lld  best %.3f ms  %.2f ns/record  result %016llx\n", which ? "head2 " : "chains", (long long)n,
           best, best * 1e6 / n, hash[which]);
  }
  printf(hash[0] == hash[1] ? "bits agree\n" : "BITS DIFFER\n");
  return 0;
}
