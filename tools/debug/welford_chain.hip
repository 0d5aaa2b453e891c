// Microbenchmark (experiments only): wall-clock ns per record of one wave running the Welford
// update chain (finalize.h k_welford_chains) over n records, timed with HIP events.
//   dep4   : 4 dependent FP64 ops per record, operands in registers (the latency floor)
//   chain  : the update with y = RN(1/k) pairs broadcast by readlane, samples from HBM
//   chainc : the same with the samples computed in registers (no memory at all)
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o welford_chain welford_chain.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

__device__ __forceinline__ double rl(double v, int l) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), l);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

__global__ void dep4(double* out, double a, long n) {
  double m = a + threadIdx.x;
  for (long i = 0; i < n; i += 16) {
#pragma unroll
    for (int u = 0; u < 16; u++) {
      const double d = a - m;
      m = m + __fma_rn(d, 1e-7, d * 1e-9);
    }
  }
  out[threadIdx.x] = m;
}

template <bool kMem>
__global__ void chain(const double* __restrict__ x, double* out, long n) {
  const int lane = threadIdx.x & 63;
  double mean = 0.0, m2 = 0.0;
  double xb[32], xn[32];
  const double* X = x + (long)lane * n;
#pragma unroll
  for (int q = 0; q < 32; q++) xb[q] = kMem ? X[q] : 0.25 + q * 1e-3;
  for (long c0 = 0; c0 < n; c0 += 64) {
    const double kd = (double)(c0 + lane + 1);
    const double yh = 1.0 / kd;
    const double yl = __fma_rn(-kd, yh, 1.0) * yh;
#pragma unroll
    for (int hb = 0; hb < 2; hb++) {
      const long c = c0 + hb * 32;
#pragma unroll
      for (int q = 0; q < 32; q++) {
        const long kq = c + 32 + q;
        xn[q] = kMem ? X[kq < n ? kq : n - 1] : xb[q] * 0.999;
      }
#pragma unroll
      for (int q = 0; q < 32; q++) {
        const double delta = xb[q] - mean;
        mean = mean + __fma_rn(delta, rl(yh, hb * 32 + q), delta * rl(yl, hb * 32 + q));
        const double delta2 = xb[q] - mean;
        m2 = m2 + delta * delta2;
      }
#pragma unroll
      for (int q = 0; q < 32; q++) xb[q] = xn[q];
    }
  }
  out[threadIdx.x] = mean + m2;
}

int main() {
  const long n = 1 << 18;  // ~ the longest cell at config 2 (272k records)
  double *x, *out;
  hipMalloc(&x, 64 * n * sizeof(double));
  hipMalloc(&out, 64 * sizeof(double));
  hipMemset(x, 0, 64 * n * sizeof(double));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float ms = 0;
  for (int rep = 0; rep < 2; rep++) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(dep4, dim3(1), dim3(64), 0, 0, out, 0.5, n);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("dep4   %.2f ns/record (%.3f ms)\n", ms * 1e6 / n, ms);
    hipEventRecord(e0);
    hipLaunchKernelGGL(chain<true>, dim3(1), dim3(64), 0, 0, x, out, n);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("chain  %.2f ns/record (%.3f ms)\n", ms * 1e6 / n, ms);
    hipEventRecord(e0);
    hipLaunchKernelGGL(chain<false>, dim3(1), dim3(64), 0, 0, x, out, n);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("chainc %.2f ns/record (%.3f ms)\n", ms * 1e6 / n, ms);
  }
  return 0;
}
