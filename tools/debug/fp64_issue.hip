// Microbenchmark (experiments only): one wave, n records, ns per record of FP64 dependency chains
// shaped like the Welford update (finalize.h), to separate latency from issue cost on gfx950.
//   k_dep4  : sub -> mul -> fma -> add, constants in SGPRs (the latency floor)
//   k_dep4v : the same with the two reciprocal words in VGPRs (per lane)
//   k_dep4x : k_dep4 plus the M2 update (sub, mul, add) beside it
//   k_full  : the Welford update as k_welford_chains issues it (VGPR pairs, x from a register ring)
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o fp64_issue tools/debug/fp64_issue.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void k_dep4(double* out, double a, long n) {
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
__global__ void k_dep4v(double* out, double a, long n) {
  double m = a + threadIdx.x;
  const double h = 1e-7 * (1 + threadIdx.x), l = 1e-9 * (1 + threadIdx.x);
  for (long i = 0; i < n; i += 16) {
#pragma unroll
    for (int u = 0; u < 16; u++) {
      const double d = a - m;
      m = m + __fma_rn(d, h, d * l);
    }
  }
  out[threadIdx.x] = m;
}
__global__ void k_dep4x(double* out, double a, long n) {
  double m = a + threadIdx.x, m2 = 0.0;
  const double h = 1e-7 * (1 + threadIdx.x), l = 1e-9 * (1 + threadIdx.x);
  for (long i = 0; i < n; i += 16) {
#pragma unroll
    for (int u = 0; u < 16; u++) {
      const double d = a - m;
      m = m + __fma_rn(d, h, d * l);
      const double d2 = a - m;
      m2 = m2 + d * d2;
    }
  }
  out[threadIdx.x] = m + m2;
}
__global__ void k_full(double* out, double a, long n) {
  double m = a + threadIdx.x, m2 = 0.0;
  double x[16];
#pragma unroll
  for (int u = 0; u < 16; u++) x[u] = a * (u + 1) * 0.01;
  for (long i = 0; i < n; i += 16) {
    const double kq = (double)(i + (threadIdx.x & 15) + 1);
    const double h = 1.0 / kq;
    const double l = __fma_rn(-kq, h, 1.0) * h;
#pragma unroll
    for (int u = 0; u < 16; u++) {
      const double d = x[u] - m;
      m = m + __fma_rn(d, h, d * l);
      const double d2 = x[u] - m;
      m2 = m2 + d * d2;
    }
#pragma unroll
    for (int u = 0; u < 16; u++) x[u] = x[u] * 0.999;
  }
  out[threadIdx.x] = m + m2;
}

int main() {
  const long n = 1 << 20;
  double* out;
  hipMalloc(&out, 64 * sizeof(double));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[4] = {"dep4", "dep4v", "dep4x", "full"};
  for (int k = 0; k < 4; k++) {
    float best = 1e30f;
    for (int r = 0; r < 3; r++) {
      hipEventRecord(e0);
      if (k == 0) hipLaunchKernelGGL(k_dep4, dim3(1), dim3(64), 0, 0, out, 0.5, n);
      if (k == 1) hipLaunchKernelGGL(k_dep4v, dim3(1), dim3(64), 0, 0, out, 0.5, n);
      if (k == 2) hipLaunchKernelGGL(k_dep4x, dim3(1), dim3(64), 0, 0, out, 0.5, n);
      if (k == 3) hipLaunchKernelGGL(k_full, dim3(1), dim3(64), 0, 0, out, 0.5, n);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    printf("%-6s %.2f ns/record\n", names[k], best * 1e6 / n);
  }
  return 0;
}
