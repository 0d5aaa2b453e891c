// Microbenchmark (experiments only): cycles per dependent FP64 / FP32 operation on one wave, and
// with 2 / 4 independent chains interleaved -- the floor of the sequential Welford update.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o fp64_chain fp64_chain.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int kChains, typename T>
__global__ void chain(T* out, T a, T b, int iters, long long* cyc) {
  T x[kChains];
  for (int c = 0; c < kChains; c++) x[c] = a + (T)(threadIdx.x + c);
  const long long t0 = clock64();
  for (int i = 0; i < iters; i += 16) {  // 16 dependent steps per loop iteration: the loop overhead amortized
#pragma unroll
    for (int u = 0; u < 16; u++) {
#pragma unroll
      for (int c = 0; c < kChains; c++) x[c] = __fma_rn(x[c], a, b);
    }
  }
  const long long t1 = clock64();
  T s = 0;
  for (int c = 0; c < kChains; c++) s += x[c];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

template <int kChains, typename T>
void run(const char* name) {
  T* out;
  long long* cyc;
  hipMalloc(&out, 64 * sizeof(T));
  hipMalloc(&cyc, sizeof(long long));
  const int iters = 1 << 20;
  hipLaunchKernelGGL((chain<kChains, T>), dim3(1), dim3(64), 0, 0, out, (T)0.999999, (T)1e-7, iters, cyc);
  hipLaunchKernelGGL((chain<kChains, T>), dim3(1), dim3(64), 0, 0, out, (T)0.999999, (T)1e-7, iters, cyc);
  long long h = 0;
  hipMemcpy(&h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  printf("%s chains=%d: %.2f cycles per dependent fma (%.2f per fma issued)\n", name, kChains,
         (double)h / iters, (double)h / iters / kChains);
  hipFree(out);
  hipFree(cyc);
}

int main() {
  run<1, double>("f64");
  run<2, double>("f64");
  run<4, double>("f64");
  run<8, double>("f64");
  run<1, float>("f32");
  run<4, float>("f32");
  return 0;
}
