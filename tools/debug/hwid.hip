// Which SIMD each wave of a workgroup lands on (HW_REG_HW_ID: wave id 3:0, SIMD 5:4, CU 11:8).
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k_hwid(unsigned* out) {
  const unsigned v = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_ID, offset 0, 32 bits
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 16 + threadIdx.x / 64] = v;
}
int main() {
  unsigned* d;
  hipMalloc(&d, 4096 * 4);
  for (int threads : {128, 192, 256}) {
    hipMemset(d, 0, 4096 * 4);
    hipLaunchKernelGGL(k_hwid, dim3(8), dim3(threads), 0, 0, d);
    unsigned h[8 * 16];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("block of %d threads:\n", threads);
    for (int b = 0; b < 4; b++) {
      printf("  block %d:", b);
      for (int w = 0; w < threads / 64; w++) {
        const unsigned v = h[b * 16 + w];
        printf(" [wave %d: simd %u cu %u wid %u]", w, (v >> 4) & 3, (v >> 8) & 15, v & 15);
      }
      printf("\n");
    }
  }
  return 0;
}
