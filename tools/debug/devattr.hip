// Prints the LDS limits the runtime reports (round 5: sizing the Welford head launch's LDS reservation).
#include <hip/hip_runtime.h>
#include <cstdio>
int main() {
  int a = 0, b = 0, c = 0;
  (void)hipDeviceGetAttribute(&a, hipDeviceAttributeMaxSharedMemoryPerBlock, 0);
  (void)hipDeviceGetAttribute(&b, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, 0);
  (void)hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, 0);
  printf("lds per block %d per CU %d CUs %d\n", a, b, c);
  return 0;
}
