// Host build of sctools_amd/csrc/fixedpt.h for tests/test_fixedpt.py (the
// same header the HIP kernels use on the device).
#include <stdint.h>

#include "../../sctools_amd/csrc/fixedpt.h"

extern "C" int fx_stats(const double* x, int64_t n, double* mean, double* var, int64_t* lanes_out) {
  int64_t lanes[sct::kStreamLanes] = {0};
  for (int64_t i = 0; i < n; i++) sct::fx_accumulate(lanes, x[i]);
  sct::fx_finalize(lanes, n, mean, var);
  if (lanes_out)
    for (int i = 0; i < sct::kStreamLanes; i++) lanes_out[i] = lanes[i];
  return 0;
}

extern "C" int fx_finalize_lanes(const int64_t* lanes, int64_t n, double* mean, double* var) {
  sct::fx_finalize(lanes, n, mean, var);
  return 0;
}
