// common.h -- shared definitions of the gfx950 metric engine.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/sctools_gpu.h"

namespace sct {

constexpr int kWave = 64;  // CDNA wavefront

// ---- partial-row layout (int64 [rows][SCT_NP]) ----
enum : int {
  P_N_READS = 0,
  P_PERFECT_UMI,
  P_EXONIC,
  P_INTRONIC,
  P_UTR,
  P_UNIQUE,
  P_MULTIPLE,
  P_DUP,
  P_SPLICED,
  P_N_MOL,
  P_MOL_SINGLE,
  P_N_FRAG,
  P_FRAG_SINGLE,
  P_N_K1,
  P_K1_MULTI,
  P_PERFECT_CB,
  P_INTERGENIC,
  P_UNMAPPED,
  P_MITO_K1,
  P_MITO_READS,
  P_NCOUNT,  // number of additive counters (20)
  P_FIRST = 20,  // RUN modes: index of the entity's first record (stored, not summed)
};
constexpr int P_FLOAT = SCT_P_FLOAT_BASE;  // 24: stream s lanes at P_FLOAT + 8*s
constexpr int kStreams = 4;                // UY frac, genomic frac, genomic mean quality, CY frac
static_assert(SCT_P_FLOAT_BASE + kStreams * 8 <= SCT_NP, "partials row too small");

struct Bits {  // key layout: [entity | k1 | k2 | hash]
  int e, k1, k2, h;
  int total() const { return e + k1 + k2 + h; }
};

}  // namespace sct
