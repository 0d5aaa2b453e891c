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

constexpr uint32_t kUnmappedValBit = 0x80000000u;  // sort value bit 31: the record is unmapped

struct Bits {  // key layout: [entity | k1' | k2 | hash], k1' = k1 * mul mod 2^k1 (a bijection)
  int e, k1, k2, h;
  uint32_t mul = 1, inv = 1;  // odd multiplier and its inverse mod 2^k1 (1, 1: identity)
  int total() const { return e + k1 + k2 + h; }
  __host__ __device__ uint32_t k1_mask() const { return k1 ? (uint32_t)((1ull << k1) - 1) : 0u; }
  __host__ __device__ uint32_t scramble(uint32_t k) const { return (k * mul) & k1_mask(); }
  __host__ __device__ uint32_t unscramble(uint32_t k) const { return (k * inv) & k1_mask(); }
};

}  // namespace sct

namespace sct {

// ---- gene view: one 16-byte contribution per record, emitted by the cell-view pass ----
// Everything GatherGeneMetrics derives per record, with the distinct-count events of the
// (gene, cell, umi) Counters already resolved in the cell-sorted order (molecules,
// fragments and (cell, gene) pairs are the same sets in both views).
enum : uint32_t {
  GF_PERFECT_UMI = 1u << 0,
  GF_EXONIC = 1u << 1,
  GF_INTRONIC = 1u << 2,
  GF_UTR = 1u << 3,
  GF_UNIQUE = 1u << 4,
  GF_MULTIPLE = 1u << 5,
  GF_DUP = 1u << 6,
  GF_SPLICED = 1u << 7,
  GF_MOL_HEAD = 1u << 8,
  GF_MOL_SINGLE = 1u << 9,
  GF_FRAG_FIRST = 1u << 10,
  GF_FRAG_SINGLE = 1u << 11,
  GF_CG_HEAD = 1u << 12,   // first record of a (cell, gene) pair -> number_cells_expressing
  GF_CG_MULTI = 1u << 13,  // ... of a pair with > 1 record -> number_cells_detected_multiple
  GF_MOL_SECOND = 1u << 14,   // -1 on molecules_with_single_read_evidence (reduce.h DF_MOL_SECOND)
  GF_FRAG_SECOND = 1u << 15,  // -1 on fragments_with_single_read_evidence
};
constexpr int kGeneFlags = 14;  // lanes: the two SECOND bits subtract from the SINGLE lanes

struct __attribute__((aligned(16))) GenePayload {
  uint32_t gene;
  uint16_t flags;
  uint8_t uy_gt30, uy_len;
  uint16_t gq_gt30, gq_len, gq_sum, pad;
};
static_assert(sizeof(GenePayload) == 16, "gene payload must be 16 bytes");

#ifndef SCT_GENES_PER_BUCKET
#define SCT_GENES_PER_BUCKET 64
#endif
constexpr int kGenesPerBucket = SCT_GENES_PER_BUCKET;  // LDS bins of one gene bucket
constexpr int kMaxGeneBuckets = 4096;  // n_gene_ids <= 262144 (gene-bucket arrays in dynamic LDS, <= 64 KB a block)

}  // namespace sct
