// reduce.h -- the sorted-order pass: the reference's Counter results from key runs.
//
// Keys are [entity | k1 | k2 | fragment hash] (segment.h).  In sorted order
//   [entity|k1|k2] runs are the molecules (_molecule_histogram, aggregator.py:264),
//   [entity|k1] runs are the genes of a cell (_genes_histogram, 530) or the cells of a
//   gene (_cells_histogram, 595),
// and the records of one fragment (ref, pos, strand; _fragment_histogram, 300-303)
// share the hash bits, so they sit in one equal-key sub-run of their molecule.  A
// mapped record alone in its sub-run is a new single-read fragment with no memory
// access beyond the sorted (key, value) pair; only records with an equal neighbour
// gather (ref, pos, strand) to resolve first occurrences exactly.
//
// The kernel adds the distinct counts to the entity partial rows and, for the gene
// view, stores the per-record distinct-count events as 16-bit flags by record index.
#pragma once
#include "fixedpt.h"
#include "util.h"

namespace sct {

constexpr int kReduceItems = 8;
constexpr int kReduceTile = kBlock * kReduceItems;  // 2048 sorted positions per block

struct RecCols {
  const int32_t* ref;
  const int32_t* pos;
  const uint16_t* gq_sum;
  const uint16_t* gq_len;
  const uint16_t* gq_gt30;
  const uint8_t* bits;
  const uint8_t* xf;
  const uint8_t* cy_gt30;
  const uint8_t* cy_len;
  const uint8_t* uy_gt30;
  const uint8_t* uy_len;
};

// distinct-count events per record (gene view flags).  The single-read counts are sums of
// +1 (SINGLE) and -1 (SECOND) events: the sorted pass sets SINGLE on the head of a one-record
// group; the hash tiles (bucket.h) set SINGLE on every head and SECOND on the record that
// first finds its group already present.
enum : uint16_t {
  DF_MOL_HEAD = 1u << 0,
  DF_MOL_SINGLE = 1u << 1,
  DF_FRAG_FIRST = 1u << 2,
  DF_FRAG_SINGLE = 1u << 3,
  DF_K1_HEAD = 1u << 4,
  DF_K1_MULTI = 1u << 5,
  DF_MOL_SECOND = 1u << 6,
  DF_FRAG_SECOND = 1u << 7,
};

// P_N_MOL, P_MOL_SINGLE, P_N_FRAG, P_FRAG_SINGLE, P_N_K1, P_K1_MULTI, P_MITO_K1
constexpr int kDistinct = 7;
__device__ __forceinline__ int distinct_slot(int i) { return i < 6 ? P_N_MOL + i : P_MITO_K1; }

__device__ __forceinline__ bool same_fragment(const RecCols& r, uint32_t a, uint32_t b) {
  return r.pos[a] == r.pos[b] && r.ref[a] == r.ref[b] &&
         ((r.bits[a] ^ r.bits[b]) & SCT_B_REVERSE) == 0;
}

template <bool kCell, bool kGene>
__global__ void __launch_bounds__(kBlock) k_reduce_sorted(const uint64_t* __restrict__ keys,
                                                          const uint32_t* __restrict__ vals, int64_t n, RecCols r,
                                                          const uint8_t* __restrict__ k1_is_mito, Bits b,
                                                          int64_t* __restrict__ partials,
                                                          uint16_t* __restrict__ dflags) {
  // stage the tile's sorted (key, value) pairs with coalesced loads; halo of one key each side
  __shared__ uint64_t s_k[kReduceTile + 2];
  __shared__ uint32_t s_v[kReduceTile];
  const int t = threadIdx.x;
  const int64_t base = (int64_t)xcd_tile(blockIdx.x, gridDim.x) * kReduceTile;
  const int tile_n = (int)((n - base) < kReduceTile ? (n - base) : kReduceTile);
  for (int q = t; q < tile_n; q += kBlock) {
    s_k[q + 1] = keys[base + q];
    s_v[q] = vals[base + q];
  }
  if (t == 0) s_k[0] = base > 0 ? keys[base - 1] : ~0ull;
  if (t == 1) s_k[tile_n + 1] = base + tile_n < n ? keys[base + tile_n] : ~0ull;
  __syncthreads();

  const int sh_e = b.k1 + b.k2 + b.h;
  const int sh_k1 = b.k2 + b.h;
  const int sh_mol = b.h;
  const uint64_t k1_mask = b.k1 ? ((1ull << b.k1) - 1) : 0;
  int64_t acc[kDistinct];
#pragma unroll
  for (int i = 0; i < kDistinct; i++) acc[i] = 0;
  int64_t cur_e = -1;
  const auto slot = [](int i) { return distinct_slot(i); };
  // blocked items: each thread owns kReduceItems consecutive sorted positions; all lanes of a
  // wave step together so entity changes flush wave-cooperatively
  const int q0 = t * kReduceItems;
#pragma unroll
  for (int j = 0; j < kReduceItems; j++) {
    const int q = q0 + j;
    const bool valid = q < tile_n;
    const uint64_t k = valid ? s_k[q + 1] : 0;
    const int64_t e = valid ? (int64_t)(k >> sh_e) : cur_e;
    wave_flush<kDistinct>(acc, valid && e != cur_e && cur_e >= 0, cur_e, partials, slot);
    if (!valid) continue;
    cur_e = e;
    const int64_t p = base + q;
    const uint64_t kprev = s_k[q];
    const uint64_t knext = s_k[q + 2];
    const bool first = (p == 0);
    const bool last = (p + 1 == n);
    const bool k1_head = first || (kprev >> sh_k1) != (k >> sh_k1);
    const bool k1_multi = k1_head && !last && (knext >> sh_k1) == (k >> sh_k1);
    const bool mol_head = first || (kprev >> sh_mol) != (k >> sh_mol);
    const bool mol_single = mol_head && (last || (knext >> sh_mol) != (k >> sh_mol));
    const uint32_t v = s_v[q];
    const uint32_t i = v & ~kUnmappedValBit;
    const bool mapped = !(v & kUnmappedValBit);
    uint16_t f = (mol_head ? DF_MOL_HEAD : 0) | (mol_single ? DF_MOL_SINGLE : 0) | (k1_head ? DF_K1_HEAD : 0) |
                 (k1_multi ? DF_K1_MULTI : 0);
    acc[0] += mol_head;
    acc[1] += mol_single;
    acc[4] += k1_head;
    acc[5] += k1_multi;
    if constexpr (kCell) {
      if (k1_head) acc[6] += k1_is_mito[b.unscramble((uint32_t)((k >> sh_k1) & k1_mask))];
    }
    if (mapped) {
      bool is_first = true, single = true;
      const bool eq_prev = !first && kprev == k;
      const bool eq_next = !last && knext == k;
      if (eq_prev) {  // an earlier record of the sub-run may hold the same fragment
        for (int64_t pq = p - 1; pq >= 0; pq--) {
          const int64_t lq = pq - base;
          const uint64_t kq = (lq >= 0) ? s_k[lq + 1] : keys[pq];
          if (kq != k) break;
          const uint32_t vq = (lq >= 0) ? s_v[lq] : vals[pq];
          if (!(vq & kUnmappedValBit) && same_fragment(r, vq, i)) {
            is_first = false;
            break;
          }
        }
      }
      if (is_first && eq_next) {
        for (int64_t pq = p + 1; pq < n; pq++) {
          const int64_t lq = pq - base;
          const uint64_t kq = (lq < tile_n) ? s_k[lq + 1] : keys[pq];
          if (kq != k) break;
          const uint32_t vq = (lq < tile_n) ? s_v[lq] : vals[pq];
          if (!(vq & kUnmappedValBit) && same_fragment(r, vq, i)) {
            single = false;
            break;
          }
        }
      }
      if (is_first) {
        acc[2] += 1;
        acc[3] += single;
        f |= DF_FRAG_FIRST | (single ? DF_FRAG_SINGLE : 0);
      }
    }
    if constexpr (kGene) dflags[i] = f;
  }
  wave_flush<kDistinct>(acc, cur_e >= 0, cur_e, partials, slot);
}

}  // namespace sct
