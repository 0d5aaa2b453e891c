// tagsort.h -- on-GPU tag sort of columnar records (TagSortBam / sort_by_tags_and_queryname).
//
// The reference sorts records by tag values then query name with Python's stable sorted()
// (bam.py:638-709, TagSortableRecord.__lt__; a missing tag sorts as ""), and checks an order
// with verify_sort (bam.py:712-724).  Dictionary ids are ranks of the sorted strings with the
// missing value first, so comparing ids compares the strings.  Here:
//
//   k_pack        SoA columns -> one 32-byte record per index (coalesced), so later gathers move
//                 whole records instead of 14 scattered column reads;
//   rounds        the sort fields, least significant first, packed greedily into <= 64-bit keys;
//                 each round is a stable LSD radix sort (radix.h) of (key, record index), the
//                 first round over the identity order, later rounds over keys gathered through
//                 the previous round's permutation -- stable rounds compose lexicographically;
//   k_unpack      records gathered through the final permutation back into SoA columns.
//
// A caller-provided tiebreak id (the query-name rank) is the least significant field; without
// it ties keep their input order, as sorted() does.
#pragma once
#include "radix.h"
#include "util.h"

namespace sct {

struct PackedRec {
  uint4 a, b;  // a: cell, umi, gene, ref; b: pos, gq_sum | gq_len << 16, gq_gt30 | bits << 16 | xf << 24,
               //    cy_gt30 | cy_len << 8 | uy_gt30 << 16 | uy_len << 24
};

__global__ void __launch_bounds__(kBlock) k_pack(sct_records_t r, uint4* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= r.n) return;
  const uint4 a = make_uint4((uint32_t)r.cell[i], (uint32_t)r.umi[i], (uint32_t)r.gene[i], (uint32_t)r.ref[i]);
  const uint4 b = make_uint4((uint32_t)r.pos[i], (uint32_t)r.gq_sum[i] | ((uint32_t)r.gq_len[i] << 16),
                             (uint32_t)r.gq_gt30[i] | ((uint32_t)r.bits[i] << 16) | ((uint32_t)r.xf[i] << 24),
                             (uint32_t)r.cy_gt30[i] | ((uint32_t)r.cy_len[i] << 8) | ((uint32_t)r.uy_gt30[i] << 16) |
                                 ((uint32_t)r.uy_len[i] << 24));
  out[2 * i] = a;
  out[2 * i + 1] = b;
}

// sort fields: 0 cell, 1 umi, 2 gene (words of PackedRec.a), 3 tiebreak (its own column)
struct KeyField {
  int which, bits;
};
struct RoundKey {
  KeyField f[4];  // most significant first
  int nf, bits;
};

__device__ __forceinline__ uint32_t field_of(const uint4& a, uint32_t tie, int which) {
  return which == 0 ? a.x : which == 1 ? a.y : which == 2 ? a.z : tie;
}

// keys of one round: record perm[j] (or j for the first round), fields packed MSB-first
__global__ void __launch_bounds__(kBlock) k_round_keys(const uint4* __restrict__ recs, const int32_t* __restrict__ tie,
                                                       const uint32_t* __restrict__ perm, int64_t n, RoundKey rk,
                                                       uint64_t* __restrict__ keys, uint32_t* __restrict__ vals) {
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j >= n) return;
  const uint32_t idx = perm ? perm[j] : (uint32_t)j;
  const uint4 a = recs[2 * (int64_t)idx];
  const uint32_t t = tie ? (uint32_t)tie[idx] : 0u;
  uint64_t k = 0;
  for (int f = 0; f < rk.nf; f++) {
    const int b = rk.f[f].bits;
    const uint64_t v = (uint64_t)field_of(a, t, rk.f[f].which) & (b >= 32 ? 0xFFFFFFFFull : ((1ull << b) - 1));
    k = b ? ((b >= 64 ? 0ull : (k << b)) | v) : k;
  }
  keys[j] = k;
  vals[j] = idx;
}

__global__ void __launch_bounds__(kBlock) k_unpack(const uint4* __restrict__ recs, const uint32_t* __restrict__ perm,
                                                   int64_t n, sct_records_t out) {
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j >= n) return;
  const int64_t i = perm ? (int64_t)perm[j] : j;
  const uint4 a = recs[2 * i];
  const uint4 b = recs[2 * i + 1];
  const_cast<int32_t*>(out.cell)[j] = (int32_t)a.x;
  const_cast<int32_t*>(out.umi)[j] = (int32_t)a.y;
  const_cast<int32_t*>(out.gene)[j] = (int32_t)a.z;
  const_cast<int32_t*>(out.ref)[j] = (int32_t)a.w;
  const_cast<int32_t*>(out.pos)[j] = (int32_t)b.x;
  const_cast<uint16_t*>(out.gq_sum)[j] = (uint16_t)(b.y & 0xFFFFu);
  const_cast<uint16_t*>(out.gq_len)[j] = (uint16_t)(b.y >> 16);
  const_cast<uint16_t*>(out.gq_gt30)[j] = (uint16_t)(b.z & 0xFFFFu);
  const_cast<uint8_t*>(out.bits)[j] = (uint8_t)(b.z >> 16);
  const_cast<uint8_t*>(out.xf)[j] = (uint8_t)(b.z >> 24);
  const_cast<uint8_t*>(out.cy_gt30)[j] = (uint8_t)b.w;
  const_cast<uint8_t*>(out.cy_len)[j] = (uint8_t)(b.w >> 8);
  const_cast<uint8_t*>(out.uy_gt30)[j] = (uint8_t)(b.w >> 16);
  const_cast<uint8_t*>(out.uy_len)[j] = (uint8_t)(b.w >> 24);
}

// verify_sort (bam.py:712-724): the first j with key(j) < key(j - 1), as a minimum over the
// grid (n when sorted).  Keys compare field by field, most significant first.
__global__ void __launch_bounds__(kBlock) k_verify_order(sct_records_t r, const int32_t* __restrict__ tie,
                                                         KeyField f0, KeyField f1, KeyField f2, int nf,
                                                         unsigned long long* __restrict__ first_bad) {
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x + 1;
  if (j >= r.n) return;
  const KeyField fs[3] = {f0, f1, f2};
  for (int f = 0; f < nf + (tie ? 1 : 0); f++) {
    const int w = f < nf ? fs[f].which : 3;
    const int32_t* col = w == 0 ? r.cell : w == 1 ? r.umi : w == 2 ? r.gene : tie;
    const uint32_t x = (uint32_t)col[j - 1], y = (uint32_t)col[j];
    if (y < x) {
      atomicMin(first_bad, (unsigned long long)j);
      return;
    }
    if (y > x) return;
  }
}

}  // namespace sct
