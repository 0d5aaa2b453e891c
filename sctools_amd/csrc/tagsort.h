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

// ---- cell order without a tiebreak: LSD passes that move whole 32-byte rows ----
// Each pass ranks a tile of kRowTile records stably on 8 bits of the cell id (wave-level
// multi-split, as radix.h), stages the rows in LDS in digit order and writes each digit's rows
// as one run.  The first pass reads the SoA columns and writes packed rows plus the cell key
// column the next pass histograms; the last pass writes the SoA columns.  No random gathers:
// about 70 streamed bytes per record per pass.
constexpr int kRowItems = 8;
constexpr int kRowTile = kBlock * kRowItems;  // 2048 records: 64 KB of rows in LDS

__global__ void __launch_bounds__(kBlock) k_row_hist(const int32_t* __restrict__ key, int64_t n, int shift,
                                                     int64_t tiles, uint32_t* __restrict__ counts) {
  __shared__ uint32_t hist[kWaves][kRadix];
  const int wid = threadIdx.x / kWave;
  for (int i = threadIdx.x; i < kWaves * kRadix; i += kBlock) (&hist[0][0])[i] = 0;
  __syncthreads();
  const unsigned tile = xcd_tile(blockIdx.x, gridDim.x);  // consecutive tiles on one XCD (radix.h)
  const int64_t base = (int64_t)tile * kRowTile;
#pragma unroll
  for (int j = 0; j < kRowItems; j++) {
    const int64_t p = base + (int64_t)j * kBlock + threadIdx.x;
    if (p < n) atomicAdd(&hist[wid][((uint32_t)key[p] >> shift) & (kRadix - 1)], 1u);
  }
  __syncthreads();
  const int d = threadIdx.x;
  uint32_t t = 0;
#pragma unroll
  for (int w = 0; w < kWaves; w++) t += hist[w][d];
  counts[(int64_t)d * tiles + tile] = t;
}

template <bool kFromSoA, bool kToSoA>
__global__ void __launch_bounds__(kBlock) k_row_scatter(sct_records_t in, const uint4* __restrict__ rows_in,
                                                        uint4* __restrict__ rows_out, int32_t* __restrict__ key_out,
                                                        sct_records_t out, int64_t n, int shift, int64_t tiles,
                                                        const uint32_t* __restrict__ offsets) {
  __shared__ uint4 s_rows[2 * kRowTile];
  __shared__ uint32_t s_whist[kWaves][kRadix];
  __shared__ uint32_t s_dstart[kRadix];
  __shared__ uint32_t s_goff[kRadix];
  __shared__ uint64_t s_scan[kWaves + 1];
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  const unsigned tile = xcd_tile(blockIdx.x, gridDim.x);  // consecutive tiles on one XCD (radix.h)
  const int64_t base = (int64_t)tile * kRowTile;
  const int tile_n = (int)((n - base) < kRowTile ? (n - base) : kRowTile);
  for (int i = threadIdx.x; i < kWaves * kRadix; i += kBlock) (&s_whist[0][0])[i] = 0;
  s_goff[threadIdx.x] = offsets[(int64_t)threadIdx.x * tiles + tile];
  __syncthreads();
  const uint64_t lt = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
  uint4 ra[kRowItems], rb[kRowItems];
  uint16_t rank[kRowItems];
  uint8_t dig[kRowItems];
  // wave `wid` owns tile positions [wid * kRowItems * 64, ...): ranks follow input order (stable)
#pragma unroll
  for (int j = 0; j < kRowItems; j++) {
    const int q = wid * (kRowItems * kWave) + j * kWave + lane;
    const int64_t p = base + q;
    uint32_t d = kRadix - 1;  // padding ranks last and is never written
    if (q < tile_n) {
      if constexpr (kFromSoA) {
        ra[j] = make_uint4((uint32_t)in.cell[p], (uint32_t)in.umi[p], (uint32_t)in.gene[p], (uint32_t)in.ref[p]);
        rb[j] = make_uint4((uint32_t)in.pos[p], (uint32_t)in.gq_sum[p] | ((uint32_t)in.gq_len[p] << 16),
                           (uint32_t)in.gq_gt30[p] | ((uint32_t)in.bits[p] << 16) | ((uint32_t)in.xf[p] << 24),
                           (uint32_t)in.cy_gt30[p] | ((uint32_t)in.cy_len[p] << 8) |
                               ((uint32_t)in.uy_gt30[p] << 16) | ((uint32_t)in.uy_len[p] << 24));
      } else {
        ra[j] = rows_in[2 * p];
        rb[j] = rows_in[2 * p + 1];
      }
      d = (ra[j].x >> shift) & (kRadix - 1);
    }
    dig[j] = (uint8_t)d;
    uint64_t peers = ~0ull;
#pragma unroll
    for (int bitn = 0; bitn < kRadixBits; bitn++) {
      const uint64_t m = __ballot((d >> bitn) & 1u);
      peers &= ((d >> bitn) & 1u) ? m : ~m;
    }
    const int leader = __ffsll((unsigned long long)peers) - 1;
    const uint32_t below = (uint32_t)__popcll(peers & lt);
    uint32_t bse = 0;
    if (lane == leader) {
      bse = s_whist[wid][d];
      s_whist[wid][d] = bse + (uint32_t)__popcll(peers);
    }
    bse = (uint32_t)__shfl((int)bse, leader);
    rank[j] = (uint16_t)(bse + below);
  }
  __syncthreads();
  {
    const int d = threadIdx.x;
    uint32_t run = 0;
    uint32_t pre[kWaves];
#pragma unroll
    for (int w = 0; w < kWaves; w++) {
      pre[w] = run;
      run += s_whist[w][d];
    }
    uint64_t tot;
    const uint64_t ds = block_exclusive_scan<uint64_t>((uint64_t)run, &tot, s_scan);
    s_dstart[d] = (uint32_t)ds;
#pragma unroll
    for (int w = 0; w < kWaves; w++) s_whist[w][d] = (uint32_t)ds + pre[w];
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kRowItems; j++) {
    const int q = wid * (kRowItems * kWave) + j * kWave + lane;
    if (q < tile_n) {
      const uint32_t lp = s_whist[wid][dig[j]] + rank[j];
      s_rows[2 * lp] = ra[j];
      s_rows[2 * lp + 1] = rb[j];
    }
  }
  __syncthreads();
  for (int q = threadIdx.x; q < tile_n; q += kBlock) {
    const uint4 a = s_rows[2 * q];
    const uint4 b = s_rows[2 * q + 1];
    const uint32_t d = (a.x >> shift) & (kRadix - 1);
    const uint64_t o = (uint64_t)s_goff[d] + (uint32_t)(q - (int)s_dstart[d]);
    if constexpr (kToSoA) {
      const_cast<int32_t*>(out.cell)[o] = (int32_t)a.x;
      const_cast<int32_t*>(out.umi)[o] = (int32_t)a.y;
      const_cast<int32_t*>(out.gene)[o] = (int32_t)a.z;
      const_cast<int32_t*>(out.ref)[o] = (int32_t)a.w;
      const_cast<int32_t*>(out.pos)[o] = (int32_t)b.x;
      const_cast<uint16_t*>(out.gq_sum)[o] = (uint16_t)(b.y & 0xFFFFu);
      const_cast<uint16_t*>(out.gq_len)[o] = (uint16_t)(b.y >> 16);
      const_cast<uint16_t*>(out.gq_gt30)[o] = (uint16_t)(b.z & 0xFFFFu);
      const_cast<uint8_t*>(out.bits)[o] = (uint8_t)(b.z >> 16);
      const_cast<uint8_t*>(out.xf)[o] = (uint8_t)(b.z >> 24);
      const_cast<uint8_t*>(out.cy_gt30)[o] = (uint8_t)b.w;
      const_cast<uint8_t*>(out.cy_len)[o] = (uint8_t)(b.w >> 8);
      const_cast<uint8_t*>(out.uy_gt30)[o] = (uint8_t)(b.w >> 16);
      const_cast<uint8_t*>(out.uy_len)[o] = (uint8_t)(b.w >> 24);
    } else {
      rows_out[2 * o] = a;
      rows_out[2 * o + 1] = b;
      key_out[o] = (int32_t)a.x;
    }
  }
}


// ---- orders whose fields fit one 64-bit key, with a tiebreak (TagSortBam: CB, UB, GE, query name) ----
// One LSD radix sort of (fields key, record index) from the SoA columns, then the tiebreak inside
// each run of equal keys (molecules, mostly a few records): runs of <= kTieShort records are
// sorted by one thread with a sorting network on (tiebreak, index) -- the index is increasing in
// a run (the sort is stable), so ties keep input order as sorted() does; longer runs are gathered
// into a compact list and radix-sorted by (run, tiebreak).  This replaces a second full radix
// round (27 query-name bits) and the gather of its keys.
constexpr int kTieShort = 16;

// The field key of every record in input order, followed by the top `th` bits of its tiebreak
// (tie_bits wide): the bits the last radix digit has free past the fields cost no pass, and they
// split most runs of equal fields (duplicates rarely share their query-name rank's top bits), so
// the run fix-up gathers the full tiebreak for far fewer records.
// ... written with the packed row, in one pass over the columns (round 4: k_pack and a separate key
// pass read the key fields twice)
__global__ void __launch_bounds__(kBlock) k_pack_field_keys(sct_records_t r, int64_t n, RoundKey rk,
                                                            const int32_t* __restrict__ tie, int tie_bits, int th,
                                                            uint4* __restrict__ rows, uint64_t* __restrict__ keys,
                                                            uint32_t* __restrict__ vals) {
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j >= n) return;
  const uint32_t f[3] = {(uint32_t)r.cell[j], (uint32_t)r.umi[j], (uint32_t)r.gene[j]};
  const uint4 a = make_uint4(f[0], f[1], f[2], (uint32_t)r.ref[j]);
  const uint4 b = make_uint4((uint32_t)r.pos[j], (uint32_t)r.gq_sum[j] | ((uint32_t)r.gq_len[j] << 16),
                             (uint32_t)r.gq_gt30[j] | ((uint32_t)r.bits[j] << 16) | ((uint32_t)r.xf[j] << 24),
                             (uint32_t)r.cy_gt30[j] | ((uint32_t)r.cy_len[j] << 8) | ((uint32_t)r.uy_gt30[j] << 16) |
                                 ((uint32_t)r.uy_len[j] << 24));
  rows[2 * j] = a;
  rows[2 * j + 1] = b;
  uint64_t k = 0;
  for (int i = 0; i < rk.nf; i++) {
    const int bb = rk.f[i].bits;
    const uint64_t v = (uint64_t)f[rk.f[i].which] & (bb >= 32 ? 0xFFFFFFFFull : ((1ull << bb) - 1));
    k = bb ? ((bb >= 64 ? 0ull : (k << bb)) | v) : k;
  }
  if (th > 0) k = (k << th) | (((uint32_t)tie[j] >> (tie_bits - th)) & ((1u << th) - 1));
  keys[j] = k;
  vals[j] = (uint32_t)j;
}

__device__ __forceinline__ void ce(uint64_t& a, uint64_t& b) {
  const uint64_t lo = a < b ? a : b, hi = a < b ? b : a;
  a = lo;
  b = hi;
}

// Batcher's odd-even merge sort on 16
constexpr int kNet16[63][2] = {
    {0, 1}, {2, 3}, {0, 2}, {1, 3}, {1, 2}, {4, 5}, {6, 7}, {4, 6}, {5, 7}, {5, 6}, {0, 4}, {2, 6}, {2, 4},
    {1, 5}, {3, 7}, {3, 5}, {1, 2}, {3, 4}, {5, 6}, {8, 9}, {10, 11}, {8, 10}, {9, 11}, {9, 10}, {12, 13},
    {14, 15}, {12, 14}, {13, 15}, {13, 14}, {8, 12}, {10, 14}, {10, 12}, {9, 13}, {11, 15}, {11, 13}, {9, 10},
    {11, 12}, {13, 14}, {0, 8}, {4, 12}, {4, 8}, {2, 10}, {6, 14}, {6, 10}, {2, 4}, {6, 8}, {10, 12}, {1, 9},
    {5, 13}, {5, 9}, {3, 11}, {7, 15}, {7, 11}, {3, 5}, {7, 9}, {11, 13}, {1, 2}, {3, 4}, {5, 6}, {7, 8},
    {9, 10}, {11, 12}, {13, 14}};

// The tiebreak inside every run of >= 2 equal keys, one wave per 64 sorted positions:
//   * runs that lie inside the wave's positions are sorted all at once by a 64-lane bitonic network
//     on (run start lane, tiebreak, lane) -- the lane is the input order inside a run (the radix
//     sort is stable), so ties of equal names keep it, as sorted() does; other lanes key on their
//     own lane and stay put;
//   * the run that crosses the wave's end is finished by its first lane (serially: <= kTieShort
//     records in registers, longer runs to the compact list, ctl[0] runs / ctl[1] records);
//     the lanes of a run that started in an earlier wave belong to that wave.
// The tiebreak gather (random) is issued only for lanes in runs of >= 2.
__device__ __forceinline__ void tie_serial(const uint64_t* __restrict__ keys, uint32_t* __restrict__ perm,
                                           const int32_t* __restrict__ tie, int64_t n, int64_t p,
                                           uint4* __restrict__ longs, uint32_t* __restrict__ ctl) {
  const uint64_t k = keys[p];
  int L = 1;
  while (L <= kTieShort && p + L < n && keys[p + L] == k) L++;
  if (L == 1) return;
  if (L > kTieShort) {
    int64_t e = p + L;
    while (e < n && keys[e] == k) e++;
    const uint32_t len = (uint32_t)(e - p);
    const uint32_t slot = atomicAdd(&ctl[0], 1u);
    const uint32_t off = atomicAdd(&ctl[1], len);
    longs[slot] = make_uint4((uint32_t)p, len, off, 0u);
    return;
  }
  uint64_t v[kTieShort];
#pragma unroll
  for (int i = 0; i < kTieShort; i++) {
    if (i < L) {
      const uint32_t idx = perm[p + i];
      v[i] = ((uint64_t)(uint32_t)tie[idx] << 32) | idx;
    } else {
      v[i] = ~0ull;  // sentinel: sorts last
    }
  }
#pragma unroll
  for (int c = 0; c < 63; c++) ce(v[kNet16[c][0]], v[kNet16[c][1]]);
#pragma unroll
  for (int i = 0; i < kTieShort; i++)
    if (i < L) perm[p + i] = (uint32_t)v[i];
}

// Round 4 (SCT_TIE_V2): runs inside the wave are sorted by odd-even transposition over their lanes
// (one compare-exchange round per record of the longest such run; most runs are 2-3 records, the
// 64-lane bitonic network is kept for waves with a run longer than kTieRounds), and the run crossing
// the wave's end is finished by the whole wave: lanes 0..kTieShort-1 load the next keys (a halo),
// the run's records are gathered one per lane and sorted by a 16-lane bitonic network -- instead of
// one lane walking the run with dependent loads (tie_serial, kept for runs longer than kTieShort).
#ifndef SCT_TIE_V2
#define SCT_TIE_V2 1
#endif
constexpr int kTieRounds = 8;

__device__ __forceinline__ void tie_bitonic64(uint64_t& key, uint32_t& idx, int lane) {
#pragma unroll
  for (int size = 2; size <= kWave; size <<= 1) {
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      const uint64_t ok = __shfl_xor(key, stride);
      const uint32_t ov = (uint32_t)__shfl_xor((int)idx, stride);
      const bool asc = (lane & size) == 0 || size == kWave;
      const bool low = (lane & stride) == 0;
      const bool take = (low == asc) ? (ok < key) : (ok > key);
      key = take ? ok : key;
      idx = take ? ov : idx;
    }
  }
}

__global__ void __launch_bounds__(kBlock) k_tie_wave2(const uint64_t* __restrict__ keys, uint32_t* __restrict__ perm,
                                                      const int32_t* __restrict__ tie, int64_t n,
                                                      uint4* __restrict__ longs, uint32_t* __restrict__ ctl) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t p0 = p - lane;
  const bool valid = p < n;
  const uint64_t k = valid ? keys[p] : 0ull;
  // the halo: the keys after the wave's last position (for the run crossing its end)
  const int64_t ph = p0 + kWave + lane;
  const uint64_t hk = (lane < kTieShort && ph < n) ? keys[ph] : 0ull;
  uint32_t idx = valid ? perm[p] : 0u;
  uint64_t kp = __shfl_up(k, 1), kn = __shfl_down(k, 1);
  if (lane == 0) kp = (p > 0 && valid) ? keys[p - 1] : ~k;
  if (lane == kWave - 1) kn = (p + 1 < n) ? keys[p + 1] : ~k;
  const bool head = !valid || k != kp;
  const bool tail = !valid || p + 1 >= n || k != kn;
  const uint64_t H = __ballot(head), T = __ballot(tail);
  const uint64_t upto = lane == kWave - 1 ? ~0ull : ((2ull << lane) - 1);
  const uint64_t from = ~((1ull << lane) - 1);
  const uint64_t hs = H & upto, ts = T & from;
  const int s0 = hs ? 63 - __clzll((long long)hs) : -1;  // first lane of the lane's run, if in this wave
  const int s1 = ts ? __ffsll((unsigned long long)ts) - 1 : -1;  // last lane of the run, if in this wave
  const bool need = valid && s0 >= 0 && s1 >= 0 && s1 > s0;
  if (__ballot(need)) {
    const uint32_t t = need ? (uint32_t)tie[idx] : 0u;
    int len = need ? s1 - s0 + 1 : 0;
#pragma unroll
    for (int off = kWave / 2; off > 0; off >>= 1) {
      const int o = __shfl_xor(len, off);
      len = o > len ? o : len;
    }
    if (len <= kTieRounds) {
      // (tiebreak, lane): ties keep input order (the radix sort is stable)
      uint64_t key = ((uint64_t)t << 32) | (uint32_t)lane;
      const int r = lane - s0;  // position inside the run (need lanes)
      for (int i = 0; i < len; i++) {
        const bool up = ((r ^ i) & 1) == 0;  // pairs (r, r + 1) with r = i mod 2
        const int partner = up ? lane + 1 : lane - 1;
        const uint64_t ok = __shfl(key, partner & (kWave - 1));
        const uint32_t ov = (uint32_t)__shfl((int)idx, partner & (kWave - 1));
        const bool in = need && partner >= s0 && partner <= s1;
        const bool take = in && (up ? (ok < key) : (ok > key));
        key = take ? ok : key;
        idx = take ? ov : idx;
      }
    } else {
      uint64_t key = ((uint64_t)(need ? s0 : lane) << 58) | ((uint64_t)t << 6) | (uint64_t)lane;
      tie_bitonic64(key, idx, lane);
    }
    if (need) perm[p] = idx;
  }
  // the run crossing the wave's end (lane 63 is not a tail) and starting in this wave
  if (!((T >> (kWave - 1)) & 1ull) && H) {
    const int h = 63 - __clzll((long long)H);
    const uint64_t kl = __shfl(k, kWave - 1);
    const uint64_t same = __ballot(lane < kTieShort && ph < n && hk == kl);
    const int ext = (int)__builtin_ctzll(~same);  // halo records continuing the run
    const int L = kWave - h + ext;
    if (L > kTieShort || ext == kTieShort) {  // a long run (or one that may be): the serial path
      if (lane == h) tie_serial(keys, perm, tie, n, p, longs, ctl);
    } else {
      const int64_t q = p0 + h + lane;  // record `lane` of the run
      const bool mine = lane < L;
      const uint32_t qi = mine ? perm[q] : 0u;
      uint64_t key = mine ? (((uint64_t)(uint32_t)tie[qi] << 32) | (uint32_t)lane) : ~0ull;
      uint32_t qv = qi;
#pragma unroll
      for (int size = 2; size <= kTieShort; size <<= 1) {
#pragma unroll
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
          const uint64_t ok = __shfl_xor(key, stride);
          const uint32_t ov = (uint32_t)__shfl_xor((int)qv, stride);
          const bool asc = (lane & size) == 0 || size == kTieShort;
          const bool low = (lane & stride) == 0;
          const bool take = (low == asc) ? (ok < key) : (ok > key);
          key = take ? ok : key;
          qv = take ? ov : qv;
        }
      }
      if (mine) perm[q] = qv;
    }
  }
}

__global__ void __launch_bounds__(kBlock) k_tie_wave(const uint64_t* __restrict__ keys, uint32_t* __restrict__ perm,
                                                     const int32_t* __restrict__ tie, int64_t n,
                                                     uint4* __restrict__ longs, uint32_t* __restrict__ ctl) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const bool valid = p < n;
  const uint64_t k = valid ? keys[p] : 0ull;
  uint64_t kp = __shfl_up(k, 1), kn = __shfl_down(k, 1);
  if (lane == 0) kp = (p > 0 && valid) ? keys[p - 1] : ~k;
  if (lane == kWave - 1) kn = (p + 1 < n) ? keys[p + 1] : ~k;
  const bool head = !valid || k != kp;
  const bool tail = !valid || p + 1 >= n || k != kn;
  const uint64_t H = __ballot(head), T = __ballot(tail);
  const uint64_t upto = lane == kWave - 1 ? ~0ull : ((2ull << lane) - 1);
  const uint64_t from = ~((1ull << lane) - 1);
  const uint64_t hs = H & upto, ts = T & from;
  const int s0 = hs ? 63 - __clzll((long long)hs) : -1;  // first lane of the lane's run, if in this wave
  const int s1 = ts ? __ffsll((unsigned long long)ts) - 1 : -1;  // last lane of the run, if in this wave
  const bool need = valid && s0 >= 0 && s1 >= 0 && s1 > s0;
  uint32_t idx = valid ? perm[p] : 0u;
  if (__ballot(need)) {
    const uint32_t t = need ? (uint32_t)tie[idx] : 0u;
    uint64_t key = ((uint64_t)(need ? s0 : lane) << 58) | ((uint64_t)t << 6) | (uint64_t)lane;
#pragma unroll
    for (int size = 2; size <= kWave; size <<= 1) {
#pragma unroll
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        const uint64_t ok = __shfl_xor(key, stride);
        const uint32_t ov = (uint32_t)__shfl_xor((int)idx, stride);
        const bool asc = (lane & size) == 0 || size == kWave;
        const bool low = (lane & stride) == 0;
        const bool take = (low == asc) ? (ok < key) : (ok > key);
        key = take ? ok : key;
        idx = take ? ov : idx;
      }
    }
    if (need) perm[p] = idx;
  }
  // the run crossing the wave's end: its first lane (in this wave) sorts all of it
  if (!((T >> (kWave - 1)) & 1ull)) {
    const int h = H ? 63 - __clzll((long long)H) : -1;
    if (h >= 0 && lane == h) tie_serial(keys, perm, tie, n, p, longs, ctl);
  }
}

// long runs, one block each: compact keys (compact offset of the run, tiebreak), values (record
// index) and the position each compact slot maps back to.  Runs own disjoint compact ranges, so
// sorted by (offset, tiebreak) every run's records stay inside its own range.
__global__ void __launch_bounds__(kBlock) k_long_keys(const uint4* __restrict__ longs, const uint32_t* __restrict__ perm,
                                                      const int32_t* __restrict__ tie, int tie_bits,
                                                      uint64_t* __restrict__ ck, uint32_t* __restrict__ cv,
                                                      uint32_t* __restrict__ pos_of) {
  const uint4 L = longs[blockIdx.x];
  for (uint32_t i = threadIdx.x; i < L.y; i += kBlock) {
    const uint32_t idx = perm[L.x + i];
    ck[L.z + i] = ((uint64_t)L.z << tie_bits) | (uint32_t)tie[idx];
    cv[L.z + i] = idx;
    pos_of[L.z + i] = L.x + i;
  }
}

// the sorted compact list back into the runs' positions of `perm`
__global__ void __launch_bounds__(kBlock) k_long_scatter(const uint32_t* __restrict__ pos_of,
                                                         const uint32_t* __restrict__ cv, int64_t m,
                                                         uint32_t* __restrict__ perm) {
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j >= m) return;
  perm[pos_of[j]] = cv[j];
}

// ---- (CB, UB, GE[, query name]) by groups (round 6) ----
// The order's key is 14 + 20 + 15 (+ 27 query-name) bits at config 5; sorting all of it by device-wide
// LSD passes took 7 passes plus a random gather of every record's tiebreak and row.  Instead:
//   k_pack_group_keys  one pass over the SoA columns: the 32-byte row (the tiebreak in the cell's word:
//                      the cell comes back from the key) and the GROUP key K1 = (cell, top `ub` umi bits);
//   radix_sort         LSD over K1 only (c + ub bits: 3 passes at config 5), stable;
//   k_group_wave       one wave per 64 sorted positions: every group (run of equal K1: ~10 records at
//                      config 5) that lies in the wave is sorted by W = (low umi bits, gene, tiebreak,
//                      lane) with one 64-lane bitonic network -- the lane is the input order inside a
//                      group (the LSD passes are stable), so ties keep it as sorted() does -- and the
//                      group crossing the wave's end (<= 64 records) by a second network; each record's
//                      row is gathered once and written to the SoA output in its final place;
//   k_group_long       groups of 65 .. kGroupCap records: one block each, a bitonic sort in LDS.
// A group longer than kGroupCap (or a cell id the key cannot hold) sets a flag, and the host sorts
// with the general path instead.
constexpr int kGroupCap = 2048;  // records of a long group sorted in one block's LDS (11 index bits)
struct GroupBits {
  int ub;   // umi bits in K1 (the top ones)
  int ul;   // umi bits below them (in W)
  int g, t; // gene and tiebreak bits (in W)
  int c, u; // cell and umi bits
};

__device__ __forceinline__ uint32_t low_bits(uint32_t v, int b) { return b >= 32 ? v : (v & ((1u << b) - 1u)); }

// W: the order inside a group, < 2^52 (the host picks ub so that ul + g + t <= 52)
__device__ __forceinline__ uint64_t group_w(uint32_t tie, uint32_t umi, uint32_t gene, const GroupBits& gb) {
  const uint64_t ul = (uint64_t)low_bits(umi, gb.ul);
  const uint64_t gv = (uint64_t)low_bits(gene, gb.g);
  const uint64_t tv = gb.t ? (uint64_t)low_bits(tie, gb.t) : 0ull;
  return (ul << (gb.g + gb.t)) | (gv << gb.t) | tv;
}

// ctl[0]: long groups listed, ctl[1]: a group longer than kGroupCap, ctl[2]: a cell id >= 2^c.
// The values are the positions: not written (the first downsweep takes them from the index).
// (Round 6, measured: counting the first radix digit here, in 2048-record blocks, to spare the first
// upsweep cost this pass as much as the upsweep it saved: 13.60 against 13.58 ms at config 5.)
__global__ void __launch_bounds__(kBlock) k_pack_group_keys(sct_records_t r, int64_t n, GroupBits gb,
                                                            const int32_t* __restrict__ tie, uint4* __restrict__ rows,
                                                            uint32_t* __restrict__ keys, uint32_t* __restrict__ ctl) {
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j >= n) return;
  const uint32_t cell = (uint32_t)r.cell[j], umi = (uint32_t)r.umi[j];
  if (low_bits(cell, gb.c) != cell) atomicOr(&ctl[2], 1u);
  rows[2 * j] = make_uint4(tie ? (uint32_t)tie[j] : 0u, umi, (uint32_t)r.gene[j], (uint32_t)r.ref[j]);
  rows[2 * j + 1] = make_uint4((uint32_t)r.pos[j], (uint32_t)r.gq_sum[j] | ((uint32_t)r.gq_len[j] << 16),
                               (uint32_t)r.gq_gt30[j] | ((uint32_t)r.bits[j] << 16) | ((uint32_t)r.xf[j] << 24),
                               (uint32_t)r.cy_gt30[j] | ((uint32_t)r.cy_len[j] << 8) | ((uint32_t)r.uy_gt30[j] << 16) |
                                   ((uint32_t)r.uy_len[j] << 24));
  const uint32_t top = gb.ub ? (low_bits(umi, gb.u) >> gb.ul) : 0u;
  keys[j] = (uint32_t)(((uint64_t)low_bits(cell, gb.c) << gb.ub) | top);  // c + ub <= 32
}

__global__ void __launch_bounds__(kBlock) k_iota(uint32_t* __restrict__ v, int64_t n) {
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j < n) v[j] = (uint32_t)j;
}

// ---- round 6: an MSD pass by the group key's top digit first (locality for the row gather) ----
// The group sort's last step gathers every record's 32-byte row at random; measured at config 5 it
// took 3.9 ms on rows in input order and 2.6 ms on rows pre-grouped by the top bits of the cell
// (tools/c5_locality_probe.py): the rows that consecutive output positions gather then share cache
// lines and MALL residency.  So the rows are written once in the order of K1's top kMsdBits bits (a
// stable multi-split, rows staged in LDS per 2048-record tile, as k_row_scatter), and the rest of K1 is
// sorted by LSD passes INSIDE those buckets (segmented: each tile belongs to one bucket, and the
// count matrix is laid out bucket-major, so one device-wide scan gives every bucket its own digit
// offsets) -- one pass fewer than sorting all of K1.  The top digit is 9 bits wide (512 buckets), so
// a 25-bit K1 -- config 5's (14-bit cell, 11 umi bits) -- takes two 8-bit segmented passes, not three.
constexpr int kMsdItems = 8;
constexpr int kMsdTile = kBlock * kMsdItems;  // 2048 records: 64 KB of rows + 8 KB of tiebreaks in LDS
constexpr int kMsdBits = 9;
constexpr int kMsdRadix = 1 << kMsdBits;  // buckets of the MSD pass
static_assert(kMsdRadix == 2 * kBlock, "two top digits per thread");
static_assert(kMsdTile <= 0xffff, "16-bit per-tile digit counts and starts");
constexpr int kSegItems = 16;
constexpr int kSegTile = kBlock * kSegItems;  // segmented LSD tiles (4096 items)

__device__ __forceinline__ uint32_t group_key(uint32_t cell, uint32_t umi, const GroupBits& gb) {
  const uint32_t top = gb.ub ? (low_bits(umi, gb.u) >> gb.ul) : 0u;
  return (uint32_t)(((uint64_t)low_bits(cell, gb.c) << gb.ub) | top);  // c + ub <= 32
}

// the top digit's count per tile (counts[d * tiles + tile]); ctl[2]: a cell id the key cannot hold
__global__ void __launch_bounds__(kBlock) k_gmsd_hist(const int32_t* __restrict__ cell, const int32_t* __restrict__ umi,
                                                      int64_t n, GroupBits gb, int sh_top, int64_t tiles,
                                                      uint32_t* __restrict__ counts, uint32_t* __restrict__ ctl) {
  __shared__ uint32_t hist[kWaves][kMsdRadix];
  const int wid = threadIdx.x / kWave;
  for (int i = threadIdx.x; i < kWaves * kMsdRadix; i += kBlock) (&hist[0][0])[i] = 0;
  __syncthreads();
  const unsigned tile = xcd_tile(blockIdx.x, gridDim.x);
  const int64_t base = (int64_t)tile * kMsdTile;
  bool bad = false;
#pragma unroll
  for (int j = 0; j < kMsdItems; j++) {
    const int64_t p = base + (int64_t)j * kBlock + threadIdx.x;
    if (p < n) {
      const uint32_t c = (uint32_t)cell[p];
      bad |= low_bits(c, gb.c) != c;
      atomicAdd(&hist[wid][(group_key(c, (uint32_t)umi[p], gb) >> sh_top) & (kMsdRadix - 1)], 1u);
    }
  }
  if (bad) atomicOr(&ctl[2], 1u);
  __syncthreads();
  for (int d = threadIdx.x; d < kMsdRadix; d += kBlock) {
    uint32_t t = 0;
#pragma unroll
    for (int w = 0; w < kWaves; w++) t += hist[w][d];
    counts[(int64_t)d * tiles + tile] = t;
  }
}

// the stable multi-split by the top digit: SoA columns + tiebreak in, rows (tiebreak in the cell's
// word) + group keys out, each digit's records of the tile written as one run (k_row_scatter's scheme).
// Per-tile counts and starts are 16-bit (<= kMsdTile), so the 512 digits' bookkeeping takes 7 KB and
// two blocks still share a CU's 160 KB of LDS.
__global__ void __launch_bounds__(kBlock) k_gmsd_scatter(sct_records_t in, const int32_t* __restrict__ tie, int64_t n,
                                                         GroupBits gb, int sh_top, int64_t tiles,
                                                         const uint32_t* __restrict__ offsets,
                                                         uint4* __restrict__ rows_out, uint32_t* __restrict__ keys_out) {
  __shared__ uint4 s_rows[2 * kMsdTile];
  __shared__ uint32_t s_tie[kMsdTile];
  __shared__ uint16_t s_whist[kWaves][kMsdRadix];
  __shared__ uint16_t s_dstart[kMsdRadix];
  __shared__ uint32_t s_goff[kMsdRadix];
  __shared__ uint64_t s_scan[kWaves + 1];
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  const unsigned tile = xcd_tile(blockIdx.x, gridDim.x);
  const int64_t base = (int64_t)tile * kMsdTile;
  const int tile_n = (int)((n - base) < kMsdTile ? (n - base) : kMsdTile);
  for (int i = threadIdx.x; i < kWaves * kMsdRadix; i += kBlock) (&s_whist[0][0])[i] = 0;
  for (int d = threadIdx.x; d < kMsdRadix; d += kBlock) s_goff[d] = offsets[(int64_t)d * tiles + tile];
  __syncthreads();
  const uint64_t lt = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
  uint4 ra[kMsdItems], rb[kMsdItems];
  uint32_t tv[kMsdItems];
  uint16_t rank[kMsdItems];
  uint16_t dig[kMsdItems];
#pragma unroll
  for (int j = 0; j < kMsdItems; j++) {
    const int q = wid * (kMsdItems * kWave) + j * kWave + lane;
    const int64_t p = base + q;
    uint32_t d = kMsdRadix - 1;  // padding ranks last and is never written
    if (q < tile_n) {
      ra[j] = make_uint4((uint32_t)in.cell[p], (uint32_t)in.umi[p], (uint32_t)in.gene[p], (uint32_t)in.ref[p]);
      rb[j] = make_uint4((uint32_t)in.pos[p], (uint32_t)in.gq_sum[p] | ((uint32_t)in.gq_len[p] << 16),
                         (uint32_t)in.gq_gt30[p] | ((uint32_t)in.bits[p] << 16) | ((uint32_t)in.xf[p] << 24),
                         (uint32_t)in.cy_gt30[p] | ((uint32_t)in.cy_len[p] << 8) | ((uint32_t)in.uy_gt30[p] << 16) |
                             ((uint32_t)in.uy_len[p] << 24));
      tv[j] = tie ? (uint32_t)tie[p] : 0u;
      d = (group_key(ra[j].x, ra[j].y, gb) >> sh_top) & (kMsdRadix - 1);
    }
    dig[j] = (uint16_t)d;
    uint64_t peers = ~0ull;
#pragma unroll
    for (int bitn = 0; bitn < kMsdBits; bitn++) {
      const uint64_t m = __ballot((d >> bitn) & 1u);
      peers &= ((d >> bitn) & 1u) ? m : ~m;
    }
    const int leader = __ffsll((unsigned long long)peers) - 1;
    const uint32_t below = (uint32_t)__popcll(peers & lt);
    uint32_t bse = 0;
    if (lane == leader) {
      bse = s_whist[wid][d];
      s_whist[wid][d] = (uint16_t)(bse + (uint32_t)__popcll(peers));
    }
    bse = (uint32_t)__shfl((int)bse, leader);
    rank[j] = (uint16_t)(bse + below);
  }
  __syncthreads();
  {
    // thread t: digits 2t and 2t + 1
    const int d0 = 2 * threadIdx.x, d1 = d0 + 1;
    uint32_t run0 = 0, run1 = 0;
    uint32_t pre0[kWaves], pre1[kWaves];
#pragma unroll
    for (int w = 0; w < kWaves; w++) {
      pre0[w] = run0;
      run0 += s_whist[w][d0];
      pre1[w] = run1;
      run1 += s_whist[w][d1];
    }
    uint64_t tot;
    const uint32_t ds0 = (uint32_t)block_exclusive_scan<uint64_t>((uint64_t)(run0 + run1), &tot, s_scan);
    const uint32_t ds1 = ds0 + run0;
    s_dstart[d0] = (uint16_t)ds0;
    s_dstart[d1] = (uint16_t)ds1;
#pragma unroll
    for (int w = 0; w < kWaves; w++) {
      s_whist[w][d0] = (uint16_t)(ds0 + pre0[w]);
      s_whist[w][d1] = (uint16_t)(ds1 + pre1[w]);
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kMsdItems; j++) {
    const int q = wid * (kMsdItems * kWave) + j * kWave + lane;
    if (q < tile_n) {
      const uint32_t lp = (uint32_t)s_whist[wid][dig[j]] + rank[j];
      s_rows[2 * lp] = ra[j];
      s_rows[2 * lp + 1] = rb[j];
      s_tie[lp] = tv[j];
    }
  }
  __syncthreads();
  for (int q = threadIdx.x; q < tile_n; q += kBlock) {
    const uint4 a = s_rows[2 * q];
    const uint4 b = s_rows[2 * q + 1];
    const uint32_t k = group_key(a.x, a.y, gb);
    const uint32_t d = (k >> sh_top) & (kMsdRadix - 1);
    const uint64_t o = (uint64_t)s_goff[d] + (uint32_t)(q - (int)s_dstart[d]);
    rows_out[2 * o] = make_uint4(s_tie[q], a.y, a.z, a.w);
    rows_out[2 * o + 1] = b;
    keys_out[o] = k;
  }
}

// one block: the buckets (digits of the MSD pass) -> their starts, sizes and first segmented tile
// (gseg[0, R) start, [R, 2R) size, [2R, 3R) tile base, gseg[3R] the tile total; R = kMsdRadix)
__global__ void __launch_bounds__(kBlock) k_gseg_plan(const uint32_t* __restrict__ offsets, int64_t tiles, int64_t n,
                                                      uint32_t* __restrict__ gseg) {
  __shared__ uint64_t s_scan[kWaves + 1];
  uint32_t st[2], sz[2], nt[2];
#pragma unroll
  for (int i = 0; i < 2; i++) {
    const int d = 2 * threadIdx.x + i;
    st[i] = offsets[(int64_t)d * tiles];
    const uint32_t nx = d + 1 < kMsdRadix ? offsets[(int64_t)(d + 1) * tiles] : (uint32_t)n;
    sz[i] = nx - st[i];
    nt[i] = (sz[i] + kSegTile - 1) / kSegTile;
  }
  uint64_t tot;
  const uint32_t tb0 = (uint32_t)block_exclusive_scan<uint64_t>((uint64_t)(nt[0] + nt[1]), &tot, s_scan);
#pragma unroll
  for (int i = 0; i < 2; i++) {
    const int d = 2 * threadIdx.x + i;
    gseg[d] = st[i];
    gseg[kMsdRadix + d] = sz[i];
    gseg[2 * kMsdRadix + d] = tb0 + (i ? nt[0] : 0u);
  }
  if (threadIdx.x == 0) gseg[3 * kMsdRadix] = (uint32_t)tot;
}

// a segmented tile's bucket and range: tile base b = the last bucket whose first tile <= tile
struct SegTile {
  int b;
  uint32_t tl, nt;  // tile inside the bucket, the bucket's tiles
  int64_t base;
  int len;
};
// (tb: the bucket tile bases, gseg[2R .. 3R], staged in LDS by the caller: seg_stage)
__device__ __forceinline__ const uint32_t* seg_stage(const uint32_t* __restrict__ gseg, uint32_t* s_tb) {
  for (int d = threadIdx.x; d < kMsdRadix; d += kBlock) s_tb[d] = gseg[2 * kMsdRadix + d];
  if (threadIdx.x == 0) s_tb[kMsdRadix] = gseg[3 * kMsdRadix];
  __syncthreads();
  return s_tb;
}
__device__ __forceinline__ bool seg_tile(const uint32_t* __restrict__ gseg, const uint32_t* tb, uint32_t tile,
                                         SegTile& st) {
  if (tile >= tb[kMsdRadix]) return false;
  int lo = 0, hi = kMsdRadix - 1;  // the last b with tb[b] <= tile (empty buckets share their successor's base)
  while (lo < hi) {
    const int mid = (lo + hi + 1) / 2;
    if (tb[mid] <= tile) lo = mid; else hi = mid - 1;
  }
  st.b = lo;
  st.tl = tile - tb[lo];
  st.nt = (lo + 1 < kMsdRadix ? tb[lo + 1] : tb[kMsdRadix]) - tb[lo];
  st.base = (int64_t)gseg[lo] + (int64_t)st.tl * kSegTile;
  const int64_t rem = (int64_t)gseg[kMsdRadix + lo] - (int64_t)st.tl * kSegTile;
  st.len = (int)(rem < kSegTile ? rem : kSegTile);
  return true;
}
// count index of (bucket, digit, tile inside the bucket): bucket-major, then digit, then tile
__device__ __forceinline__ int64_t seg_cidx(const uint32_t* tb, const SegTile& st, uint32_t d) {
  return (int64_t)kRadix * tb[st.b] + (int64_t)d * st.nt + st.tl;
}

__global__ void __launch_bounds__(kBlock) k_gseg_upsweep(const uint32_t* __restrict__ keys, int shift,
                                                         const uint32_t* __restrict__ gseg,
                                                         uint32_t* __restrict__ counts) {
  __shared__ uint32_t hist[kWaves][kRadix];
  __shared__ uint32_t s_tb[kMsdRadix + 1];
  const uint32_t* tb = seg_stage(gseg, s_tb);
  SegTile st;
  // consecutive tiles on one XCD (radix.h): their digit runs' partly written lines meet in one L2
  if (!seg_tile(gseg, tb, xcd_tile(blockIdx.x, gridDim.x), st)) return;  // block-uniform
  const int wid = threadIdx.x / kWave;
  for (int i = threadIdx.x; i < kWaves * kRadix; i += kBlock) (&hist[0][0])[i] = 0;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kSegItems; j++) {
    const int q = j * kBlock + threadIdx.x;
    if (q < st.len) atomicAdd(&hist[wid][(keys[st.base + q] >> shift) & (kRadix - 1)], 1u);
  }
  __syncthreads();
  const int d = threadIdx.x;
  uint32_t t = 0;
#pragma unroll
  for (int w = 0; w < kWaves; w++) t += hist[w][d];
  counts[seg_cidx(tb, st, (uint32_t)d)] = t;
}

// k_radix_downsweep on a segmented tile (kIdx: the values are the positions)
template <bool kIdx>
__global__ void __launch_bounds__(kBlock) k_gseg_downsweep(const uint32_t* __restrict__ keys_in,
                                                           const uint32_t* __restrict__ vals_in,
                                                           uint32_t* __restrict__ keys_out,
                                                           uint32_t* __restrict__ vals_out, int shift,
                                                           const uint32_t* __restrict__ gseg,
                                                           const uint32_t* __restrict__ offsets) {
  __shared__ uint32_t s_keys[kSegTile];
  __shared__ uint32_t s_vals[kSegTile];
  __shared__ uint32_t s_whist[kWaves][kRadix];
  __shared__ uint32_t s_dstart[kRadix];
  __shared__ uint32_t s_goff[kRadix];
  __shared__ uint64_t s_scan[kWaves + 1];
  // the bucket tile bases are staged in s_vals: read only before the barrier after s_goff (s_vals is
  // written two barriers later), so the block stays at 40 KB of LDS, 4 blocks per CU
  static_assert(kSegTile >= kMsdRadix + 1, "tile bases fit s_vals");
  const uint32_t* tb = seg_stage(gseg, s_vals);
  SegTile st;
  // consecutive tiles on one XCD (radix.h): their digit runs' partly written lines meet in one L2
  if (!seg_tile(gseg, tb, xcd_tile(blockIdx.x, gridDim.x), st)) return;  // block-uniform
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  const int tile_n = st.len;
  for (int i = threadIdx.x; i < kWaves * kRadix; i += kBlock) (&s_whist[0][0])[i] = 0;
  s_goff[threadIdx.x] = offsets[seg_cidx(tb, st, (uint32_t)threadIdx.x)];
  __syncthreads();
  const uint64_t lt = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
  uint32_t k[kSegItems], v[kSegItems];
  uint16_t rank[kSegItems];
  uint8_t dig[kSegItems];
#pragma unroll
  for (int j = 0; j < kSegItems; j++) {
    const int q = wid * (kSegItems * kWave) + j * kWave + lane;
    const int64_t p = st.base + q;
    if (q < tile_n) {
      k[j] = keys_in[p];
      v[j] = kIdx ? (uint32_t)p : vals_in[p];
    } else {
      k[j] = ~0u;  // padding: digit 255, ranked after every real item, never written
      v[j] = 0;
    }
    const uint32_t d = (k[j] >> shift) & (kRadix - 1);
    dig[j] = (uint8_t)d;
    uint64_t peers = ~0ull;
#pragma unroll
    for (int bitn = 0; bitn < kRadixBits; bitn++) {
      const uint64_t m = __ballot((d >> bitn) & 1u);
      peers &= ((d >> bitn) & 1u) ? m : ~m;
    }
    const int leader = __ffsll((unsigned long long)peers) - 1;
    const uint32_t below = (uint32_t)__popcll(peers & lt);
    uint32_t bse = 0;
    if (lane == leader) {
      bse = s_whist[wid][d];
      s_whist[wid][d] = bse + (uint32_t)__popcll(peers);
    }
    bse = (uint32_t)__shfl((int)bse, leader);
    rank[j] = (uint16_t)(bse + below);
  }
  __syncthreads();
  {
    const int d = threadIdx.x;
    uint32_t run = 0;
    uint32_t pre[kWaves];
#pragma unroll
    for (int w = 0; w < kWaves; w++) {
      pre[w] = run;
      run += s_whist[w][d];
    }
    uint64_t tot;
    const uint64_t ds = block_exclusive_scan<uint64_t>((uint64_t)run, &tot, s_scan);
    s_dstart[d] = (uint32_t)ds;
#pragma unroll
    for (int w = 0; w < kWaves; w++) s_whist[w][d] = (uint32_t)ds + pre[w];
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kSegItems; j++) {
    const uint32_t lp = s_whist[wid][dig[j]] + rank[j];
    s_keys[lp] = k[j];
    s_vals[lp] = v[j];
  }
  __syncthreads();
  for (int q = threadIdx.x; q < tile_n; q += kBlock) {
    const uint32_t kk = s_keys[q];
    const uint32_t d = (kk >> shift) & (kRadix - 1);
    const uint64_t o = (uint64_t)s_goff[d] + (uint32_t)(q - (int)s_dstart[d]);
    keys_out[o] = kk;
    vals_out[o] = s_vals[q];
  }
}

// one record to the SoA output (its cell from the group key, the rest from its row)
__device__ __forceinline__ void group_store(const sct_records_t& out, int64_t j, uint32_t cell, const uint4& a,
                                            const uint4& b) {
  const_cast<int32_t*>(out.cell)[j] = (int32_t)cell;
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

// 64-lane bitonic sort of one 64-bit key per lane, ascending by lane
__device__ __forceinline__ uint64_t bitonic64_key(uint64_t key, int lane) {
#pragma unroll
  for (int size = 2; size <= kWave; size <<= 1) {
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      const uint64_t ok = __shfl_xor(key, stride);
      const bool asc = (lane & size) == 0 || size == kWave;
      const bool low = (lane & stride) == 0;
      key = (low == asc) ? (ok < key ? ok : key) : (ok > key ? ok : key);
    }
  }
  return key;
}

// the row of lane `src`
__device__ __forceinline__ void row_from(int src, uint4& a, uint4& b) {
  a.y = (uint32_t)__shfl((int)a.y, src);
  a.z = (uint32_t)__shfl((int)a.z, src);
  a.w = (uint32_t)__shfl((int)a.w, src);
  b.x = (uint32_t)__shfl((int)b.x, src);
  b.y = (uint32_t)__shfl((int)b.y, src);
  b.z = (uint32_t)__shfl((int)b.z, src);
  b.w = (uint32_t)__shfl((int)b.w, src);
}

// The group crossing the wave's end is found from a halo of the next 64 keys, so its records' loads
// are issued together with the wave's own (one round of dependent loads, not two).
__global__ void __launch_bounds__(kBlock) k_group_wave(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ perm,
                                                       const uint4* __restrict__ rows, int64_t n, GroupBits gb,
                                                       sct_records_t out, uint2* __restrict__ longs,
                                                       uint32_t* __restrict__ ctl) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t p0 = p - lane;
  const bool valid = p < n;
  const uint32_t k = valid ? keys[p] : 0u;
  const int64_t ph = p + kWave;
  const uint32_t hk = ph < n ? keys[ph] : 0u;  // the halo
  uint32_t kp = (uint32_t)__shfl_up((int)k, 1), kn = (uint32_t)__shfl_down((int)k, 1);
  if (lane == 0) kp = (p > 0 && valid) ? keys[p - 1] : ~k;
  if (lane == kWave - 1) kn = (p + 1 < n) ? keys[p + 1] : ~k;
  const bool head = !valid || k != kp;
  const bool tail = !valid || p + 1 >= n || k != kn;
  const uint64_t H = __ballot(head), T = __ballot(tail);
  const uint64_t upto = lane == kWave - 1 ? ~0ull : ((2ull << lane) - 1);
  const uint64_t from = ~((1ull << lane) - 1);
  const uint64_t hs = H & upto, ts = T & from;
  const int s0 = hs ? 63 - __clzll((long long)hs) : -1;  // first lane of the lane's group, if in this wave
  const int s1 = ts ? __ffsll((unsigned long long)ts) - 1 : -1;  // last lane of the group, if in this wave
  const bool inside = valid && s0 >= 0 && s1 >= 0;  // the lane's group lies in the wave: written here
  // the group crossing the wave's end, if it starts in this wave (else an earlier wave owns it)
  const bool cross = !((T >> (kWave - 1)) & 1ull) && H != 0;  // wave-uniform
  const int h = cross ? 63 - __clzll((long long)H) : 0;
  const uint32_t kl = (uint32_t)__shfl((int)k, kWave - 1);
  const uint64_t same = __ballot(ph < n && hk == kl);
  const int ext = same == ~0ull ? kWave : __builtin_ctzll(~same);
  const int64_t g0 = p0 + h;
  const int L = kWave - h + ext;
  const bool small = cross && ext < kWave && L <= kWave;
  uint32_t idx = 0, idx2 = 0;
  if (inside) idx = perm[p];
  const bool in2 = small && lane < L;
  if (in2) idx2 = perm[g0 + lane];
  uint4 a = make_uint4(0, 0, 0, 0), b = make_uint4(0, 0, 0, 0), a2 = a, b2 = a;
  if (inside) {
    a = rows[2 * (int64_t)idx];
    b = rows[2 * (int64_t)idx + 1];
  }
  if (in2) {
    a2 = rows[2 * (int64_t)idx2];
    b2 = rows[2 * (int64_t)idx2 + 1];
  }
  const bool need = inside && s1 > s0;
  if (__ballot(need)) {
    // (group start lane | W | lane): lanes outside groups key on their own lane and stay put
    const uint64_t w = need ? group_w(a.x, a.y, a.z, gb) : 0ull;
    const uint64_t key = bitonic64_key(((uint64_t)(need ? s0 : lane) << 58) | (w << 6) | (uint64_t)lane, lane);
    row_from((int)(key & 63u), a, b);
  }
  if (inside) group_store(out, p, k >> gb.ub, a, b);
  if (!cross) return;  // wave-uniform
  if (small) {
    const uint64_t key = bitonic64_key(in2 ? ((group_w(a2.x, a2.y, a2.z, gb) << 6) | (uint64_t)lane) : ~0ull, lane);
    row_from((int)(key & 63u), a2, b2);
    if (in2) group_store(out, g0 + lane, kl >> gb.ub, a2, b2);
    return;
  }
  // longer than a wave: its end, 64 keys at a time past the halo (bounded by kGroupCap)
  int64_t e = ph - lane + ext;
  if (ext == kWave) {
    while (true) {
      const int64_t q = e + lane;
      const uint64_t m = __ballot(q < n && keys[q] == kl);
      const int x = m == ~0ull ? kWave : __builtin_ctzll(~m);
      e += x;
      if (x < kWave || e - g0 > kGroupCap) break;
    }
  }
  const int64_t len = e - g0;
  if (len > kGroupCap) {
    if (lane == 0) atomicOr(&ctl[1], 1u);  // too long: the host sorts on the general path
  } else if (lane == 0) {
    longs[atomicAdd(&ctl[0], 1u)] = make_uint2((uint32_t)g0, (uint32_t)len);
  }
}

// one block per long group (65 .. kGroupCap records): (W, index) bitonic-sorted in LDS
__global__ void __launch_bounds__(kBlock) k_group_long(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ perm,
                                                       const uint4* __restrict__ rows, GroupBits gb,
                                                       const uint2* __restrict__ longs, sct_records_t out) {
  __shared__ uint64_t s_k[kGroupCap];
  const uint2 G = longs[blockIdx.x];
  const int len = (int)G.y;
  int np2 = kWave;
  while (np2 < len) np2 <<= 1;
  for (int i = threadIdx.x; i < np2; i += kBlock) {
    uint64_t v = ~0ull;
    if (i < len) {
      const uint4 a = rows[2 * (int64_t)perm[G.x + i]];
      v = (group_w(a.x, a.y, a.z, gb) << 11) | (uint64_t)i;
    }
    s_k[i] = v;
  }
  __syncthreads();
  for (int size = 2; size <= np2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = threadIdx.x; i < np2 / 2; i += kBlock) {
        const int lo = 2 * i - (i & (stride - 1));  // pair (lo, lo + stride)
        const int hi = lo + stride;
        const bool asc = (lo & size) == 0;
        const uint64_t x = s_k[lo], y = s_k[hi];
        if ((x > y) == asc) {
          s_k[lo] = y;
          s_k[hi] = x;
        }
      }
      __syncthreads();
    }
  }
  const uint32_t cell = keys[G.x] >> gb.ub;
  for (int j = threadIdx.x; j < len; j += kBlock) {
    const uint32_t idx = perm[G.x + (uint32_t)(s_k[j] & (kGroupCap - 1))];
    group_store(out, (int64_t)G.x + j, cell, rows[2 * (int64_t)idx], rows[2 * (int64_t)idx + 1]);
  }
}

}  // namespace sct

