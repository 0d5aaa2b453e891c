// segment.h -- the input-order pass: entity runs (bam.iter_tag_groups, bam.py:492-540),
// packed sort keys, and every per-record additive metric of the entity.
//
// One block owns a tile of kTile consecutive records.  The entity column is staged
// into LDS with coalesced loads, run heads are found on blocked items, and a block
// scan numbers the runs.  Then each thread walks the tile in striped order (all
// column loads coalesced), builds the key [run | k1 | k2 | fragment hash] and the
// value (record index, bit 31 = unmapped), and sums the metrics that are plain
// per-record sums in the reference (aggregator.py:259-334, 507-530) into the run's
// partial row: n_reads, barcode / alignment counters, and the exact fixed-point
// lanes of the quality streams (fixedpt.h).  Runs are contiguous in input order, so
// a thread flushes once per run it touches and a wave once per tile.
#pragma once
#include <type_traits>
#include "bucket.h"
#include "fixedpt.h"
#include "radix.h"
#include "reduce.h"
#include "util.h"

namespace sct {

// heads per tile.  With `seen` set (grouped gene partials), every run head also bumps
// seen[entity value]; a value seen twice means the column is not sorted into single
// runs and *dup_flag gets bit 0; a value outside [0, n_ids) sets bit 1.
__global__ void k_heads(const int32_t* __restrict__ key, int64_t n, uint64_t* __restrict__ tile_cnt,
                        uint32_t* __restrict__ seen, uint32_t n_ids, uint64_t* __restrict__ dup_flag) {
  const int64_t base = (int64_t)blockIdx.x * kTile;
  uint64_t c = 0;
#pragma unroll 4
  for (int j = 0; j < kItems; j++) {
    const int64_t p = base + (int64_t)j * kBlock + threadIdx.x;
    if (p < n) {
      const int32_t v = key[p];
      const bool h = (p == 0 || v != key[p - 1]);
      c += h ? 1 : 0;
      if (h && seen) {
        if ((uint32_t)v >= n_ids) atomicOr((unsigned long long*)dup_flag, 2ull);  // id outside the dictionary
        else if (atomicAdd(&seen[v], 1u) != 0u) atomicOr((unsigned long long*)dup_flag, 1ull);
      }
    }
  }
  __shared__ uint64_t red[kWaves];
  c = wave_sum(c);
  if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t t = 0;
    for (int w = 0; w < kWaves; w++) t += red[w];
    tile_cnt[blockIdx.x] = t;
  }
}

// k_heads with 16-byte loads: thread t of item j owns records [4(j*kBlock + t), +4) of the
// tile; the record before its first comes from the previous lane (lane 0 loads it).  Needs a
// 16-byte aligned column (the host checks and falls back to k_heads).
__global__ void __launch_bounds__(kBlock) k_heads4(const int32_t* __restrict__ key, int64_t n,
                                                   uint64_t* __restrict__ tile_cnt, uint32_t* __restrict__ seen,
                                                   uint32_t n_ids, uint64_t* __restrict__ dup_flag) {
  constexpr int kVec = kItems / 4;
  const int64_t base = (int64_t)blockIdx.x * kTile;
  const int lane = threadIdx.x & (kWave - 1);
  int4 v[kVec];
#pragma unroll
  for (int j = 0; j < kVec; j++) {  // every load issued before any compare
    const int64_t p = base + 4 * ((int64_t)j * kBlock + threadIdx.x);
    if (p + 3 < n) {
      v[j] = *reinterpret_cast<const int4*>(key + p);
    } else {
      v[j].x = p < n ? key[p] : 0;
      v[j].y = p + 1 < n ? key[p + 1] : 0;
      v[j].z = p + 2 < n ? key[p + 2] : 0;
      v[j].w = 0;
    }
  }
  uint64_t c = 0;
#pragma unroll
  for (int j = 0; j < kVec; j++) {
    const int64_t p = base + 4 * ((int64_t)j * kBlock + threadIdx.x);
    int32_t prev = __shfl_up(v[j].w, 1);
    if (lane == 0 && p > 0 && p < n) prev = key[p - 1];
    const int32_t r[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const bool in = p + i < n;
      const bool h = in && (p + i == 0 || r[i] != (i == 0 ? prev : r[i - 1]));
      c += h ? 1 : 0;
      if (h && seen) {
        if ((uint32_t)r[i] >= n_ids) atomicOr((unsigned long long*)dup_flag, 2ull);  // id outside the dictionary
        else if (atomicAdd(&seen[r[i]], 1u) != 0u) atomicOr((unsigned long long*)dup_flag, 1ull);
      }
    }
  }
  __shared__ uint64_t red[kWaves];
  c = wave_sum(c);
  if (lane == 0) red[threadIdx.x / kWave] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t t = 0;
    for (int w = 0; w < kWaves; w++) t += red[w];
    tile_cnt[blockIdx.x] = t;
  }
}

struct KeyCols {
  const int32_t* ent;  // column whose runs are the entities
  const int32_t* k1;
  const int32_t* k2;
  uint32_t n_k1, n_k2;  // dictionary sizes: ids outside them set bit 1 of *err
};

__device__ __forceinline__ uint64_t make_key(uint64_t e, uint32_t k1, uint32_t k2, uint32_t hash, const Bits& b) {
  const uint64_t hv = b.h ? (uint64_t)(hash >> (32 - b.h)) : 0;  // top bits of the fragment mix
  const uint64_t ev = b.e ? (e << (b.k1 + b.k2 + b.h)) : 0;  // bucket path: entities are record ranges
  return ev | ((uint64_t)b.scramble(k1) << (b.k2 + b.h)) | ((uint64_t)k2 << b.h) | hv;
}

// per-record additive counters of one run
template <bool kCell>
struct AddAcc {
  static constexpr int kK = kCell ? 13 : 9;
  int32_t v[kK];  // per thread: at most kKItems records between flushes
  // counter i -> partial slot: 0..8 are P_N_READS..P_SPLICED; 9..12 are P_PERFECT_CB, P_INTERGENIC,
  // P_UNMAPPED, P_MITO_READS
  static __device__ __forceinline__ int slot(int i) {
    return i < 9 ? i : (i < 12 ? P_PERFECT_CB + (i - 9) : P_MITO_READS);
  }
  __device__ __forceinline__ void clear() {
#pragma unroll
    for (int i = 0; i < kK; i++) v[i] = 0;
  }
};


// The key pass (k_build_keys_run) owns kKTile records per block, kKItems per thread: twice the
// heads tile (k_heads / tile offsets are per kTile), which halves the per-block costs (run-id
// scan, the wave flushes that end each quality stream, the gene-bucket histogram flush).
constexpr int kKItems = 2 * kItems;  // 32: the blocked head masks are 32-bit
constexpr int kKTile = kBlock * kKItems;
constexpr int kKTilesPerBlock = kKTile / kTile;
constexpr int kRunBatch = 8;  // striped rounds whose entity loads are in flight together
static_assert(kKItems == 32, "head masks are 32-bit; two threads per 64-position word of s_hb");
static_assert(kKItems % kRunBatch == 0, "whole batches");
static_assert(kKTile <= 65535, "local run ids are 16-bit");

// Number the runs of the tile.  Run ids are local: the run of tile position q is the returned base
// (tile_off - 1) plus the number of heads at positions <= q (local 0 = the run continuing from the
// previous tile).  Heads are found on striped, coalesced loads (the previous record comes from the
// neighbouring lane; lane 0 re-reads it, a cache hit) and kept as one bit per position (s_hb:
// kKTile / 64 words, ballots); a block scan counts each thread's 32 blocked positions' heads, and
// s_wpre gets the heads before each 64-position word, so loc_of() reads any position's run id off
// two LDS words.  Writes ent_start[run] for heads when ent_start is set.  Block-wide (barriers).
// Also returns the thread's blocked head mask (*my_heads) and the local id of the run before its
// first position (*my_ex): the run of position 32t + j is ebase + my_ex + popc(heads & bits 0..j).
__device__ __forceinline__ int64_t tile_run_ids(const int32_t* __restrict__ ent, int64_t base, int tile_n,
                                                uint64_t tile_off, uint64_t* s_hb, uint64_t* s_scan,
                                                int64_t* __restrict__ ent_start, uint32_t* my_heads,
                                                uint32_t* my_ex, uint32_t* n_heads, uint16_t* s_wpre) {
  const int t = threadIdx.x, lane = t & (kWave - 1), w = t / kWave;
  for (int j0 = 0; j0 < kKItems; j0 += kRunBatch) {
    int32_t v[kRunBatch], pv[kRunBatch];
#pragma unroll
    for (int u = 0; u < kRunBatch; u++) {
      const int q = (j0 + u) * kBlock + t;
      const int64_t p = base + (q < tile_n ? q : 0);
      v[u] = ent[p];
      pv[u] = (lane == 0 && p > 0) ? ent[p - 1] : 0;
    }
#pragma unroll
    for (int u = 0; u < kRunBatch; u++) {
      const int q = (j0 + u) * kBlock + t;
      const int32_t up = __shfl_up(v[u], 1);
      const int32_t prev = lane == 0 ? pv[u] : up;
      const bool h = q < tile_n && (base + q == 0 || v[u] != prev);
      const uint64_t m = __ballot(h);
      if (lane == 0) s_hb[(j0 + u) * kWaves + w] = m;  // positions 64 ((j0 + u) kWaves + w) + [0, 64)
    }
  }
  __syncthreads();
  const uint32_t heads = reinterpret_cast<const uint32_t*>(s_hb)[t];  // blocked positions 32t .. 32t+31
  uint64_t tot;
  const uint64_t ex = block_exclusive_scan<uint64_t>((uint64_t)__popc(heads), &tot, s_scan);  // has barriers
  const int64_t ebase = (int64_t)tile_off - 1;
  *my_heads = heads;
  *my_ex = (uint32_t)ex;
  *n_heads = (uint32_t)tot;  // the tile's last run has local id n_heads
  if (!(t & 1)) s_wpre[t >> 1] = (uint16_t)ex;  // thread 2i starts word i (kKItems == 32)
  if (ent_start) {
    const int q0 = t * kKItems;
    for (uint32_t hb = heads; hb; hb &= hb - 1) {
      const int j = __ffs(hb) - 1;
      ent_start[ebase + (uint32_t)ex + (uint32_t)__popc(heads & ((2u << j) - 1u))] = base + q0 + j;
    }
  }
  __syncthreads();
  return ebase;
}

// The local run id of tile position q (tile_run_ids' convention) from the head bits: the heads
// before q's 64-position word plus those of the word at positions <= q.
__device__ __forceinline__ uint32_t loc_of(int q, const uint64_t* s_hb, const uint16_t* s_wpre) {
  const uint64_t m = s_hb[q >> 6];
  const int bit = q & 63;
  return (uint32_t)s_wpre[q >> 6] + (uint32_t)__popcll(bit == 63 ? m : (m & ((2ull << bit) - 1ull)));
}

// ---- the first partition level, planned before the key pass (bucket.h) ----
// Level-0 segments are entities of more than kBigCap records (k_bucket_level0).  Their first
// partition level is planned from the entity and k1 columns alone, so that the key pass writes
// every payload of a segment straight into its level-1 child instead of writing it in input order
// for k_bucket_scatter to move once more (aggregator.py:264, 300-303: the molecule and fragment
// Counters this grouping serves):
//   k_level1_plan      per key-pass tile: run ids (ent_start), each record's level-1 digit counted
//                      per (entity, digit) in l1.hist (the children's sizes), and the tile's range
//                      inside every child it feeds, reserved with one atomic per (slot, digit): l1.toff;
//   k_bucket_classify  (level 1) turns l1.hist into the children's starts, in place, marked kL1Seg;
//   k_build_keys_run   ranks each segment record inside its tile's range with one LDS atomic.
// Only runs that can be segments get a slot: the tile's first and last runs and the runs of more
// than kBigCap records inside it (at most two: a tile holds kKTile < 3 (kBigCap + 1) records).
// The digit is the top kRadixBits of key' = [k1' | k2 | hash]; the host takes this path when they
// come from k1' alone (k1 >= kRadixBits bits): digit = k1' >> (k1 - kRadixBits).
constexpr int kL1Slots = 4;
constexpr uint32_t kL1NoSlot = 0xffffu;
constexpr uint32_t kL1Seg = kL1SegMark;  // l1.hist entry of a classified segment: child start | kL1Seg
static_assert(kKTile < 3 * (kBigCap + 1) + 2, "at most two inner segment runs per key-pass tile");
struct L1Plan {
  uint32_t* hist;  // [entity][kRadix] (nullptr: payloads are written in input order)
  uint32_t* toff;  // [tile][kL1Slots][kRadix]: the tile's offset inside each child it feeds
  uint2* tslot;    // [tile]: the slots' local run ids, 16 bits each (kL1NoSlot: none)
  Pay* pay_b;      // the level-1 children's buffer (B)
};
__device__ __forceinline__ uint32_t l1_slot_loc(uint2 ts, int k) {
  return ((k < 2 ? ts.x : ts.y) >> (16 * (k & 1))) & 0xffffu;
}

template <int kN>
__device__ __forceinline__ int slot_of(uint32_t loc, const uint32_t (&sl)[kN]) {
  int r = -1;
#pragma unroll
  for (int k = kN - 1; k >= 0; k--) r = loc == sl[k] ? k : r;
  return r;
}

__global__ void __launch_bounds__(kBlock) k_level1_plan(const int32_t* __restrict__ ent, const int32_t* __restrict__ k1col,
                                                        uint32_t n_k1, int64_t n, const uint64_t* __restrict__ tile_off,
                                                        Bits b, int dshift, int64_t* __restrict__ ent_start,
                                                        L1Plan l1) {
  __shared__ uint64_t s_scan[kWaves + 1];
  __shared__ uint64_t s_hb[kKTile / 64];
  __shared__ uint16_t s_wpre[kKTile / 64];
  __shared__ uint32_t s_h[kL1Slots * kRadix];
  __shared__ uint32_t s_slot[kL1Slots];
  __shared__ uint32_t s_nmid;
  static_assert(kBlock == kRadix, "one thread per digit");
  const int t = threadIdx.x;
  const int64_t base = (int64_t)blockIdx.x * kKTile;
  const int tile_n = (int)((n - base) < kKTile ? (n - base) : kKTile);
  for (int i = t; i < kL1Slots * kRadix; i += kBlock) s_h[i] = 0;
  if (t < kL1Slots) s_slot[t] = kL1NoSlot;
  if (t == 0) s_nmid = 0;
  uint32_t heads, ex, n_heads;  // (tile_run_ids' barriers publish the initialisation above)
  const int64_t ebase = tile_run_ids(ent, base, tile_n, tile_off[(size_t)blockIdx.x * kKTilesPerBlock], s_hb,
                                     s_scan, ent_start, &heads, &ex, &n_heads, s_wpre);
  const uint32_t first = loc_of(0, s_hb, s_wpre);  // the run at the tile's first position
  // inner runs with more than kBigCap records in the tile: head h and position h + kBigCap in one run
  for (uint32_t hb = heads; hb; hb &= hb - 1) {
    const int j = __ffs(hb) - 1;
    const uint32_t l = ex + (uint32_t)__popc(heads & ((2u << j) - 1u));
    const int h = t * kKItems + j;
    if (l != first && l != n_heads && h + kBigCap < tile_n && loc_of(h + kBigCap, s_hb, s_wpre) == l) {
      const uint32_t k = atomicAdd(&s_nmid, 1u);
      if (k < kL1Slots - 2) s_slot[1 + k] = l;
    }
  }
  if (t == 0) {
    s_slot[0] = first;
    if (n_heads != first) s_slot[kL1Slots - 1] = n_heads;
  }
  __syncthreads();
  uint32_t sl[kL1Slots];
#pragma unroll
  for (int k = 0; k < kL1Slots; k++) sl[k] = s_slot[k];
  for (int j0 = 0; j0 < kKItems; j0 += kRunBatch) {  // striped, loads of kRunBatch rounds in flight
    uint32_t v[kRunBatch];
#pragma unroll
    for (int u = 0; u < kRunBatch; u++) {
      const int q = (j0 + u) * kBlock + t;
      v[u] = (uint32_t)k1col[base + (q < tile_n ? q : 0)];
    }
    // round 4: a wave whose positions in this batch lie in one run (the common case: runs are cells
    // of thousands of records) takes that run's slot once, not per record (as the key pass does)
    const int wo = t & ~(kWave - 1);
    const int lo = j0 * kBlock + wo, hi = (j0 + kRunBatch - 1) * kBlock + wo + kWave - 1;
    int ku = -2;  // the wave's uniform slot (-1: none), or -2: per record
    if (hi < tile_n) {
      const uint32_t llo = loc_of(lo, s_hb, s_wpre), lhi = loc_of(hi, s_hb, s_wpre);
      if (__builtin_amdgcn_readfirstlane((int)llo) == __builtin_amdgcn_readfirstlane((int)lhi))
        ku = slot_of(__builtin_amdgcn_readfirstlane((int)llo), sl);
    }
    if (ku >= 0) {
      uint32_t* h = &s_h[ku * kRadix];
#pragma unroll
      for (int u = 0; u < kRunBatch; u++) {
        const uint32_t k1 = v[u] < n_k1 ? v[u] : 0u;  // the key pass's rule for an invalid id
        atomicAdd(&h[b.scramble(k1) >> dshift], 1u);
      }
    } else if (ku == -2) {
#pragma unroll
      for (int u = 0; u < kRunBatch; u++) {
        const int q = (j0 + u) * kBlock + t;
        if (q >= tile_n) continue;
        const uint32_t k1 = v[u] < n_k1 ? v[u] : 0u;
        const int k = slot_of(loc_of(q, s_hb, s_wpre), sl);
        if (k >= 0) atomicAdd(&s_h[k * kRadix + (b.scramble(k1) >> dshift)], 1u);
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kL1Slots; k++) {
    const uint32_t c = s_h[k * kRadix + t];
    if (sl[k] != kL1NoSlot && c)
      l1.toff[((size_t)blockIdx.x * kL1Slots + k) * kRadix + t] =
          atomicAdd(&l1.hist[(size_t)(ebase + sl[k]) * kRadix + t], c);
  }
  if (t == 0) l1.tslot[blockIdx.x] = make_uint2(sl[0] | (sl[1] << 16), sl[2] | (sl[3] << 16));
}

// Exact-lane increments of RN(a / B) for one denominator B per barcode stream and tile (the tile's
// first record's): a sample with that denominator adds 8 table words instead of computing them
// (fx_increments).  Barcode lengths are fixed in a chemistry; any other denominator is computed
// in place (a rare divergent branch).  Table entries are computed with the same ratio_y /
// fx_increments as the computed samples, so the lanes are bit-identical either way.  The genomic
// streams keep the arithmetic: soft-clipped reads change gq_len on ~1 record in 8, so a wave would
// run both paths every round.
constexpr int kTabU8 = 32;  // uy / cy (uint8 lengths): a = 0 .. 31
constexpr int kTabN = 2 * kTabU8;
constexpr uint32_t kNoTab = 0xffffffffu;
struct StreamTabs {
  uint4 inc[kTabN][2];  // the 8 lane increments of a (inc7 < 2^32: a <= B means x <= 1)
  uint32_t den[2];      // per table (uy, cy): the tabulated denominator, or kNoTab
};
static_assert(kTabN <= kBlock, "one entry per thread");

template <bool kCell>
__device__ __forceinline__ void fill_stream_tabs(const RecCols& r, int64_t base, StreamTabs* s) {
  const int t = threadIdx.x;
  if (t >= kTabN) return;
  const int tb = t / kTabU8;
  const uint32_t a = (uint32_t)(t % kTabU8);
  const uint32_t B = tb == 0 ? (uint32_t)r.uy_len[base] : (kCell ? (uint32_t)r.cy_len[base] : 0u);
#ifndef SCT_TAB_MASK
#define SCT_TAB_MASK 3  // experiments: which tables are used (bit 0 uy, bit 1 cy)
#endif
  const bool on = B < (uint32_t)kTabU8 && (kCell || tb == 0) && ((SCT_TAB_MASK >> tb) & 1);
  if (a == 0) s->den[tb] = on ? B : kNoTab;
  const double x = (on && B != 0 && a <= B) ? ratio_y(a, B, 1.0 / (double)B) : 0.0;  // = ratio_rcp(a, B)
  uint32_t inc[kStreamLanes - 1];
  uint64_t inc7;
  fx_increments(x, inc, inc7);
  s->inc[t][0] = make_uint4(inc[0], inc[1], inc[2], inc[3]);
  s->inc[t][1] = make_uint4(inc[4], inc[5], inc[6], (uint32_t)inc7);
}

// The exact fixed-point lanes of the quality streams for one tile: blocked items (kItems
// consecutive records per thread, two halves of the thread's kKItems) with 16-byte vector loads;
// the streams are summed one after another so only 8 lanes are live per thread.  Runs come from
// the thread's head mask (tile_run_ids: `heads`, `ex`), not from LDS: a half whose wave holds no
// run boundary (almost all of them: runs are cells of thousands of records) sums its 16 samples
// with no flush test at all.
// gwide (gene view): set when an operand exceeds the narrow gene payload (gene.h gene_payload8).
template <bool kCell>
__device__ __forceinline__ void stream_tile(const RecCols& r, int64_t base, int tile_n, uint32_t heads, uint32_t ex,
                                            int64_t ebase, const double* s_rcp, const StreamTabs* s_tab,
                                            int64_t* __restrict__ partials, uint32_t* __restrict__ gwide) {
  const int t = threadIdx.x;
  constexpr int ns = kCell ? 4 : 3;
  // numerator / denominator columns of half h of stream st: items q0 .. q0 + kItems - 1 of the thread's kKItems
  // (zeros past the tile: a zero sample adds nothing)
  const auto load = [&](int st, int h, uint32_t (&wn)[8], uint32_t (&wd)[8]) {
    const int q0 = t * kKItems + h * kItems;
    const int64_t p0 = base + q0;
    const bool full = q0 + kItems <= tile_n;
    const void* num = st == 0 ? (const void*)r.uy_gt30 : st == 1 ? (const void*)r.gq_gt30
                    : st == 2 ? (const void*)r.gq_sum : (const void*)r.cy_gt30;
    const void* den = st == 0 ? (const void*)r.uy_len : (st == 1 || st == 2) ? (const void*)r.gq_len
                    : (const void*)r.cy_len;
    const bool wide = (st == 1 || st == 2);  // uint16 columns
    if (full) {
      if (wide) {
        const uint4 a0 = reinterpret_cast<const uint4*>((const uint16_t*)num + p0)[0];
        const uint4 a1 = reinterpret_cast<const uint4*>((const uint16_t*)num + p0)[1];
        const uint4 b0 = reinterpret_cast<const uint4*>((const uint16_t*)den + p0)[0];
        const uint4 b1 = reinterpret_cast<const uint4*>((const uint16_t*)den + p0)[1];
        wn[0] = a0.x, wn[1] = a0.y, wn[2] = a0.z, wn[3] = a0.w, wn[4] = a1.x, wn[5] = a1.y, wn[6] = a1.z, wn[7] = a1.w;
        wd[0] = b0.x, wd[1] = b0.y, wd[2] = b0.z, wd[3] = b0.w, wd[4] = b1.x, wd[5] = b1.y, wd[6] = b1.z, wd[7] = b1.w;
      } else {
        const uint4 a0 = *reinterpret_cast<const uint4*>((const uint8_t*)num + p0);
        const uint4 b0 = *reinterpret_cast<const uint4*>((const uint8_t*)den + p0);
        wn[0] = a0.x, wn[1] = a0.y, wn[2] = a0.z, wn[3] = a0.w, wn[4] = wn[5] = wn[6] = wn[7] = 0;
        wd[0] = b0.x, wd[1] = b0.y, wd[2] = b0.z, wd[3] = b0.w, wd[4] = wd[5] = wd[6] = wd[7] = 0;
      }
    } else {
#pragma unroll
      for (int k = 0; k < 8; k++) wn[k] = wd[k] = 0;
#pragma unroll
      for (int j = 0; j < kItems; j++) {
        const bool ok = q0 + j < tile_n;
        const uint32_t a = !ok ? 0u : wide ? ((const uint16_t*)num)[p0 + j] : ((const uint8_t*)num)[p0 + j];
        const uint32_t d = !ok ? 0u : wide ? ((const uint16_t*)den)[p0 + j] : ((const uint8_t*)den)[p0 + j];
        if (wide) {
          wn[j / 2] |= a << (16 * (j % 2));
          wd[j / 2] |= d << (16 * (j % 2));
        } else {
          wn[j / 4] |= a << (8 * (j % 4));
          wd[j / 4] |= d << (8 * (j % 4));
        }
      }
    }
  };
  // a thread with no position in the tile holds no run (its lanes stay zero and never flush)
  const bool mine = t * kKItems < tile_n;
  int64_t lanes[kStreamLanes];
  int64_t cur_e = -1;
  // a stream's lanes run over both halves and are flushed once.  (Loading the next half's columns
  // before summing this one costs 16 VGPRs: the kernel then runs at 4 waves per SIMD instead of 5,
  // 1.34 against 1.25 ms)
  uint32_t wn[8], wd[8];
  uint32_t over = 0;  // operand bits above the narrow payload's fields (uy 5 bits, gq 9, gq_sum 15)
#pragma unroll 1
  for (int sh = 0; sh < 2 * ns; sh++) {
    const int st = sh >> 1, h = sh & 1;
    const bool wide = (st == 1 || st == 2);
    load(st, h, wn, wd);
    if (h == 0) {
#pragma unroll
      for (int i = 0; i < kStreamLanes; i++) lanes[i] = 0;
      cur_e = mine ? ebase + (int64_t)ex + (int64_t)(heads & 1u) : -1;  // the run of the thread's first position
    }
    {  // on the packed columns: uy (u8) above 31, gq_gt30 / gq_len (u16) above 511, gq_sum above 32767
      const uint32_t m = st == 0 ? 0xE0E0E0E0u : st == 1 ? 0xFE00FE00u : st == 2 ? 0x80008000u : 0u;
      uint32_t o = 0;
#pragma unroll
      for (int k = 0; k < 8; k++) o |= wn[k] | (st < 2 ? wd[k] : 0u);
      over |= o & m;
    }
    const int slot0 = P_FLOAT + st * kStreamLanes;
    const auto slot = [slot0](int i) { return slot0 + i; };
    const int tb = st == 0 ? 0 : st == 3 ? 1 : -1;
    const uint32_t B = tb >= 0 ? s_tab->den[tb] : kNoTab;  // block-uniform
    const uint4* tab = &s_tab->inc[tb >= 0 ? tb * kTabU8 : 0][0];
    const auto sample = [&](int j) {
      const uint32_t a = wide ? (wn[j / 2] >> (16 * (j % 2))) & 0xffffu : (wn[j / 4] >> (8 * (j % 4))) & 0xffu;
      const uint32_t d = wide ? (wd[j / 2] >> (16 * (j % 2))) & 0xffffu : (wd[j / 4] >> (8 * (j % 4))) & 0xffu;
      if (B != kNoTab && d == B && a <= B) {
        const uint4 i0 = tab[2 * a], i1 = tab[2 * a + 1];
        lanes[0] += i0.x, lanes[1] += i0.y, lanes[2] += i0.z, lanes[3] += i0.w;
        lanes[4] += i1.x, lanes[5] += i1.y, lanes[6] += i1.z, lanes[7] += i1.w;
      } else {
        fx_accumulate(lanes, ratio_rcp(a, d, s_rcp));
      }
    };
    // run changes inside this half: head bits of its positions (the first position of the thread
    // opened cur_e already)
    const uint32_t ch = ((heads >> (h * kItems)) & ((1u << kItems) - 1u)) & (h == 0 ? ~1u : ~0u);
    if (!__ballot(ch != 0)) {
#pragma unroll
      for (int j = 0; j < kItems; j++) sample(j);
    } else {
      // a run boundary inside the thread's own items: only this thread's lanes change runs, so it
      // adds them to the ending run's row by itself (8 atomics, no wave-wide reduction per item)
#pragma unroll
      for (int j = 0; j < kItems; j++) {
        if ((ch >> j) & 1u) {
#pragma unroll
          for (int i = 0; i < kStreamLanes; i++) {
            atomicAdd((unsigned long long*)&partials[cur_e * SCT_NP + slot(i)], (unsigned long long)lanes[i]);
            lanes[i] = 0;
          }
          cur_e += 1;
        }
        sample(j);
      }
    }
    if (h == 1) wave_flush<kStreamLanes>(lanes, cur_e >= 0, cur_e, partials, slot);
  }
  if (gwide && __ballot(over != 0) && (threadIdx.x & (kWave - 1)) == 0) atomicOr(gwide, 1u);
}

// kBucket: write the bucket path's 16-byte payload (bucket.h: w0 = key' | ref | strand |
// mapped, w1 = index | pos; a mapped ref id >= 2^kRefBits raises *err): a segment's record (l1.hist
// set: the first partition level planned by k_level1_plan) into its level-1 child in buffer B, any
// other record at its own position in buffer A.  Otherwise the global sort's (key with entity
// bits, u32 value with bit 31 = unmapped).
// Segment records are staged per batch of kKeyBatch rounds (kStage records): ranked in LDS by
// (batch slot, digit), placed in child order, and written out as contiguous runs per child -- a
// wave's store then covers a few runs instead of 64 scattered lines.  A batch holds at most two
// segment runs (its first and its last: a run inside it has < kStage <= kBigCap records).
// kStreams: also the exact quality-stream lanes of the runs (stream_tile), reusing the tile's
// run ids: the stream ALU work overlaps the key pass's memory traffic in one launch.
constexpr int kKeyBatch = 4;  // striped rounds whose column loads are issued together (8: occupancy 3, slower)
constexpr int kStage = kKeyBatch * kBlock;
static_assert(kKItems % kKeyBatch == 0, "whole batches");
static_assert(kStage <= kBigCap, "a run inside a batch is never a segment");
static_assert(kStage < (1 << 16), "16-bit ranks");
constexpr uint32_t kDirect = 0xffffffffu;

template <bool kCell, bool kGene, bool kBucket, bool kStreams>
// 5 waves per SIMD (<= 96 VGPRs)
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(5))) k_build_keys_run(KeyCols c, RecCols r, const uint8_t* __restrict__ k1_is_mito,
                                                           int64_t n, const uint64_t* __restrict__ tile_off, Bits b,
                                                           uint64_t* __restrict__ keys, void* __restrict__ vals,
                                                           int64_t* __restrict__ ent_start,
                                                           int64_t* __restrict__ partials,
                                                           uint32_t* __restrict__ gene_counts, int n_buckets,
                                                           uint32_t* __restrict__ err, uint32_t* __restrict__ gwide,
                                                           uint32_t* __restrict__ gtoff, L1Plan l1) {
  static_assert(!kGene || kCell, "gene buckets come from the cell view");
  __shared__ uint64_t s_scan[kWaves + 1];
  __shared__ uint64_t s_hb[kKTile / 64];      // tile_run_ids' head bits
  __shared__ uint16_t s_wpre[kKTile / 64];    // heads before each word of s_hb (loc_of)
  using TabT = typename std::conditional<kStreams, StreamTabs, uint32_t>::type;
  __shared__ TabT s_tab_[1];
  StreamTabs* s_tab = reinterpret_cast<StreamTabs*>(s_tab_);
  uint32_t* s_hist = sct_dyn_lds;  // kGene: n_buckets counters (dynamic LDS)
  __shared__ double s_rcp[kStreams ? kRcpN : 1];
  const int t = threadIdx.x;
  const int64_t base = (int64_t)blockIdx.x * kKTile;
  const int tile_n = (int)((n - base) < kKTile ? (n - base) : kKTile);
  if (kGene)
    for (int i = t; i < n_buckets; i += kBlock) s_hist[i] = 0;
  if constexpr (kStreams) {  // visible after tile_run_ids' barriers
    fill_rcp(s_rcp);
    fill_stream_tabs<kCell>(r, base, s_tab);
  }
  // level-1 children (l1.hist set): per slot whose run is a segment, the next position of each
  // child inside this tile's range; s_lslot = the slot's local run id, or kL1NoSlot.  A batch's
  // staging: s_bc counts, then child-order starts, per (batch slot, digit); s_gd the distance from
  // a staged position to its destination.
  constexpr int kL1 = kBucket ? 1 : 0;
  __shared__ uint32_t s_pos[kL1 ? kL1Slots * kRadix : 1];
  __shared__ uint32_t s_lslot[kL1Slots];
  __shared__ Pay s_stage[kL1 ? kStage : 1];
  __shared__ uint32_t s_bc[kL1 ? 2 * kRadix : 1];
  __shared__ uint32_t s_gd[kL1 ? 2 * kRadix : 1];
  const int KB = b.k1 + b.k2 + b.h;
  const int bits1 = KB < kRadixBits ? KB : kRadixBits;
  const int sh1 = KB - bits1;
  const uint32_t dmask = (1u << bits1) - 1u;
  const uint64_t tile_off0 = tile_off[(size_t)blockIdx.x * kKTilesPerBlock];
  const bool planned = kBucket && l1.hist != nullptr;  // uniform
  if constexpr (kBucket) {
    if (planned) {
      static_assert(kBlock == kRadix, "one thread per digit");
      const uint2 ts = l1.tslot[blockIdx.x];
#pragma unroll
      for (int k = 0; k < kL1Slots; k++) {
        const uint32_t l = l1_slot_loc(ts, k);
        bool seg = false;
        if (l != kL1NoSlot) {
          const uint32_t v = l1.hist[(size_t)((int64_t)tile_off0 - 1 + l) * kRadix + t];
          seg = (v & kL1Seg) != 0;  // every digit of a classified segment carries the mark
          if (seg) s_pos[k * kRadix + t] = (v & ~kL1Seg) + l1.toff[((size_t)blockIdx.x * kL1Slots + k) * kRadix + t];
        }
        if (t == 0) s_lslot[k] = seg ? l : kL1NoSlot;
      }
      s_bc[t] = 0;
      s_bc[kRadix + t] = 0;
    }
  }
  // 1-2. run index of every record of the tile
  uint32_t my_heads, my_ex, n_heads;
  const int64_t ebase = tile_run_ids(c.ent, base, tile_n, tile_off0, s_hb, s_scan, planned ? nullptr : ent_start,
                                     &my_heads, &my_ex, &n_heads, s_wpre);
  uint32_t lsl[kL1Slots];
#pragma unroll
  for (int k = 0; k < kL1Slots; k++) lsl[k] = planned ? s_lslot[k] : kL1NoSlot;

  // 3. striped pass: keys, values and the run's additive metrics.  Runs are contiguous, so
  // in a round the wave's lanes cross a run boundary together: flush wave-cooperatively.
  using A = AddAcc<kCell>;
  A acc;
  acc.clear();
  int64_t cur_e = -1;
  const auto slot = [](int i) { return A::slot(i); };
  // The columns of kKeyBatch rounds are loaded together (clamped, unconditional loads: all in
  // flight at once), then the rounds are processed: the wait for memory is paid once per batch.
  for (int j0 = 0; j0 < kKItems; j0 += kKeyBatch) {
    const int qlo = j0 * kBlock;
    if (qlo >= tile_n) break;  // block-uniform
    int32_t vk1[kKeyBatch], vk2[kKeyBatch], vref[kKeyBatch], vpos[kKeyBatch];
    uint8_t vbt[kKeyBatch], vxf[kKeyBatch];
#pragma unroll
    for (int u = 0; u < kKeyBatch; u++) {
      const int q = (j0 + u) * kBlock + t;
      const int64_t p = base + (q < tile_n ? q : 0);
      vk1[u] = c.k1[p];
      vk2[u] = c.k2[p];
      vbt[u] = r.bits[p];
      vxf[u] = r.xf[p];
      vref[u] = r.ref[p];
      vpos[u] = r.pos[p];
    }
    // One run across the wave's batch: the run ids of its lowest position (the lanes' previous
    // round) and its highest agree (wave-uniform LDS reads): no per-record run id or flush test.
    bool one_run = false;
#ifndef SCT_KEY_FASTPATH
#define SCT_KEY_FASTPATH 1
#endif
    if (SCT_KEY_FASTPATH && tile_n == kKTile) {  // block-uniform
      const int wo = t & ~(kWave - 1) & (kBlock - 1);
      const int lo = (j0 == 0 ? 0 : (j0 - 1) * kBlock) + wo;
      const int hi = (j0 + kKeyBatch - 1) * kBlock + wo + kWave - 1;
      const int elo = __builtin_amdgcn_readfirstlane((int)loc_of(lo, s_hb, s_wpre));
      const int ehi = __builtin_amdgcn_readfirstlane((int)loc_of(hi, s_hb, s_wpre));
      one_run = elo == ehi;
      if (one_run) cur_e = ebase + elo;
    }
    // the batch's segment runs (block-uniform): its first and its last run, if segments
    uint32_t blo = kL1NoSlot, bhi = kL1NoSlot;
    int bs0 = -1, bs1 = -1;
    if (planned) {
      const int qhi = (qlo + kStage < tile_n ? qlo + kStage : tile_n) - 1;
      blo = loc_of(qlo, s_hb, s_wpre);
      bhi = loc_of(qhi, s_hb, s_wpre);
      bs0 = slot_of(blo, lsl);
      bs1 = bhi != blo ? slot_of(bhi, lsl) : -1;
    }
    const bool stage = bs0 >= 0 || bs1 >= 0;
    uint32_t rk[kKeyBatch];  // staged records: batch slot << 16 | rank in (slot, digit); else kDirect
    uint32_t t0 = 0, n_staged = 0;
    if constexpr (kBucket) {
      if (stage) {
#pragma unroll
        for (int u = 0; u < kKeyBatch; u++) {
          const int q = (j0 + u) * kBlock + t;
          rk[u] = kDirect;
          if (q >= tile_n) continue;
          const uint32_t loc = one_run ? (uint32_t)(cur_e - ebase) : loc_of(q, s_hb, s_wpre);
          const int ls = (loc == blo && bs0 >= 0) ? 0 : (loc == bhi && bs1 >= 0) ? 1 : -1;
          if (ls < 0) continue;
          const uint32_t k1 = (uint32_t)vk1[u] < c.n_k1 ? (uint32_t)vk1[u] : 0u;  // (the rule below)
          const uint32_t dg = (uint32_t)(((uint64_t)b.scramble(k1) << (b.k2 + b.h)) >> sh1) & dmask;
          rk[u] = ((uint32_t)ls << 16) | atomicAdd(&s_bc[ls * kRadix + dg], 1u);
        }
        __syncthreads();
        // child-order starts per (batch slot, digit); the tile's child positions advance
        const uint32_t c0 = s_bc[t], c1 = s_bc[kRadix + t];
        uint64_t tot;
        const uint64_t ex = block_exclusive_scan<uint64_t>((uint64_t)c0 | ((uint64_t)c1 << 32), &tot, s_scan);
        t0 = (uint32_t)tot;
        n_staged = t0 + (uint32_t)(tot >> 32);
        const uint32_t st0 = (uint32_t)ex, st1 = t0 + (uint32_t)(ex >> 32);
        s_bc[t] = st0;
        s_bc[kRadix + t] = st1;
        if (c0) {  // thread t alone owns digit t of the batch's slots
          const uint32_t g = s_pos[bs0 * kRadix + t];
          s_pos[bs0 * kRadix + t] = g + c0;
          s_gd[t] = g - st0;
        }
        if (c1) {
          const uint32_t g = s_pos[bs1 * kRadix + t];
          s_pos[bs1 * kRadix + t] = g + c1;
          s_gd[kRadix + t] = g - st1;
        }
        __syncthreads();
      }
    }
#pragma unroll
    for (int u = 0; u < kKeyBatch; u++) {
      const int q = (j0 + u) * kBlock + t;
      const bool valid = q < tile_n;
      const int64_t p = base + q;
      int64_t e = cur_e;
      if (!one_run) {
        e = valid ? ebase + (int64_t)loc_of(q, s_hb, s_wpre) : cur_e;
#ifndef SCT_PACKED_FLUSH
#define SCT_PACKED_FLUSH 1
#endif
        if (SCT_PACKED_FLUSH)  // per-lane counts <= kKItems between flushes: 16-bit fields suffice
          wave_flush_packed16<A::kK>(acc.v, valid && e != cur_e && cur_e >= 0, cur_e, partials, slot);
        else
          wave_flush<A::kK>(acc.v, valid && e != cur_e && cur_e >= 0, cur_e, partials, slot);
        if (!valid) continue;
        cur_e = e;
      }
      uint32_t k1 = (uint32_t)vk1[u];
      uint32_t k2 = (uint32_t)vk2[u];
      if (k1 >= c.n_k1 || k2 >= c.n_k2) {  // invalid input: reported, never used as an index
        atomicOr(err, 2u);
        k1 = k1 < c.n_k1 ? k1 : 0u;  // (k_level1_plan applies the same rule to k1)
        k2 = k2 < c.n_k2 ? k2 : 0u;
      }
      const uint8_t bt = vbt[u];
      const uint8_t xf = vxf[u];
      const bool mapped = !(bt & SCT_B_UNMAPPED);
      const int32_t ref = vref[u];
      const int32_t pos = vpos[u];
      const bool rev = bt & SCT_B_REVERSE;
      const uint32_t hsh = mapped ? frag_hash(ref, pos, rev ? 1u : 0u) : 0u;
      if constexpr (kBucket) {
        const bool mito = kCell ? k1_is_mito[k1] != 0 : false;
        const uint64_t kp = make_key(0, k1, k2, hsh, b);
        const Pay x{payload_w0(kp, ref, rev, mapped, mito), ((uint64_t)p << 32) | (uint32_t)pos};
        if (stage && rk[u] != kDirect) {
          const uint32_t ls = rk[u] >> 16;
          const uint32_t dg = (uint32_t)(kp >> sh1) & dmask;
          s_stage[s_bc[ls * kRadix + dg] + (rk[u] & 0xffffu)] = x;
        } else {
          reinterpret_cast<Pay*>(keys)[p] = x;  // (the bucket path's keys are payload buffer A)
        }
        if (mapped && (uint32_t)ref >= (1u << kRefBits)) atomicOr(err, 1u);
      } else {
        keys[p] = make_key((uint64_t)e, k1, k2, hsh, b);
        static_cast<uint32_t*>(vals)[p] = (uint32_t)p | (mapped ? 0u : kUnmappedValBit);
      }
      if (kGene) atomicAdd(&s_hist[k1 / kGenesPerBucket], 1u);
      // MetricAggregator.parse_molecule (aggregator.py:259-334)
      acc.v[0] += 1;
      acc.v[1] += (bt & SCT_B_PERFECT_UMI) ? 1 : 0;
      if (mapped) {
        const bool nh1 = bt & SCT_B_NH1;
        acc.v[2] += (xf == SCT_XF_CODING);
        acc.v[3] += (xf == SCT_XF_INTRONIC);
        acc.v[4] += (xf == SCT_XF_UTR);
        acc.v[5] += nh1 ? 1 : 0;
        acc.v[6] += nh1 ? 0 : 1;
        acc.v[7] += (bt & SCT_B_DUPLICATE) ? 1 : 0;
        acc.v[8] += (bt & SCT_B_SPLICED) ? 1 : 0;
      }
      if constexpr (kCell) {
        // CellMetrics.parse_extra_fields (aggregator.py:507-530) + mito reads (463-490)
        acc.v[9] += ((bt & SCT_B_HAS_CB) && (bt & SCT_B_PERFECT_CB)) ? 1 : 0;
        acc.v[10] += (xf == SCT_XF_INTERGENIC);
        acc.v[11] += (xf == SCT_XF_ABSENT);
        acc.v[12] += k1_is_mito[k1];
      }
    }
    if constexpr (kBucket) {
      if (stage) {  // the staged records, child by child (contiguous runs), to buffer B
        __syncthreads();
        s_bc[t] = 0;  // (the next batch's counters: every read of the starts is done)
        s_bc[kRadix + t] = 0;
        for (uint32_t q = t; q < n_staged; q += kBlock) {
          const Pay x = s_stage[q];
          const uint32_t dg = (uint32_t)(x.w0 >> (sh1 + kKeyShift)) & dmask;
          l1.pay_b[s_gd[(q >= t0 ? kRadix : 0) + dg] + q] = x;
        }
        __syncthreads();
      }
    }
  }
  if (SCT_PACKED_FLUSH)
    wave_flush_packed16<A::kK>(acc.v, cur_e >= 0, cur_e, partials, slot);
  else
    wave_flush<A::kK>(acc.v, cur_e >= 0, cur_e, partials, slot);
  if (kGene) {
    __syncthreads();
    // the tile's range in each present bucket: its offset inside the bucket (k_gene_emit)
    for (int i = t; i < n_buckets; i += kBlock)
      if (s_hist[i]) gtoff[(size_t)blockIdx.x * n_buckets + i] = atomicAdd(&gene_counts[i], s_hist[i]);
  }
  if constexpr (kStreams) stream_tile<kCell>(r, base, tile_n, my_heads, my_ex, ebase, s_rcp, s_tab, partials,
                                                 kGene ? gwide : nullptr);
}

}  // namespace sct
