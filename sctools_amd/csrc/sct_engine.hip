// sct_engine.hip -- MI355X (gfx950) per-cell / per-gene metric engine.
//
// Replaces the per-record Python loop of the reference
// (GatherCellMetrics / GatherGeneMetrics.extract_metrics, gatherer.py:116-232,
// driving MetricAggregator.parse_molecule, aggregator.py:236-334, and
// finalize, aggregator.py:342-387, 463-490, 571-578) with:
//
//   1. run segmentation of the entity column (bam.iter_tag_groups,
//      bam.py:492-540): a head-flag count per 4096-record tile, a scan of the
//      tile counts, and a tile-local scan that numbers the runs;
//   2. a packed 64-bit key per record, [entity | k1 | k2 | fragment hash]
//      (cell: k1 = gene, k2 = umi; gene: k1 = cell, k2 = umi), bits trimmed to
//      the dictionary sizes;
//   3. an LSD radix sort of (key, record index), 8-bit digits, LDS-staged
//      tiles with wave-level multi-split ranking (ballot-based match on the
//      64-lane wave) and coalesced bucket writes;
//   4. one pass over the sorted keys that turns key runs into the Counter
//      results (molecules = runs of [entity|k1|k2], k1 runs, fragment
//      first-occurrences inside a molecule's equal-hash sub-run) and sums every
//      per-record metric into int64 partial rows with integer atomics (exact,
//      so the result does not depend on scheduling);
//   5. finalize: ratios and the mean / variance of each stream, either from
//      exact fixed-point sums (SCT_FLOAT_EXACT_SUM, fixedpt.h) or by a
//      sequential Welford walk per entity in record order (SCT_FLOAT_WELFORD,
//      bit-identical to stats.py:82-99).
//
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -shared.
// -ffp-contract=off keeps every Welford operation separately rounded, as
// Python does.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <utility>
#include <vector>

#include "common.h"
#include "fixedpt.h"

using namespace sct;

namespace {

constexpr int kBlock = 256;
constexpr int kItems = 16;
constexpr int kTile = kBlock * kItems;  // 4096 records per tile
constexpr int kRadixBits = 8;
constexpr int kRadix = 1 << kRadixBits;
constexpr int kReduceItems = 8;
constexpr int kReduceTile = kBlock * kReduceItems;  // 2048 sorted positions per block
constexpr int kScanChunk = 4096;

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIPCHK(expr)                                                                      \
  do {                                                                                    \
    hipError_t _e = (expr);                                                               \
    if (_e != hipSuccess)                                                                 \
      return fail(SCT_EHIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__, \
                  __LINE__);                                                              \
  } while (0)

#define LAUNCHCHK() HIPCHK(hipGetLastError())

// ---- optional per-kernel timing with HIP events on the launch stream (sct_profile_*) ----
struct ProfEntry {
  std::string name;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;
};
thread_local bool g_prof = false;
thread_local std::vector<ProfEntry> g_prof_entries;

struct ProfScope {
  hipEvent_t a = nullptr, b = nullptr;
  hipStream_t s;
  const char* name;
  ProfScope(const char* n, hipStream_t st) : s(st), name(n) {
    if (g_prof && hipEventCreate(&a) == hipSuccess && hipEventCreate(&b) == hipSuccess) (void)hipEventRecord(a, s);
  }
  ~ProfScope() {
    if (!g_prof || !a || !b) return;
    (void)hipEventRecord(b, s);
    for (auto& e : g_prof_entries)
      if (e.name == name) {
        e.ev.emplace_back(a, b);
        return;
      }
    g_prof_entries.push_back(ProfEntry{name, {{a, b}}});
  }
};

#define LAUNCH(name, kern, grid, block, strm, ...)                      \
  do {                                                                  \
    ProfScope _ps(name, strm);                                          \
    hipLaunchKernelGGL(kern, grid, block, 0, strm, __VA_ARGS__);        \
  } while (0);                                                          \
  LAUNCHCHK()

inline int bitlen(uint64_t v) {  // bits for ids 0..v-1 (v>=1); 0 when v <= 1
  return v <= 1 ? 0 : 64 - __builtin_clzll(v - 1);
}

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ======================================================================================
// block-level helpers
// ======================================================================================

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
  for (int off = kWave / 2; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

// exclusive scan over the block (kBlock threads); returns the total in *total
template <typename T>
__device__ __forceinline__ T block_exclusive_scan(T v, T* total, T* lds /*kBlock/kWave + 1*/) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  // inclusive wave scan
  T x = v;
  for (int off = 1; off < kWave; off <<= 1) {
    T y = __shfl_up(x, off);
    if (lane >= off) x += y;
  }
  if (lane == kWave - 1) lds[wid] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    T run = 0;
    for (int w = 0; w < kBlock / kWave; w++) {
      T t = lds[w];
      lds[w] = run;
      run += t;
    }
    lds[kBlock / kWave] = run;
  }
  __syncthreads();
  T res = lds[wid] + x - v;
  *total = lds[kBlock / kWave];
  __syncthreads();
  return res;
}

// ======================================================================================
// device-wide exclusive scan of uint32 counts -> uint32 offsets (3 kernels)
// ======================================================================================

__global__ void k_scan_reduce(const uint32_t* __restrict__ in, int64_t m, uint64_t* __restrict__ sums) {
  const int64_t base = (int64_t)blockIdx.x * kScanChunk;
  uint64_t s = 0;
  for (int i = threadIdx.x; i < kScanChunk; i += kBlock) {
    const int64_t p = base + i;
    if (p < m) s += in[p];
  }
  __shared__ uint64_t red[kBlock / kWave];
  s = wave_sum(s);
  if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t t = 0;
    for (int w = 0; w < kBlock / kWave; w++) t += red[w];
    sums[blockIdx.x] = t;
  }
}

// single block: exclusive scan of m uint64 (in place), total -> out_total
__global__ void k_scan_small(uint64_t* __restrict__ data, int64_t m, uint64_t* __restrict__ out_total) {
  __shared__ uint64_t lds[kBlock / kWave + 1];
  uint64_t carry = 0;
  for (int64_t base = 0; base < m; base += kBlock) {
    const int64_t p = base + threadIdx.x;
    const uint64_t v = p < m ? data[p] : 0;
    uint64_t tot;
    const uint64_t ex = block_exclusive_scan<uint64_t>(v, &tot, lds);
    if (p < m) data[p] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0 && out_total) *out_total = carry;
}

__global__ void k_scan_apply(const uint32_t* __restrict__ in, int64_t m,
                             const uint64_t* __restrict__ block_off, uint32_t* __restrict__ out) {
  __shared__ uint64_t lds[kBlock / kWave + 1];
  const int64_t base = (int64_t)blockIdx.x * kScanChunk;
  uint64_t carry = block_off[blockIdx.x];
  // each thread owns kScanChunk / kBlock consecutive entries
  constexpr int per = kScanChunk / kBlock;
  uint32_t v[per];
  uint64_t s = 0;
  const int64_t p0 = base + (int64_t)threadIdx.x * per;
#pragma unroll
  for (int j = 0; j < per; j++) {
    const int64_t p = p0 + j;
    v[j] = p < m ? in[p] : 0;
    s += v[j];
  }
  uint64_t tot;
  uint64_t ex = block_exclusive_scan<uint64_t>(s, &tot, lds) + carry;
#pragma unroll
  for (int j = 0; j < per; j++) {
    const int64_t p = p0 + j;
    if (p < m) out[p] = (uint32_t)ex;
    ex += v[j];
  }
}

// ======================================================================================
// 1. run segmentation
// ======================================================================================

__global__ void k_heads(const int32_t* __restrict__ key, int64_t n, uint64_t* __restrict__ tile_cnt) {
  const int64_t base = (int64_t)blockIdx.x * kTile;
  uint64_t c = 0;
#pragma unroll 4
  for (int j = 0; j < kItems; j++) {
    const int64_t p = base + (int64_t)j * kBlock + threadIdx.x;
    if (p < n) c += (p == 0 || key[p] != key[p - 1]) ? 1 : 0;
  }
  __shared__ uint64_t red[kBlock / kWave];
  c = wave_sum(c);
  if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t t = 0;
    for (int w = 0; w < kBlock / kWave; w++) t += red[w];
    tile_cnt[blockIdx.x] = t;
  }
}

__device__ __forceinline__ uint32_t frag_hash(int32_t ref, int32_t pos, uint32_t strand) {
  uint32_t h = (uint32_t)ref * 0x9E3779B1u ^ ((uint32_t)pos * 0x85EBCA77u) ^ (strand * 0xC2B2AE3Du);
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  h *= 0x297A2D39u;
  h ^= h >> 15;
  return h;
}

struct KeyCols {
  const int32_t* ent;  // RUN: column whose runs are entities; GROUPED: entity id column
  const int32_t* k1;
  const int32_t* k2;
  const int32_t* ref;
  const int32_t* pos;
  const uint8_t* bits;
};

__device__ __forceinline__ uint64_t make_key(uint64_t e, uint32_t k1, uint32_t k2, uint32_t hash,
                                             const Bits& b) {
  const uint64_t hmask = b.h ? ((1ull << b.h) - 1) : 0;
  // the hash takes the TOP bits of the 32-bit mix
  const uint64_t hv = b.h ? ((uint64_t)(hash >> (32 - b.h)) & hmask) : 0;
  return (e << (b.k1 + b.k2 + b.h)) | ((uint64_t)k1 << (b.k2 + b.h)) | ((uint64_t)k2 << b.h) | hv;
}

// RUN modes: entity id = run index (needs the tile offsets of head counts)
__global__ void k_build_keys_run(KeyCols c, int64_t n, const uint64_t* __restrict__ tile_off, Bits b,
                                 uint64_t* __restrict__ keys, uint32_t* __restrict__ vals,
                                 int64_t* __restrict__ ent_start) {
  __shared__ uint64_t lds[kBlock / kWave + 1];
  const int64_t base = (int64_t)blockIdx.x * kTile;
  const int64_t p0 = base + (int64_t)threadIdx.x * kItems;
  int32_t kv[kItems];
  uint32_t heads = 0;
#pragma unroll
  for (int j = 0; j < kItems; j++) {
    const int64_t p = p0 + j;
    kv[j] = p < n ? c.ent[p] : 0;
  }
  int32_t prev = (p0 > 0 && p0 - 1 < n) ? c.ent[p0 - 1] : 0;
#pragma unroll
  for (int j = 0; j < kItems; j++) {
    const int64_t p = p0 + j;
    const bool h = p < n && (p == 0 || kv[j] != (j ? kv[j - 1] : prev));
    heads |= (h ? 1u : 0u) << j;
  }
  uint64_t tot;
  const uint64_t ex = block_exclusive_scan<uint64_t>((uint64_t)__popc(heads), &tot, lds);
  int64_t e = (int64_t)(tile_off[blockIdx.x] + ex) - 1;
#pragma unroll
  for (int j = 0; j < kItems; j++) {
    const int64_t p = p0 + j;
    if (p >= n) break;
    if (heads & (1u << j)) {
      e += 1;
      ent_start[e] = p;
    }
    const uint8_t bt = c.bits[p];
    const uint32_t hsh = (bt & SCT_B_UNMAPPED) ? 0u : frag_hash(c.ref[p], c.pos[p], (bt & SCT_B_REVERSE) ? 1u : 0u);
    keys[p] = make_key((uint64_t)e, (uint32_t)c.k1[p], (uint32_t)c.k2[p], hsh, b);
    vals[p] = (uint32_t)p;
  }
}

// GROUPED mode: entity id = the id column itself
__global__ void k_build_keys_grouped(KeyCols c, int64_t n, Bits b, uint64_t* __restrict__ keys,
                                     uint32_t* __restrict__ vals) {
  for (int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x; p < n; p += (int64_t)gridDim.x * kBlock) {
    const uint8_t bt = c.bits[p];
    const uint32_t hsh = (bt & SCT_B_UNMAPPED) ? 0u : frag_hash(c.ref[p], c.pos[p], (bt & SCT_B_REVERSE) ? 1u : 0u);
    keys[p] = make_key((uint64_t)(uint32_t)c.ent[p], (uint32_t)c.k1[p], (uint32_t)c.k2[p], hsh, b);
    vals[p] = (uint32_t)p;
  }
}

// ======================================================================================
// 3. LSD radix sort (key u64, value u32), 8-bit digits
// ======================================================================================

// per-tile digit histogram -> counts[digit * num_tiles + tile]
__global__ void k_radix_upsweep(const uint64_t* __restrict__ keys, int64_t n, int shift, int64_t num_tiles,
                                uint32_t* __restrict__ counts) {
  __shared__ uint32_t hist[kBlock / kWave][kRadix];
  const int wid = threadIdx.x / kWave;
  for (int i = threadIdx.x; i < (kBlock / kWave) * kRadix; i += kBlock) (&hist[0][0])[i] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kTile;
#pragma unroll 4
  for (int j = 0; j < kItems; j++) {
    const int64_t p = base + (int64_t)j * kBlock + threadIdx.x;
    if (p < n) atomicAdd(&hist[wid][(keys[p] >> shift) & (kRadix - 1)], 1u);
  }
  __syncthreads();
  for (int d = threadIdx.x; d < kRadix; d += kBlock) {
    uint32_t t = 0;
#pragma unroll
    for (int w = 0; w < kBlock / kWave; w++) t += hist[w][d];
    counts[(int64_t)d * num_tiles + blockIdx.x] = t;
  }
}

// stable scatter of one tile: wave-level multi-split ranking, LDS staging, coalesced writes
__global__ void __launch_bounds__(kBlock) k_radix_downsweep(
    const uint64_t* __restrict__ keys_in, const uint32_t* __restrict__ vals_in, uint64_t* __restrict__ keys_out,
    uint32_t* __restrict__ vals_out, int64_t n, int shift, int64_t num_tiles,
    const uint32_t* __restrict__ offsets) {
  constexpr int kWaves = kBlock / kWave;
  __shared__ uint64_t s_keys[kTile];
  __shared__ uint32_t s_vals[kTile];
  __shared__ uint32_t s_whist[kWaves][kRadix];
  __shared__ uint32_t s_dstart[kRadix];
  __shared__ uint64_t s_scan[kWaves + 1];

  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  const int64_t base = (int64_t)blockIdx.x * kTile;
  const int tile_n = (int)((n - base) < kTile ? (n - base) : kTile);

  for (int i = threadIdx.x; i < kWaves * kRadix; i += kBlock) (&s_whist[0][0])[i] = 0;
  __syncthreads();

  const uint64_t lt = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
  uint64_t k[kItems];
  uint32_t v[kItems];
  uint16_t rank[kItems];
  uint8_t dig[kItems];
  // wave `wid` owns tile positions [wid*kItems*kWave, (wid+1)*kItems*kWave), round j covers 64 of them
#pragma unroll
  for (int j = 0; j < kItems; j++) {
    const int q = wid * (kItems * kWave) + j * kWave + lane;
    const int64_t p = base + q;
    if (q < tile_n) {
      k[j] = keys_in[p];
      v[j] = vals_in[p];
    } else {
      k[j] = ~0ull;  // padding sorts last (digit 255 at every shift) and is never written
      v[j] = 0;
    }
    const uint32_t d = (uint32_t)(k[j] >> shift) & (kRadix - 1);
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
  // digit totals -> digit starts (exclusive), and per-wave prefixes inside each digit
  {
    const int d = threadIdx.x;  // kBlock == kRadix
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
  for (int j = 0; j < kItems; j++) {
    const uint32_t lp = s_whist[wid][dig[j]] + rank[j];
    s_keys[lp] = k[j];
    s_vals[lp] = v[j];
  }
  __syncthreads();
  for (int q = threadIdx.x; q < tile_n; q += kBlock) {
    const uint64_t kk = s_keys[q];
    const uint32_t d = (uint32_t)(kk >> shift) & (kRadix - 1);
    const uint64_t o = (uint64_t)offsets[(int64_t)d * num_tiles + blockIdx.x] + (uint32_t)(q - (int)s_dstart[d]);
    keys_out[o] = kk;
    vals_out[o] = s_vals[q];
  }
}

// ======================================================================================
// 4. reduction over the sorted keys
// ======================================================================================

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

__device__ __forceinline__ double ratio(uint32_t a, uint32_t b) {
  return b ? (double)a / (double)b : 0.0;
}

template <bool kCell, bool kExact>
struct Acc {
  int32_t c[P_NCOUNT];
  int64_t l[kExact ? kStreams * kStreamLanes : 1];
  __device__ __forceinline__ void clear() {
#pragma unroll
    for (int i = 0; i < P_NCOUNT; i++) c[i] = 0;
    if (kExact) {
#pragma unroll
      for (int i = 0; i < kStreams * kStreamLanes; i++) l[i] = 0;
    }
  }
  __device__ __forceinline__ void flush(int64_t* __restrict__ row) const {
#pragma unroll
    for (int i = 0; i < P_NCOUNT; i++)
      if (c[i]) atomicAdd((unsigned long long*)&row[i], (unsigned long long)(int64_t)c[i]);
    if (kExact) {
      constexpr int ns = kCell ? 4 : 3;
#pragma unroll
      for (int i = 0; i < ns * kStreamLanes; i++)
        if (l[i]) atomicAdd((unsigned long long*)&row[P_FLOAT + i], (unsigned long long)l[i]);
    }
  }
};

template <bool kCell, bool kExact>
__global__ void __launch_bounds__(kBlock) k_reduce_sorted(const uint64_t* __restrict__ keys,
                                                          const uint32_t* __restrict__ vals, int64_t n,
                                                          RecCols r, const uint8_t* __restrict__ k1_is_mito,
                                                          Bits b, int64_t* __restrict__ partials) {
  const int sh_e = b.k1 + b.k2 + b.h;
  const int sh_k1 = b.k2 + b.h;
  const int sh_mol = b.h;
  const int64_t p0 = (int64_t)blockIdx.x * kReduceTile + (int64_t)threadIdx.x * kReduceItems;

  Acc<kCell, kExact> acc;
  acc.clear();
  int64_t cur_e = -1;
  uint64_t kprev = (p0 > 0 && p0 <= n) ? keys[p0 - 1] : ~0ull;

  for (int j = 0; j < kReduceItems; j++) {
    const int64_t p = p0 + j;
    if (p >= n) break;
    const uint64_t k = keys[p];
    const uint64_t knext = (p + 1 < n) ? keys[p + 1] : ~0ull;
    const int64_t e = (int64_t)(k >> sh_e);
    if (e != cur_e) {
      if (cur_e >= 0) acc.flush(partials + cur_e * SCT_NP);
      acc.clear();
      cur_e = e;
    }
    const bool first = (p == 0);
    const bool k1_head = first || (kprev >> sh_k1) != (k >> sh_k1);
    const bool k1_multi = k1_head && (p + 1 < n) && (knext >> sh_k1) == (k >> sh_k1);
    const bool mol_head = first || (kprev >> sh_mol) != (k >> sh_mol);
    const bool mol_single = mol_head && ((p + 1 >= n) || (knext >> sh_mol) != (k >> sh_mol));

    const uint32_t i = vals[p];
    const uint8_t bt = r.bits[i];
    const uint8_t xf = r.xf[i];
    const bool mapped = !(bt & SCT_B_UNMAPPED);

    acc.c[P_N_READS] += 1;
    acc.c[P_PERFECT_UMI] += (bt & SCT_B_PERFECT_UMI) ? 1 : 0;
    acc.c[P_N_MOL] += mol_head;
    acc.c[P_MOL_SINGLE] += mol_single;
    acc.c[P_N_K1] += k1_head;
    acc.c[P_K1_MULTI] += k1_multi;
    if (kCell) {
      acc.c[P_PERFECT_CB] += ((bt & SCT_B_HAS_CB) && (bt & SCT_B_PERFECT_CB)) ? 1 : 0;
      acc.c[P_INTERGENIC] += (xf == SCT_XF_INTERGENIC);
      acc.c[P_UNMAPPED] += (xf == SCT_XF_ABSENT);
      const uint32_t k1 = (uint32_t)((k >> sh_k1) & ((1ull << b.k1) - 1));
      const int mito = k1_is_mito[b.k1 ? k1 : 0];
      acc.c[P_MITO_K1] += (k1_head && mito) ? 1 : 0;
      acc.c[P_MITO_READS] += mito;
    }
    if (mapped) {
      acc.c[P_EXONIC] += (xf == SCT_XF_CODING);
      acc.c[P_INTRONIC] += (xf == SCT_XF_INTRONIC);
      acc.c[P_UTR] += (xf == SCT_XF_UTR);
      acc.c[P_UNIQUE] += (bt & SCT_B_NH1) ? 1 : 0;
      acc.c[P_MULTIPLE] += (bt & SCT_B_NH1) ? 0 : 1;
      acc.c[P_DUP] += (bt & SCT_B_DUPLICATE) ? 1 : 0;
      acc.c[P_SPLICED] += (bt & SCT_B_SPLICED) ? 1 : 0;
      // fragment (ref, pos, strand) inside the molecule: first occurrence / single read.
      // Equal fragments share the hash, so they sit in the same equal-key sub-run.
      const int32_t rf = r.ref[i];
      const int32_t ps = r.pos[i];
      const uint8_t st = bt & SCT_B_REVERSE;
      bool is_first = true;
      for (int64_t q = p - 1; q >= 0; q--) {
        if (keys[q] != k) break;
        const uint32_t jq = vals[q];
        const uint8_t bq = r.bits[jq];
        if (!(bq & SCT_B_UNMAPPED) && (bq & SCT_B_REVERSE) == st && r.pos[jq] == ps && r.ref[jq] == rf) {
          is_first = false;
          break;
        }
      }
      if (is_first) {
        bool single = true;
        for (int64_t q = p + 1; q < n; q++) {
          if (keys[q] != k) break;
          const uint32_t jq = vals[q];
          const uint8_t bq = r.bits[jq];
          if (!(bq & SCT_B_UNMAPPED) && (bq & SCT_B_REVERSE) == st && r.pos[jq] == ps && r.ref[jq] == rf) {
            single = false;
            break;
          }
        }
        acc.c[P_N_FRAG] += 1;
        acc.c[P_FRAG_SINGLE] += single;
      }
    }
    if (kExact) {
      fx_accumulate(acc.l + 0 * kStreamLanes, ratio(r.uy_gt30[i], r.uy_len[i]));
      const uint32_t gl = r.gq_len[i];
      fx_accumulate(acc.l + 1 * kStreamLanes, ratio(r.gq_gt30[i], gl));
      fx_accumulate(acc.l + 2 * kStreamLanes, ratio(r.gq_sum[i], gl));
      if (kCell) fx_accumulate(acc.l + 3 * kStreamLanes, ratio(r.cy_gt30[i], r.cy_len[i]));
    }
    kprev = k;
  }
  // wave-level combine when every lane of the wave ends on the same entity.  All 64 lanes
  // stay active for the shuffles; lanes without items hold zeros and cur_e == -1.
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t e0 = __shfl(cur_e, 0);
  const bool uniform = __all(cur_e == e0 || cur_e < 0);
  if (e0 < 0) return;  // wave-uniform: lane 0 had no items, so no lane had
  if (uniform) {
#pragma unroll
    for (int c = 0; c < P_NCOUNT; c++) acc.c[c] = wave_sum(acc.c[c]);
    if (kExact) {
      constexpr int ns = kCell ? 4 : 3;
#pragma unroll
      for (int c = 0; c < ns * kStreamLanes; c++) acc.l[c] = wave_sum(acc.l[c]);
    }
    if (lane == 0) acc.flush(partials + cur_e * SCT_NP);
  } else if (cur_e >= 0) {
    acc.flush(partials + cur_e * SCT_NP);
  }
}

// ======================================================================================
// 5. finalize
// ======================================================================================

__global__ void k_finalize(const int64_t* __restrict__ partials, int64_t rows, int mode, int exact,
                           const int64_t* __restrict__ ent_start, int64_t* __restrict__ out_i,
                           double* __restrict__ out_f) {
  const int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (r >= rows) return;
  const int64_t* P = partials + r * SCT_NP;
  int64_t* I = out_i + r * SCT_NI;
  double* F = out_f + r * SCT_NF;
  const int64_t n_reads = P[P_N_READS];
  const int64_t n_mol = P[P_N_MOL];
  const int64_t n_frag = P[P_N_FRAG];
  I[SCT_I_N_READS] = n_reads;
  I[SCT_I_NOISE_READS] = 0;
  I[SCT_I_PERFECT_MOLECULE_BARCODES] = P[P_PERFECT_UMI];
  I[SCT_I_READS_MAPPED_EXONIC] = P[P_EXONIC];
  I[SCT_I_READS_MAPPED_INTRONIC] = P[P_INTRONIC];
  I[SCT_I_READS_MAPPED_UTR] = P[P_UTR];
  I[SCT_I_READS_MAPPED_UNIQUELY] = P[P_UNIQUE];
  I[SCT_I_READS_MAPPED_MULTIPLE] = P[P_MULTIPLE];
  I[SCT_I_DUPLICATE_READS] = P[P_DUP];
  I[SCT_I_SPLICED_READS] = P[P_SPLICED];
  I[SCT_I_ANTISENSE_READS] = 0;
  I[SCT_I_N_MOLECULES] = n_mol;
  I[SCT_I_N_FRAGMENTS] = n_frag;
  I[SCT_I_FRAGMENTS_SINGLE] = P[P_FRAG_SINGLE];
  I[SCT_I_MOLECULES_SINGLE] = P[P_MOL_SINGLE];
  I[SCT_I_PERFECT_CELL_BARCODES] = P[P_PERFECT_CB];
  I[SCT_I_READS_MAPPED_INTERGENIC] = P[P_INTERGENIC];
  I[SCT_I_READS_UNMAPPED] = P[P_UNMAPPED];
  I[SCT_I_READS_TOO_MANY_LOCI] = 0;
  I[SCT_I_N_K1] = P[P_N_K1];
  I[SCT_I_K1_MULTIPLE] = P[P_K1_MULTI];
  I[SCT_I_N_MITO_GENES] = P[P_MITO_K1];
  I[SCT_I_N_MITO_MOLECULES] = P[P_MITO_READS];
  I[SCT_I_ENTITY] = ent_start ? ent_start[r] : r;

  const double qnan = __builtin_nan("");
  F[SCT_F_READS_PER_MOLECULE] = n_mol ? (double)n_reads / (double)n_mol : qnan;
  F[SCT_F_READS_PER_FRAGMENT] = n_frag ? (double)n_reads / (double)n_frag : qnan;
  F[SCT_F_FRAGMENTS_PER_MOLECULE] = n_mol ? (double)n_frag / (double)n_mol : qnan;
  const int64_t mito = P[P_MITO_READS];
  F[SCT_F_PCT_MITO] = mito ? ((double)mito / (double)n_reads) * 100.0 : 0.0;
  if (exact) {
    fx_finalize(P + P_FLOAT + 0 * kStreamLanes, n_reads, &F[SCT_F_UY_MEAN], &F[SCT_F_UY_VAR]);
    fx_finalize(P + P_FLOAT + 1 * kStreamLanes, n_reads, &F[SCT_F_GQF_MEAN], &F[SCT_F_GQF_VAR]);
    fx_finalize(P + P_FLOAT + 2 * kStreamLanes, n_reads, &F[SCT_F_GQ_MEAN], &F[SCT_F_GQ_VAR]);
    if (mode == SCT_MODE_CELL) {
      fx_finalize(P + P_FLOAT + 3 * kStreamLanes, n_reads, &F[SCT_F_CY_MEAN], &F[SCT_F_CY_VAR]);
    } else {
      F[SCT_F_CY_MEAN] = 0.0;
      F[SCT_F_CY_VAR] = 0.0;
    }
  }
}

// Sequential Welford per entity in record order (stats.py:82-87): one lane per entity.
struct Welford {
  double mean, m2;
  __device__ __forceinline__ void update(double x, double cnt) {
    const double delta = x - mean;
    mean += delta / cnt;
    const double delta2 = x - mean;
    m2 += delta * delta2;
  }
};

template <bool kCell>
__global__ void k_welford(RecCols r, const int64_t* __restrict__ ent_start, int64_t n_ent, int64_t n,
                          double* __restrict__ out_f) {
  const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (e >= n_ent) return;
  const int64_t s = ent_start[e];
  const int64_t t = (e + 1 < n_ent) ? ent_start[e + 1] : n;
  Welford wu{0.0, 0.0}, wf{0.0, 0.0}, wq{0.0, 0.0}, wc{0.0, 0.0};
  double cnt = 0.0;
  for (int64_t i = s; i < t; i++) {
    cnt += 1.0;
    const uint32_t gl = r.gq_len[i];
    if (kCell) wc.update(ratio(r.cy_gt30[i], r.cy_len[i]), cnt);
    wu.update(ratio(r.uy_gt30[i], r.uy_len[i]), cnt);
    wf.update(ratio(r.gq_gt30[i], gl), cnt);
    wq.update(ratio(r.gq_sum[i], gl), cnt);
  }
  const double qnan = __builtin_nan("");
  const double dn1 = cnt - 1.0;
  double* F = out_f + e * SCT_NF;
  F[SCT_F_UY_MEAN] = wu.mean;
  F[SCT_F_UY_VAR] = cnt < 2.0 ? qnan : wu.m2 / dn1;
  F[SCT_F_GQF_MEAN] = wf.mean;
  F[SCT_F_GQF_VAR] = cnt < 2.0 ? qnan : wf.m2 / dn1;
  F[SCT_F_GQ_MEAN] = wq.mean;
  F[SCT_F_GQ_VAR] = cnt < 2.0 ? qnan : wq.m2 / dn1;
  if (kCell) {
    F[SCT_F_CY_MEAN] = wc.mean;
    F[SCT_F_CY_VAR] = cnt < 2.0 ? qnan : wc.m2 / dn1;
  } else {
    F[SCT_F_CY_MEAN] = 0.0;
    F[SCT_F_CY_VAR] = 0.0;
  }
}

// ======================================================================================
// host side
// ======================================================================================

struct Layout {
  size_t keys_a, keys_b, vals_a, vals_b, tile_cnt, scan_sums, counts, offsets, ent_start, partials,
      scalars, total;
  int64_t num_tiles, num_chunks, max_ent;
};

inline size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

Layout layout_for(const sct_plan_t* plan) {
  Layout L;
  const int64_t n = plan->n_records > 0 ? plan->n_records : 0;
  L.num_tiles = cdiv(n > 0 ? n : 1, kTile);
  const int64_t m = (int64_t)kRadix * L.num_tiles;
  L.num_chunks = cdiv(m, kScanChunk);
  L.max_ent = plan->mode == SCT_MODE_GENE_GROUPED ? 0
              : (plan->max_entities > 0 ? plan->max_entities : (n > 0 ? n : 1));
  size_t off = 0;
  auto take = [&](size_t bytes) {
    size_t o = off;
    off += align_up(bytes);
    return o;
  };
  // the prefix [0, scalars + 256) is all sct_count_entities touches
  L.tile_cnt = take(sizeof(uint64_t) * (size_t)(L.num_tiles + 1));
  L.scalars = take(256);
  L.scan_sums = take(sizeof(uint64_t) * (size_t)(L.num_chunks + 1));
  L.keys_a = take(sizeof(uint64_t) * (size_t)(n > 0 ? n : 1));
  L.keys_b = take(sizeof(uint64_t) * (size_t)(n > 0 ? n : 1));
  L.vals_a = take(sizeof(uint32_t) * (size_t)(n > 0 ? n : 1));
  L.vals_b = take(sizeof(uint32_t) * (size_t)(n > 0 ? n : 1));
  L.counts = take(sizeof(uint32_t) * (size_t)m);
  L.offsets = take(sizeof(uint32_t) * (size_t)m);
  L.ent_start = take(sizeof(int64_t) * (size_t)(L.max_ent + 1));
  L.partials = take(sizeof(int64_t) * SCT_NP * (size_t)(L.max_ent > 0 ? L.max_ent : 1));
  L.total = off;
  return L;
}

// size of the workspace prefix needed by sct_count_entities
size_t count_bytes(const Layout& L) { return L.scalars + 256; }

int check_plan(const sct_plan_t* plan, const sct_records_t* rec) {
  if (!plan) return fail(SCT_EINVAL, "plan is NULL");
  if (plan->mode < SCT_MODE_CELL || plan->mode > SCT_MODE_GENE_GROUPED)
    return fail(SCT_EINVAL, "unknown mode %d", plan->mode);
  if (plan->float_mode != SCT_FLOAT_EXACT_SUM && plan->float_mode != SCT_FLOAT_WELFORD)
    return fail(SCT_EINVAL, "unknown float_mode %d", plan->float_mode);
  if (plan->float_mode == SCT_FLOAT_WELFORD && plan->mode == SCT_MODE_GENE_GROUPED)
    return fail(SCT_EINVAL, "SCT_FLOAT_WELFORD needs a RUN mode (record order defines Welford order)");
  if (plan->n_records < 0 || plan->n_records > (int64_t)0xFFFFFFFF)
    return fail(SCT_EINVAL, "n_records %lld out of range [0, 2^32)", (long long)plan->n_records);
  if (plan->n_cell_ids <= 0 || plan->n_gene_ids <= 0 || plan->n_umi_ids <= 0)
    return fail(SCT_EINVAL, "dictionary sizes must be positive");
  if (rec) {
    if (rec->n != plan->n_records) return fail(SCT_EINVAL, "records.n != plan.n_records");
    if (rec->n > 0 && (!rec->cell || !rec->umi || !rec->gene || !rec->ref || !rec->pos || !rec->gq_sum ||
                       !rec->gq_len || !rec->gq_gt30 || !rec->bits || !rec->xf || !rec->cy_gt30 ||
                       !rec->cy_len || !rec->uy_gt30 || !rec->uy_len))
      return fail(SCT_EINVAL, "a record column pointer is NULL");
  }
  return SCT_OK;
}

template <typename T>
T* at(void* ws, size_t off) {
  return reinterpret_cast<T*>(static_cast<char*>(ws) + off);
}

// device-wide exclusive scan of m uint32 counts into offsets
int scan_counts(const uint32_t* in, int64_t m, uint32_t* out, uint64_t* sums, hipStream_t s) {
  const int64_t chunks = cdiv(m, kScanChunk);
  LAUNCH("scan", k_scan_reduce, dim3((unsigned)chunks), dim3(kBlock), s, in, m, sums);
  LAUNCH("scan", k_scan_small, dim3(1), dim3(kBlock), s, sums, chunks, (uint64_t*)nullptr);
  LAUNCH("scan", k_scan_apply, dim3((unsigned)chunks), dim3(kBlock), s, in, m, (const uint64_t*)sums, out);
  return SCT_OK;
}

// LSD sort of (keys, vals) over the low `bits` bits; returns the buffer index (0 = a, 1 = b) holding the result
int radix_sort(void* ws, const Layout& L, int64_t n, int bits, int* which, hipStream_t s) {
  uint64_t* ka = at<uint64_t>(ws, L.keys_a);
  uint64_t* kb = at<uint64_t>(ws, L.keys_b);
  uint32_t* va = at<uint32_t>(ws, L.vals_a);
  uint32_t* vb = at<uint32_t>(ws, L.vals_b);
  uint32_t* counts = at<uint32_t>(ws, L.counts);
  uint32_t* offs = at<uint32_t>(ws, L.offsets);
  uint64_t* sums = at<uint64_t>(ws, L.scan_sums);
  const int passes = (bits + kRadixBits - 1) / kRadixBits;
  const int64_t tiles = cdiv(n, kTile);
  int cur = 0;
  for (int ps = 0; ps < passes; ps++) {
    const int shift = ps * kRadixBits;
    uint64_t* kin = cur ? kb : ka;
    uint32_t* vin = cur ? vb : va;
    uint64_t* kout = cur ? ka : kb;
    uint32_t* vout = cur ? va : vb;
    LAUNCH("radix_upsweep", k_radix_upsweep, dim3((unsigned)tiles), dim3(kBlock), s, (const uint64_t*)kin, n, shift,
                       L.num_tiles, counts);
    int rc = scan_counts(counts, (int64_t)kRadix * L.num_tiles, offs, sums, s);
    if (rc) return rc;
    LAUNCH("radix_downsweep", k_radix_downsweep, dim3((unsigned)tiles), dim3(kBlock), s, (const uint64_t*)kin,
                       (const uint32_t*)vin, kout, vout, n, shift, L.num_tiles, (const uint32_t*)offs);
    cur ^= 1;
  }
  *which = cur;
  return SCT_OK;
}

int run_heads(const sct_plan_t* plan, const sct_records_t* rec, void* ws, const Layout& L, hipStream_t s) {
  const int32_t* ent = plan->mode == SCT_MODE_CELL ? rec->cell : rec->gene;
  const int64_t n = rec->n;
  const int64_t tiles = cdiv(n, kTile);
  uint64_t* tc = at<uint64_t>(ws, L.tile_cnt);
  LAUNCH("heads", k_heads, dim3((unsigned)tiles), dim3(kBlock), s, ent, n, tc);
  LAUNCH("scan", k_scan_small, dim3(1), dim3(kBlock), s, tc, tiles, at<uint64_t>(ws, L.scalars));
  return SCT_OK;
}

// keys + sort + reduce into zeroed partial rows; returns rows via *n_ent (host)
int build_and_reduce(const sct_plan_t* plan, const sct_records_t* rec, const uint8_t* gene_is_mito, void* ws,
                     const Layout& L, int64_t n_ent, int64_t* partials, hipStream_t s) {
  const int64_t n = rec->n;
  const int mode = plan->mode;
  const bool cell = mode == SCT_MODE_CELL;
  Bits b;
  const int64_t ent_ids = mode == SCT_MODE_GENE_GROUPED ? plan->n_gene_ids : n_ent;
  b.e = bitlen((uint64_t)ent_ids);
  b.k1 = bitlen((uint64_t)(cell ? plan->n_gene_ids : plan->n_cell_ids));
  b.k2 = bitlen((uint64_t)plan->n_umi_ids);
  const int used = b.e + b.k1 + b.k2;
  if (used > 64) return fail(SCT_EINVAL, "packed key needs %d bits (> 64)", used);
  // fill the last radix digit with fragment-hash bits (free: same pass count)
  const int padded = ((used + kRadixBits - 1) / kRadixBits) * kRadixBits;
  b.h = (padded > 63 ? 63 : padded) - used;  // keep every shift < 64
  if (b.h < 0) b.h = 0;
  if (b.h > 32) b.h = 32;
  const int bits = used + b.h;

  KeyCols kc;
  kc.ent = mode == SCT_MODE_CELL ? rec->cell : rec->gene;
  kc.k1 = cell ? rec->gene : rec->cell;
  kc.k2 = rec->umi;
  kc.ref = rec->ref;
  kc.pos = rec->pos;
  kc.bits = rec->bits;
  uint64_t* ka = at<uint64_t>(ws, L.keys_a);
  uint32_t* va = at<uint32_t>(ws, L.vals_a);
  const int64_t tiles = cdiv(n, kTile);
  if (mode == SCT_MODE_GENE_GROUPED) {
    const int64_t blocks = cdiv(n, kBlock) < 65536 ? cdiv(n, kBlock) : 65536;
    LAUNCH("build_keys", k_build_keys_grouped, dim3((unsigned)blocks), dim3(kBlock), s, kc, n, b, ka, va);
  } else {
    LAUNCH("build_keys", k_build_keys_run, dim3((unsigned)tiles), dim3(kBlock), s, kc, n,
                       (const uint64_t*)at<uint64_t>(ws, L.tile_cnt), b, ka, va, at<int64_t>(ws, L.ent_start));
  }
  int which = 0;
  int rc = radix_sort(ws, L, n, bits, &which, s);
  if (rc) return rc;
  const uint64_t* keys = which ? at<uint64_t>(ws, L.keys_b) : ka;
  const uint32_t* vals = which ? at<uint32_t>(ws, L.vals_b) : va;

  const int64_t rows = mode == SCT_MODE_GENE_GROUPED ? plan->n_gene_ids : n_ent;
  HIPCHK(hipMemsetAsync(partials, 0, sizeof(int64_t) * SCT_NP * (size_t)rows, s));
  RecCols rc2{rec->ref, rec->pos, rec->gq_sum, rec->gq_len, rec->gq_gt30, rec->bits, rec->xf,
              rec->cy_gt30, rec->cy_len, rec->uy_gt30, rec->uy_len};
  const bool exact = plan->float_mode == SCT_FLOAT_EXACT_SUM;
  const int64_t rblocks = cdiv(n, kReduceTile);
  if (cell && exact) {
    LAUNCH("reduce_sorted", (k_reduce_sorted<true, true>), dim3((unsigned)rblocks), dim3(kBlock), s, keys, vals, n,
           rc2, gene_is_mito, b, partials);
  } else if (cell) {
    LAUNCH("reduce_sorted", (k_reduce_sorted<true, false>), dim3((unsigned)rblocks), dim3(kBlock), s, keys, vals, n,
           rc2, gene_is_mito, b, partials);
  } else if (exact) {
    LAUNCH("reduce_sorted", (k_reduce_sorted<false, true>), dim3((unsigned)rblocks), dim3(kBlock), s, keys, vals, n,
           rc2, gene_is_mito, b, partials);
  } else {
    LAUNCH("reduce_sorted", (k_reduce_sorted<false, false>), dim3((unsigned)rblocks), dim3(kBlock), s, keys, vals, n,
           rc2, gene_is_mito, b, partials);
  }
  return SCT_OK;
}

}  // namespace

// ======================================================================================
// C-ABI
// ======================================================================================

extern "C" {

int sct_abi_version(void) { return SCT_ABI_VERSION; }

int sct_profile_enable(int on) {
  g_prof = on != 0;
  return SCT_OK;
}

int sct_profile_read(const char** names, double* ms, int64_t* launches, int max_kernels) {
  // waits for the recorded events, returns per-kernel totals, and resets the counters
  static thread_local std::vector<std::string> held;
  held.clear();
  int k = 0;
  for (auto& e : g_prof_entries) {
    double tot = 0.0;
    for (auto& pr : e.ev) {
      float t = 0.f;
      if (hipEventSynchronize(pr.second) == hipSuccess && hipEventElapsedTime(&t, pr.first, pr.second) == hipSuccess)
        tot += t;
      (void)hipEventDestroy(pr.first);
      (void)hipEventDestroy(pr.second);
    }
    held.push_back(e.name);
    if (k < max_kernels) {
      if (ms) ms[k] = tot;
      if (launches) launches[k] = (int64_t)e.ev.size();
    }
    k++;
  }
  for (int i = 0; i < k && i < max_kernels; i++)
    if (names) names[i] = held[i].c_str();
  g_prof_entries.clear();
  return k;
}

const char* sct_last_error(void) { return g_err.c_str(); }

int sct_workspace_size(const sct_plan_t* plan, size_t* bytes) {
  int rc = check_plan(plan, nullptr);
  if (rc) return rc;
  if (!bytes) return fail(SCT_EINVAL, "bytes is NULL");
  *bytes = layout_for(plan).total;
  return SCT_OK;
}

int sct_count_entities(const sct_plan_t* plan, const sct_records_t* rec, void* workspace, size_t workspace_bytes,
                       int64_t* n_entities, void* stream) {
  g_err.clear();
  int rc = check_plan(plan, rec);
  if (rc) return rc;
  if (!n_entities) return fail(SCT_EINVAL, "n_entities is NULL");
  if (plan->mode == SCT_MODE_GENE_GROUPED) {
    *n_entities = plan->n_gene_ids;
    return SCT_OK;
  }
  if (rec->n == 0) {
    *n_entities = 0;
    return SCT_OK;
  }
  sct_plan_t p1 = *plan;
  p1.max_entities = 1;  // the count only needs the prefix of the layout
  const Layout L = layout_for(&p1);
  if (!workspace || workspace_bytes < count_bytes(L))
    return fail(SCT_ENOMEM, "workspace too small for counting (%zu < %zu)", workspace_bytes, count_bytes(L));
  hipStream_t s = (hipStream_t)stream;
  rc = run_heads(&p1, rec, workspace, L, s);
  if (rc) return rc;
  uint64_t total = 0;
  HIPCHK(hipMemcpyAsync(&total, at<uint64_t>(workspace, L.scalars), sizeof(uint64_t), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  *n_entities = (int64_t)total;
  return SCT_OK;
}

int sct_compute_metrics(const sct_plan_t* plan, const sct_records_t* rec, const uint8_t* gene_is_mito,
                        const uint8_t* gene_is_multi, void* workspace, size_t workspace_bytes, int64_t* out_ints,
                        double* out_floats, int64_t capacity, int64_t* n_rows, void* stream) {
  (void)gene_is_multi;  // multi-gene rows are dropped by the caller (gatherer.py:210-212)
  g_err.clear();
  int rc = check_plan(plan, rec);
  if (rc) return rc;
  if (plan->mode == SCT_MODE_GENE_GROUPED)
    return fail(SCT_EINVAL, "sct_compute_metrics handles RUN modes; use sct_gene_partials for GROUPED");
  if (!n_rows) return fail(SCT_EINVAL, "n_rows is NULL");
  if (plan->mode == SCT_MODE_CELL && !gene_is_mito) return fail(SCT_EINVAL, "gene_is_mito is NULL");
  const int64_t n = rec->n;
  if (n == 0) {
    *n_rows = 0;
    return SCT_OK;
  }
  const Layout L = layout_for(plan);
  if (!workspace || workspace_bytes < L.total)
    return fail(SCT_ENOMEM, "workspace too small (%zu < %zu)", workspace_bytes, L.total);
  hipStream_t s = (hipStream_t)stream;
  rc = run_heads(plan, rec, workspace, L, s);
  if (rc) return rc;
  uint64_t total = 0;
  HIPCHK(hipMemcpyAsync(&total, at<uint64_t>(workspace, L.scalars), sizeof(uint64_t), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  const int64_t n_ent = (int64_t)total;
  if (n_ent > L.max_ent) return fail(SCT_ENOMEM, "%lld entities exceed plan.max_entities %lld", (long long)n_ent,
                                     (long long)L.max_ent);
  if (n_ent > capacity)
    return fail(SCT_EINVAL, "%lld entities exceed output capacity %lld", (long long)n_ent, (long long)capacity);
  int64_t* partials = at<int64_t>(workspace, L.partials);
  rc = build_and_reduce(plan, rec, gene_is_mito, workspace, L, n_ent, partials, s);
  if (rc) return rc;
  const bool exact = plan->float_mode == SCT_FLOAT_EXACT_SUM;
  const int64_t* ent_start = at<int64_t>(workspace, L.ent_start);
  LAUNCH("finalize", k_finalize, dim3((unsigned)cdiv(n_ent, kBlock)), dim3(kBlock), s, (const int64_t*)partials,
                     n_ent, plan->mode, exact ? 1 : 0, ent_start, out_ints, out_floats);
  if (!exact) {
    RecCols rc2{rec->ref, rec->pos, rec->gq_sum, rec->gq_len, rec->gq_gt30, rec->bits, rec->xf,
                rec->cy_gt30, rec->cy_len, rec->uy_gt30, rec->uy_len};
    if (plan->mode == SCT_MODE_CELL) {
      LAUNCH("welford", k_welford<true>, dim3((unsigned)cdiv(n_ent, kBlock)), dim3(kBlock), s, rc2, ent_start, n_ent,
             n, out_floats);
    } else {
      LAUNCH("welford", k_welford<false>, dim3((unsigned)cdiv(n_ent, kBlock)), dim3(kBlock), s, rc2, ent_start,
             n_ent, n, out_floats);
    }
  }
  *n_rows = n_ent;
  return SCT_OK;
}

int sct_gene_partials(const sct_plan_t* plan, const sct_records_t* rec, void* workspace, size_t workspace_bytes,
                      int64_t* partials, void* stream) {
  g_err.clear();
  int rc = check_plan(plan, rec);
  if (rc) return rc;
  if (plan->mode != SCT_MODE_GENE_GROUPED) return fail(SCT_EINVAL, "sct_gene_partials needs SCT_MODE_GENE_GROUPED");
  if (plan->float_mode != SCT_FLOAT_EXACT_SUM) return fail(SCT_EINVAL, "GROUPED partials need SCT_FLOAT_EXACT_SUM");
  if (!partials) return fail(SCT_EINVAL, "partials is NULL");
  hipStream_t s = (hipStream_t)stream;
  if (rec->n == 0) {
    HIPCHK(hipMemsetAsync(partials, 0, sizeof(int64_t) * SCT_NP * (size_t)plan->n_gene_ids, s));
    return SCT_OK;
  }
  const Layout L = layout_for(plan);
  if (!workspace || workspace_bytes < L.total)
    return fail(SCT_ENOMEM, "workspace too small (%zu < %zu)", workspace_bytes, L.total);
  return build_and_reduce(plan, rec, nullptr, workspace, L, 0, partials, s);
}

int sct_finalize_partials(int32_t mode, const int64_t* partials, int64_t rows, int64_t* out_ints, double* out_floats,
                          void* stream) {
  g_err.clear();
  if (mode < SCT_MODE_CELL || mode > SCT_MODE_GENE_GROUPED) return fail(SCT_EINVAL, "unknown mode %d", mode);
  if (rows < 0 || (rows > 0 && (!partials || !out_ints || !out_floats)))
    return fail(SCT_EINVAL, "bad finalize arguments");
  if (rows == 0) return SCT_OK;
  hipStream_t s = (hipStream_t)stream;
  LAUNCH("finalize", k_finalize, dim3((unsigned)cdiv(rows, kBlock)), dim3(kBlock), s, partials, rows, (int)mode, 1,
                     (const int64_t*)nullptr, out_ints, out_floats);
  return SCT_OK;
}

}  // extern "C"
