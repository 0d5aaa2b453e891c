// radix.h -- device-wide LSD radix sort of (uint64 key, uint32 value), 8-bit digits.
//
// Per pass: an upsweep of per-tile digit counts, a device-wide scan of the
// digit-major count matrix, and a downsweep that ranks each tile stably with
// wave-level multi-split (8 ballots give every lane the mask of lanes holding
// its digit; the lowest such lane updates the wave's digit counter in LDS),
// stages the tile in LDS in digit order and writes each digit bucket as a
// contiguous run.
#pragma once
#include "scan.h"
#include "util.h"

namespace sct {

constexpr int kItems = 16;
constexpr int kTile = kBlock * kItems;  // 4096 records per tile (entity-run heads, key pass)
// LSD radix sort tiles: 2048 items (24 KB of keys / values staged in LDS, so 6 blocks fit a CU)
// 12 / 16 items (3072 / 4096-item tiles, 2 blocks per CU): config 5 20.3 / 21.9 ms vs 19.7.  The
// macro exists for tests/native/libsct_engine_si4.so (1024-item tiles: the tiling that exposed the
// round-3 tag-sort workspace bug, tests/test_gpu_tagsort.py::test_tag_sort_small_radix_tiles).
#ifndef SCT_SORT_ITEMS
#define SCT_SORT_ITEMS 8
#endif
constexpr int kSortItems = SCT_SORT_ITEMS;
constexpr int kSortTile = kBlock * kSortItems;
constexpr int kRadixBits = 8;
constexpr int kRadix = 1 << kRadixBits;
static_assert(kRadix == kBlock, "digit-per-thread scan assumes kRadix == kBlock");

// K: uint64_t, or uint32_t for keys of <= 32 bits (round 6: the group tag sort's K1 -- a third less
// traffic per pass)
template <typename K = uint64_t, int kIt = kSortItems>
__global__ void k_radix_upsweep(const K* __restrict__ keys, int64_t n, int shift, int64_t num_tiles,
                                uint32_t* __restrict__ counts) {
  __shared__ uint32_t hist[kWaves][kRadix];
  const int wid = threadIdx.x / kWave;
  for (int i = threadIdx.x; i < kWaves * kRadix; i += kBlock) (&hist[0][0])[i] = 0;
  __syncthreads();
  const unsigned tile = xcd_tile(blockIdx.x, gridDim.x);  // consecutive tiles on one XCD
  const int64_t base = (int64_t)tile * (kBlock * kIt);
#pragma unroll
  for (int j = 0; j < kIt; j++) {
    const int64_t p = base + (int64_t)j * kBlock + threadIdx.x;
    if (p < n) atomicAdd(&hist[wid][(keys[p] >> shift) & (kRadix - 1)], 1u);
  }
  __syncthreads();
  for (int d = threadIdx.x; d < kRadix; d += kBlock) {
    uint32_t t = 0;
#pragma unroll
    for (int w = 0; w < kWaves; w++) t += hist[w][d];
    counts[(int64_t)d * num_tiles + tile] = t;
  }
}

// kIdx: the values are the input positions (the first pass over freshly packed keys): not read
template <typename K = uint64_t, bool kIdx = false, int kIt = kSortItems>
__global__ void __launch_bounds__(kBlock) k_radix_downsweep(const K* __restrict__ keys_in,
                                                            const uint32_t* __restrict__ vals_in,
                                                            K* __restrict__ keys_out,
                                                            uint32_t* __restrict__ vals_out, int64_t n, int shift,
                                                            int64_t num_tiles, const uint32_t* __restrict__ offsets) {
  constexpr int kTileN = kBlock * kIt;
  __shared__ K s_keys[kTileN];
  __shared__ uint32_t s_vals[kTileN];
  __shared__ uint32_t s_whist[kWaves][kRadix];
  __shared__ uint32_t s_dstart[kRadix];
  __shared__ uint32_t s_goff[kRadix];  // this tile's output offset per digit (one global read each)
  __shared__ uint64_t s_scan[kWaves + 1];

  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  // consecutive tiles on one XCD: a digit's runs of neighbouring tiles are neighbours in the
  // output, so their partly written lines meet in that XCD's L2 instead of two L2s
  const unsigned tile = xcd_tile(blockIdx.x, gridDim.x);
  const int64_t base = (int64_t)tile * kTileN;
  const int tile_n = (int)((n - base) < kTileN ? (n - base) : kTileN);

  for (int i = threadIdx.x; i < kWaves * kRadix; i += kBlock) (&s_whist[0][0])[i] = 0;
  s_goff[threadIdx.x] = offsets[(int64_t)threadIdx.x * num_tiles + tile];  // kRadix == kBlock
  __syncthreads();

  const uint64_t lt = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
  K k[kIt];
  uint32_t v[kIt];
  uint16_t rank[kIt];
  uint8_t dig[kIt];
  // wave `wid` owns tile positions [wid*kIt*kWave, ...); round j covers 64 of them
#pragma unroll
  for (int j = 0; j < kIt; j++) {
    const int q = wid * (kIt * kWave) + j * kWave + lane;
    const int64_t p = base + q;
    if (q < tile_n) {
      k[j] = keys_in[p];
      v[j] = kIdx ? (uint32_t)p : vals_in[p];
    } else {
      k[j] = (K)~0ull;  // padding: digit 255 at every shift, ranked after all real items, never written
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
  for (int j = 0; j < kIt; j++) {
    const uint32_t lp = s_whist[wid][dig[j]] + rank[j];
    s_keys[lp] = k[j];
    s_vals[lp] = v[j];
  }
  __syncthreads();
  for (int q = threadIdx.x; q < tile_n; q += kBlock) {
    const K kk = s_keys[q];
    const uint32_t d = (uint32_t)(kk >> shift) & (kRadix - 1);
    const uint64_t o = (uint64_t)s_goff[d] + (uint32_t)(q - (int)s_dstart[d]);
    keys_out[o] = kk;
    vals_out[o] = s_vals[q];
  }
}

// ---- onesweep (round 4): every pass's digit histogram in one read, tile offsets by look-back ----
// k_radix_hist_all counts the digits of all passes at once (the histogram of a digit is the same
// in every pass's input order), k_radix_bases turns them into each pass's digit starts, and each
// pass is one kernel: a block takes the next tile by ticket, ranks it as k_radix_downsweep does,
// and finds its output offset per digit by decoupled look-back over the earlier tiles' published
// counts (status words: 2 flag bits + a 30-bit count; kLbAgg = the tile's own count, kLbPre = the
// inclusive prefix) -- no per-tile count matrix, no upsweep pass and no device-wide scan.
// Tickets are handed out in block start order, so a tile only ever waits on tiles whose blocks
// have started (forward progress without co-residency).
constexpr uint32_t kLbAgg = 1u << 30, kLbPre = 2u << 30, kLbVal = (1u << 30) - 1u;
constexpr int kMaxPasses = 8;
constexpr int kHistAllBlocks = 2048;
#ifndef SCT_LOOKAHEAD
#define SCT_LOOKAHEAD 8
#endif
constexpr int kLookAhead = SCT_LOOKAHEAD;

__global__ void __launch_bounds__(kBlock) k_radix_hist_all(const uint64_t* __restrict__ keys, int64_t n, int passes,
                                                           uint32_t* __restrict__ ghist) {
  __shared__ uint32_t h[kMaxPasses][kRadix];
  for (int i = threadIdx.x; i < kMaxPasses * kRadix; i += kBlock) (&h[0][0])[i] = 0;
  __syncthreads();
  for (int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x; p < n; p += (int64_t)gridDim.x * kBlock) {
    const uint64_t k = keys[p];
    for (int ps = 0; ps < passes; ps++) atomicAdd(&h[ps][(k >> (ps * kRadixBits)) & (kRadix - 1)], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < passes * kRadix; i += kBlock) {
    const uint32_t c = (&h[0][0])[i];
    if (c) atomicAdd(&ghist[i], c);
  }
}

// gbase[ps][d] = exclusive prefix of ghist[ps][.] (one block, kRadix == kBlock)
__global__ void __launch_bounds__(kBlock) k_radix_bases(const uint32_t* __restrict__ ghist, int passes,
                                                        uint32_t* __restrict__ gbase) {
  __shared__ uint64_t s_scan[kWaves + 1];
  for (int ps = 0; ps < passes; ps++) {
    uint64_t tot;
    const uint64_t ex = block_exclusive_scan<uint64_t>((uint64_t)ghist[ps * kRadix + threadIdx.x], &tot, s_scan);
    gbase[ps * kRadix + threadIdx.x] = (uint32_t)ex;
  }
}

__device__ __forceinline__ uint32_t lb_load(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lb_store(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void __launch_bounds__(kBlock) k_radix_onesweep(const uint64_t* __restrict__ keys_in,
                                                           const uint32_t* __restrict__ vals_in,
                                                           uint64_t* __restrict__ keys_out,
                                                           uint32_t* __restrict__ vals_out, int64_t n, int shift,
                                                           const uint32_t* __restrict__ gbase,
                                                           uint32_t* __restrict__ status,
                                                           uint32_t* __restrict__ ticket) {
  __shared__ uint64_t s_keys[kSortTile];
  __shared__ uint32_t s_vals[kSortTile];
  __shared__ uint32_t s_whist[kWaves][kRadix];
  __shared__ uint32_t s_dstart[kRadix];
  __shared__ uint32_t s_goff[kRadix];
  __shared__ uint64_t s_scan[kWaves + 1];
  __shared__ uint32_t s_tile;
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  if (threadIdx.x == 0) s_tile = atomicAdd(ticket, 1u);
  for (int i = threadIdx.x; i < kWaves * kRadix; i += kBlock) (&s_whist[0][0])[i] = 0;
  __syncthreads();
  const uint32_t tile = s_tile;
  const int64_t base = (int64_t)tile * kSortTile;
  const int tile_n = (int)((n - base) < kSortTile ? (n - base) : kSortTile);

  const uint64_t lt = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
  uint64_t k[kSortItems];
  uint32_t v[kSortItems];
  uint16_t rank[kSortItems];
  uint8_t dig[kSortItems];
#pragma unroll
  for (int j = 0; j < kSortItems; j++) {
    const int q = wid * (kSortItems * kWave) + j * kWave + lane;
    const int64_t p = base + q;
    if (q < tile_n) {
      k[j] = keys_in[p];
      v[j] = vals_in[p];
    } else {
      k[j] = ~0ull;  // padding: digit 255, ranked after every real item, never written
      v[j] = 0;
    }
  }
#pragma unroll
  for (int j = 0; j < kSortItems; j++) {
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
  {
    const int d = threadIdx.x;
    uint32_t run = 0;
    uint32_t pre[kWaves];
#pragma unroll
    for (int w = 0; w < kWaves; w++) {
      pre[w] = run;
      run += s_whist[w][d];
    }
    // the padding of a partial last tile was counted in digit 255: only real items are published
    const uint32_t real = (d == kRadix - 1) ? run - (uint32_t)(kSortTile - tile_n) : run;
    uint32_t* st = status + (size_t)tile * kRadix + d;
    uint32_t excl = 0;
    if (tile == 0) {
      lb_store(st, kLbPre | real);
    } else {
      lb_store(st, kLbAgg | real);
      // kLookAhead predecessors' words loaded together per step (their latencies overlap);
      // consumed in order up to the first unpublished one (retried) or an inclusive prefix
      int64_t j = (int64_t)tile - 1;
      while (true) {
        uint32_t w[kLookAhead];
#pragma unroll
        for (int u = 0; u < kLookAhead; u++)
          w[u] = j - u >= 0 ? lb_load(status + (size_t)(j - u) * kRadix + d) : kLbPre;
        int u = 0;
        bool done = false;
#pragma unroll
        for (int v = 0; v < kLookAhead; v++) {
          if (u != v || done) continue;  // (a gap stopped the scan)
          if (!(w[v] & (kLbAgg | kLbPre))) continue;
          excl += w[v] & kLbVal;
          done = (w[v] & kLbPre) != 0;
          u = v + 1;
        }
        if (done) break;
        j -= u;
        if (u == 0) __builtin_amdgcn_s_sleep(1);
      }
      lb_store(st, kLbPre | (excl + real));
    }
    s_goff[d] = gbase[d] + excl;
    uint64_t tot;
    const uint64_t ds = block_exclusive_scan<uint64_t>((uint64_t)run, &tot, s_scan);
    s_dstart[d] = (uint32_t)ds;
#pragma unroll
    for (int w = 0; w < kWaves; w++) s_whist[w][d] = (uint32_t)ds + pre[w];
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kSortItems; j++) {
    const uint32_t lp = s_whist[wid][dig[j]] + rank[j];
    s_keys[lp] = k[j];
    s_vals[lp] = v[j];
  }
  __syncthreads();
  for (int q = threadIdx.x; q < tile_n; q += kBlock) {
    const uint64_t kk = s_keys[q];
    const uint32_t d = (uint32_t)(kk >> shift) & (kRadix - 1);
    const uint64_t o = (uint64_t)s_goff[d] + (uint32_t)(q - (int)s_dstart[d]);
    keys_out[o] = kk;
    vals_out[o] = s_vals[q];
  }
}

struct SortBuffers {
  uint64_t *ka, *kb;
  uint32_t *va, *vb;
  uint32_t *counts, *offsets;  // count_cap entries each (>= kRadix * cdiv(n, kSortTile))
  uint64_t* sums;              // cdiv(count_cap, kScanChunk) + 1
  int64_t count_cap;
};

// LSD sort of (ka, va) over the low `bits` bits; *which = 0 if the result is in (ka, va), 1 if in (kb, vb)
inline int radix_sort(const SortBuffers& B, int64_t n, int bits, int* which, hipStream_t s) {
  const int passes = (bits + kRadixBits - 1) / kRadixBits;
  const int64_t tiles = cdiv(n, kSortTile);
  if ((int64_t)kRadix * tiles > B.count_cap)  // (the round-3 tag-sort layout violated this)
    return fail(SCT_EINVAL, "radix_sort: %lld digit counts exceed the workspace's %lld", (long long)(kRadix * tiles),
                (long long)B.count_cap);
  int cur = 0;
  // onesweep when the counts fit its 30-bit status words and the offsets buffer holds the
  // histograms (ghist, gbase: kMaxPasses x kRadix each, + a ticket per pass)
  static const char* one_env = getenv("SCT_RADIX_ONESWEEP");
  const bool onesweep = (one_env && one_env[0] == '1') && n < (int64_t)kLbVal && passes <= kMaxPasses &&
                        B.count_cap >= (int64_t)(2 * kMaxPasses * kRadix + kMaxPasses);
  if (onesweep) {
    uint32_t* ghist = B.offsets;
    uint32_t* gbase = B.offsets + kMaxPasses * kRadix;
    uint32_t* tickets = B.offsets + 2 * kMaxPasses * kRadix;
    HIPCHK(hipMemsetAsync(B.offsets, 0, sizeof(uint32_t) * (2 * kMaxPasses * kRadix + kMaxPasses), s));
    const int64_t hb = tiles < kHistAllBlocks ? tiles : kHistAllBlocks;
    LAUNCH_N("radix_hist_all", n, k_radix_hist_all, dim3((unsigned)hb), dim3(kBlock), s, (const uint64_t*)B.ka, n,
             passes, ghist);
    LAUNCH("radix_bases", k_radix_bases, dim3(1), dim3(kBlock), s, (const uint32_t*)ghist, passes, gbase);
    for (int ps = 0; ps < passes; ps++) {
      const uint64_t* kin = cur ? B.kb : B.ka;
      const uint32_t* vin = cur ? B.vb : B.va;
      uint64_t* kout = cur ? B.ka : B.kb;
      uint32_t* vout = cur ? B.va : B.vb;
      HIPCHK(hipMemsetAsync(B.counts, 0, sizeof(uint32_t) * (size_t)kRadix * (size_t)tiles, s));
      LAUNCH_N("radix_onesweep", n, k_radix_onesweep, dim3((unsigned)tiles), dim3(kBlock), s, kin, vin, kout, vout, n,
               ps * kRadixBits, (const uint32_t*)(gbase + ps * kRadix), B.counts, tickets + ps);
      cur ^= 1;
    }
    *which = cur;
    return SCT_OK;
  }
  for (int ps = 0; ps < passes; ps++) {
    const int shift = ps * kRadixBits;
    const uint64_t* kin = cur ? B.kb : B.ka;
    const uint32_t* vin = cur ? B.vb : B.va;
    uint64_t* kout = cur ? B.ka : B.kb;
    uint32_t* vout = cur ? B.va : B.vb;
    LAUNCH_N("radix_upsweep", n, k_radix_upsweep<uint64_t>, dim3((unsigned)tiles), dim3(kBlock), s, kin, n, shift,
             tiles, B.counts);
    int rc = scan_counts(B.counts, (int64_t)kRadix * tiles, B.offsets, B.sums, s);
    if (rc) return rc;
    LAUNCH_N("radix_downsweep", n, k_radix_downsweep<uint64_t>, dim3((unsigned)tiles), dim3(kBlock), s, kin, vin, kout,
             vout, n, shift, tiles, (const uint32_t*)B.offsets);
    cur ^= 1;
  }
  *which = cur;
  return SCT_OK;
}

// items per thread of radix_sort32's tiles: 32-bit keys halve the tile's key staging, so a tile of
// 4096 items (16 per digit on average, against 8 at 2048) takes the LDS of a 2048-item 64-bit tile
#ifndef SCT_SORT_ITEMS32
#define SCT_SORT_ITEMS32 16
#endif
constexpr int kSortItems32 = SCT_SORT_ITEMS32;
static_assert(kSortItems32 >= kSortItems, "radix_sort32's tile counts fit the workspace's count_cap");
// the same over 32-bit keys (bits <= 32) held in the key buffers (ka / kb reinterpreted).
// positions: the values are the input positions (nothing in va): the first pass takes them from
// the index.
inline int radix_sort32(const SortBuffers& B, int64_t n, int bits, int* which, hipStream_t s,
                        bool positions = false) {
  if (bits > 32) return fail(SCT_EINVAL, "radix_sort32: %d key bits", bits);
  const int passes = (bits + kRadixBits - 1) / kRadixBits;
  const int64_t tiles = cdiv(n, kBlock * kSortItems32);
  if ((int64_t)kRadix * tiles > B.count_cap)
    return fail(SCT_EINVAL, "radix_sort32: %lld digit counts exceed the workspace's %lld", (long long)(kRadix * tiles),
                (long long)B.count_cap);
  uint32_t* ka = reinterpret_cast<uint32_t*>(B.ka);
  uint32_t* kb = reinterpret_cast<uint32_t*>(B.kb);
  int cur = 0;
  for (int ps = 0; ps < passes; ps++) {
    const int shift = ps * kRadixBits;
    const uint32_t* kin = cur ? kb : ka;
    const uint32_t* vin = cur ? B.vb : B.va;
    uint32_t* kout = cur ? ka : kb;
    uint32_t* vout = cur ? B.va : B.vb;
    const bool pre = positions && ps == 0;
    LAUNCH_N("radix_upsweep", n, (k_radix_upsweep<uint32_t, kSortItems32>), dim3((unsigned)tiles), dim3(kBlock), s,
             kin, n, shift, tiles, B.counts);
    int rc = scan_counts(B.counts, (int64_t)kRadix * tiles, B.offsets, B.sums, s);
    if (rc) return rc;
    if (pre) {
      LAUNCH_N("radix_downsweep", n, (k_radix_downsweep<uint32_t, true, kSortItems32>), dim3((unsigned)tiles),
               dim3(kBlock), s, kin, vin, kout, vout, n, shift, tiles, (const uint32_t*)B.offsets);
    } else {
      LAUNCH_N("radix_downsweep", n, (k_radix_downsweep<uint32_t, false, kSortItems32>), dim3((unsigned)tiles),
               dim3(kBlock), s, kin, vin, kout, vout, n, shift, tiles, (const uint32_t*)B.offsets);
    }
    cur ^= 1;
  }
  *which = cur;
  return SCT_OK;
}

}  // namespace sct
