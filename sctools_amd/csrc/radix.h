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

__global__ void k_radix_upsweep(const uint64_t* __restrict__ keys, int64_t n, int shift, int64_t num_tiles,
                                uint32_t* __restrict__ counts) {
  __shared__ uint32_t hist[kWaves][kRadix];
  const int wid = threadIdx.x / kWave;
  for (int i = threadIdx.x; i < kWaves * kRadix; i += kBlock) (&hist[0][0])[i] = 0;
  __syncthreads();
  const unsigned tile = xcd_tile(blockIdx.x, gridDim.x);  // consecutive tiles on one XCD
  const int64_t base = (int64_t)tile * kSortTile;
#pragma unroll
  for (int j = 0; j < kSortItems; j++) {
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

__global__ void __launch_bounds__(kBlock) k_radix_downsweep(const uint64_t* __restrict__ keys_in,
                                                            const uint32_t* __restrict__ vals_in,
                                                            uint64_t* __restrict__ keys_out,
                                                            uint32_t* __restrict__ vals_out, int64_t n, int shift,
                                                            int64_t num_tiles, const uint32_t* __restrict__ offsets) {
  __shared__ uint64_t s_keys[kSortTile];
  __shared__ uint32_t s_vals[kSortTile];
  __shared__ uint32_t s_whist[kWaves][kRadix];
  __shared__ uint32_t s_dstart[kRadix];
  __shared__ uint32_t s_goff[kRadix];  // this tile's output offset per digit (one global read each)
  __shared__ uint64_t s_scan[kWaves + 1];

  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  // consecutive tiles on one XCD: a digit's runs of neighbouring tiles are neighbours in the
  // output, so their partly written lines meet in that XCD's L2 instead of two L2s
  const unsigned tile = xcd_tile(blockIdx.x, gridDim.x);
  const int64_t base = (int64_t)tile * kSortTile;
  const int tile_n = (int)((n - base) < kSortTile ? (n - base) : kSortTile);

  for (int i = threadIdx.x; i < kWaves * kRadix; i += kBlock) (&s_whist[0][0])[i] = 0;
  s_goff[threadIdx.x] = offsets[(int64_t)threadIdx.x * num_tiles + tile];  // kRadix == kBlock
  __syncthreads();

  const uint64_t lt = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
  uint64_t k[kSortItems];
  uint32_t v[kSortItems];
  uint16_t rank[kSortItems];
  uint8_t dig[kSortItems];
  // wave `wid` owns tile positions [wid*kSortItems*kWave, ...); round j covers 64 of them
#pragma unroll
  for (int j = 0; j < kSortItems; j++) {
    const int q = wid * (kSortItems * kWave) + j * kWave + lane;
    const int64_t p = base + q;
    if (q < tile_n) {
      k[j] = keys_in[p];
      v[j] = vals_in[p];
    } else {
      k[j] = ~0ull;  // padding: digit 255 at every shift, ranked after all real items, never written
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
  for (int ps = 0; ps < passes; ps++) {
    const int shift = ps * kRadixBits;
    const uint64_t* kin = cur ? B.kb : B.ka;
    const uint32_t* vin = cur ? B.vb : B.va;
    uint64_t* kout = cur ? B.ka : B.kb;
    uint32_t* vout = cur ? B.va : B.vb;
    LAUNCH_N("radix_upsweep", n, k_radix_upsweep, dim3((unsigned)tiles), dim3(kBlock), s, kin, n, shift, tiles, B.counts);
    int rc = scan_counts(B.counts, (int64_t)kRadix * tiles, B.offsets, B.sums, s);
    if (rc) return rc;
    LAUNCH_N("radix_downsweep", n, k_radix_downsweep, dim3((unsigned)tiles), dim3(kBlock), s, kin, vin, kout, vout, n,
           shift, tiles, (const uint32_t*)B.offsets);
    cur ^= 1;
  }
  *which = cur;
  return SCT_OK;
}

}  // namespace sct
