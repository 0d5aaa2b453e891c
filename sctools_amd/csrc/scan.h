// scan.h -- device-wide exclusive scans (reduce / small scan / apply).
#pragma once
#include "util.h"

namespace sct {

constexpr int kScanChunk = 4096;

// Chunk sums.  kVec: `in` is 16-byte aligned, so whole 4-count groups load as one uint4
// (lane t of round r reads group r * kBlock + t: coalesced 16-byte loads, all issued at once).
template <bool kVec>
__global__ void __launch_bounds__(kBlock) k_scan_reduce(const uint32_t* __restrict__ in, int64_t m,
                                                        uint64_t* __restrict__ sums) {
  const int64_t base = (int64_t)blockIdx.x * kScanChunk;
  uint64_t s = 0;
  if (kVec && base + kScanChunk <= m) {
    const uint4* src = reinterpret_cast<const uint4*>(in + base);
    uint4 a[kScanChunk / (4 * kBlock)];
#pragma unroll
    for (int r = 0; r < kScanChunk / (4 * kBlock); r++) a[r] = src[r * kBlock + threadIdx.x];
#pragma unroll
    for (int r = 0; r < kScanChunk / (4 * kBlock); r++) s += (uint64_t)a[r].x + a[r].y + a[r].z + a[r].w;
  } else {
    for (int i = threadIdx.x; i < kScanChunk; i += kBlock) {
      const int64_t p = base + i;
      if (p < m) s += in[p];
    }
  }
  __shared__ uint64_t red[kWaves];
  s = wave_sum(s);
  if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t t = 0;
    for (int w = 0; w < kWaves; w++) t += red[w];
    sums[blockIdx.x] = t;
  }
}

// one block: exclusive scan of m uint64 in place; the total goes to *out_total (if set)
__global__ void k_scan_small(uint64_t* __restrict__ data, int64_t m, uint64_t* __restrict__ out_total) {
  __shared__ uint64_t lds[kWaves + 1];
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

// one 1024-thread block: exclusive scan of m uint64 in place (the per-tile run counts, ~25K
// elements at 100M records).  Chunks of kScanWChunk are loaded coalesced (the next chunk's
// loads in flight while the current one is scanned), transposed through LDS so each thread
// scans kScanPer consecutive elements, and stored coalesced; the total goes to *out_total.
// (Each thread walking its own contiguous run straight from HBM serialised ~24 dependent
// loads per thread: 45-240 us.)
constexpr int kScanWide = 1024;
constexpr int kScanPer = 4;
constexpr int kScanWChunk = kScanWide * kScanPer;  // 32 KB of LDS
__global__ void __launch_bounds__(kScanWide) k_scan_wide(uint64_t* __restrict__ data, int64_t m,
                                                         uint64_t* __restrict__ out_total) {
  __shared__ uint64_t s_v[kScanWChunk];
  __shared__ uint64_t lds[kScanWide / kWave + 1];
  const int t = threadIdx.x;
  uint64_t nxt[kScanPer];
#pragma unroll
  for (int k = 0; k < kScanPer; k++) {
    const int64_t p = (int64_t)k * kScanWide + t;
    nxt[k] = p < m ? data[p] : 0;
  }
  uint64_t carry = 0;
  for (int64_t base = 0; base < m; base += kScanWChunk) {
#pragma unroll
    for (int k = 0; k < kScanPer; k++) s_v[k * kScanWide + t] = nxt[k];
#pragma unroll
    for (int k = 0; k < kScanPer; k++) {
      const int64_t p = base + kScanWChunk + (int64_t)k * kScanWide + t;
      nxt[k] = p < m ? data[p] : 0;
    }
    __syncthreads();
    uint64_t v[kScanPer];
    uint64_t sum = 0;
#pragma unroll
    for (int k = 0; k < kScanPer; k++) {
      v[k] = s_v[t * kScanPer + k];
      sum += v[k];
    }
    uint64_t tot;
    uint64_t run = carry + block_exclusive_scan_n<kScanWide, uint64_t>(sum, &tot, lds);
#pragma unroll
    for (int k = 0; k < kScanPer; k++) {
      s_v[t * kScanPer + k] = run;
      run += v[k];
    }
    carry += tot;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kScanPer; k++) {
      const int64_t p = base + (int64_t)k * kScanWide + t;
      if (p < m) data[p] = s_v[k * kScanWide + t];
    }
    __syncthreads();  // the next chunk overwrites s_v
  }
  if (t == 0 && out_total) *out_total = carry;
}

// kVec: `in` and `out` are 16-byte aligned; a full chunk's thread loads and stores its 16
// consecutive counts as four uint4.
template <bool kVec>
__global__ void __launch_bounds__(kBlock) k_scan_apply(const uint32_t* __restrict__ in, int64_t m,
                                                       const uint64_t* __restrict__ block_off,
                                                       uint32_t* __restrict__ out) {
  __shared__ uint64_t lds[kWaves + 1];
  const int64_t base = (int64_t)blockIdx.x * kScanChunk;
  const uint64_t carry = block_off[blockIdx.x];
  constexpr int per = kScanChunk / kBlock;
  static_assert(per % 4 == 0, "uint4 groups");
  const bool full = kVec && base + kScanChunk <= m;
  uint32_t v[per];
  uint64_t s = 0;
  const int64_t p0 = base + (int64_t)threadIdx.x * per;
  if (full) {
    const uint4* src = reinterpret_cast<const uint4*>(in + p0);
#pragma unroll
    for (int g = 0; g < per / 4; g++) {
      const uint4 a = src[g];
      v[4 * g] = a.x;
      v[4 * g + 1] = a.y;
      v[4 * g + 2] = a.z;
      v[4 * g + 3] = a.w;
    }
  } else {
#pragma unroll
    for (int j = 0; j < per; j++) {
      const int64_t p = p0 + j;
      v[j] = p < m ? in[p] : 0;
    }
  }
#pragma unroll
  for (int j = 0; j < per; j++) s += v[j];
  uint64_t tot;
  uint64_t ex = block_exclusive_scan<uint64_t>(s, &tot, lds) + carry;
  if (full) {
    uint4* dst = reinterpret_cast<uint4*>(out + p0);
#pragma unroll
    for (int g = 0; g < per / 4; g++) {
      uint4 o;
      o.x = (uint32_t)ex;
      ex += v[4 * g];
      o.y = (uint32_t)ex;
      ex += v[4 * g + 1];
      o.z = (uint32_t)ex;
      ex += v[4 * g + 2];
      o.w = (uint32_t)ex;
      ex += v[4 * g + 3];
      dst[g] = o;
    }
  } else {
#pragma unroll
    for (int j = 0; j < per; j++) {
      const int64_t p = p0 + j;
      if (p < m) out[p] = (uint32_t)ex;
      ex += v[j];
    }
  }
}

// exclusive scan of m uint32 counts into `out`; `sums` needs cdiv(m, kScanChunk) entries
inline int scan_counts(const uint32_t* in, int64_t m, uint32_t* out, uint64_t* sums, hipStream_t s) {
  const int64_t chunks = cdiv(m, kScanChunk);
  if ((((uintptr_t)in | (uintptr_t)out) & 15) == 0) {
    LAUNCH("scan", k_scan_reduce<true>, dim3((unsigned)chunks), dim3(kBlock), s, in, m, sums);
    LAUNCH("scan", k_scan_small, dim3(1), dim3(kBlock), s, sums, chunks, (uint64_t*)nullptr);
    LAUNCH("scan", k_scan_apply<true>, dim3((unsigned)chunks), dim3(kBlock), s, in, m, (const uint64_t*)sums, out);
  } else {
    LAUNCH("scan", k_scan_reduce<false>, dim3((unsigned)chunks), dim3(kBlock), s, in, m, sums);
    LAUNCH("scan", k_scan_small, dim3(1), dim3(kBlock), s, sums, chunks, (uint64_t*)nullptr);
    LAUNCH("scan", k_scan_apply<false>, dim3((unsigned)chunks), dim3(kBlock), s, in, m, (const uint64_t*)sums, out);
  }
  return SCT_OK;
}

}  // namespace sct
