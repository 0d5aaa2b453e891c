// exchange.h -- records binned by cell for the exchange between devices.
//
// The reference makes cell-disjoint chunks of an unsorted BAM with SplitBam: every barcode gets a
// bin (bam.py:439-448), each input file is written out bin by bin (write_barcodes_to_bins,
// bam.py:454-463) and the pieces of a bin are merged (bam.py:465-480); each chunk is then
// TagSortBam-ed (platform.py:55-97) and measured.  Across devices here:
//
//   k_bin_hist     per tile of kBinTile records: how many go to each bin;
//   (scan)         bin-major exclusive scan of the tile counts -> each tile's offset per bin;
//   k_bin_scatter  each tile ranked stably by bin (wave multi-split on the bin's bits, as the
//                  radix passes do), staged in LDS in bin order and written as one run per bin --
//                  SoA in, SoA out, the optional tiebreak column (query-name rank) carried along;
//   k_bin_totals   the records of each bin.
//
// Bins keep input order inside (stable), so a device that receives bin r of every device in
// device order holds its cells' records in file order -- the same order one device would see, so
// the tag sort that follows (stable, tagsort.h) gives the same records in the same order.
#pragma once
#include "radix.h"
#include "util.h"

namespace sct {

constexpr int kMaxBins = 256;
constexpr int kBinItems = 4;
constexpr int kBinTile = kBlock * kBinItems;  // 1024 records: 36 KB of rows and ties in LDS

// bin of a cell id: the caller's table, or contiguous id ranges (cell * n_bins / n_cell_ids; ids
// are ranks of the sorted barcodes, so bin order is barcode order)
__device__ __forceinline__ uint32_t cell_bin(uint32_t cell, const uint8_t* __restrict__ table, uint32_t n_bins,
                                             uint32_t n_cell_ids) {
  const uint32_t c = cell < n_cell_ids ? cell : n_cell_ids - 1;  // (ids are checked on the host)
  if (table) {
    const uint32_t b = table[c];
    return b < n_bins ? b : n_bins - 1;
  }
  return (uint32_t)(((uint64_t)c * n_bins) / n_cell_ids);
}

__global__ void __launch_bounds__(kBlock) k_bin_hist(const int32_t* __restrict__ cell, int64_t n,
                                                     const uint8_t* __restrict__ table, uint32_t n_bins,
                                                     uint32_t n_cell_ids, int64_t tiles, uint32_t* __restrict__ counts) {
  __shared__ uint32_t hist[kWaves][kMaxBins];
  const int wid = threadIdx.x / kWave;
  for (int i = threadIdx.x; i < kWaves * kMaxBins; i += kBlock) (&hist[0][0])[i] = 0;
  __syncthreads();
  const unsigned tile = xcd_tile(blockIdx.x, gridDim.x);
  const int64_t base = (int64_t)tile * kBinTile;
#pragma unroll
  for (int j = 0; j < kBinItems; j++) {
    const int64_t p = base + (int64_t)j * kBlock + threadIdx.x;
    if (p < n) atomicAdd(&hist[wid][cell_bin((uint32_t)cell[p], table, n_bins, n_cell_ids)], 1u);
  }
  __syncthreads();
  const uint32_t d = threadIdx.x;  // kMaxBins == kBlock
  if (d < n_bins) {
    uint32_t t = 0;
#pragma unroll
    for (int w = 0; w < kWaves; w++) t += hist[w][d];
    counts[(int64_t)d * tiles + tile] = t;
  }
}
static_assert(kMaxBins == kBlock, "one thread per bin");

template <bool kTie>
__global__ void __launch_bounds__(kBlock) k_bin_scatter(sct_records_t in, const int32_t* __restrict__ tie_in,
                                                        sct_records_t out, int32_t* __restrict__ tie_out, int64_t n,
                                                        const uint8_t* __restrict__ table, uint32_t n_bins,
                                                        uint32_t n_cell_ids, int bin_bits, int64_t tiles,
                                                        const uint32_t* __restrict__ offsets) {
  __shared__ uint4 s_rows[2 * kBinTile];
  __shared__ uint32_t s_tie[kTie ? kBinTile : 1];
  __shared__ uint8_t s_dig[kBinTile];
  __shared__ uint32_t s_whist[kWaves][kMaxBins];
  __shared__ uint32_t s_dstart[kMaxBins];
  __shared__ uint32_t s_goff[kMaxBins];
  __shared__ uint64_t s_scan[kWaves + 1];
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  const unsigned tile = xcd_tile(blockIdx.x, gridDim.x);
  const int64_t base = (int64_t)tile * kBinTile;
  const int tile_n = (int)((n - base) < kBinTile ? (n - base) : kBinTile);
  for (int i = threadIdx.x; i < kWaves * kMaxBins; i += kBlock) (&s_whist[0][0])[i] = 0;
  s_goff[threadIdx.x] = threadIdx.x < n_bins ? offsets[(int64_t)threadIdx.x * tiles + tile] : 0u;
  __syncthreads();
  const uint64_t lt = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
  uint4 ra[kBinItems], rb[kBinItems];
  uint32_t tv[kBinItems];
  uint16_t rank[kBinItems];
  uint8_t dig[kBinItems];
  // wave `wid` owns tile positions [wid * kBinItems * 64, ...): ranks follow input order (stable)
#pragma unroll
  for (int j = 0; j < kBinItems; j++) {
    const int q = wid * (kBinItems * kWave) + j * kWave + lane;
    const int64_t p = base + q;
    uint32_t d = kMaxBins - 1;  // padding: ranked last, never written
    tv[j] = 0;
    if (q < tile_n) {
      ra[j] = make_uint4((uint32_t)in.cell[p], (uint32_t)in.umi[p], (uint32_t)in.gene[p], (uint32_t)in.ref[p]);
      rb[j] = make_uint4((uint32_t)in.pos[p], (uint32_t)in.gq_sum[p] | ((uint32_t)in.gq_len[p] << 16),
                         (uint32_t)in.gq_gt30[p] | ((uint32_t)in.bits[p] << 16) | ((uint32_t)in.xf[p] << 24),
                         (uint32_t)in.cy_gt30[p] | ((uint32_t)in.cy_len[p] << 8) | ((uint32_t)in.uy_gt30[p] << 16) |
                             ((uint32_t)in.uy_len[p] << 24));
      if constexpr (kTie) tv[j] = (uint32_t)tie_in[p];
      d = cell_bin(ra[j].x, table, n_bins, n_cell_ids);
    }
    dig[j] = (uint8_t)d;
    // lanes with the same bin: ballots on the bin's bits (the padding's all-ones value included)
    uint64_t peers = ~0ull;
    for (int bitn = 0; bitn < kRadixBits; bitn++) {
      if (bitn >= bin_bits) {  // (wave-uniform)
        // bits above the bins' width: only padding lanes set them
        const uint64_t m = __ballot(d >= n_bins);
        peers &= (d >= n_bins) ? m : ~m;
        break;
      }
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
  for (int j = 0; j < kBinItems; j++) {
    const int q = wid * (kBinItems * kWave) + j * kWave + lane;
    if (q < tile_n) {
      const uint32_t lp = s_whist[wid][dig[j]] + rank[j];
      s_rows[2 * lp] = ra[j];
      s_rows[2 * lp + 1] = rb[j];
      s_dig[lp] = dig[j];
      if constexpr (kTie) s_tie[lp] = tv[j];
    }
  }
  __syncthreads();
  for (int q = threadIdx.x; q < tile_n; q += kBlock) {
    const uint4 a = s_rows[2 * q];
    const uint4 b = s_rows[2 * q + 1];
    const uint32_t d = s_dig[q];
    const uint64_t o = (uint64_t)s_goff[d] + (uint32_t)(q - (int)s_dstart[d]);
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
    if constexpr (kTie) tie_out[o] = (int32_t)s_tie[q];
  }
}

// records per bin from the scanned (bin-major) tile offsets
__global__ void k_bin_totals(const uint32_t* __restrict__ offsets, int64_t tiles, uint32_t n_bins, int64_t n,
                             int64_t* __restrict__ bin_counts) {
  const uint32_t b = threadIdx.x;
  if (b >= n_bins) return;
  const int64_t lo = offsets[(int64_t)b * tiles];
  const int64_t hi = b + 1 < n_bins ? (int64_t)offsets[(int64_t)(b + 1) * tiles] : n;
  bin_counts[b] = hi - lo;
}

}  // namespace sct
