// gene.h -- grouped per-gene partials (the gene view of a cell-sharded shard).
//
// GatherGeneMetrics over the same records (gatherer.py:189-232) needs, per gene, the
// plain per-record sums plus distinct counts over (gene, cell, umi) keys.  Those keys
// are the cell view's (cell, gene, umi) keys, so the distinct-count events come from
// the cell-view sorted pass (reduce.h, DF_* flags by record index).  Here:
//   k_gene_emit    input order, coalesced: one 16-byte GenePayload per record into its
//                  gene bucket (kGenesPerBucket genes) at offsets from the per-tile
//                  bucket count matrix (segment.h) -- no atomics across blocks;
//   k_gene_plan    bucket extents -> block work list;
//   k_gene_reduce  each block streams a slice of one bucket through LDS, sums runs of
//                  equal gene in registers (a (cell, gene) pair's records stay
//                  adjacent), adds runs into LDS bins, and the bins into the rows.
// Per-gene rows are additive over cell shards: the RCCL all-reduce replaces
// MergeGeneMetrics' CSV merge (merge.py:74-191).
#pragma once
#include "fixedpt.h"
#include "radix.h"
#include "reduce.h"
#include "util.h"

namespace sct {

constexpr int kGeneChunk = 65536;  // payloads per reduce block
constexpr int kGeneSub = 2048;     // payloads staged in LDS at a time
constexpr int kGeneItems = kGeneSub / kBlock;

__global__ void __launch_bounds__(kBlock) k_gene_emit(const int32_t* __restrict__ gene, RecCols r,
                                                      const uint16_t* __restrict__ dflags, int64_t n,
                                                      const uint32_t* __restrict__ offsets, int n_buckets,
                                                      GenePayload* __restrict__ pay) {
  __shared__ uint32_t s_cnt[kMaxGeneBuckets];
  const int t = threadIdx.x;
  const int64_t base = (int64_t)blockIdx.x * kTile;
  const int64_t tiles = gridDim.x;
  for (int i = t; i < n_buckets; i += kBlock) s_cnt[i] = 0;
  __syncthreads();
  for (int j = 0; j < kItems; j++) {
    const int64_t p = base + (int64_t)j * kBlock + t;
    if (p >= n) break;
    const uint32_t g = (uint32_t)gene[p];
    const uint8_t bt = r.bits[p];
    const uint8_t xf = r.xf[p];
    const uint16_t df = dflags[p];
    uint32_t f = (bt & SCT_B_PERFECT_UMI) ? GF_PERFECT_UMI : 0;
    if (!(bt & SCT_B_UNMAPPED)) {
      f |= (xf == SCT_XF_CODING ? GF_EXONIC : 0) | (xf == SCT_XF_INTRONIC ? GF_INTRONIC : 0) |
           (xf == SCT_XF_UTR ? GF_UTR : 0) | ((bt & SCT_B_NH1) ? GF_UNIQUE : GF_MULTIPLE) |
           ((bt & SCT_B_DUPLICATE) ? GF_DUP : 0) | ((bt & SCT_B_SPLICED) ? GF_SPLICED : 0);
    }
    f |= (df & DF_MOL_HEAD ? GF_MOL_HEAD : 0) | (df & DF_MOL_SINGLE ? GF_MOL_SINGLE : 0) |
         (df & DF_FRAG_FIRST ? GF_FRAG_FIRST : 0) | (df & DF_FRAG_SINGLE ? GF_FRAG_SINGLE : 0) |
         (df & DF_K1_HEAD ? GF_CG_HEAD : 0) | (df & DF_K1_MULTI ? GF_CG_MULTI : 0) |
         (df & DF_MOL_SECOND ? GF_MOL_SECOND : 0) | (df & DF_FRAG_SECOND ? GF_FRAG_SECOND : 0);
    GenePayload gp;
    gp.gene = g;
    gp.flags = (uint16_t)f;
    gp.uy_gt30 = r.uy_gt30[p];
    gp.uy_len = r.uy_len[p];
    gp.gq_gt30 = r.gq_gt30[p];
    gp.gq_len = r.gq_len[p];
    gp.gq_sum = r.gq_sum[p];
    gp.pad = 0;
    const uint32_t bk = g / kGenesPerBucket;
    const uint32_t rank = atomicAdd(&s_cnt[bk], 1u);
    pay[(uint64_t)offsets[(int64_t)bk * tiles + blockIdx.x] + rank] = gp;
  }
}

// one block: bucket extents from the scanned count matrix -> block work list
__global__ void k_gene_plan(const uint32_t* __restrict__ offsets, int64_t tiles, int n_buckets, int64_t n,
                            int64_t* __restrict__ work, int64_t* __restrict__ n_work) {
  __shared__ uint64_t lds[kWaves + 1];
  uint64_t carry_w = 0;
  for (int base = 0; base < n_buckets; base += kBlock) {
    const int bk = base + threadIdx.x;
    uint64_t beg = 0, end = 0;
    if (bk < n_buckets) {
      beg = offsets[(int64_t)bk * tiles];
      end = bk + 1 < n_buckets ? offsets[(int64_t)(bk + 1) * tiles] : (uint64_t)n;
    }
    const uint64_t nw = (end - beg + kGeneChunk - 1) / kGeneChunk;
    uint64_t tot_w;
    const uint64_t woff = block_exclusive_scan<uint64_t>(nw, &tot_w, lds) + carry_w;
    for (uint64_t k = 0; k < nw; k++) {
      const uint64_t b0 = beg + k * kGeneChunk;
      const uint64_t b1 = (b0 + kGeneChunk < end) ? b0 + kGeneChunk : end;
      work[3 * (woff + k) + 0] = bk;
      work[3 * (woff + k) + 1] = (int64_t)b0;
      work[3 * (woff + k) + 2] = (int64_t)b1;
    }
    carry_w += tot_w;
  }
  if (threadIdx.x == 0) *n_work = (int64_t)carry_w;
}

struct GeneAcc {
  int32_t c[1 + kGeneFlags];
  int64_t l[3 * kStreamLanes];
  __device__ __forceinline__ void clear() {
#pragma unroll
    for (int i = 0; i < 1 + kGeneFlags; i++) c[i] = 0;
#pragma unroll
    for (int i = 0; i < 3 * kStreamLanes; i++) l[i] = 0;
  }
  __device__ __forceinline__ void flush(unsigned long long* bin) const {
#pragma unroll
    for (int i = 0; i < 1 + kGeneFlags; i++)
      if (c[i]) atomicAdd(&bin[i], (unsigned long long)(int64_t)c[i]);  // may be negative
#pragma unroll
    for (int i = 0; i < 3 * kStreamLanes; i++)
      if (l[i]) atomicAdd(&bin[1 + kGeneFlags + i], (unsigned long long)l[i]);
  }
};

__global__ void __launch_bounds__(kBlock) k_gene_reduce(const GenePayload* __restrict__ pay,
                                                        const int64_t* __restrict__ work,
                                                        const int64_t* __restrict__ n_work, int32_t n_gene_ids,
                                                        int64_t* __restrict__ partials) {
  __shared__ unsigned long long bins[kGenesPerBucket * kGeneLanes];
  __shared__ uint4 tile[kGeneSub];
  if ((int64_t)blockIdx.x >= *n_work) return;  // block-uniform
  const int bucket = (int)work[3 * blockIdx.x + 0];
  const int64_t beg = work[3 * blockIdx.x + 1];
  const int64_t end = work[3 * blockIdx.x + 2];
  const uint32_t g0 = (uint32_t)bucket * kGenesPerBucket;
  for (int i = threadIdx.x; i < kGenesPerBucket * kGeneLanes; i += kBlock) bins[i] = 0;
  const uint4* src = reinterpret_cast<const uint4*>(pay);
  for (int64_t sub = beg; sub < end; sub += kGeneSub) {
    const int cnt = (int)((end - sub) < kGeneSub ? (end - sub) : kGeneSub);
    __syncthreads();
    for (int i = threadIdx.x; i < cnt; i += kBlock) tile[i] = src[sub + i];
    __syncthreads();
    GeneAcc acc;
    acc.clear();
    int cur = -1;
    const int j0 = threadIdx.x * kGeneItems;
    for (int j = j0; j < j0 + kGeneItems && j < cnt; j++) {
      const GenePayload g = reinterpret_cast<const GenePayload*>(tile)[j];
      const int lg = (int)(g.gene - g0);
      if (lg != cur) {
        if (cur >= 0) acc.flush(&bins[cur * kGeneLanes]);
        acc.clear();
        cur = lg;
      }
      acc.c[0] += 1;
#pragma unroll
      for (int f = 0; f < kGeneFlags; f++) acc.c[1 + f] += (g.flags >> f) & 1u;
      acc.c[1 + 9] -= (g.flags >> 14) & 1u;   // GF_MOL_SECOND on the GF_MOL_SINGLE lane
      acc.c[1 + 11] -= (g.flags >> 15) & 1u;  // GF_FRAG_SECOND on the GF_FRAG_SINGLE lane
      fx_accumulate(acc.l + 0 * kStreamLanes, ratio(g.uy_gt30, g.uy_len));
      fx_accumulate(acc.l + 1 * kStreamLanes, ratio(g.gq_gt30, g.gq_len));
      fx_accumulate(acc.l + 2 * kStreamLanes, ratio(g.gq_sum, g.gq_len));
    }
    if (cur >= 0) acc.flush(&bins[cur * kGeneLanes]);
  }
  __syncthreads();
  // bins -> partial rows: lanes 0..14 are partial slots 0..14; stream lanes follow P_FLOAT
  for (int i = threadIdx.x; i < kGenesPerBucket * kGeneLanes; i += kBlock) {
    const unsigned long long v = bins[i];
    if (!v) continue;
    const int lg = i / kGeneLanes, lane = i % kGeneLanes;
    const uint32_t gene = g0 + (uint32_t)lg;
    if ((int32_t)gene >= n_gene_ids) continue;
    const int slot = lane < 1 + kGeneFlags ? lane : P_FLOAT + (lane - 1 - kGeneFlags);
    atomicAdd((unsigned long long*)&partials[(int64_t)gene * SCT_NP + slot], v);
  }
}

}  // namespace sct
