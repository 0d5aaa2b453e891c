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
//   k_gene_reduce  each block counting-sorts sub-tiles of one bucket's payloads by gene in
//                  LDS, sums each thread's runs of equal gene in registers, adds runs into
//                  LDS bins, and the bins into the rows.
// Per-gene rows are additive over cell shards: the RCCL all-reduce replaces
// MergeGeneMetrics' CSV merge (merge.py:74-191).
#pragma once
#include "fixedpt.h"
#include "radix.h"
#include "reduce.h"
#include "util.h"

namespace sct {

constexpr int kGeneChunk = 16384;  // payloads per reduce block
constexpr int kGeneSub = 1024;     // payloads sorted in LDS at a time
constexpr int kGeneItems = kGeneSub / kBlock;
constexpr int kGeneCnt = 1 + kGeneFlags;  // n_reads + flag counts (32-bit bins)
constexpr int kGeneCntPad = 16;

// Lanes of the wave holding the same `key` (nbits bits) among the lanes with `valid` set.
__device__ __forceinline__ uint64_t wave_peers(uint32_t key, int nbits, bool valid) {
  uint64_t peers = __ballot(valid);
  for (int bitn = 0; bitn < nbits; bitn++) {
    const uint64_t m = __ballot((key >> bitn) & 1u);
    peers &= ((key >> bitn) & 1u) ? m : ~m;
  }
  return peers;
}

// Rank of a lane among the block's items with the same key: one LDS atomic per distinct key in
// the wave (the lowest peer adds the group's size), so a hot key does not serialize the wave.
__device__ __forceinline__ uint32_t block_rank(uint32_t key, int nbits, bool valid, uint32_t* cnt) {
  const int lane = threadIdx.x & (kWave - 1);
  const uint64_t lt = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
  const uint64_t peers = wave_peers(key, nbits, valid);
  const int leader = peers ? __ffsll((unsigned long long)peers) - 1 : 0;
  uint32_t base = 0;
  if (valid && lane == leader) base = atomicAdd(&cnt[key], (uint32_t)__popcll(peers));
  base = (uint32_t)__shfl((int)base, leader);
  return base + (uint32_t)__popcll(peers & lt);
}

__global__ void __launch_bounds__(kBlock) k_gene_emit(const int32_t* __restrict__ gene, RecCols r,
                                                      const uint16_t* __restrict__ dflags, int64_t n,
                                                      const uint32_t* __restrict__ offsets, int n_buckets,
                                                      GenePayload* __restrict__ pay) {
  __shared__ uint32_t s_cnt[kMaxGeneBuckets];
  __shared__ uint32_t s_off[kMaxGeneBuckets];
  const int t = threadIdx.x;
  const int64_t base = (int64_t)blockIdx.x * kTile;
  const int64_t tiles = gridDim.x;
  int nbb = 0;
  while ((1 << nbb) < n_buckets) nbb++;
  for (int i = t; i < n_buckets; i += kBlock) {
    s_cnt[i] = 0;
    s_off[i] = offsets[(int64_t)i * tiles + blockIdx.x];
  }
  __syncthreads();
#pragma unroll 4
  for (int j = 0; j < kItems; j++) {
    const int64_t p = base + (int64_t)j * kBlock + t;
    const bool valid = p < n;
    GenePayload gp{};
    uint32_t bk = 0;
    if (valid) {
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
      gp.gene = g;
      gp.flags = (uint16_t)f;
      gp.uy_gt30 = r.uy_gt30[p];
      gp.uy_len = r.uy_len[p];
      gp.gq_gt30 = r.gq_gt30[p];
      gp.gq_len = r.gq_len[p];
      gp.gq_sum = r.gq_sum[p];
      gp.pad = 0;
      bk = g / kGenesPerBucket;
    }
    const uint32_t rank = block_rank(bk, nbb, valid, s_cnt);
    if (valid) reinterpret_cast<uint4*>(pay)[(uint64_t)s_off[bk] + rank] = *reinterpret_cast<const uint4*>(&gp);
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
  int32_t c[kGeneCnt];
  int64_t l[3 * kStreamLanes];
  __device__ __forceinline__ void clear() {
#pragma unroll
    for (int i = 0; i < kGeneCnt; i++) c[i] = 0;
#pragma unroll
    for (int i = 0; i < 3 * kStreamLanes; i++) l[i] = 0;
  }
  __device__ __forceinline__ void add(const GenePayload& g, double x0, double x1, double x2) {
    c[0] += 1;
#pragma unroll
    for (int f = 0; f < kGeneFlags; f++) c[1 + f] += (g.flags >> f) & 1u;
    c[1 + 9] -= (g.flags >> 14) & 1u;   // GF_MOL_SECOND on the GF_MOL_SINGLE lane
    c[1 + 11] -= (g.flags >> 15) & 1u;  // GF_FRAG_SECOND on the GF_FRAG_SINGLE lane
    fx_accumulate(l + 0 * kStreamLanes, x0);
    fx_accumulate(l + 1 * kStreamLanes, x1);
    fx_accumulate(l + 2 * kStreamLanes, x2);
  }
  __device__ __forceinline__ void flush(int32_t* cbin, unsigned long long* lbin) const {
#pragma unroll
    for (int i = 0; i < kGeneCnt; i++)
      if (c[i]) atomicAdd(&cbin[i], c[i]);
#pragma unroll
    for (int i = 0; i < 3 * kStreamLanes; i++)
      if (l[i]) atomicAdd(&lbin[i], (unsigned long long)l[i]);
  }
};

// One work item = (gene bucket, range of its payloads).  Each sub-tile of kGeneSub payloads is
// counting-sorted in LDS by local gene id, so every thread's kGeneItems consecutive payloads are
// long runs of one gene: registers accumulate a run and flush it into the LDS bins once.
__global__ void __launch_bounds__(kBlock) k_gene_reduce(const GenePayload* __restrict__ pay,
                                                        const int64_t* __restrict__ work,
                                                        const int64_t* __restrict__ n_work, int32_t n_gene_ids,
                                                        int64_t* __restrict__ partials) {
  __shared__ uint4 s_sorted[kGeneSub];
  __shared__ int32_t s_cbin[kGenesPerBucket * kGeneCntPad];
  __shared__ unsigned long long s_lbin[kGenesPerBucket * 3 * kStreamLanes];
  __shared__ uint32_t s_cnt[kGenesPerBucket];
  __shared__ uint32_t s_start[kGenesPerBucket];
  __shared__ uint64_t s_scan[kWaves + 1];
  if ((int64_t)blockIdx.x >= *n_work) return;  // block-uniform
  const int t = threadIdx.x;
  const int bucket = (int)work[3 * blockIdx.x + 0];
  const int64_t beg = work[3 * blockIdx.x + 1];
  const int64_t end = work[3 * blockIdx.x + 2];
  const uint32_t g0 = (uint32_t)bucket * kGenesPerBucket;
  for (int i = t; i < kGenesPerBucket * kGeneCntPad; i += kBlock) s_cbin[i] = 0;
  for (int i = t; i < kGenesPerBucket * 3 * kStreamLanes; i += kBlock) s_lbin[i] = 0ull;
  const uint4* src = reinterpret_cast<const uint4*>(pay);
  // A thread's run accumulator survives sub-tiles: sorted sub-tiles of one bucket put the same
  // genes at similar positions, so a thread keeps adding to one gene and flushes on change.
  GeneAcc acc;
  acc.clear();
  int cur = -1;
  for (int64_t sub = beg; sub < end; sub += kGeneSub) {
    const int cnt = (int)((end - sub) < kGeneSub ? (end - sub) : kGeneSub);
    if (t < kGenesPerBucket) s_cnt[t] = 0;
    uint4 v[kGeneItems];
    uint32_t rk[kGeneItems];
#pragma unroll
    for (int j = 0; j < kGeneItems; j++) {
      const int q = j * kBlock + t;
      if (q < cnt) v[j] = src[sub + q];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kGeneItems; j++) {
      const int q = j * kBlock + t;
      const bool valid = q < cnt;
      const uint32_t lg = valid ? v[j].x - g0 : 0u;  // GenePayload.gene is the first word
      rk[j] = block_rank(lg, 6, valid, s_cnt);
    }
    __syncthreads();
    {
      uint64_t tot;
      const uint32_t c = t < kGenesPerBucket ? s_cnt[t] : 0u;
      const uint32_t st = (uint32_t)block_exclusive_scan<uint64_t>((uint64_t)c, &tot, s_scan);
      if (t < kGenesPerBucket) s_start[t] = st;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kGeneItems; j++) {
      const int q = j * kBlock + t;
      if (q < cnt) s_sorted[s_start[v[j].x - g0] + rk[j]] = v[j];
    }
    __syncthreads();
    // the thread's kGeneItems sorted payloads; all divisions first (independent, overlapped)
    const int j0 = t * kGeneItems;
    GenePayload gs[kGeneItems];
    double xs[kGeneItems][3];
#pragma unroll
    for (int k = 0; k < kGeneItems; k++) {
      const uint4 w = j0 + k < cnt ? s_sorted[j0 + k] : make_uint4(0xFFFFFFFFu, 0, 0, 0);
      gs[k] = *reinterpret_cast<const GenePayload*>(&w);
#ifndef SCT_EXP_NO_DIV
      xs[k][0] = ratio(gs[k].uy_gt30, gs[k].uy_len);
      xs[k][1] = ratio(gs[k].gq_gt30, gs[k].gq_len);
      xs[k][2] = ratio(gs[k].gq_sum, gs[k].gq_len);
#else
      xs[k][0] = (double)gs[k].uy_gt30;
      xs[k][1] = (double)gs[k].gq_gt30;
      xs[k][2] = (double)gs[k].gq_sum;
#endif
    }
#pragma unroll
    for (int k = 0; k < kGeneItems; k++) {
      if (j0 + k >= cnt) break;
      const int lg = (int)(gs[k].gene - g0);
      if (lg != cur) {
        if (cur >= 0) acc.flush(&s_cbin[cur * kGeneCntPad], &s_lbin[cur * 3 * kStreamLanes]);
        acc.clear();
        cur = lg;
      }
#ifndef SCT_EXP_SORT_ONLY
      acc.add(gs[k], xs[k][0], xs[k][1], xs[k][2]);
#else
      acc.c[0] += (int)xs[k][0];
#endif
    }
    __syncthreads();  // s_sorted / s_cnt are reused by the next sub-tile
  }
  if (cur >= 0) acc.flush(&s_cbin[cur * kGeneCntPad], &s_lbin[cur * 3 * kStreamLanes]);
  __syncthreads();
  // bins -> partial rows: counter lanes 0..14 are partial slots 0..14; stream lanes follow P_FLOAT
  for (int i = t; i < kGenesPerBucket * kGeneCnt; i += kBlock) {
    const int lg = i / kGeneCnt, lane = i % kGeneCnt;
    const int32_t v = s_cbin[lg * kGeneCntPad + lane];
    const uint32_t gene = g0 + (uint32_t)lg;
    if (!v || (int32_t)gene >= n_gene_ids) continue;
    atomicAdd((unsigned long long*)&partials[(int64_t)gene * SCT_NP + lane], (unsigned long long)(int64_t)v);
  }
  for (int i = t; i < kGenesPerBucket * 3 * kStreamLanes; i += kBlock) {
    const int lg = i / (3 * kStreamLanes), lane = i % (3 * kStreamLanes);
    const unsigned long long v = s_lbin[i];
    const uint32_t gene = g0 + (uint32_t)lg;
    if (!v || (int32_t)gene >= n_gene_ids) continue;
    atomicAdd((unsigned long long*)&partials[(int64_t)gene * SCT_NP + P_FLOAT + lane], v);
  }
}

}  // namespace sct
