// gene.h -- grouped per-gene partials (the gene view of a cell-sharded shard).
//
// GatherGeneMetrics over the same records (gatherer.py:189-232) needs, per gene, the
// plain per-record sums plus distinct counts over (gene, cell, umi) keys.  Those keys
// are the cell view's (cell, gene, umi) keys, so the distinct-count events come from
// the cell-view sorted pass (reduce.h, DF_* flags by record index).  Here:
//   k_gene_plan    bucket starts from the per-bucket record counts (build_keys) -> the
//                  emit cursors and the reduce work list;
//   k_gene_emit    input order, coalesced: one payload per record into its gene bucket
//                  (kGenesPerBucket genes), at the range build_keys reserved per (tile, bucket); 8 bytes
//                  (gene_payload8) when the stream operands fit, else 16 (GenePayload);
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

// payloads per reduce work item (each item ends with up to kGenesPerBucket x 39 global atomics into
// the gene rows; 65536-payload items measured 0.87-0.89 ms against 0.85 at config 2)
#ifndef SCT_GENE_CHUNK
#define SCT_GENE_CHUNK 16384
#endif
constexpr int kGeneChunk = SCT_GENE_CHUNK;
// Round 4: a bucket of >= kGeneHotBucket payloads (the Zipf head holds ~55 % of the records in one
// bucket at config 2, the other buckets ~100k each) is reduced in items of kGeneChunkHot payloads:
// each item ends with up to kGenesPerBucket x 39 global atomics on its bucket's 64 gene rows, so
// fewer, larger items cut that write traffic (PMC writes 115 MB -> 63 MB with 64K items for the
// head bucket alone); smaller buckets keep kGeneChunk
#ifndef SCT_GENE_CHUNK_HOT
#define SCT_GENE_CHUNK_HOT 65536
#endif
constexpr int kGeneChunkHot = SCT_GENE_CHUNK_HOT;
constexpr uint64_t kGeneHotBucket = kGeneChunkHot;
__device__ __forceinline__ uint64_t gene_chunk(uint64_t c) { return c >= kGeneHotBucket ? kGeneChunkHot : kGeneChunk; }
constexpr int kGeneSub = 2048;  // 16-byte payloads sorted in LDS at a time (32 KB)
constexpr int kGeneCnt = 1 + kGeneFlags;  // n_reads + flag counts (32-bit bins)
constexpr int kGeneCntPad = 16;

// the GF flags of one record: its own bits plus the distinct-count events of the cell view
__device__ __forceinline__ uint32_t gene_flags(uint8_t bt, uint8_t xf, uint16_t df) {
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
  return f;
}

// The wide payload: 16 bytes (GenePayload) -- everything GatherGeneMetrics derives from a record.
__device__ __forceinline__ uint4 gene_payload(uint32_t g, uint32_t f, uint8_t uy_gt30, uint8_t uy_len,
                                              uint16_t gq_gt30, uint16_t gq_len, uint16_t gq_sum) {
  GenePayload gp;
  gp.gene = g;
  gp.flags = (uint16_t)f;
  gp.uy_gt30 = uy_gt30;
  gp.uy_len = uy_len;
  gp.gq_gt30 = gq_gt30;
  gp.gq_len = gq_len;
  gp.gq_sum = gq_sum;
  gp.pad = 0;
  return *reinterpret_cast<const uint4*>(&gp);
}

// The narrow payload: the same in 8 bytes, used when every record's stream operands fit (the
// exact-stream pass of build_keys checks them and sets *gwide otherwise; stream_tile):
//   bits 0-5 the local gene (gene mod kGenesPerBucket: the bucket is the payload's region),
//   6-20 the GF flags with EXONIC / INTRONIC / UTR (exclusive) as a 2-bit code (1, 2, 3),
//   21-25 uy_gt30, 26-30 uy_len, 31-39 gq_gt30, 40-48 gq_len, 49-63 gq_sum.
constexpr uint32_t kNarrowUy = 31, kNarrowGq = 511, kNarrowGqSum = 32767;
__device__ __forceinline__ uint64_t gene_payload8(uint32_t g, uint32_t f, uint32_t uy_gt30, uint32_t uy_len,
                                                  uint32_t gq_gt30, uint32_t gq_len, uint32_t gq_sum) {
  const uint32_t code = ((f >> 1) & 1u) | ((f >> 1) & 2u) | ((f >> 3) & 1u) * 3u;
  const uint32_t f15 = (f & 1u) | (code << 1) | ((f >> 4) << 3);
  return (uint64_t)(g & (kGenesPerBucket - 1)) | ((uint64_t)f15 << 6) | ((uint64_t)uy_gt30 << 21) |
         ((uint64_t)uy_len << 26) | ((uint64_t)gq_gt30 << 31) | ((uint64_t)gq_len << 40) | ((uint64_t)gq_sum << 49);
}

// kEmitVec consecutive elements of a column for one lane: one 4- to 16-byte load in a full
// tile (kFull: block-uniform, so no per-lane branches and no wait after every load), element
// by element with zeros past n in the last tile.  The columns are allocated 16-byte aligned.
constexpr int kEmitVec = 4;  // (the rank packing below assumes 4)
template <bool kFull, int V, typename T>
__device__ __forceinline__ void load_vec(const T* __restrict__ col, int64_t p0, int64_t n, T (&v)[V]) {
  constexpr int kW = sizeof(T) * V > 16 ? 16 / (int)sizeof(T) : V;  // elements per load (<= 16 bytes)
  struct alignas(sizeof(T) * kW) Vec {
    T x[kW];
  };
  if constexpr (kFull) {
#pragma unroll
    for (int c = 0; c < V; c += kW) {
      const Vec w = *reinterpret_cast<const Vec*>(col + p0 + c);
#pragma unroll
      for (int k = 0; k < kW; k++) v[c + k] = w.x[k];
    }
  } else {
#pragma unroll
    for (int k = 0; k < V; k++) v[k] = p0 + k < n ? col[p0 + k] : (T)0;
  }
}

// the columns gene_emit reads for one lane's V consecutive records
template <int V>
struct EmitInV {
  int32_t g[V];
  uint8_t bt[V], xf[V], ug[V], ul[V];
  uint16_t df[V], gg[V], gl[V], gs[V];
  template <bool kFull>
  __device__ __forceinline__ void load(const int32_t* __restrict__ gene, const RecCols& r,
                                       const uint16_t* __restrict__ dflags, int64_t p0, int64_t n) {
    load_vec<kFull, V>(gene, p0, n, g);
    load_vec<kFull, V>(r.bits, p0, n, bt);
    load_vec<kFull, V>(r.xf, p0, n, xf);
    load_vec<kFull, V>(r.uy_gt30, p0, n, ug);
    load_vec<kFull, V>(r.uy_len, p0, n, ul);
    load_vec<kFull, V>(dflags, p0, n, df);
    load_vec<kFull, V>(r.gq_gt30, p0, n, gg);
    load_vec<kFull, V>(r.gq_len, p0, n, gl);
    load_vec<kFull, V>(r.gq_sum, p0, n, gs);
  }
};
using EmitIn = EmitInV<kEmitVec>;

// One block per key-pass tile (kEmitTile = build_keys' kKTile records, input order, coalesced).
// build_keys counted the tile's records per gene bucket and reserved the tile's range in each
// bucket with one atomic (gtoff[tile][bucket]: the range's offset inside the bucket), so a single
// pass ranks each record within its bucket (an LDS atomic: any order inside a range is fine, the
// reduction is order-free) and writes its payload at bucket start + offset + rank; the gene column
// is read once.  Each lane takes kEmitVec consecutive records per round, so every column is read
// with one 4- to 16-byte load per lane; same-bucket lanes of one store get consecutive ranks (LDS
// atomics on one address return in lane order), so the stores coalesce.
constexpr int kEmitTile = 2 * kTile;
constexpr int kEmitRounds = kEmitTile / (kBlock * kEmitVec);

template <bool kFull, bool k8>
__device__ __forceinline__ void gene_emit_tile(const int32_t* __restrict__ gene, const RecCols& r,
                                               const uint16_t* __restrict__ dflags, int64_t n, int64_t base,
                                               const uint32_t* __restrict__ bstart, const uint32_t* __restrict__ toff,
                                               int n_buckets, void* __restrict__ pay, uint32_t* s_cnt,
                                               uint32_t* s_off) {
  const int t = threadIdx.x;
  // (entries of buckets absent from the tile were never written: read, never used)
  for (int i = t; i < n_buckets; i += kBlock) {
    s_cnt[i] = 0;
    s_off[i] = bstart[i] + toff[i];
  }
  __syncthreads();
  // software-pipelined: round j + 1's column loads are issued before round j's stores (vmcnt
  // counts stores too, so loads issued after them would wait for them)
  EmitIn cur;
  cur.load<kFull>(gene, r, dflags, base + t * kEmitVec, n);
#pragma unroll 2
  for (int j = 0; j < kEmitRounds; j++) {
    const int q0 = (j * kBlock + t) * kEmitVec;
    const int64_t p0 = base + q0;
    EmitIn nxt;
    if (j + 1 < kEmitRounds) nxt.load<kFull>(gene, r, dflags, p0 + kBlock * kEmitVec, n);
#pragma unroll
    for (int k = 0; k < kEmitVec; k++) {
      if (kFull || p0 + k < n) {
        const uint32_t gk = (uint32_t)cur.g[k];
        const uint32_t bk = gk / kGenesPerBucket;
        const uint32_t f = gene_flags(cur.bt[k], cur.xf[k], cur.df[k]);
        const uint64_t at = (uint64_t)s_off[bk] + atomicAdd(&s_cnt[bk], 1u);
        if constexpr (k8)
          reinterpret_cast<uint64_t*>(pay)[at] = gene_payload8(gk, f, cur.ug[k], cur.ul[k], cur.gg[k], cur.gl[k],
                                                               cur.gs[k]);
        else
          reinterpret_cast<uint4*>(pay)[at] = gene_payload(gk, f, cur.ug[k], cur.ul[k], cur.gg[k], cur.gl[k],
                                                           cur.gs[k]);
      }
    }
    if (j + 1 < kEmitRounds) cur = nxt;
  }
}

// The narrow payloads staged in LDS (round 4): the tile's records go out in halves of
// kEmitHalf, each counting-sorted by bucket in LDS (an atomic rank, a scan of the bucket counts)
// and written as one contiguous run per bucket range.  Written straight from registers, the 64
// lanes of a store hit ~64 buckets -- 64 cache lines per store instruction -- and the emit stalled
// on issuing its stores (SQ: wait_inst 0.69, profiles/r04/a_gene_reduce_ablation/).
#ifndef SCT_EMIT_STAGE
#define SCT_EMIT_STAGE 4096
#endif
#ifndef SCT_EMIT_VEC
#define SCT_EMIT_VEC 4
#endif
constexpr int kEmitHalf = SCT_EMIT_STAGE;  // records staged at a time
constexpr int kEmitParts = kEmitTile / kEmitHalf;
constexpr int kSVec = SCT_EMIT_VEC;  // consecutive records per lane per round
constexpr int kEmitPer = kEmitHalf / (kBlock * kSVec);  // rounds of kSVec records per stage
static_assert(kEmitHalf <= 4096 && kEmitTile % kEmitHalf == 0 && kEmitPer >= 1, "12-bit ranks, whole stages");
template <bool kFull>
__device__ __forceinline__ void gene_emit_staged(const int32_t* __restrict__ gene, const RecCols& r,
                                                 const uint16_t* __restrict__ dflags, int64_t n, int64_t base,
                                                 const uint32_t* __restrict__ bstart, const uint32_t* __restrict__ toff,
                                                 int n_buckets, uint64_t* __restrict__ pay, uint32_t* s_cnt,
                                                 uint32_t* s_off, uint32_t* s_loc, uint64_t* s_pay, uint16_t* s_bkt,
                                                 uint64_t* s_scan) {
  const int t = threadIdx.x;
  for (int i = t; i < n_buckets; i += kBlock) {
    s_cnt[i] = 0;
    s_off[i] = bstart[i] + toff[i];
  }
  __syncthreads();
  for (int h = 0; h < kEmitParts; h++) {
    const int64_t hb = base + (int64_t)h * kEmitHalf;
    uint64_t pv[kEmitPer * kSVec];
    uint32_t br[kEmitPer * kSVec];  // bucket << 12 | rank; ~0u: past n
    // software-pipelined: round j + 1's column loads in flight while round j is ranked
    EmitInV<kSVec> cur;
    cur.load<kFull>(gene, r, dflags, hb + t * kSVec, n);
#pragma unroll
    for (int j = 0; j < kEmitPer; j++) {
      const int64_t p0 = hb + (j * kBlock + t) * kSVec;
      EmitInV<kSVec> nxt;
      if (j + 1 < kEmitPer) nxt.load<kFull>(gene, r, dflags, p0 + kBlock * kSVec, n);
#pragma unroll
      for (int k = 0; k < kSVec; k++) {
        const int i = j * kSVec + k;
        br[i] = ~0u;
        pv[i] = 0;
        if (kFull || p0 + k < n) {
          const uint32_t gk = (uint32_t)cur.g[k];
          const uint32_t bk = gk / kGenesPerBucket;
          const uint32_t f = gene_flags(cur.bt[k], cur.xf[k], cur.df[k]);
          pv[i] = gene_payload8(gk, f, cur.ug[k], cur.ul[k], cur.gg[k], cur.gl[k], cur.gs[k]);
          br[i] = (bk << 12) | atomicAdd(&s_cnt[bk], 1u);
        }
      }
      if (j + 1 < kEmitPer) cur = nxt;
    }
    __syncthreads();
    // bucket counts -> staging starts (s_loc), in chunks of kBlock buckets
    uint64_t carry = 0;
    for (int b0 = 0; b0 < n_buckets; b0 += kBlock) {
      const int b = b0 + t;
      const uint64_t c = b < n_buckets ? s_cnt[b] : 0;
      uint64_t tot;
      const uint64_t ex = block_exclusive_scan<uint64_t>(c, &tot, s_scan) + carry;
      carry += tot;
      if (b < n_buckets) s_loc[b] = (uint32_t)ex;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kEmitPer * kSVec; i++) {
      if (br[i] == ~0u) continue;
      const uint32_t q = s_loc[br[i] >> 12] + (br[i] & 0xfffu);
      s_pay[q] = pv[i];
      s_bkt[q] = (uint16_t)(br[i] >> 12);
    }
    __syncthreads();
    const int cnt = (int)carry;
    for (int q = t; q < cnt; q += kBlock) {
      const uint32_t b = s_bkt[q];
      pay[(uint64_t)s_off[b] + (uint32_t)(q - (int)s_loc[b])] = s_pay[q];
    }
    __syncthreads();
    for (int i = t; i < n_buckets; i += kBlock) {
      s_off[i] += s_cnt[i];
      s_cnt[i] = 0;
    }
    __syncthreads();
  }
}

// bstart: the bucket starts (k_gene_plan); gtoff: build_keys' per-(tile, bucket) range offsets
// (narrow payloads: staged in LDS, gene_emit_staged, when the bucket arrays fit (staged); wide:
// written from registers)
constexpr int kEmitStagedBuckets = 2048;  // 3 x 8 KB of bucket arrays beside the 40 KB staging
__global__ void __launch_bounds__(kBlock) k_gene_emit(const int32_t* __restrict__ gene, RecCols r,
                                                      const uint16_t* __restrict__ dflags, int64_t n,
                                                      const uint32_t* __restrict__ bstart,
                                                      const uint32_t* __restrict__ gtoff, int n_buckets,
                                                      const uint32_t* __restrict__ gwide, int staged,
                                                      void* __restrict__ pay) {
  __shared__ uint64_t s_pay[kEmitHalf];
  __shared__ uint16_t s_bkt[kEmitHalf];
  __shared__ uint64_t s_scan[kWaves + 1];
  uint32_t* s_cnt = sct_dyn_lds;                  // n_buckets each (dynamic LDS)
  uint32_t* s_off = sct_dyn_lds + n_buckets;
  uint32_t* s_loc = sct_dyn_lds + 2 * n_buckets;
  const int64_t base = (int64_t)blockIdx.x * kEmitTile;
  const uint32_t* toff = gtoff + (size_t)blockIdx.x * n_buckets;
  const bool full = base + kEmitTile <= n, wide = *gwide != 0;  // block-uniform
  if (wide) {
    if (full) gene_emit_tile<true, false>(gene, r, dflags, n, base, bstart, toff, n_buckets, pay, s_cnt, s_off);
    else gene_emit_tile<false, false>(gene, r, dflags, n, base, bstart, toff, n_buckets, pay, s_cnt, s_off);
  } else if (!staged) {  // (more buckets than the staging's LDS allows)
    if (full) gene_emit_tile<true, true>(gene, r, dflags, n, base, bstart, toff, n_buckets, pay, s_cnt, s_off);
    else gene_emit_tile<false, true>(gene, r, dflags, n, base, bstart, toff, n_buckets, pay, s_cnt, s_off);
  } else {
    uint64_t* p8 = reinterpret_cast<uint64_t*>(pay);
    if (full)
      gene_emit_staged<true>(gene, r, dflags, n, base, bstart, toff, n_buckets, p8, s_cnt, s_off, s_loc, s_pay, s_bkt,
                             s_scan);
    else
      gene_emit_staged<false>(gene, r, dflags, n, base, bstart, toff, n_buckets, p8, s_cnt, s_off, s_loc, s_pay,
                              s_bkt, s_scan);
  }
}

// one block: bucket starts (exclusive scan of the bucket counts) -> the emit cursors and the
// reduce work list (chunks of <= kGeneChunk payloads of one bucket), written by all threads
__global__ void __launch_bounds__(kBlock) k_gene_plan(const uint32_t* __restrict__ counts, int n_buckets,
                                                      uint32_t* __restrict__ cursor, int64_t* __restrict__ work,
                                                      int64_t* __restrict__ n_work) {
  __shared__ uint64_t lds[kWaves + 1];
  uint32_t* s_beg = sct_dyn_lds;                   // n_buckets + 1 (dynamic LDS)
  uint32_t* s_woff = sct_dyn_lds + n_buckets + 1;  // n_buckets + 1
  uint64_t carry = 0, carry_w = 0;
  for (int base = 0; base < n_buckets; base += kBlock) {
    const int bk = base + threadIdx.x;
    const uint64_t c = bk < n_buckets ? counts[bk] : 0;
    uint64_t tot;
    const uint64_t beg = block_exclusive_scan<uint64_t>(c, &tot, lds) + carry;
    carry += tot;
    const uint64_t nw = (c + gene_chunk(c) - 1) / gene_chunk(c);
    uint64_t tot_w;
    const uint64_t woff = block_exclusive_scan<uint64_t>(nw, &tot_w, lds) + carry_w;
    carry_w += tot_w;
    if (bk < n_buckets) {
      cursor[bk] = (uint32_t)beg;
      s_beg[bk] = (uint32_t)beg;
      s_woff[bk] = (uint32_t)woff;
    }
  }
  if (threadIdx.x == 0) {
    s_beg[n_buckets] = (uint32_t)carry;
    s_woff[n_buckets] = (uint32_t)carry_w;
    *n_work = (int64_t)carry_w;
  }
  __syncthreads();
  for (uint32_t w = threadIdx.x; w < (uint32_t)carry_w; w += kBlock) {
    int lo = 0, hi = n_buckets - 1;  // the bucket with s_woff[b] <= w < s_woff[b + 1]
    while (lo < hi) {
      const int mid = (lo + hi + 1) / 2;
      if (s_woff[mid] <= w) lo = mid; else hi = mid - 1;
    }
    const uint64_t e = s_beg[lo + 1];
    const uint64_t ch = gene_chunk(e - s_beg[lo]);
    const uint64_t b0 = (uint64_t)s_beg[lo] + (uint64_t)(w - s_woff[lo]) * ch;
    work[3 * w + 0] = lo;
    work[3 * w + 1] = (int64_t)b0;
    work[3 * w + 2] = (int64_t)(b0 + ch < e ? b0 + ch : e);
  }
}

// One payload as the reduction uses it: the local gene, the 16 counted flag bits and the three
// stream operand pairs.
struct GeneItem {
  uint32_t lg, f, ua, ub, qa, qb, qs;
};

// The two payload formats.  kSub payloads of a sub-tile are sorted in the same 32 KB of LDS;
// slot(i) is the LDS slot of sorted position i: within each 128-byte group of payloads the slot
// is XORed with the group index, so the 64 lanes reading their k-th payload (thread t owns
// positions kItems t .. kItems t + kItems - 1) spread over the banks.
template <bool k8>
struct GeneFmt;
template <>
struct GeneFmt<false> {  // GenePayload; counted flag bit f is GF bit f
  using W = uint4;
  static constexpr int kSub = 2048;
  __device__ static uint32_t slot(uint32_t i) { return i ^ ((i >> 3) & 7u); }
  __device__ static uint32_t local(const W* p, int q, uint32_t g0) {
    return reinterpret_cast<const uint32_t*>(p)[4 * q] - g0;  // GenePayload.gene is the first word
  }
  __device__ static GeneItem item(const W& w, uint32_t g0) {
    const GenePayload& g = *reinterpret_cast<const GenePayload*>(&w);
    return GeneItem{g.gene - g0, g.flags, g.uy_gt30, g.uy_len, g.gq_gt30, g.gq_len, g.gq_sum};
  }
  template <typename B>
  __device__ static void counts(B byte, int32_t n, int32_t (&c)[kGeneCnt]) {
    c[0] = n;
#pragma unroll
    for (int f = 0; f < kGeneFlags; f++) c[1 + f] = byte(f);
    c[1 + 9] -= byte(14);   // GF_MOL_SECOND
    c[1 + 11] -= byte(15);  // GF_FRAG_SECOND
  }
};
template <>
struct GeneFmt<true> {  // gene_payload8; counted bits: 0 PERFECT, 1-2 the xf code, 3-14 GF 4-15, 15 UTR
  using W = uint2;
  static constexpr int kSub = 4096;
  __device__ static uint32_t slot(uint32_t i) { return i ^ ((i >> 4) & 15u); }
  __device__ static uint32_t local(const W* p, int q, uint32_t) {
    return reinterpret_cast<const uint32_t*>(p)[2 * q] & (kGenesPerBucket - 1);
  }
  __device__ static GeneItem item(const W& w, uint32_t) {
    const uint32_t f15 = (w.x >> 6) & 0x7fffu;
    return GeneItem{w.x & (kGenesPerBucket - 1), f15 | (((f15 >> 1) & (f15 >> 2) & 1u) << 15), (w.x >> 21) & 31u,
                    (w.x >> 26) & 31u, (w.x >> 31) | ((w.y & 0xffu) << 1), (w.y >> 8) & 511u, w.y >> 17};
  }
  template <typename B>
  __device__ static void counts(B byte, int32_t n, int32_t (&c)[kGeneCnt]) {
    c[0] = n;
    c[1] = byte(0);              // GF_PERFECT_UMI
    c[2] = byte(1) - byte(15);   // GF_EXONIC: code 1
    c[3] = byte(2) - byte(15);   // GF_INTRONIC: code 2
    c[4] = byte(15);             // GF_UTR: code 3
#pragma unroll
    for (int f = 4; f < kGeneFlags; f++) c[1 + f] = byte(f - 1);
    c[1 + 9] -= byte(13);   // GF_MOL_SECOND
    c[1 + 11] -= byte(14);  // GF_FRAG_SECOND
  }
};
static_assert(kGeneFlags == 14, "flag bits 14 and 15 are the SECOND events");

// The uy stream's exact-lane increments for one denominator (barcode lengths are fixed in a
// chemistry): entry a holds fx_increments(RN(a / B)), computed as the other samples are, so a
// table hit adds the same 8 words the arithmetic would.
constexpr int kUyTab = 32;
constexpr uint32_t kNoUyTab = 0xffffffffu;
__device__ __forceinline__ void fill_uy_tab(uint32_t B, uint4* tab) {
  const uint32_t a = threadIdx.x;
  if (a >= (uint32_t)kUyTab) return;
  const double x = (B != 0 && a <= B) ? ratio_y(a, B, 1.0 / (double)B) : 0.0;  // = ratio_rcp(a, B)
  uint32_t inc[kStreamLanes - 1];
  uint64_t inc7;
  fx_increments(x, inc, inc7);
  tab[2 * a] = make_uint4(inc[0], inc[1], inc[2], inc[3]);
  tab[2 * a + 1] = make_uint4(inc[4], inc[5], inc[6], (uint32_t)inc7);
}

// A thread's open run of one gene.  The 16 counted flag bits are counted in bytes of pk (a run
// stays open over the sub-tiles of one work item, and is flushed before it could reach
// kRunCap payloads), two 64-bit adds per payload instead of one extract-and-add per flag.
// Round 5: a payload's 16 flag bits reach the byte counters as four nibbles, each spread to four
// bytes by a 16-entry LDS table (one 32-bit read and add per nibble, in place of two 64-bit
// shift-or-mask spreads): 0.891 -> 0.886 ms at config 2, 1.069 -> 1.052 at config 4.  (A gq_gt30
// increment table like uy's, its 3.2 KB of LDS taken from the sort buffer to keep 3 blocks per CU,
// was slower: 0.999 ms.  The reduce is not VALU-bound: profiles/r05/gene_reduce/.)
__device__ __forceinline__ void fill_nib_tab(uint32_t* tab) {
  const uint32_t v = threadIdx.x;
  if (v < 16) tab[v] = (v & 1u) | ((v >> 1) & 1u) << 8 | ((v >> 2) & 1u) << 16 | ((v >> 3) & 1u) << 24;
}
struct GeneAcc {
  uint32_t pk[4];  // byte f % 4 of pk[f / 4]: #payloads with counted bit f
  int32_t n;       // n_reads
  int64_t l[3 * kStreamLanes];
  __device__ __forceinline__ void clear() {
    pk[0] = pk[1] = pk[2] = pk[3] = 0;
    n = 0;
#pragma unroll
    for (int i = 0; i < 3 * kStreamLanes; i++) l[i] = 0;
  }
  // uy_tab: the uy lane increments of a = 0 .. kUyTab - 1 over the work item's uy denominator uy_b
  // (kNoUyTab: none); other denominators are computed
  __device__ __forceinline__ void add(const GeneItem& g, const double* s_rcp, const uint4* uy_tab, uint32_t uy_b,
                                      const uint32_t* nib) {
    n += 1;
#pragma unroll
    for (int j = 0; j < 4; j++) pk[j] += nib[(g.f >> (4 * j)) & 15u];
    if (g.ub == uy_b && g.ua <= uy_b) {
      const uint4 i0 = uy_tab[2 * g.ua], i1 = uy_tab[2 * g.ua + 1];
      l[0] += i0.x, l[1] += i0.y, l[2] += i0.z, l[3] += i0.w;
      l[4] += i1.x, l[5] += i1.y, l[6] += i1.z, l[7] += i1.w;
    } else {
      fx_accumulate(l + 0 * kStreamLanes, ratio_rcp(g.ua, g.ub, s_rcp));
    }
    const double yq = rcp_of(g.qb, s_rcp);  // the two gq quotients share the reciprocal
    fx_accumulate(l + 1 * kStreamLanes, ratio_y(g.qa, g.qb, yq));
    fx_accumulate(l + 2 * kStreamLanes, ratio_y(g.qs, g.qb, yq));
  }
  __device__ __forceinline__ int32_t byte(int f) const { return (int32_t)((pk[f / 4] >> (8 * (f % 4))) & 0xffu); }
  // unconditional adds (zeros included): a per-lane test would cost an exec-mask round per lane
  template <bool k8>
  __device__ __forceinline__ void flush(int32_t* cbin, unsigned long long* lbin) const {
    int32_t c[kGeneCnt];
    GeneFmt<k8>::counts([this](int f) { return byte(f); }, n, c);
#pragma unroll
    for (int i = 0; i < kGeneCnt; i++) atomicAdd(&cbin[i], c[i]);
#pragma unroll
    for (int i = 0; i < 3 * kStreamLanes; i++) atomicAdd(&lbin[i], (unsigned long long)l[i]);
  }
};
constexpr int kRunCap = 255;  // byte counters
static_assert(GeneFmt<false>::kSub / kBlock <= kRunCap / 2 && GeneFmt<true>::kSub / kBlock <= kRunCap / 2,
              "a sub-tile adds at most kItems payloads to an open run");

// Segmented inclusive DPP scan over the wave: lanes hold partial sums of the segment (adjacent
// lanes with equal keys) that starts at lane `seg`.  Step j adds the value of the lane 1, 2, 4, 8
// lanes back inside the row (row_shr), then of lane 15 of the previous row (row_bcast:15, rows 1
// and 3) and of lane 31 (row_bcast:31, rows 2 and 3), where that lane lies in the segment
// (m[j]); a step no lane needs is skipped (wave-uniform).  Afterwards the last lane of every
// segment holds the segment's sum.  The DPP moves have no `old` operand: lanes whose source is
// invalid are exactly the lanes with m[j] false.
constexpr int kGenePack = 9;  // counted flags as 16-bit pairs (8 words) + n_reads

template <int kCtrl, int kRowMask>
__device__ __forceinline__ uint32_t dpp_raw(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, kCtrl, kRowMask, 0xf, false);
}

template <int kCtrl, int kRowMask>
__device__ __forceinline__ void seg_step(uint32_t (&c)[kGenePack], int64_t (&l)[3 * kStreamLanes], bool m) {
#pragma unroll
  for (int i = 0; i < kGenePack; i++) {
    const uint32_t x = dpp_raw<kCtrl, kRowMask>(c[i]);
    c[i] += m ? x : 0u;
  }
#pragma unroll
  for (int i = 0; i < 3 * kStreamLanes; i++) {
    const uint64_t v = (uint64_t)l[i];
    const uint64_t x = ((uint64_t)dpp_raw<kCtrl, kRowMask>((uint32_t)(v >> 32)) << 32) |
                       dpp_raw<kCtrl, kRowMask>((uint32_t)v);
    l[i] += m ? (int64_t)x : 0;
  }
}

// Flush the wave's run accumulators: lane runs of gene `key` (< 0: nothing to flush; the lane's
// accumulator is left as it is).  Segments are maximal groups of adjacent lanes with one key;
// after the segmented scan the last lane of each segment adds its gene's sums to the LDS bins --
// one atomic per (segment, value), no two lanes on one address.  Every lane must call it, all
// active; lanes with key >= 0 must clear their accumulator afterwards.
template <bool k8>
__device__ __forceinline__ void gene_wave_flush(GeneAcc& acc, int key, int32_t* s_cbin, unsigned long long* s_lbin) {
  const int lane = threadIdx.x & (kWave - 1);
  const int prev = __shfl_up(key, 1);
  const uint64_t heads = __ballot(lane == 0 || prev != key);
  const uint64_t upto = lane == kWave - 1 ? ~0ull : ((1ull << (lane + 1)) - 1);
  const int seg = kWave - 1 - __clzll((unsigned long long)(heads & upto));
  const int p = lane & 15;
  const bool m0 = p >= 1 && seg <= lane - 1, m1 = p >= 2 && seg <= lane - 2;
  const bool m2 = p >= 4 && seg <= lane - 4, m3 = p >= 8 && seg <= lane - 8;
  const bool m4 = ((lane >> 4) & 1) && seg < (lane & ~15), m5 = lane >= 32 && seg <= 31;
  // counted flags in 16-bit halves (a lane's run has < 256 payloads, a segment < 2^16)
  uint32_t c[kGenePack];
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const uint32_t w = acc.pk[j / 2] >> (16 * (j % 2));
    c[j] = (w & 0xffu) | (((w >> 8) & 0xffu) << 16);
  }
  c[8] = (uint32_t)acc.n;
  if (__ballot(m0)) seg_step<0x111, 0xf>(c, acc.l, m0);  // row_shr:1
  if (__ballot(m1)) seg_step<0x112, 0xf>(c, acc.l, m1);  // row_shr:2
  if (__ballot(m2)) seg_step<0x114, 0xf>(c, acc.l, m2);  // row_shr:4
  if (__ballot(m3)) seg_step<0x118, 0xf>(c, acc.l, m3);  // row_shr:8
  if (__ballot(m4)) seg_step<0x142, 0xa>(c, acc.l, m4);  // row_bcast:15
  if (__ballot(m5)) seg_step<0x143, 0xc>(c, acc.l, m5);  // row_bcast:31
  const bool tail = lane == kWave - 1 || ((heads >> (lane + 1)) & 1ull);
  if (tail && key >= 0) {
    int32_t* cb = &s_cbin[key * kGeneCntPad];
    unsigned long long* lb = &s_lbin[key * 3 * kStreamLanes];
    int32_t cnt[kGeneCnt];
    GeneFmt<k8>::counts([&c](int f) { return (int32_t)((c[f / 2] >> (16 * (f % 2))) & 0xffffu); }, (int32_t)c[8],
                        cnt);
#pragma unroll
    for (int i = 0; i < kGeneCnt; i++) atomicAdd(&cb[i], cnt[i]);
#pragma unroll
    for (int i = 0; i < 3 * kStreamLanes; i++) atomicAdd(&lb[i], (unsigned long long)acc.l[i]);
  }
}

// One work item = (gene bucket, range [beg, end) of its payloads).  Each sub-tile of kSub
// payloads is counting-sorted in LDS by local gene id, so every thread's kItems consecutive
// payloads are long runs of one gene: registers accumulate a run; a run that ends inside the
// thread's payloads goes to the LDS bins directly.  The run still open at the end of a sub-tile
// stays in registers (in the next sub-tile the thread's positions mostly hold the same gene:
// sub-tiles of one bucket have the same gene mix); lanes whose next payloads start another gene
// flush together through the segmented DPP scan (gene_wave_flush), as do all open runs at the
// end of the work item.
template <bool k8>
__device__ __forceinline__ void gene_reduce_item(const void* __restrict__ pay, int64_t beg, int64_t end, uint32_t g0,
                                                 uint4* s_buf, int32_t* s_cbin, unsigned long long* s_lbin,
                                                 uint32_t* s_cnt, uint32_t* s_start, uint64_t* s_scan,
                                                 const double* s_rcp, uint4* s_uytab, const uint32_t* s_nib) {
  using F = GeneFmt<k8>;
  using W = typename F::W;
  constexpr int kSub = F::kSub, kItems = kSub / kBlock;
  static_assert(kSub * sizeof(W) == kGeneSub * sizeof(uint4), "one LDS buffer");
  const W* src = reinterpret_cast<const W*>(pay);
  W* s_sorted = reinterpret_cast<W*>(s_buf);
  const int t = threadIdx.x;
#ifndef SCT_GENE_UYTAB
#define SCT_GENE_UYTAB 1
#endif
  // the work item's first payload's uy denominator (block-uniform), tabulated when < kUyTab
  const uint32_t ub0 = F::item(src[beg], g0).ub;
  const uint32_t uy_b = (SCT_GENE_UYTAB && ub0 < (uint32_t)kUyTab) ? ub0 : kNoUyTab;
  if (uy_b != kNoUyTab) fill_uy_tab(uy_b, s_uytab);  // visible after the first sub-tile's barriers
  GeneAcc acc;
  acc.clear();
  int cur = -1;
  for (int64_t sub = beg; sub < end; sub += kSub) {
    const int cnt = (int)((end - sub) < kSub ? (end - sub) : kSub);
    if (t < kGenesPerBucket) s_cnt[t] = 0;
    // rank on the gene word alone (clamped, unconditional loads: all in flight at once), then
    // re-read the whole payload for the LDS scatter (an L2 hit)
    uint32_t vx[kItems];  // local gene, then | rank << 8 (one register per item)
#pragma unroll
    for (int j = 0; j < kItems; j++) {
      const int q = j * kBlock + t;
      vx[j] = F::local(src + sub, q < cnt ? q : cnt - 1, g0);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kItems; j++) {
      const int q = j * kBlock + t;
      const bool valid = q < cnt;
      vx[j] |= (valid ? atomicAdd(&s_cnt[vx[j]], 1u) : 0u) << 8;  // LDS atomics: faster than wave-aggregated ranks
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
    for (int j = 0; j < kItems; j++) {
      const int q = j * kBlock + t;
      if (q < cnt) s_sorted[F::slot(s_start[vx[j] & 0xffu] + (vx[j] >> 8))] = src[sub + q];
    }
    __syncthreads();
    // the thread's kItems consecutive sorted payloads; its open run continues if they start with
    // its gene, else the wave's changed runs are flushed together first
    const int j0 = t * kItems;
    const int my_n = cnt - j0 < 0 ? 0 : (cnt - j0 < kItems ? cnt - j0 : kItems);
    {
      // a run continues into this sub-tile if it starts with the run's gene and its byte
      // counters have room for kItems more payloads
      const int first = my_n > 0 ? (int)F::item(s_sorted[F::slot(j0)], g0).lg : cur;
      const bool changed = cur >= 0 && (first != cur || acc.n > kRunCap - kItems);
      if (__ballot(changed)) {
        gene_wave_flush<k8>(acc, changed ? cur : -2 - (t & (kWave - 1)), s_cbin, s_lbin);
        if (changed) {
          acc.clear();
          cur = -1;
        }
      }
    }
    for (int k = 0; k < my_n; k++) {
      const GeneItem g = F::item(s_sorted[F::slot(j0 + k)], g0);
      if ((int)g.lg != cur) {  // a gene boundary inside the thread's payloads: its own bin, no conflict
        if (cur >= 0) acc.flush<k8>(&s_cbin[cur * kGeneCntPad], &s_lbin[cur * 3 * kStreamLanes]);
        acc.clear();
        cur = (int)g.lg;
      }
      acc.add(g, s_rcp, s_uytab, uy_b, s_nib);
    }
    __syncthreads();  // s_sorted / s_cnt are reused by the next sub-tile
  }
  // the threads' open runs, combined across each wave
  gene_wave_flush<k8>(acc, cur, s_cbin, s_lbin);
}

// 3 waves per SIMD (the LDS allows 3 blocks per CU): <= 168 VGPRs, a few spills off the item loop
// (measured 1.07 ms against 1.26 ms at the unconstrained 200 VGPRs, config 2)
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(3))) k_gene_reduce(const void* __restrict__ pay, const int64_t* __restrict__ work,
                                                        const int64_t* __restrict__ n_work, int32_t n_gene_ids,
                                                        const uint32_t* __restrict__ gwide,
                                                        int64_t* __restrict__ partials) {
  __shared__ uint4 s_buf[kGeneSub];
  __shared__ int32_t s_cbin[kGenesPerBucket * kGeneCntPad];
  __shared__ unsigned long long s_lbin[kGenesPerBucket * 3 * kStreamLanes];
  __shared__ uint32_t s_cnt[kGenesPerBucket];
  __shared__ uint32_t s_start[kGenesPerBucket];
  __shared__ uint64_t s_scan[kWaves + 1];
  __shared__ double s_rcp[kRcpN];
  __shared__ uint4 s_uytab[2 * kUyTab];
  __shared__ uint32_t s_nib[16];
  if ((int64_t)blockIdx.x >= *n_work) return;  // block-uniform
  const int t = threadIdx.x;
  fill_rcp(s_rcp);  // visible after the first sub-tile's barriers
  fill_nib_tab(s_nib);
  const int bucket = (int)work[3 * blockIdx.x + 0];
  const int64_t beg = work[3 * blockIdx.x + 1];
  const int64_t end = work[3 * blockIdx.x + 2];
  const uint32_t g0 = (uint32_t)bucket * kGenesPerBucket;
  for (int i = t; i < kGenesPerBucket * kGeneCntPad; i += kBlock) s_cbin[i] = 0;
  for (int i = t; i < kGenesPerBucket * 3 * kStreamLanes; i += kBlock) s_lbin[i] = 0ull;
  if (*gwide)  // block-uniform
    gene_reduce_item<false>(pay, beg, end, g0, s_buf, s_cbin, s_lbin, s_cnt, s_start, s_scan, s_rcp, s_uytab, s_nib);
  else
    gene_reduce_item<true>(pay, beg, end, g0, s_buf, s_cbin, s_lbin, s_cnt, s_start, s_scan, s_rcp, s_uytab, s_nib);
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
