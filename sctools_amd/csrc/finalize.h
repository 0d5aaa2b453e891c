// finalize.h -- partial rows -> output rows, and the sequential-Welford float path.
#pragma once
#include "fixedpt.h"
#include "reduce.h"
#include "util.h"

namespace sct {

// MetricAggregator.finalize (aggregator.py:342-387), CellMetrics.finalize (463-490),
// GeneMetrics.finalize (571-578): kFinThreads threads per row -- thread 0 the integer columns and
// ratios, thread s the exact mean / variance of stream s (each a few big-integer divisions, so a
// row's four streams run side by side).  Launch with rows * kFinThreads threads.
constexpr int kFinThreads = 4;
static_assert(kFinThreads == kStreams, "one thread per quality stream");
__global__ void k_finalize(const int64_t* __restrict__ partials, int64_t rows, int mode, int exact,
                           const int64_t* __restrict__ ent_start, int64_t* __restrict__ out_i,
                           double* __restrict__ out_f) {
  const int64_t idx = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t r = idx / kFinThreads;
  const int st = (int)(idx % kFinThreads);
  if (r >= rows) return;
  const int64_t* P = partials + r * SCT_NP;
  int64_t* I = out_i + r * SCT_NI;
  double* F = out_f + r * SCT_NF;
  if (exact) {
    const int mean_col = st == 0 ? SCT_F_UY_MEAN : st == 1 ? SCT_F_GQF_MEAN : st == 2 ? SCT_F_GQ_MEAN : SCT_F_CY_MEAN;
    const int var_col = st == 0 ? SCT_F_UY_VAR : st == 1 ? SCT_F_GQF_VAR : st == 2 ? SCT_F_GQ_VAR : SCT_F_CY_VAR;
    if (st < 3 || mode == SCT_MODE_CELL) {
      fx_finalize(P + P_FLOAT + st * kStreamLanes, P[P_N_READS], &F[mean_col], &F[var_col]);
    } else {
      F[mean_col] = 0.0;
      F[var_col] = 0.0;
    }
  }
  if (st != 0) return;
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
}

// OnlineGaussianSufficientStatistic.update (stats.py:82-87), one operation per rounding
struct Welford {
  double mean, m2;
  __device__ __forceinline__ void update(double x, double cnt) {
    const double delta = x - mean;
    mean += delta / cnt;
    const double delta2 = x - mean;
    m2 += delta * delta2;
  }
};

// Sequential Welford per entity in record order.  Welford is a rounding recurrence: record k's
// update depends on record k-1's rounded mean, so an entity's chain cannot be split.  What can
// run in parallel is everything off the chain, and entities run side by side:
//   * entities of < kWfWave records: one lane each (k_welford);
//   * larger ones: one lane per (entity, stream) chain (k_welford_chains), largest first
//     (k_welford_bins / _order put them in descending log2-size order, waves dequeue groups of
//     them), over the stream values x = RN(a / b) computed once for every record (k_welford_x).
//     The chain's division delta / k uses a double-double reciprocal 1/k ~ y_hi + y_lo
//     (y_hi = RN(1/k), y_lo = RN(fma(-k, y_hi, 1) y_hi)): q = fma(delta, y_hi, RN(delta y_lo)) is
//     within 2^-104 of delta / k, which is never that close to a rounding midpoint unless it is a
//     double, so q = RN(delta / k) (tests/native/welfdiv.c checks it against IEEE division) and
//     each update is bit-identical to Python's.  The longest entity's chain bounds the time: 4
//     dependent FP64 operations per record (sub, mul, fma, add), no memory or LDS latency on it,
//     with the M2 update of each record issued beside the next record's chain.
constexpr int kWfWave = 48;  // records from which an entity gets a wave of its own
constexpr int kWfBins = 32;  // log2 size classes
struct WelfordCtl {
  uint32_t count[kWfBins];
  uint32_t cursor[kWfBins];
  uint32_t head;
  uint32_t n_big;
  uint32_t started;  // (the head queue's) head blocks resident so far (k_welford_head2 -> k_wf_gate)
};

__device__ __forceinline__ int64_t ent_end(const int64_t* __restrict__ ent_start, int64_t e, int64_t n_ent,
                                           int64_t n) {
  return (e + 1 < n_ent) ? ent_start[e + 1] : n;
}

// big entities counted per log2 size class
// (round 5: counted per block in LDS first -- one global atomic per (block, size class) instead of
// one per entity on 32 addresses: 0.2 ms each at config 4)
__global__ void __launch_bounds__(kBlock) k_welford_bins(const int64_t* __restrict__ ent_start, int64_t n_ent,
                                                         int64_t n, WelfordCtl* __restrict__ ctl) {
  __shared__ uint32_t s_c[kWfBins];
  if (threadIdx.x < kWfBins) s_c[threadIdx.x] = 0;
  __syncthreads();
  const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (e < n_ent) {
    const int64_t sz = ent_end(ent_start, e, n_ent, n) - ent_start[e];
    if (sz >= kWfWave) atomicAdd(&s_c[63 - __clzll((unsigned long long)sz)], 1u);
  }
  __syncthreads();
  if (threadIdx.x < kWfBins && s_c[threadIdx.x]) atomicAdd(&ctl->count[threadIdx.x], s_c[threadIdx.x]);
}

// big entity ids into `order`, larger size classes first (ranks in LDS, one global range per
// (block, size class))
__global__ void __launch_bounds__(kBlock) k_welford_order(const int64_t* __restrict__ ent_start, int64_t n_ent,
                                                          int64_t n, WelfordCtl* __restrict__ ctl,
                                                          uint32_t* __restrict__ order) {
  __shared__ uint32_t s_base[kWfBins], s_c[kWfBins];
  if (threadIdx.x < kWfBins) {
    uint32_t b = 0;
    for (int k = threadIdx.x + 1; k < kWfBins; k++) b += ctl->count[k];
    s_base[threadIdx.x] = b;
    s_c[threadIdx.x] = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) ctl->n_big = b + ctl->count[0];
  }
  __syncthreads();
  const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  int bin = -1;
  uint32_t rank = 0;
  if (e < n_ent) {
    const int64_t sz = ent_end(ent_start, e, n_ent, n) - ent_start[e];
    if (sz >= kWfWave) {
      bin = 63 - __clzll((unsigned long long)sz);
      rank = atomicAdd(&s_c[bin], 1u);
    }
  }
  __syncthreads();
  if (threadIdx.x < kWfBins && s_c[threadIdx.x])
    s_base[threadIdx.x] += atomicAdd(&ctl->cursor[threadIdx.x], s_c[threadIdx.x]);
  __syncthreads();
  if (bin >= 0) order[s_base[bin] + rank] = (uint32_t)e;
}

// the stream values of record i: x[0] UY, x[1] genomic fraction, x[2] genomic mean, x[3] CY
template <bool kCell>
__device__ __forceinline__ void welford_samples(const RecCols& r, int64_t i, const double* s_rcp, double (&x)[4]) {
  const uint32_t gl = r.gq_len[i];
  x[0] = ratio_rcp(r.uy_gt30[i], r.uy_len[i], s_rcp);
  x[1] = ratio_rcp(r.gq_gt30[i], gl, s_rcp);
  x[2] = ratio_rcp(r.gq_sum[i], gl, s_rcp);
  x[3] = kCell ? ratio_rcp(r.cy_gt30[i], r.cy_len[i], s_rcp) : 0.0;
}

template <bool kCell>
__device__ __forceinline__ void welford_store(double* F, int st, double mean, double m2, int64_t cnt) {
  const double var = cnt < 2 ? __builtin_nan("") : m2 / ((double)cnt - 1.0);
  const int mslot = st == 0 ? SCT_F_UY_MEAN : st == 1 ? SCT_F_GQF_MEAN : st == 2 ? SCT_F_GQ_MEAN : SCT_F_CY_MEAN;
  const int vslot = st == 0 ? SCT_F_UY_VAR : st == 1 ? SCT_F_GQF_VAR : st == 2 ? SCT_F_GQ_VAR : SCT_F_CY_VAR;
  F[mslot] = mean;
  F[vslot] = var;
}

// The stream values of every record, once, in parallel: xs[4 i + st] = x[st] of record i
// (welford_samples), a record's four streams side by side, so the 4 chain lanes of one entity load
// 32 contiguous bytes (a wave's load touches 16 lines, not 64).  The chains below load one double
// per record; xs holds kWfPad records of slack past n for their unclamped reads.
constexpr int kWfPad = 64;
constexpr int kWfHeadGroups = 4;
constexpr int kWfHeadEnts = kWfHeadGroups * (kWave / 4);
static_assert(kWfHeadEnts == kWave, "one lane per head entity");
// (round 5) records of the head entities are skipped: k_welford_x_ents wrote their samples on the
// head stream, whose chains read them while this kernel runs (the same bits rewritten
// under a concurrent read).  The first wave finds the head ranges that meet the block's records.
template <bool kCell>
__global__ void __launch_bounds__(kBlock) k_welford_x(RecCols r, int64_t n, double* __restrict__ xs,
                                                      const int64_t* __restrict__ ent_start, int64_t n_ent,
                                                      const uint32_t* __restrict__ order,
                                                      const uint32_t* __restrict__ n_head) {
  __shared__ double s_rcp[kRcpN];
  __shared__ int64_t s_lo[kWfHeadEnts], s_hi[kWfHeadEnts];
  __shared__ uint64_t s_meet;
  fill_rcp(s_rcp);
  const int64_t b0 = (int64_t)blockIdx.x * kBlock, b1 = b0 + kBlock < n ? b0 + kBlock : n;
  if (threadIdx.x < kWave) {
    const int k = threadIdx.x, m = (int)*n_head;
    int64_t lo = 0, hi = 0;
    if (k < m) {
      const int64_t e = order[k];
      lo = ent_start[e];
      hi = (e + 1 < n_ent) ? ent_start[e + 1] : n;
    }
    s_lo[k] = lo;
    s_hi[k] = hi;
    const uint64_t meet = __ballot(k < m && lo < b1 && hi > b0);
    if (k == 0) s_meet = meet;
  }
  __syncthreads();
  const int64_t i = b0 + threadIdx.x;
  if (i >= n) return;
  for (uint64_t mk = s_meet; mk; mk &= mk - 1) {
    const int k = __ffsll((unsigned long long)mk) - 1;
    if (i >= s_lo[k] && i < s_hi[k]) return;  // a head entity's record
  }
  double x[4];
  welford_samples<kCell>(r, i, s_rcp, x);
  double2* o = reinterpret_cast<double2*>(xs + 4 * i);
  o[0] = make_double2(x[0], x[1]);
  o[1] = make_double2(x[2], kCell ? x[3] : 0.0);
}

// Round 4: the head groups (the kWfHeadGroups x kWfGroup largest entities: the longest chains decide
// the drop-in's time) get their samples first and their chains launched at once; the rest follows
// on another stream.  k_welford_split gives the head groups their own queue (ctl_head) and starts
// the main queue after them; k_welford_x_ents computes the samples of the head entities' records
// only (a grid-stride loop over their concatenation).
__global__ void k_welford_split(WelfordCtl* __restrict__ ctl, WelfordCtl* __restrict__ ctl_head) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const uint32_t nb = ctl->n_big;
  ctl_head->n_big = nb < (uint32_t)kWfHeadEnts ? nb : (uint32_t)kWfHeadEnts;
  ctl_head->head = 0;
  ctl->head = kWfHeadGroups;  // the first kWfHeadGroups groups are the head queue's
}
template <bool kCell>
__global__ void __launch_bounds__(kBlock) k_welford_x_ents(RecCols r, const int64_t* __restrict__ ent_start,
                                                           int64_t n_ent, int64_t n, const uint32_t* __restrict__ order,
                                                           const WelfordCtl* __restrict__ ctl_head,
                                                           double* __restrict__ xs) {
  __shared__ double s_rcp[kRcpN];
  __shared__ int64_t s_beg[kWfHeadEnts], s_pre[kWfHeadEnts + 1];
  fill_rcp(s_rcp);
  const int m = (int)ctl_head->n_big;  // <= kWfHeadEnts
  if (threadIdx.x < kWfHeadEnts) {
    int64_t b = 0, len = 0;
    if ((int)threadIdx.x < m) {
      const int64_t e = order[threadIdx.x];
      b = ent_start[e];
      len = ent_end(ent_start, e, n_ent, n) - b;
    }
    s_beg[threadIdx.x] = b;
    s_pre[threadIdx.x + 1] = len;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    s_pre[0] = 0;
    for (int k = 1; k <= kWfHeadEnts; k++) s_pre[k] += s_pre[k - 1];
  }
  __syncthreads();
  const int64_t total = s_pre[m];
  for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < total; j += (int64_t)gridDim.x * kBlock) {
    int lo = 0, hi = m - 1;  // the entity k with s_pre[k] <= j < s_pre[k + 1]
    while (lo < hi) {
      const int mid = (lo + hi + 1) / 2;
      if (s_pre[mid] <= j) lo = mid; else hi = mid - 1;
    }
    const int64_t i = s_beg[lo] + (j - s_pre[lo]);
    double x[4];
    welford_samples<kCell>(r, i, s_rcp, x);
    double2* o = reinterpret_cast<double2*>(xs + 4 * i);
    o[0] = make_double2(x[0], x[1]);
    o[1] = make_double2(x[2], kCell ? x[3] : 0.0);
  }
}

// Big entities: one lane per (entity, stream) chain, kWfGroup entities x 4 streams per wave, groups
// of similar sizes (the order is by descending log2 size), waves dequeue groups.  Every lane steps
// the same record index k together, so RN(1 / k) is the same for all of them: the wave computes 64
// of them at a time, one per lane in registers (one division per lane per 64 records), and record
// q's pair reaches the chain by readlane (reading it from LDS put the LDS latency on the chain every
// few records: 22 ms at config 2).  Per record a lane loads its sample (kWfBatch records per batch;
// the next batch's loads, unconditional with clamped addresses, are in flight while this batch's
// kWfBatch updates run) and runs the update: 4 dependent FP64 operations, nothing on them waiting
// for memory or LDS.
constexpr int kWfGroup = kWave / 4;
constexpr int kWfBatch = 32;
static_assert(kWave % kWfBatch == 0, "batches tile the 64-record y chunks");
constexpr int kWfBlocks = 2048;  // persistent grid (waves dequeue groups)
// lane l's double, broadcast (l a compile-time constant after unrolling)
__device__ __forceinline__ double readlane_f64(double v, int l) {
  const uint64_t b = (uint64_t)__double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), l);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// SCT_WF_PAIRS: how record q's reciprocal pair reaches the chain lanes.  0: four v_readlane per
// record (round 3); 1: one broadcast ds_read_b128 from a per-wave LDS row; 2 (round 4): no transfer
// at all -- every row of 16 lanes computes the pairs of the same 16 records, and the two FP64 FMAs
// of the division read record q's pair from lane q of their own row as a DPP operand
// (v_fmac_f64_dpp row_newbcast:q): the lone wave that carries the longest entity is issue-bound,
// and the readlanes were 4 of its 11 instructions per record.  t = RN(l d) is taken as
// fma(l, d, +0), which rounds the same product once (a zero product gives +0 instead of -0 only
// where the next fma's sum is +0 either way).
#ifndef SCT_WF_PAIRS
#define SCT_WF_PAIRS 2
#endif
#define SCT_WF_DPP_CASE(Q)                                                                                     \
  case Q:                                                                                                      \
    if (Q == 0)                                                                                                \
      asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:" #Q " row_mask:0xf bank_mask:0xf"     \
                   : "+v"(t)                                                                                   \
                   : "v"(y), "v"(d));                                                                          \
    else                                                                                                       \
      asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:" #Q " row_mask:0xf bank_mask:0xf"                  \
                   : "+v"(t)                                                                                   \
                   : "v"(y), "v"(d));                                                                          \
    break;
// t += y[lane q of this row] * d (q a compile-time constant after unrolling: the switch folds).  y is
// written at q == 0 only (a sub-chunk's pairs): the s_nop there covers the DPP read-after-VALU-write
// hazard on it.
__device__ __forceinline__ void fmac_row_bcast(double& t, double y, double d, int q) {
  switch (q) {
    SCT_WF_DPP_CASE(0) SCT_WF_DPP_CASE(1) SCT_WF_DPP_CASE(2) SCT_WF_DPP_CASE(3) SCT_WF_DPP_CASE(4)
    SCT_WF_DPP_CASE(5) SCT_WF_DPP_CASE(6) SCT_WF_DPP_CASE(7) SCT_WF_DPP_CASE(8) SCT_WF_DPP_CASE(9)
    SCT_WF_DPP_CASE(10) SCT_WF_DPP_CASE(11) SCT_WF_DPP_CASE(12) SCT_WF_DPP_CASE(13) SCT_WF_DPP_CASE(14)
    SCT_WF_DPP_CASE(15)
    default: break;
  }
}
#undef SCT_WF_DPP_CASE
template <bool kCell>
__global__ void __launch_bounds__(kBlock) k_welford_chains(const int64_t* __restrict__ ent_start, int64_t n_ent,
                                                           int64_t n, const uint32_t* __restrict__ order,
                                                           WelfordCtl* __restrict__ ctl,
                                                           const double* __restrict__ xs, double* __restrict__ out_f) {
  constexpr int ns = kCell ? 4 : 3;
  __shared__ double2 s_y_all[kWaves][kWave];
  const int lane = threadIdx.x & (kWave - 1);
  const int st = lane & 3;
  double2* s_y = s_y_all[threadIdx.x / kWave];
  const uint32_t n_big = ctl->n_big;
  const uint32_t n_groups = (n_big + kWfGroup - 1) / kWfGroup;
  while (true) {
    uint32_t g = 0;
    if (lane == 0) g = atomicAdd(&ctl->head, 1u);
    g = (uint32_t)__shfl((int)g, 0);
    if (g >= n_groups) break;  // wave-uniform: every wave reaches it once the queue is drained
    const uint32_t k = g * kWfGroup + (uint32_t)(lane >> 2);
    const bool mine = k < n_big && st < ns;
    int64_t e = 0, s = 0, len = 0;
    if (mine) {
      e = order[k];
      s = ent_start[e];
      len = ent_end(ent_start, e, n_ent, n) - s;
    }
    int64_t kmax = len;  // the wave's longest chain
    for (int off = kWave / 2; off > 0; off >>= 1) {
      const int64_t o = __shfl_xor(kmax, off);
      kmax = o > kmax ? o : kmax;
    }
    // a lane without a chain steps along over records 0 .. kmax - 1 (in bounds: kmax <= n), its
    // result unused
    const double* X = xs + 4 * s + st;
    const int64_t clen = mine ? len : kmax;
    const int64_t lastx = clen > 0 ? clen - 1 : 0;
    double mean = 0.0, m2 = 0.0;
    // the pending M2 term of the last record updated (zeros add exactly 0.0 to m2 = 0.0)
    double pdelta = 0.0, px = 0.0;
    bool pact = true;
    // the samples of two batches, ping-pong: batch hb of a 64-record chunk reads xq[hb] while the
    // next batch's loads land in xq[hb ^ 1] (round 4: no copy of the next batch into the current)
    double xq[2][kWfBatch];
#pragma unroll
    for (int q = 0; q < kWfBatch; q++) xq[0][q] = X[4 * (q < lastx ? q : lastx)];
    for (int64_t c0 = 0; c0 < kmax; c0 += kWave) {
      // 1 / k for this chunk's 64 record indices, as y_hi + y_lo, lane i holding k = c0 + i + 1;
      // the chain reads record q's pair with readlane (a compile-time lane: no LDS latency on it)
      const double kd = (double)(c0 + lane + 1);
      const double yh = 1.0 / kd;
      const double yl = __fma_rn(-kd, yh, 1.0) * yh;
      if (SCT_WF_PAIRS == 1) {
        __builtin_amdgcn_wave_barrier();  // the previous chunk's reads of the row are done (in order per wave)
        s_y[lane] = make_double2(yh, yl);
        __builtin_amdgcn_wave_barrier();
      }
#pragma unroll
      for (int hb = 0; hb < kWave / kWfBatch; hb++) {
        const int64_t c = c0 + hb * kWfBatch;
        if (c >= kmax) break;  // wave-uniform
        {  // the next batch's samples: records nb .. nb + kWfBatch - 1
          const int64_t nb = c + kWfBatch;
          const bool part = nb < clen && nb + kWfBatch > clen;  // this lane's chain ends inside it
          if (__builtin_amdgcn_ballot_w64(part) == 0) {  // wave-uniform: one base per lane, no clamps
            const double* B = nb + kWfBatch <= clen ? X + 4 * nb : xs;  // past its end: unused values
#pragma unroll
            for (int q = 0; q < kWfBatch; q++) xq[hb ^ 1][q] = B[4 * q];
          } else {
#pragma unroll
            for (int q = 0; q < kWfBatch; q++) {
              const int64_t kq = nb + q;
              xq[hb ^ 1][q] = X[4 * (kq < lastx ? kq : lastx)];
            }
          }
        }
        // Record q's M2 term (x_q - mean_q) delta_q runs at record q + 1, beside its mean chain:
        // waves issue in order, and after the mean add the M2 sub -> mul -> add would otherwise hold
        // the next record's ops behind two more dependent FP64 latencies (12.9 against 14.3 ms
        // at config 2, profiles/r03/s_welford_m2_pipelined/).  Same operations on the same values.
        // SCT_WF_PAIRS 2: each row's lane j holds the pair of record c + 16 i + j for the batch's
        // sub-chunk i of 16 records
        double yh16 = 0.0, yl16 = 0.0;
        const auto update = [&](int q, bool act, bool fast) {
          const double x = xq[hb][q];
          if (SCT_WF_PAIRS == 2) {
            if ((q & 15) == 0) {
              const double kq = (double)(c + q + (lane & 15) + 1);
              yh16 = 1.0 / kq;
              yl16 = __fma_rn(-kq, yh16, 1.0) * yh16;
            }
            // (no empty-asm ordering here: with the DPP FMAs the compiler's own schedule is 8 %
            // faster, 31.0 against 33.6 ns per record, tools/debug/welford_micro.hip)
            const double delta = x - mean;
            const double d2 = px - mean;
            double t = 0.0;
            fmac_row_bcast(t, yl16, delta, q & 15);  // RN(l delta)
            const double p2 = pdelta * d2;
            fmac_row_bcast(t, yh16, delta, q & 15);  // RN(h delta + RN(l delta)) = RN(delta / k)
            const double pm2 = m2 + p2;
            m2 = fast || pact ? pm2 : m2;
            const double nm = mean + t;
            mean = act ? nm : mean;
            pdelta = delta, px = x, pact = act;
            return;
          }
          double h, l;
          if (SCT_WF_PAIRS == 1) {
            const double2 y = s_y[hb * kWfBatch + q];  // one broadcast read (every lane, one address)
            h = y.x;
            l = y.y;
          } else {
            h = readlane_f64(yh, hb * kWfBatch + q);
            l = readlane_f64(yl, hb * kWfBatch + q);
          }
          // the issue order is pinned by empty asm statements (the scheduler would put the M2 ops
          // back between two records): the two subs, the two muls, the fma and the M2 add, then
          // the mean add
          double delta = x - mean;
          double d2 = px - mean;
          asm volatile("" : "+v"(delta), "+v"(d2));
          double t = delta * l;
          double p2 = pdelta * d2;
          asm volatile("" : "+v"(t), "+v"(p2));
          double f = __fma_rn(delta, h, t);  // RN(delta / k)
          double pm2 = m2 + p2;
          asm volatile("" : "+v"(f), "+v"(pm2));
          m2 = fast || pact ? pm2 : m2;
          const double nm = mean + f;
          mean = act ? nm : mean;
          pdelta = delta, px = x, pact = act;
        };
        // no lane-divergent branch around the updates: readlane must see y of every lane (a
        // value computed under a partial exec mask would be stale in the inactive lanes)
        if (__builtin_amdgcn_ballot_w64(c + kWfBatch > clen) == 0) {  // wave-uniform
#pragma unroll
          for (int q = 0; q < kWfBatch; q++) update(q, true, true);
        } else {
#pragma unroll
          for (int q = 0; q < kWfBatch; q++) update(q, c + q < clen, false);
        }
      }
    }
    m2 = pact ? m2 + pdelta * (px - mean) : m2;  // the last record's pending M2 term
    if (mine) {
      double* F = out_f + e * SCT_NF;
      welford_store<kCell>(F, st, mean, m2, len);
      if (!kCell && st == 0) {
        F[SCT_F_CY_MEAN] = 0.0;
        F[SCT_F_CY_VAR] = 0.0;
      }
    }
  }
}

// Round 5: the head entities' chains on one block of 16 waves each (k_welford_head2), kW2Ents
// entities per block.  Inside the pipeline the lone wave of k_welford_chains carrying the longest
// entity ran at 1.7x (config 2) its pace alone; beside an HBM copy on every CU a chain runs at 2.6x,
// beside FP64 work on its SIMD at 2.4x (tools/debug/welford_head2_micro.hip).  Here
//   wave 0 (mean)   runs the mean chain alone on plain FP64 operations: per chunk of kW2Chunk records
//                   it reads the chunk's samples and reciprocal pairs from LDS into registers, steps
//                   the means (delta = x - mean, t = RN(l delta), q = RN(h delta + t), mean += q: the
//                   operations of k_welford_chains, so the same bits) and writes every mean to LDS.
//                   No selects: a lane past its chain's end steps on over repeated samples, unused;
//   wave 1 (M2)     one chunk behind: per record delta = x - mean_{k-1}, d2 = x - mean_k,
//                   m2 += delta * d2 (stats.py:82-87: the same roundings in the same order) from the
//                   staged samples and means; a lane's final mean is taken here at its last record
//                   (chunks a lane finishes take a slower path with selects; finished lanes sit out);
//   waves 2, 3      the loaders, kW2Depth chunks ahead (224 records at 16 entities per block: ~6 us
//   (loaders)       of the chain), copy the samples HBM -> LDS with direct-to-LDS loads (16 B per
//                   lane, 32 / kW2Ents records of the block's entities per load, no registers in
//                   flight; each loader holds <= 63 loads in flight, vmcnt's limit) and compute the
//                   chunk's reciprocal pairs; loader w takes the chunks j with j % 2 == w;
//   waves 4 - 15    hold the CU's registers (below).
// The waves meet at one block barrier per chunk (LDS writes done first; the loader of the chunk the
// next phase reads waits for it).  16 entities per block measured best (4 / 8 per block have deeper
// rings but more blocks: profiles/r05/welford/head_ents_per_block_c2.txt); the ~148 KB of LDS and
// the register-holding waves give every head block a CU of its own, and welford_stage starts the
// key pass only once the head blocks are resident (k_wf_gate).
#ifndef SCT_W2_CHUNK
#define SCT_W2_CHUNK 16
#endif
#ifndef SCT_W2_ENTS
#define SCT_W2_ENTS 16
#endif
constexpr int kW2Chunk = SCT_W2_CHUNK;         // records per chunk
constexpr int kW2Ents = SCT_W2_ENTS;           // entities per block
constexpr int kW2Lanes = 4 * kW2Ents;          // chain lanes (4 streams per entity)
constexpr int kW2PerLoad = 32 / kW2Ents;       // records per 64 x 16-byte load
constexpr int kW2Loads = kW2Chunk / kW2PerLoad;  // loads per chunk
constexpr int kW2Slots = 64 * 16 / kW2Chunk * 4 / kW2Ents;  // ~128 KB of samples
constexpr int kW2Depth = (kW2Slots - 2) & ~1;  // chunks in flight ahead of the mean chain
#ifndef SCT_W2_FILL
#define SCT_W2_FILL 12
#endif
constexpr int kW2Work = 4;                     // mean, M2, two loaders
constexpr int kW2Waves = kW2Work + SCT_W2_FILL;  // + waves that only hold the CU (see below)
static_assert(kW2Ents >= 1 && kW2Ents <= 16 && (kW2Ents & (kW2Ents - 1)) == 0, "entities per block: power of 2");
static_assert(kW2Chunk % kW2PerLoad == 0 && kWfHeadEnts % kW2Ents == 0, "whole loads per chunk, whole blocks");
static_assert((kW2Slots & (kW2Slots - 1)) == 0 && kW2Slots >= kW2Depth + 2, "slots: chunks p - 1 .. p + depth");
constexpr int kW2InFlight = (kW2Depth / 2) * kW2Loads;  // a loader's loads in flight after issuing
constexpr int kW2After = (kW2Depth / 2 - 1) * kW2Loads;  // ... after its chunk the next phase reads
static_assert(kW2InFlight <= 63, "a loader's loads in flight fit vmcnt");  // (56 at 16 entities)
// The block barrier of k_welford_head2: LDS writes done, then s_barrier -- without the fence of
// __syncthreads(), which also waits for every load in flight.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
#ifdef SCT_W2_PROF  // experiments (tools/debug/welford_head2_micro.hip): per-wave ticks in barriers and in all
__device__ unsigned long long sct_w2_prof[2 * 4 + 2];
#define W2_BARRIER()                           \
  do {                                         \
    const long long _t = wall_clock64();       \
    lds_barrier();                             \
    w2_wait += wall_clock64() - _t;            \
  } while (0)
#else
#define W2_BARRIER() lds_barrier()
#endif
template <bool kCell>
__global__ void __launch_bounds__(kW2Waves * kWave) k_welford_head2(const int64_t* __restrict__ ent_start,
                                                                      int64_t n_ent, int64_t n,
                                                                      const uint32_t* __restrict__ order,
                                                                      WelfordCtl* __restrict__ ctl_head,
                                                                      const double* __restrict__ xs,
                                                                      double* __restrict__ out_f) {
  constexpr int ns = kCell ? 4 : 3;
  constexpr int C = kW2Chunk;
  __shared__ double s_x[kW2Slots][C][kW2Lanes];  // samples: chunk j in slot j % kW2Slots, [record][lane]
  __shared__ double s_m[2][C][kW2Lanes];         // means: chunk j in slot j & 1
  __shared__ double2 s_y[kW2Slots][C];           // the reciprocal pairs of chunk j's record indices
#ifdef SCT_W2_PROF
  long long w2_wait = 0;
  const long long w2_t0 = wall_clock64();
  const long long w2_c0 = clock64();
#endif
  const int lane = threadIdx.x & (kWave - 1);
  const int cl = lane & (kW2Lanes - 1);  // the chain lane this lane mirrors (lanes >= kW2Lanes: copies)
  const int role = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave));  // 0 mean, 1 M2, 2-3 loaders
  const int st = lane & 3;
  if (threadIdx.x == 0) atomicAdd(&ctl_head->started, 1u);  // resident (k_wf_gate)
  const uint32_t n_big = ctl_head->n_big;
  if (blockIdx.x * (uint32_t)kW2Ents >= n_big) return;  // block-uniform
  // the block's entity `slot` (4 lanes per entity, one per stream)
  const auto entity = [&](int slot, int64_t& e, int64_t& s, int64_t& len) {
    const uint32_t k = blockIdx.x * (uint32_t)kW2Ents + (uint32_t)slot;
    e = 0, s = 0, len = 0;
    if (k < n_big) {
      e = order[k];
      s = ent_start[e];
      len = ent_end(ent_start, e, n_ent, n) - s;
    }
  };
  int64_t e, s, len;
  entity(cl >> 2, e, s, len);
  const bool mine = lane < kW2Lanes && len > 0 && st < ns;
  int64_t kmax = len;  // the block's longest chain (the same in every wave)
  for (int off = kWave / 2; off > 0; off >>= 1) {
    const int64_t o = __shfl_xor(kmax, off);
    kmax = o > kmax ? o : kmax;
  }
  const int64_t clen = mine ? len : kmax;  // a lane without a chain steps along, its result unused
  const int64_t P = (kmax + C - 1) / C;
  double m2 = 0.0, mprev = 0.0, fin = 0.0;  // the M2 wave's results
  // one loop per role (the waves meet at P + 2 barriers: the prologue's and one per phase 0 .. P)
  if (role >= kW2Work) {
    // The block's other waves do nothing but meet the barriers: with them the block holds every
    // SIMD's registers (4 waves x 128 VGPRs each), so no wave of another kernel shares the CU.  The
    // LDS alone does not ensure it: kernels without LDS (the other chains, the fills) landed beside
    // the chain and their FP64 work delayed its operations.
    for (int64_t p = 0; p <= P + 1; p++) W2_BARRIER();
  } else if (role >= 2) {
    // loader lane i moves 16 bytes: streams 2 (i & 1) .. +1 of entity (i / 2) % kW2Ents, at record
    // offset i / (2 kW2Ents) of the load's kW2PerLoad records (LDS row = kW2Lanes doubles)
    const int w = role - 2;
    int64_t le, ls, llen;
    entity((lane >> 1) & (kW2Ents - 1), le, ls, llen);
    const int64_t llast = (llen > 0 ? llen : kmax) - 1;
    const double* LX = xs + 4 * ls + 2 * (lane & 1);
    const int rofs = lane / (2 * kW2Ents);
    const auto issue = [&](int64_t j) {  // chunk j: kW2Loads loads, and its reciprocal pairs
      const int sl = (int)(j & (kW2Slots - 1));
#pragma unroll
      for (int u = 0; u < kW2Loads; u++) {
        const int64_t kq = j * C + u * kW2PerLoad + rofs;
        __builtin_amdgcn_global_load_lds(LX + 4 * (kq < llast ? kq : llast), &s_x[sl][u * kW2PerLoad][0], 16, 0, 0);
      }
      if (lane < C) {  // 1 / k as yh + yl for k = j C + lane + 1 (the pairs k_welford_chains computes)
        const double kq = (double)(j * C + lane + 1);
        const double yh = 1.0 / kq;
        s_y[sl][lane] = make_double2(yh, __fma_rn(-kq, yh, 1.0) * yh);
      }
    };
    for (int j = w; j < kW2Depth; j += 2) issue(j);
    if (w == 0) asm volatile("s_waitcnt vmcnt(%0)" : : "n"(kW2After) : "memory");  // chunk 0 landed
    W2_BARRIER();
    for (int64_t p = 0; p <= P; p++) {
      if ((int)(p & 1) == w) issue(p + kW2Depth);                                   // its chunk p was waited for
      else asm volatile("s_waitcnt vmcnt(%0)" : : "n"(kW2After) : "memory");  // chunk p + 1 landed
      W2_BARRIER();
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no load may land in LDS after the block ends
  } else if (role == 0) {  // the mean chain, chunk p in phase p
    W2_BARRIER();
    double mean = 0.0;
    for (int64_t p = 0; p < P; p++) {
      const int xs_slot = (int)(p & (kW2Slots - 1)), ms_slot = (int)(p & 1);
      double xv[C];
      double2 yv[C];
#pragma unroll
      for (int q = 0; q < C; q++) {
        xv[q] = s_x[xs_slot][q][cl];
        yv[q] = s_y[xs_slot][q];
      }
#pragma unroll
      for (int q = 0; q < C; q++) {
        const double delta = xv[q] - mean;
        const double t = yv[q].y * delta;               // RN(l delta)
        const double qd = __fma_rn(delta, yv[q].x, t);  // RN(h delta + RN(l delta)) = RN(delta / k)
        mean = mean + qd;
        if (lane < kW2Lanes) s_m[ms_slot][q][cl] = mean;
      }
      W2_BARRIER();
    }
    W2_BARRIER();  // (phase P: the M2 wave's last chunk)
  } else {  // the M2 terms, chunk p - 1 in phase p
    W2_BARRIER();
    W2_BARRIER();  // (phase 0)
    for (int64_t p = 1; p <= P; p++) {
      const int64_t c = (p - 1) * C;
      const int xs_slot = (int)((p - 1) & (kW2Slots - 1)), ms_slot = (int)((p - 1) & 1);
      const bool full = c + C < clen, part = c < clen && !full;  // part: the lane's last record is in it
      double xb[C], mb[C];  // the chunk's samples and means into registers first
#pragma unroll
      for (int q = 0; q < C; q++) {
        xb[q] = s_x[xs_slot][q][cl];
        mb[q] = s_m[ms_slot][q][cl];
      }
      if (__builtin_amdgcn_ballot_w64(part) != 0) {  // some lane's chain ends in this chunk
#pragma unroll
        for (int q = 0; q < C; q++) {
          const double delta = xb[q] - mprev;
          const double d2 = xb[q] - mb[q];
          const double p2 = delta * d2;
          m2 = (c + q < clen) ? m2 + p2 : m2;
          fin = (c + q == clen - 1) ? mb[q] : fin;
          mprev = mb[q];
        }
      } else if (full) {  // (lanes already past their end sit out)
#pragma unroll
        for (int q = 0; q < C; q++) {
          const double delta = xb[q] - mprev;
          const double d2 = xb[q] - mb[q];
          m2 = m2 + delta * d2;
          mprev = mb[q];
        }
      }
      W2_BARRIER();
    }
  }
#ifdef SCT_W2_PROF
  if (lane == 0 && role < kW2Work) {
    sct_w2_prof[2 * role] = (unsigned long long)w2_wait;
    sct_w2_prof[2 * role + 1] = (unsigned long long)(wall_clock64() - w2_t0);
    if (role == 0) sct_w2_prof[8] = (unsigned long long)(clock64() - w2_c0);
  }
#endif
  if (role != 1 || !mine) return;
  double* F = out_f + e * SCT_NF;
  const int mslot = st == 0 ? SCT_F_UY_MEAN : st == 1 ? SCT_F_GQF_MEAN : st == 2 ? SCT_F_GQ_MEAN : SCT_F_CY_MEAN;
  const int vslot = st == 0 ? SCT_F_UY_VAR : st == 1 ? SCT_F_GQF_VAR : st == 2 ? SCT_F_GQ_VAR : SCT_F_CY_VAR;
  F[mslot] = fin;
  F[vslot] = len < 2 ? __builtin_nan("") : m2 / ((double)len - 1.0);
  if (!kCell && st == 0) {
    F[SCT_F_CY_MEAN] = 0.0;
    F[SCT_F_CY_VAR] = 0.0;
  }
}

// Waits until `want` head blocks are resident (*started, k_welford_head2) or ~kWfGateTicks of the
// 100 MHz wall clock have passed, whichever is first (a scheduling aid: see welford_stage).
constexpr int64_t kWfGateTicks = 400000;  // 4 ms
__global__ void __launch_bounds__(kWave) k_wf_gate(const uint32_t* started, uint32_t want, int64_t max_ticks) {
  const int64_t t0 = wall_clock64();
  // (the index term is always 0: it keeps the poll a per-lane vector load, which sees the head
  // blocks' global atomics, where a scalar-cache load of a uniform address might not)
  while (__hip_atomic_load(started + (threadIdx.x & kWave), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < want &&
         wall_clock64() - t0 < max_ticks)
    __builtin_amdgcn_s_sleep(4);
}

// Entities of < kWfWave records: one lane each (the big ones are left to k_welford_wave).
template <bool kCell>
__global__ void k_welford(RecCols r, const int64_t* __restrict__ ent_start, int64_t n_ent, int64_t n,
                          double* __restrict__ out_f) {
  __shared__ double s_rcp[kRcpN];
  fill_rcp(s_rcp);
  __syncthreads();
  const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (e >= n_ent) return;
  const int64_t s = ent_start[e];
  const int64_t t = ent_end(ent_start, e, n_ent, n);
  if (t - s >= kWfWave) return;
  Welford wu{0.0, 0.0}, wf{0.0, 0.0}, wq{0.0, 0.0}, wc{0.0, 0.0};
  double cnt = 0.0;
  for (int64_t i = s; i < t; i++) {
    cnt += 1.0;
    const uint32_t gl = r.gq_len[i];
    if (kCell) wc.update(ratio_rcp(r.cy_gt30[i], r.cy_len[i], s_rcp), cnt);
    wu.update(ratio_rcp(r.uy_gt30[i], r.uy_len[i], s_rcp), cnt);
    wf.update(ratio_rcp(r.gq_gt30[i], gl, s_rcp), cnt);
    wq.update(ratio_rcp(r.gq_sum[i], gl, s_rcp), cnt);
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

}  // namespace sct
