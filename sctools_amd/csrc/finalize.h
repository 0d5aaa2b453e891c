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
//   * larger ones: one wave each (k_welford_wave), largest first (k_welford_bins / _order put
//     them in descending log2-size order, waves dequeue them): per chunk of 64 records all 64
//     lanes load the columns (coalesced) and compute the stream values x = RN(a / b) and
//     y = RN(1 / k) in parallel; then one lane per stream runs the chain over the chunk from LDS.
//     The chain's division delta / k is RN(q0 + r y) with q0 = RN(delta y), r = fma(-q0, k, delta)
//     (exact), the correctly rounded quotient for y = RN(1/k) (Markstein; tests/native/welfdiv.c
//     checks it against IEEE division), so each update is bit-identical to Python's.
constexpr int kWfWave = 48;  // records from which an entity gets a wave of its own
constexpr int kWfBins = 32;  // log2 size classes
struct WelfordCtl {
  uint32_t count[kWfBins];
  uint32_t cursor[kWfBins];
  uint32_t head;
  uint32_t n_big;
};

__device__ __forceinline__ int64_t ent_end(const int64_t* __restrict__ ent_start, int64_t e, int64_t n_ent,
                                           int64_t n) {
  return (e + 1 < n_ent) ? ent_start[e + 1] : n;
}

// big entities counted per log2 size class (wave-aggregated)
__global__ void k_welford_bins(const int64_t* __restrict__ ent_start, int64_t n_ent, int64_t n,
                               WelfordCtl* __restrict__ ctl) {
  const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (e >= n_ent) return;
  const int64_t sz = ent_end(ent_start, e, n_ent, n) - ent_start[e];
  if (sz < kWfWave) return;
  atomicAdd(&ctl->count[63 - __clzll((unsigned long long)sz)], 1u);
}

// big entity ids into `order`, larger size classes first
__global__ void k_welford_order(const int64_t* __restrict__ ent_start, int64_t n_ent, int64_t n,
                                WelfordCtl* __restrict__ ctl, uint32_t* __restrict__ order) {
  __shared__ uint32_t s_base[kWfBins];
  if (threadIdx.x < kWfBins) {
    uint32_t b = 0;
    for (int k = threadIdx.x + 1; k < kWfBins; k++) b += ctl->count[k];
    s_base[threadIdx.x] = b;
    if (blockIdx.x == 0 && threadIdx.x == 0) ctl->n_big = b + ctl->count[0];
  }
  __syncthreads();
  const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (e >= n_ent) return;
  const int64_t sz = ent_end(ent_start, e, n_ent, n) - ent_start[e];
  if (sz < kWfWave) return;
  const int bin = 63 - __clzll((unsigned long long)sz);
  order[s_base[bin] + atomicAdd(&ctl->cursor[bin], 1u)] = (uint32_t)e;
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

// Persistent: each wave dequeues big entities (largest first) until the queue is empty.
constexpr int kWfBlocks = 2048;
template <bool kCell>
__global__ void __launch_bounds__(kBlock) k_welford_wave(RecCols r, const int64_t* __restrict__ ent_start,
                                                         int64_t n_ent, int64_t n, const uint32_t* __restrict__ order,
                                                         WelfordCtl* __restrict__ ctl, double* __restrict__ out_f) {
  constexpr int ns = kCell ? 4 : 3;
  __shared__ double s_x[kWaves][4][kWave + 2];  // +2: the 4 chain lanes read 4 different banks
  __shared__ double s_y[kWaves][kWave];
  __shared__ double s_rcp[kRcpN];
  fill_rcp(s_rcp);
  __syncthreads();
  const int lane = threadIdx.x & (kWave - 1);
  const int wv = threadIdx.x / kWave;
  const uint32_t n_big = ctl->n_big;
  while (true) {
    uint32_t k = 0;
    if (lane == 0) k = atomicAdd(&ctl->head, 1u);
    k = (uint32_t)__shfl((int)k, 0);
    if (k >= n_big) break;  // wave-uniform: every wave reaches it once the queue is drained
    const int64_t e = order[k];
    const int64_t s = ent_start[e];
    const int64_t t = ent_end(ent_start, e, n_ent, n);
    double mean = 0.0, m2 = 0.0, cnt = 0.0;
    double x[4], xn[4];
    if (s + lane < t) welford_samples<kCell>(r, s + lane, s_rcp, x);
    for (int64_t c = s; c < t; c += kWave) {
      // this chunk's samples and reciprocals to LDS; the next chunk's loads go out meanwhile
      const int64_t j = c + lane;
#pragma unroll
      for (int st = 0; st < 4; st++) s_x[wv][st][lane] = x[st];
      s_y[wv][lane] = 1.0 / (double)(j - s + 1);
      if (c + kWave + lane < t) welford_samples<kCell>(r, c + kWave + lane, s_rcp, xn);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const int m = (int)((t - c) < kWave ? (t - c) : kWave);
      if (lane < ns) {
        for (int q = 0; q < m; q++) {
          const double xv = s_x[wv][lane][q];
          const double y = s_y[wv][q];
          cnt += 1.0;
          const double delta = xv - mean;
          const double q0 = delta * y;
          const double rr = __fma_rn(-q0, cnt, delta);
          mean = mean + __fma_rn(rr, y, q0);  // == mean + delta / cnt
          const double delta2 = xv - mean;
          m2 = m2 + delta * delta2;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int st = 0; st < 4; st++) x[st] = xn[st];
    }
    double* F = out_f + e * SCT_NF;
    if (lane < ns) welford_store<kCell>(F, lane, mean, m2, t - s);
    if (!kCell && lane == 0) {
      F[SCT_F_CY_MEAN] = 0.0;
      F[SCT_F_CY_VAR] = 0.0;
    }
  }
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
