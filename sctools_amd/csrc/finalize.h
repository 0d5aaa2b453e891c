// finalize.h -- partial rows -> output rows, and the sequential-Welford float path.
#pragma once
#include "fixedpt.h"
#include "reduce.h"
#include "util.h"

namespace sct {

// MetricAggregator.finalize (aggregator.py:342-387), CellMetrics.finalize (463-490),
// GeneMetrics.finalize (571-578): one thread per row.
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

// Sequential Welford per entity in record order: one lane per entity.
template <bool kCell>
__global__ void k_welford(RecCols r, const int64_t* __restrict__ ent_start, int64_t n_ent, int64_t n,
                          double* __restrict__ out_f) {
  __shared__ double s_rcp[kRcpN];
  fill_rcp(s_rcp);
  __syncthreads();
  const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (e >= n_ent) return;
  const int64_t s = ent_start[e];
  const int64_t t = (e + 1 < n_ent) ? ent_start[e + 1] : n;
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
