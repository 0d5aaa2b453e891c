// countmat.h -- cells x genes molecule-count matrix (CountMatrix.from_sorted_tagged_bam,
// count.py:134-328) as a sort-and-count over 64-bit molecule keys.
//
// The reference walks query-name groups in file order, keeps a Python set of the
// (cell, molecule, gene) triples seen so far and appends one COO entry per new triple; the
// CSR conversion then sums the entries of each (cell, gene).  That is order-free except for
// the row order (a cell's row is numbered when its first molecule is counted), so:
//
//   k_cm_groups   one lane per query-name group head: the group's molecule key
//                 [cell | column | umi] or a "dropped" top bit; atomicMin of the group's
//                 record index per cell (row order) and over unknown genes (the KeyError)
//   radix.h       LSD sort of the keys (cbits + colbits + ubits + 1 bits)
//   k_cm_pairs    triple heads / (cell, column) pair heads in the sorted keys
//   scan.h        exclusive scan of the pair-head flags -> pair index
//   k_cm_emit     per pair: cell, column, molecule count (triples of the pair)
//   k_cm_rowkeys  (first record index, cell) per counted cell -> radix.h -> row order
//   k_cm_rows     row -> cell, cell -> row, pairs per row; scan -> CSR indptr
//   k_cm_scatter  pairs (cell-id order) -> CSR rows (first-molecule order)
//
// HBM-bound integer work: ~14 bytes read per record in k_cm_groups, 12 bytes written, then
// the radix passes over 12-byte (key, value) items.
#pragma once
#include "radix.h"
#include "scan.h"
#include "util.h"

namespace sct {

struct CountKey {
  int cbits, colbits, ubits, total;  // total = cbits + colbits + ubits; bit `total` = dropped
};

struct CountCols {
  const int32_t *cell, *umi, *gene;
  const uint8_t *xf, *qhead;
  const int32_t* gene_col;
  int64_t n;
  int32_t n_cell, n_umi, n_gene, cell_none, umi_none, n_cols;
};

constexpr uint8_t kXfAbsent = 0, kXfIntergenic = 4;  // SCT_XF_ABSENT / SCT_XF_INTERGENIC

// count.py:222-270 for the group starting at record i (qhead[i] == 1): cell / molecule of its
// first record; the implicated gene names are the single-name GE values of alignments with
// an XF tag other than INTERGENIC (gene_col != SKIP covers "has GE" and "no ','"); the group
// counts when exactly one distinct name is implicated -- for a one-alignment group that is
// the same test.
__global__ void k_cm_groups(CountCols c, CountKey K, uint64_t* __restrict__ keys, uint32_t* __restrict__ vals,
                            uint32_t* __restrict__ cell_first, unsigned long long* __restrict__ unknown,
                            uint32_t* __restrict__ err) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= c.n) return;
  uint64_t key = 1ull << K.total;
  if (c.qhead[i] || i == 0) {
    const int32_t cell = c.cell[i], umi = c.umi[i];
    if ((uint32_t)cell >= (uint32_t)c.n_cell || (uint32_t)umi >= (uint32_t)c.n_umi) {
      atomicOr(err, 1u);
    } else if (cell != c.cell_none && umi != c.umi_none) {
      int32_t sel = -1;
      bool multi = false;
      for (int64_t j = i; j < c.n && (j == i || !c.qhead[j]); j++) {
        const int32_t g = c.gene[j];
        if ((uint32_t)g >= (uint32_t)c.n_gene) {
          atomicOr(err, 1u);
          sel = -1;
          break;
        }
        const uint8_t x = c.xf[j];
        if (x == kXfAbsent || x == kXfIntergenic || c.gene_col[g] == -1) continue;
        if (sel < 0) sel = g;
        else if (g != sel) multi = true;
      }
      if (sel >= 0 && !multi) {
        int32_t col = c.gene_col[sel];
        if (col < 0 || col >= c.n_cols) {  // the reference's gene_name_to_index[gene_name] KeyError
          atomicMin(unknown, (unsigned long long)i);
          col = 0;
        }
        key = ((uint64_t)cell << (K.colbits + K.ubits)) | ((uint64_t)col << K.ubits) | (uint64_t)umi;
        atomicMin(&cell_first[cell], (uint32_t)i);
      }
    }
  }
  keys[i] = key;
  vals[i] = (uint32_t)i;
}

struct CmHead {
  bool triple, pair, first_of_cell;
};

__device__ inline CmHead cm_head(const uint64_t* keys, int64_t i, CountKey K) {
  const uint64_t k = keys[i];
  CmHead h{false, false, false};
  if (k >> K.total) return h;  // dropped (sorted last)
  if (i == 0) return CmHead{true, true, true};
  const uint64_t p = keys[i - 1];  // valid: dropped keys sort after every valid one
  h.triple = p != k;
  h.pair = h.triple && (p >> K.ubits) != (k >> K.ubits);
  h.first_of_cell = h.pair && (p >> (K.ubits + K.colbits)) != (k >> (K.ubits + K.colbits));
  return h;
}

__global__ void k_cm_pairs(const uint64_t* __restrict__ keys, int64_t n, CountKey K, uint32_t* __restrict__ flags) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  flags[i] = cm_head(keys, i, K).pair ? 1u : 0u;
}

// pair index of a triple head = (pair heads before it, inclusive) - 1
__global__ void k_cm_emit(const uint64_t* __restrict__ keys, int64_t n, CountKey K, const uint32_t* __restrict__ flags,
                          const uint32_t* __restrict__ offs, int32_t* __restrict__ pair_cell,
                          int32_t* __restrict__ pair_col, uint32_t* __restrict__ pair_count,
                          uint32_t* __restrict__ cell_pstart, uint32_t* __restrict__ cell_npairs,
                          uint64_t* __restrict__ n_pairs) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (i == n - 1) *n_pairs = (uint64_t)offs[i] + flags[i];
  const CmHead h = cm_head(keys, i, K);
  if (!h.triple) return;
  const uint64_t k = keys[i];
  const uint32_t p = offs[i] + (h.pair ? 0u : 0xFFFFFFFFu);
  atomicAdd(&pair_count[p], 1u);
  if (!h.pair) return;
  const int32_t cell = (int32_t)(k >> (K.ubits + K.colbits));
  pair_cell[p] = cell;
  pair_col[p] = (int32_t)((k >> K.ubits) & ((1ull << K.colbits) - 1));
  atomicAdd(&cell_npairs[cell], 1u);
  if (h.first_of_cell) cell_pstart[cell] = p;
}

__global__ void k_cm_rowkeys(const uint32_t* __restrict__ cell_first, int32_t n_cell, uint64_t* __restrict__ keys,
                             uint32_t* __restrict__ vals, uint64_t* __restrict__ n_rows) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool counted = c < n_cell && cell_first[c] != 0xFFFFFFFFu;
  const uint64_t rows = wave_sum<uint64_t>(counted ? 1ull : 0ull);
  if ((threadIdx.x & (kWave - 1)) == 0 && rows) atomicAdd((unsigned long long*)n_rows, (unsigned long long)rows);
  if (c >= n_cell) return;
  keys[c] = cell_first[c];  // uncounted cells (0xFFFFFFFF) sort last
  vals[c] = (uint32_t)c;
}

__global__ void k_cm_rows(const uint32_t* __restrict__ sorted_cells, int64_t n_rows,
                          const uint32_t* __restrict__ cell_npairs, int32_t* __restrict__ row_cell,
                          uint32_t* __restrict__ row_of, uint32_t* __restrict__ row_pairs) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_rows) return;
  const uint32_t c = sorted_cells[r];
  row_cell[r] = (int32_t)c;
  row_of[c] = (uint32_t)r;
  row_pairs[r] = cell_npairs[c];
}

__global__ void k_cm_scatter(int64_t nnz, const int32_t* __restrict__ pair_cell, const int32_t* __restrict__ pair_col,
                             const uint32_t* __restrict__ pair_count, const uint32_t* __restrict__ cell_pstart,
                             const uint32_t* __restrict__ row_of, const int32_t* __restrict__ indptr,
                             int32_t* __restrict__ indices, uint32_t* __restrict__ data) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= nnz) return;
  const int32_t c = pair_cell[p];
  const int64_t dst = (int64_t)indptr[row_of[c]] + (p - (int64_t)cell_pstart[c]);
  indices[dst] = pair_col[p];
  data[dst] = pair_count[p];
}

__global__ void k_cm_set_tail(int32_t* __restrict__ indptr, int64_t n_rows, int64_t nnz) {
  if (threadIdx.x == 0) indptr[n_rows] = (int32_t)nnz;
}

}  // namespace sct
