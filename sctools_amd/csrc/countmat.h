// countmat.h -- cells x genes molecule-count matrix (CountMatrix.from_sorted_tagged_bam,
// count.py:134-328) as a sort-and-count over 64-bit molecule keys.
//
// The reference walks query-name groups in file order, keeps a Python set of the
// (cell, molecule, gene) triples seen so far and appends one COO entry per new triple; the
// CSR conversion then sums the entries of each (cell, gene).  That is order-free except for
// the row order (a cell's row is numbered when its first molecule is counted), so:
//
//   k_cm_groups    one lane per query-name group head: the group's molecule key
//                  [cell | column | umi] and a keep flag; a wave-aggregated atomicMin of
//                  the group's record index per cell (row order) and over unknown genes
//   scan + k_cm_compact   kept keys -> a dense array (about half the records)
//   radix.h        LSD sort of the kept keys (cbits + colbits + ubits bits)
//   k_cm_heads     triple-head and (cell, column) pair-head flags; two scans number them
//   k_cm_emit      per pair: cell, column, index of its first triple, first pair of a cell
//   k_cm_cells     pairs per cell (from the cell's last pair)
//   k_cm_rowkeys   (first record index, cell) per counted cell -> radix.h -> row order
//   k_cm_rows      row -> cell, cell -> row, pairs per row; scan -> CSR indptr
//   k_cm_scatter   pairs (cell-id order) -> CSR rows (first-molecule order); the count of a
//                  pair = triples between its first triple and the next pair's
//
// No global atomics on the hot arrays: counts come from scans, so cell-sorted input (every
// lane of a wave on the same cell) costs the same as shuffled input.  HBM-bound integer
// work; see DESIGN.md §10 for the bytes per record of each kernel.
#pragma once
#include "radix.h"
#include "scan.h"
#include "util.h"

namespace sct {

struct CountKey {
  int cbits, colbits, ubits, total;  // total = cbits + colbits + ubits
};

struct CountCols {
  const int32_t *cell, *umi, *gene;
  const uint8_t *xf, *qhead;
  const int32_t* gene_col;
  int64_t n;
  int32_t n_cell, n_umi, n_gene, cell_none, umi_none, n_cols;
};

constexpr uint8_t kXfAbsent = 0, kXfIntergenic = 4;  // SCT_XF_ABSENT / SCT_XF_INTERGENIC

template <typename T>
__device__ __forceinline__ T wave_min(T v) {
  for (int off = kWave / 2; off > 0; off >>= 1) {
    const T o = __shfl_xor(v, off);
    v = o < v ? o : v;
  }
  return v;
}

// atomicMin(&dst[slot], v) for the lanes with `on`, combined across lanes with equal slots:
// a few leader rounds (cell-grouped input puts one or two cells in a wave), then per lane.
// Call from every lane of the wave.
__device__ __forceinline__ void wave_atomic_min(uint32_t* dst, bool on, uint32_t slot, uint32_t v) {
  const int lane = threadIdx.x & (kWave - 1);
  bool mine = on;
  for (int round = 0; round < 4; round++) {
    const uint64_t active = __ballot(mine);
    if (!active) return;
    const int leader = __ffsll((unsigned long long)active) - 1;
    const uint32_t s = __shfl(slot, leader);
    const bool take = mine && slot == s;
    const uint32_t m = wave_min(take ? v : 0xFFFFFFFFu);
    if (lane == leader) atomicMin(&dst[s], m);
    if (take) mine = false;
  }
  if (mine) atomicMin(&dst[slot], v);
}

// count.py:222-270 for the group starting at record i (qhead[i] == 1): cell / molecule of its
// first record; the implicated gene names are the single-name gene values of alignments with
// an XF tag other than INTERGENIC (gene_col != SKIP covers "has the tag" and "no ','"); the
// group counts when exactly one distinct name is implicated -- for a one-alignment group that
// is the same test.
//
// One lane per record: every lane loads its own alignment (coalesced) and classifies it; a group
// that closes inside the wave is resolved with ballots over its lanes (first implicated gene,
// any other implicated gene, any gene id outside the dictionary).  Only a group still open at
// the wave's last lane walks its remaining records in a loop.
__device__ __forceinline__ void cm_classify(const CountCols& c, int64_t j, int32_t& g, bool& implicated, bool& bad) {
  g = c.gene[j];
  bad = (uint32_t)g >= (uint32_t)c.n_gene;
  const uint8_t x = c.xf[j];
  implicated = !bad && x != kXfAbsent && x != kXfIntergenic && c.gene_col[g] != -1;
}

__global__ void __launch_bounds__(kBlock) k_cm_groups(CountCols c, CountKey K, uint64_t* __restrict__ keys,
                                                      uint32_t* __restrict__ keep, uint32_t* __restrict__ cell_first,
                                                      unsigned long long* __restrict__ unknown,
                                                      uint32_t* __restrict__ err) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t wbase = i - lane;
  const bool in = i < c.n;
  const bool head = in && (i == 0 || c.qhead[i]);
  int32_t g = 0;
  bool impl = false, badg = false;
  if (in) cm_classify(c, i, g, impl, badg);
  const uint64_t H = __ballot(head);
  const uint64_t I = __ballot(impl);
  const uint64_t Bm = __ballot(badg);
  // this lane's group within the wave: lanes [hd, nx)
  const uint64_t upto = lane == kWave - 1 ? ~0ull : ((2ull << lane) - 1);
  const uint64_t hbelow = H & upto;
  const int hd = hbelow ? 63 - __clzll((long long)hbelow) : -1;
  const uint64_t habove = H & ~upto;
  const int nx = habove ? __ffsll((unsigned long long)habove) - 1 : kWave;
  const uint64_t seg = hd < 0 ? 0ull : ((nx == kWave ? ~0ull : ((1ull << nx) - 1)) & ~((1ull << hd) - 1));
  const uint64_t Iseg = I & seg;
  const int first = Iseg ? __ffsll((unsigned long long)Iseg) - 1 : lane;
  const int32_t sel_w = __shfl(g, first);
  const uint64_t D = __ballot(impl && hd >= 0 && g != sel_w);
  bool kept = false;
  int32_t cell = 0;
  if (head) {
    cell = c.cell[i];
    const int32_t umi = c.umi[i];
    if ((uint32_t)cell >= (uint32_t)c.n_cell || (uint32_t)umi >= (uint32_t)c.n_umi) {
      atomicOr(err, 1u);
    } else if (cell != c.cell_none && umi != c.umi_none) {
      int32_t sel = Iseg ? sel_w : -1;
      bool multi = (D & seg) != 0;
      bool bad = (Bm & seg) != 0;
      const int64_t past = wbase + kWave;  // the group may continue past the wave's last lane
      if (!bad && nx == kWave && past < c.n && !c.qhead[past]) {
        for (int64_t j = past; j < c.n && !c.qhead[j]; j++) {
          int32_t gj;
          bool ij, bj;
          cm_classify(c, j, gj, ij, bj);
          if (bj) {
            bad = true;
            break;
          }
          if (!ij) continue;
          if (sel < 0) sel = gj;
          else if (gj != sel) multi = true;
        }
      }
      if (bad) {
        atomicOr(err, 1u);
      } else if (sel >= 0 && !multi) {
        int32_t col = c.gene_col[sel];
        if (col < 0 || col >= c.n_cols) {  // the reference's gene_name_to_index[gene_name] KeyError
          atomicMin(unknown, (unsigned long long)i);
          col = 0;
        }
        keys[i] = ((uint64_t)cell << (K.colbits + K.ubits)) | ((uint64_t)col << K.ubits) | (uint64_t)umi;
        kept = true;
      }
    }
  }
  if (in) keep[i] = kept ? 1u : 0u;
  wave_atomic_min(cell_first, kept, (uint32_t)cell, (uint32_t)i);
}

__global__ void k_cm_compact(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ keep,
                             const uint32_t* __restrict__ offs, int64_t n, uint64_t* __restrict__ out,
                             uint32_t* __restrict__ out_vals, uint64_t* __restrict__ n_kept) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (i == n - 1) *n_kept = (uint64_t)offs[i] + keep[i];
  if (!keep[i]) return;
  out[offs[i]] = keys[i];
  out_vals[offs[i]] = (uint32_t)i;
}

__global__ void k_cm_heads(const uint64_t* __restrict__ keys, int64_t m, CountKey K, uint32_t* __restrict__ triple,
                           uint32_t* __restrict__ pair) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const uint64_t k = keys[i];
  const uint64_t p = i ? keys[i - 1] : ~k;
  triple[i] = p != k ? 1u : 0u;
  pair[i] = (p >> K.ubits) != (k >> K.ubits) ? 1u : 0u;
}

__global__ void k_cm_emit(const uint64_t* __restrict__ keys, int64_t m, CountKey K, const uint32_t* __restrict__ pair,
                          const uint32_t* __restrict__ pair_off, const uint32_t* __restrict__ triple,
                          const uint32_t* __restrict__ triple_off, int32_t* __restrict__ pair_cell,
                          int32_t* __restrict__ pair_col, uint32_t* __restrict__ pair_tri,
                          uint32_t* __restrict__ cell_pstart, uint64_t* __restrict__ totals) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  if (i == m - 1) {
    totals[0] = (uint64_t)pair_off[i] + pair[i];
    totals[1] = (uint64_t)triple_off[i] + triple[i];
  }
  if (!pair[i]) return;
  const uint64_t k = keys[i];
  const uint32_t p = pair_off[i];
  const int cs = K.ubits + K.colbits;
  const int32_t cell = (int32_t)(k >> cs);
  pair_cell[p] = cell;
  pair_col[p] = (int32_t)((k >> K.ubits) & ((1ull << K.colbits) - 1));
  pair_tri[p] = triple_off[i];
  if (i == 0 || (keys[i - 1] >> cs) != (k >> cs)) cell_pstart[cell] = p;
}

__global__ void k_cm_cells(const int32_t* __restrict__ pair_cell, int64_t nnz, const uint32_t* __restrict__ cell_pstart,
                           uint32_t* __restrict__ cell_npairs) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= nnz) return;
  const int32_t c = pair_cell[p];
  if (p == nnz - 1 || pair_cell[p + 1] != c) cell_npairs[c] = (uint32_t)(p + 1 - cell_pstart[c]);
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

__global__ void k_cm_scatter(int64_t nnz, uint64_t n_triples, const int32_t* __restrict__ pair_cell,
                             const int32_t* __restrict__ pair_col, const uint32_t* __restrict__ pair_tri,
                             const uint32_t* __restrict__ cell_pstart, const uint32_t* __restrict__ row_of,
                             const int32_t* __restrict__ indptr, int32_t* __restrict__ indices,
                             uint32_t* __restrict__ data) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= nnz) return;
  const int32_t c = pair_cell[p];
  const int64_t dst = (int64_t)indptr[row_of[c]] + (p - (int64_t)cell_pstart[c]);
  const uint64_t next = p + 1 < nnz ? (uint64_t)pair_tri[p + 1] : n_triples;
  indices[dst] = pair_col[p];
  data[dst] = (uint32_t)(next - pair_tri[p]);
}

__global__ void k_cm_set_tail(int32_t* __restrict__ indptr, int64_t n_rows, int64_t nnz) {
  if (threadIdx.x == 0) indptr[n_rows] = (int32_t)nnz;
}

}  // namespace sct
