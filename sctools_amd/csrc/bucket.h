// bucket.h -- distinct counts without a device-wide sort.
//
// The reference's Counters (aggregator.py:264, 300-303, 530, 595) need, per entity,
// the records grouped by [k1 | k2 | fragment hash].  Records already arrive grouped by
// entity (cell-sorted input, iter_tag_groups, bam.py:492-540), so only a SEGMENTED sort
// is needed, and only far enough to make every group small:
//
//   level 0   entities of <= kBCap records are terminal buckets as they stand;
//   level L   larger segments are split MSD-first on the next 8 key bits: a per-segment
//             digit histogram, a scan into cursors, and a scatter that ranks each chunk
//             in LDS and reserves one range per (chunk, digit) with a single atomic;
//             children of <= kBCap records become terminal buckets, larger ones the next
//             level's segments (records ping-pong between the A and B buffers);
//   tile      one block per window of kWin record positions takes every terminal bucket
//             that starts in the window (<= kTileCap records), sorts them in LDS on
//             [bucket | key'] with wave-level multi-split passes over only the bits that
//             vary in the tile, and computes the distinct-count events of reduce.h from
//             neighbours -- every group is complete inside the tile;
//   giant     a bucket whose whole key is fixed but still > kBCap records (one molecule
//             with > 2047 reads at one hashed fragment) is resolved by one block.
//
// A k1 group or molecule split across sibling buckets (only when a single k1 value or
// molecule has > kBCap records) carries flags so exactly one piece counts its head and
// every piece knows the group has >= 2 records.
//
// Keys: key' = [k1' | k2 | hash] with k1' = k1 * odd mod 2^k1 (Bits::scramble), so heavy
// genes with neighbouring ids do not pile into one top digit.  KB = k1 + k2 + h <= 40
// leaves room for the 11-bit bucket ordinal and the 12-bit tile position in 64 bits.
#pragma once
#include "radix.h"
#include "reduce.h"
#include "util.h"

namespace sct {

constexpr int kBCap = 2047;                 // records of a terminal bucket (11-bit count)
constexpr int kWin = 2048;                  // a tile owns the buckets starting in kWin positions
constexpr int kTileCap = kWin + kBCap - 1;  // 4094 records per tile at most
constexpr int kChunk = kTile;               // records per partition work item
constexpr int kMaxKeyBits = 40;             // KB + 11 (ordinal) + 12 (position) <= 63
static_assert(kTileCap <= kTile, "tile capacity");
static_assert(kBCap < (1 << 11), "count field");

// terminal bucket descriptor, stored (u16) at the bucket's first record position
enum : uint16_t {
  BD_COUNT = 0x07FF,
  BD_PARITY = 1u << 11,     // records live in buffer B
  BD_K1_NOHEAD = 1u << 12,  // single-k1 piece that is not its k1 group's first piece
  BD_K1_MULTI = 1u << 13,   // single-k1 piece of a k1 group with >= 2 records
  BD_MOL_NOHEAD = 1u << 14,
  BD_MOL_MULTI = 1u << 15,
};

struct Seg {
  uint32_t start, cnt, ent, flags;
};
struct Work {
  uint32_t seg, chunk;
};
struct BucketCtl {  // device counters of one level (n_giant accumulates over levels)
  uint32_t n_seg, n_work, n_giant, pad;
};

__device__ __forceinline__ void push_segment(const Seg& sg, Seg* __restrict__ seg, Work* __restrict__ work,
                                             BucketCtl* ctl) {
  const uint32_t id = atomicAdd(&ctl->n_seg, 1u);
  seg[id] = sg;
  const uint32_t nw = (sg.cnt + kChunk - 1) / kChunk;
  const uint32_t w0 = atomicAdd(&ctl->n_work, nw);
  for (uint32_t k = 0; k < nw; k++) work[w0 + k] = Work{id, k};
}

// level 0: small entities are terminal buckets; larger ones become segments
__global__ void k_bucket_level0(const int64_t* __restrict__ ent_start, int64_t n_ent, int64_t n,
                                uint16_t* __restrict__ bdesc, Seg* __restrict__ seg, Work* __restrict__ work,
                                BucketCtl* ctl) {
  const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (e >= n_ent) return;
  const int64_t s0 = ent_start[e];
  const int64_t s1 = e + 1 < n_ent ? ent_start[e + 1] : n;
  const uint32_t c = (uint32_t)(s1 - s0);
  if (c <= (uint32_t)kBCap) {
    bdesc[s0] = (uint16_t)c;
    return;
  }
  push_segment(Seg{(uint32_t)s0, c, (uint32_t)e, 0u}, seg, work, ctl);
}

__global__ void __launch_bounds__(kBlock) k_bucket_hist(const uint64_t* __restrict__ keys, const Seg* __restrict__ seg,
                                                        const Work* __restrict__ work, int shift, int bits,
                                                        uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[kWaves][kRadix];
  const int wid = threadIdx.x / kWave;
  for (int i = threadIdx.x; i < kWaves * kRadix; i += kBlock) (&h[0][0])[i] = 0;
  const Work wk = work[xcd_tile(blockIdx.x, gridDim.x)];
  const Seg sg = seg[wk.seg];
  const uint32_t beg = sg.start + wk.chunk * (uint32_t)kChunk;
  const uint32_t end = (sg.start + sg.cnt - beg) < (uint32_t)kChunk ? sg.start + sg.cnt : beg + kChunk;
  const uint64_t mask = (1ull << bits) - 1;
  __syncthreads();
  for (uint32_t p = beg + threadIdx.x; p < end; p += kBlock) atomicAdd(&h[wid][(keys[p] >> shift) & mask], 1u);
  __syncthreads();
  const int d = threadIdx.x;
  uint32_t tot = 0;
#pragma unroll
  for (int w = 0; w < kWaves; w++) tot += h[w][d];
  if (tot) atomicAdd(&hist[(size_t)wk.seg * kRadix + d], tot);
}

// cursors: bucket bases of every segment (exclusive scan of its digit counts)
__global__ void __launch_bounds__(kBlock) k_bucket_segscan(const Seg* __restrict__ seg,
                                                           const uint32_t* __restrict__ hist,
                                                           uint32_t* __restrict__ cur) {
  __shared__ uint64_t lds[kWaves + 1];
  const size_t i = (size_t)blockIdx.x * kRadix + threadIdx.x;
  uint64_t tot;
  const uint64_t ex = block_exclusive_scan<uint64_t>((uint64_t)hist[i], &tot, lds);
  cur[i] = seg[blockIdx.x].start + (uint32_t)ex;
}

// Stable wave-level multi-split rank of one item: `peers` = lanes of the wave holding the
// same digit; the lowest such lane bumps the wave's counter for the digit.
__device__ __forceinline__ uint32_t wlms_rank(uint32_t d, int nbits, uint32_t* whist_w) {
  const int lane = threadIdx.x & (kWave - 1);
  const uint64_t lt = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
  uint64_t peers = ~0ull;
  for (int bitn = 0; bitn < nbits; bitn++) {
    const uint64_t m = __ballot((d >> bitn) & 1u);
    peers &= ((d >> bitn) & 1u) ? m : ~m;
  }
  const int leader = __ffsll((unsigned long long)peers) - 1;
  const uint32_t below = (uint32_t)__popcll(peers & lt);
  uint32_t bse = 0;
  if (lane == leader) {
    bse = whist_w[d];
    whist_w[d] = bse + (uint32_t)__popcll(peers);
  }
  bse = (uint32_t)__shfl((int)bse, leader);
  return bse + below;
}

// Turn the per-wave digit counts into per-wave digit starts (block-wide; barriers).  Returns,
// for thread d, the number of items with digit d and writes the digit start to dstart[d].
__device__ __forceinline__ uint32_t digit_starts(uint32_t (*whist)[kRadix], uint32_t* dstart, uint64_t* s_scan) {
  const int d = threadIdx.x;
  uint32_t run = 0;
  uint32_t pre[kWaves];
#pragma unroll
  for (int w = 0; w < kWaves; w++) {
    pre[w] = run;
    run += whist[w][d];
  }
  uint64_t tot;
  const uint64_t ds = block_exclusive_scan<uint64_t>((uint64_t)run, &tot, s_scan);
  if (dstart) dstart[d] = (uint32_t)ds;
#pragma unroll
  for (int w = 0; w < kWaves; w++) whist[w][d] = (uint32_t)ds + pre[w];
  return run;
}

// One level's scatter: rank a chunk in LDS on the level digit, reserve one output range per
// present digit with one atomic on the segment's cursor, and write each digit's records as a
// contiguous run (LDS-staged, coalesced).
__global__ void __launch_bounds__(kBlock) k_bucket_scatter(const uint64_t* __restrict__ kin,
                                                           const uint32_t* __restrict__ vin,
                                                           uint64_t* __restrict__ kout, uint32_t* __restrict__ vout,
                                                           const Seg* __restrict__ seg, const Work* __restrict__ work,
                                                           int shift, int bits, uint32_t* __restrict__ cur) {
  __shared__ uint64_t s_keys[kTile];
  __shared__ uint32_t s_vals[kTile];
  __shared__ uint32_t s_whist[kWaves][kRadix];
  __shared__ uint32_t s_dstart[kRadix];
  __shared__ uint32_t s_gbase[kRadix];
  __shared__ uint64_t s_scan[kWaves + 1];
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  const Work wk = work[xcd_tile(blockIdx.x, gridDim.x)];
  const Seg sg = seg[wk.seg];
  const uint32_t beg = sg.start + wk.chunk * (uint32_t)kChunk;
  const int tile_n = (int)((sg.start + sg.cnt - beg) < (uint32_t)kChunk ? (sg.start + sg.cnt - beg) : kChunk);
  const uint32_t mask = (1u << bits) - 1;
  for (int i = threadIdx.x; i < kWaves * kRadix; i += kBlock) (&s_whist[0][0])[i] = 0;
  __syncthreads();
  uint64_t k[kItems];
  uint32_t v[kItems];
  uint16_t rank[kItems];
  uint8_t dig[kItems];
#pragma unroll
  for (int j = 0; j < kItems; j++) {
    const int q = wid * (kItems * kWave) + j * kWave + lane;
    if (q < tile_n) {
      k[j] = kin[beg + q];
      v[j] = vin[beg + q];
    } else {
      k[j] = ~0ull;  // padding: the top digit, ranked after every real item
      v[j] = 0;
    }
    const uint32_t d = (uint32_t)(k[j] >> shift) & mask;
    dig[j] = (uint8_t)d;
    rank[j] = (uint16_t)wlms_rank(d, bits, s_whist[wid]);
  }
  __syncthreads();
  {
    uint32_t run = digit_starts(s_whist, s_dstart, s_scan);
    const uint32_t d = threadIdx.x;
    if (d == mask) run -= (uint32_t)(kTile - tile_n);  // padding sits at the end of the top digit
    if (run) s_gbase[d] = atomicAdd(&cur[(size_t)wk.seg * kRadix + d], run);
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kItems; j++) {
    const uint32_t lp = s_whist[wid][dig[j]] + rank[j];
    s_keys[lp] = k[j];
    s_vals[lp] = v[j];
  }
  __syncthreads();
  for (int q = threadIdx.x; q < tile_n; q += kBlock) {
    const uint64_t kk = s_keys[q];
    const uint32_t d = (uint32_t)(kk >> shift) & mask;
    const uint32_t o = s_gbase[d] + (uint32_t)(q - (int)s_dstart[d]);
    kout[o] = kk;
    vout[o] = s_vals[q];
  }
}

// Split flags of child digit d for the group boundary at Kb key bits (k1: K1; molecule:
// K1 + K2), when the parent fixes `depth` bits and the child `depth1`.  s_c = child counts.
__device__ __forceinline__ uint32_t split_flags(int Kb, int depth, int depth1, int d, uint32_t pflags,
                                                const uint32_t* s_c, uint32_t nohead, uint32_t multi) {
  if (depth1 <= Kb) return 0;  // the child holds whole groups
  const bool inherit = depth >= Kb;  // the parent already is one group's piece
  int lo = 0, hi = kRadix;
  if (!inherit) {
    const int g = depth1 - Kb;
    lo = (d >> g) << g;
    hi = lo + (1 << g);
  }
  int before = 0, total = 0;
  for (int x = lo; x < hi; x++) {
    const int ne = s_c[x] != 0;
    total += ne;
    before += (x < d) ? ne : 0;
  }
  uint32_t f = 0;
  if (inherit) {  // the group has > kBCap records
    f |= multi;
    if ((pflags & nohead) || before) f |= nohead;
  } else if (total >= 2) {
    f |= multi;
    if (before) f |= nohead;
  }
  return f;
}

// one block per segment, one thread per child digit
__global__ void __launch_bounds__(kBlock) k_bucket_classify(const Seg* __restrict__ seg,
                                                            const uint32_t* __restrict__ hist,
                                                            const uint32_t* __restrict__ cur, int depth, int bits,
                                                            int K1, int KM, int KB, int parity,
                                                            uint16_t* __restrict__ bdesc, Seg* __restrict__ nseg,
                                                            Work* __restrict__ nwork, Seg* __restrict__ giants,
                                                            BucketCtl* ctl) {
  __shared__ uint32_t s_c[kRadix];
  const int d = threadIdx.x;
  const size_t i = (size_t)blockIdx.x * kRadix + d;
  const Seg sg = seg[blockIdx.x];
  const uint32_t c = hist[i];
  s_c[d] = c;
  __syncthreads();
  if (c == 0) return;
  const uint32_t start = cur[i] - c;
  const int depth1 = depth + bits;
  uint32_t fl = split_flags(K1, depth, depth1, d, sg.flags, s_c, BD_K1_NOHEAD, BD_K1_MULTI);
  fl |= split_flags(KM, depth, depth1, d, sg.flags, s_c, BD_MOL_NOHEAD, BD_MOL_MULTI);
  const uint32_t par = parity ? BD_PARITY : 0u;
  if (c <= (uint32_t)kBCap) {
    bdesc[start] = (uint16_t)(c | fl | par);
  } else if (depth1 >= KB) {
    const uint32_t id = atomicAdd(&ctl->n_giant, 1u);
    giants[id] = Seg{start, c, sg.ent, fl | par};
  } else {
    push_segment(Seg{start, c, sg.ent, fl}, nseg, nwork, ctl);
  }
}

__device__ __forceinline__ uint32_t entity_of(const int64_t* __restrict__ ent_start, int64_t n_ent, int64_t pos) {
  int64_t lo = 0, hi = n_ent - 1;  // largest e with ent_start[e] <= pos
  while (lo < hi) {
    const int64_t mid = (lo + hi + 1) >> 1;
    if (ent_start[mid] <= pos)
      lo = mid;
    else
      hi = mid - 1;
  }
  return (uint32_t)lo;
}

// first entity of every window: entity of record position w * kWin (w = 0..n_win; entry n_win is
// the entity of the last record).  Tiles then search only their own slice of ent_start.
__global__ void k_window_entities(const int64_t* __restrict__ ent_start, int64_t n_ent, int64_t n, int64_t n_win,
                                  uint32_t* __restrict__ win_ent) {
  const int64_t w = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (w > n_win) return;
  const int64_t p = w * kWin < n ? w * kWin : n - 1;
  win_ent[w] = entity_of(ent_start, n_ent, p);
}

// exclusive max-scan over the block (values >= 0); lds needs kWaves entries; barriers inside
__device__ __forceinline__ uint32_t block_exclusive_max(uint32_t v, uint32_t* lds) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  uint32_t x = v;
  for (int off = 1; off < kWave; off <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)x, off);
    if (lane >= off) x = y > x ? y : x;
  }
  if (lane == kWave - 1) lds[wid] = x;
  __syncthreads();
  uint32_t carry = 0;
  for (int w = 0; w < wid; w++) carry = lds[w] > carry ? lds[w] : carry;
  uint32_t ex = (uint32_t)__shfl_up((int)x, 1);
  if (lane == 0) ex = 0;
  __syncthreads();
  return ex > carry ? ex : carry;
}

template <bool kCell, bool kGene>
__global__ void __launch_bounds__(kBlock) k_bucket_tile(const uint16_t* __restrict__ bdesc,
                                                        const uint64_t* __restrict__ keys_a,
                                                        const uint32_t* __restrict__ vals_a,
                                                        const uint64_t* __restrict__ keys_b,
                                                        const uint32_t* __restrict__ vals_b, int64_t n,
                                                        const int64_t* __restrict__ ent_start,
                                                        const uint32_t* __restrict__ win_ent, RecCols r,
                                                        const uint8_t* __restrict__ k1_is_mito, Bits b,
                                                        int64_t* __restrict__ partials,
                                                        uint16_t* __restrict__ dflags) {
  __shared__ uint64_t s_x[kTile];     // sort keys [bucket | key' | tile position]; scratch before the sort
  __shared__ uint32_t s_val[kTile];   // values by tile position
  __shared__ uint32_t s_bpos[kWin];   // bucket start (record position)
  __shared__ uint16_t s_boff[kWin + 1];
  __shared__ uint16_t s_bd[kWin];
  __shared__ uint32_t s_bent[kWin];
  __shared__ uint32_t s_whist[kWaves][kRadix];
  __shared__ uint64_t s_scan[kWaves + 1];
  __shared__ uint64_t s_red[2][kWaves];
  __shared__ uint32_t s_edge[4][kWaves];
  uint32_t* s_es = reinterpret_cast<uint32_t*>(s_x);                  // entity starts of the window
  uint16_t* s_bid = reinterpret_cast<uint16_t*>(s_x) + 2 * (kWin + 8);  // bucket of each tile position
  constexpr int kPer = kWin / kBlock;
  const int t = threadIdx.x;
  const int lane = t & (kWave - 1);
  const int wid = t / kWave;
  const unsigned wb = xcd_tile(blockIdx.x, gridDim.x);
  const int64_t w0 = (int64_t)wb * kWin;
  const int win_n = (int)((n - w0) < kWin ? (n - w0) : kWin);

  // 1. bucket starts in the window, in position order
  uint16_t dsc[kPer];
  uint32_t nv = 0;
#pragma unroll
  for (int j = 0; j < kPer; j++) {
    const int q = t * kPer + j;
    dsc[j] = q < win_n ? bdesc[w0 + q] : (uint16_t)0;
    nv += dsc[j] != 0;
  }
  uint64_t tot;
  uint32_t bi = (uint32_t)block_exclusive_scan<uint64_t>(nv, &tot, s_scan);
  const int nb = (int)tot;
#pragma unroll
  for (int j = 0; j < kPer; j++) {
    if (dsc[j]) {
      s_bpos[bi] = (uint32_t)(w0 + t * kPer + j);
      s_bd[bi] = dsc[j];
      bi++;
    }
  }
  __syncthreads();
  // 2. tile offsets of the buckets; the window's slice of entity starts
  uint32_t cnt[kPer];
  uint32_t sum = 0;
#pragma unroll
  for (int j = 0; j < kPer; j++) {
    const int x = t * kPer + j;
    cnt[j] = x < nb ? (uint32_t)(s_bd[x] & BD_COUNT) : 0u;
    sum += cnt[j];
  }
  uint32_t off = (uint32_t)block_exclusive_scan<uint64_t>(sum, &tot, s_scan);
  const int tn = (int)tot;
#pragma unroll
  for (int j = 0; j < kPer; j++) {
    const int x = t * kPer + j;
    if (x < nb) s_boff[x] = (uint16_t)off;
    off += cnt[j];
  }
  if (t == 0) s_boff[nb] = (uint16_t)tn;
  const uint32_t e_lo = win_ent[wb];
  const int ne = (int)(win_ent[wb + 1] - e_lo) + 1;  // <= kWin + 1
  for (int x = t; x < ne; x += kBlock) s_es[x] = (uint32_t)ent_start[e_lo + x];
  for (int q = t; q < tn; q += kBlock) s_bid[q] = 0;
  __syncthreads();
  if (tn == 0) return;  // block-uniform
  for (int x = t; x < nb; x += kBlock) {
    s_bid[s_boff[x]] = (uint16_t)x;  // bucket start marker
    const uint32_t pos = s_bpos[x];
    int lo = 0, hi = ne - 1;  // entity: largest slice index with start <= pos
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (s_es[mid] <= pos)
        lo = mid;
      else
        hi = mid - 1;
    }
    s_bent[x] = e_lo + (uint32_t)lo;
  }
  __syncthreads();
  {  // fill: bucket id of every tile position = running max of the start markers
    uint32_t run = 0;
#pragma unroll
    for (int j = 0; j < kItems; j++) {
      const int q = t * kItems + j;
      if (q < tn) run = s_bid[q] > run ? s_bid[q] : run;
    }
    uint32_t m = block_exclusive_max(run, &s_whist[0][0]);
#pragma unroll
    for (int j = 0; j < kItems; j++) {
      const int q = t * kItems + j;
      if (q < tn) {
        m = s_bid[q] > m ? s_bid[q] : m;
        s_bid[q] = (uint16_t)m;
      }
    }
  }
  __syncthreads();

  // 3. load the records in the wave-major item layout (wave w owns positions [w*per, (w+1)*per))
  const int KB = b.k1 + b.k2 + b.h;
  const int per = ((tn + kBlock - 1) / kBlock) * kWave;  // items per wave, a multiple of 64
  const int rounds = per / kWave;
  const uint64_t kbm = (1ull << KB) - 1;
  uint64_t k[kItems];
  uint64_t vor = 0, vand = ~0ull;
#pragma unroll
  for (int j = 0; j < kItems; j++) {
    k[j] = ~0ull;
    if (j < rounds) {
      const int q = wid * per + j * kWave + lane;
      if (q < tn) {
        const int bk = s_bid[q];
        const uint32_t gp = s_bpos[bk] + (uint32_t)(q - (int)s_boff[bk]);
        const bool pb = s_bd[bk] & BD_PARITY;
        // ids >= the dictionary sizes must not reach the ordinal bits
        const uint64_t kk = (pb ? keys_b[gp] : keys_a[gp]) & kbm;
        s_val[q] = pb ? vals_b[gp] : vals_a[gp];
        k[j] = ((uint64_t)bk << (KB + 12)) | (kk << 12) | (uint64_t)q;
        vor |= k[j];
        vand &= k[j];
      }
    }
  }
  // bits that vary across the tile: only those need sorting
  for (int o = kWave / 2; o > 0; o >>= 1) {
    vor |= __shfl_xor(vor, o);
    vand &= __shfl_xor(vand, o);
  }
  if (lane == 0) {
    s_red[0][wid] = vor;
    s_red[1][wid] = vand;
  }
  __syncthreads();
  uint64_t vary = 0;
  {
    uint64_t o = 0, a = ~0ull;
#pragma unroll
    for (int w = 0; w < kWaves; w++) {
      o |= s_red[0][w];
      a &= s_red[1][w];
    }
    vary = (o ^ a) >> 12 << 12;
  }
  const int hb = vary ? 63 - __builtin_clzll(vary) : -1;

  // 4. LSD passes in LDS over bits [12, hb]; items stay in registers between passes
  for (int shift = 12; shift <= hb; shift += kRadixBits) {
    const int nbits = (hb + 1 - shift) < kRadixBits ? (hb + 1 - shift) : kRadixBits;
    const uint32_t mask = (1u << nbits) - 1;
    for (int i = t; i < kWaves * kRadix; i += kBlock) (&s_whist[0][0])[i] = 0;
    __syncthreads();
    uint16_t rank[kItems];
    uint8_t dig[kItems];
#pragma unroll
    for (int j = 0; j < kItems; j++) {
      if (j < rounds) {
        const uint32_t d = (uint32_t)(k[j] >> shift) & mask;
        dig[j] = (uint8_t)d;
        rank[j] = (uint16_t)wlms_rank(d, nbits, s_whist[wid]);
      }
    }
    __syncthreads();
    digit_starts(s_whist, nullptr, s_scan);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kItems; j++)
      if (j < rounds) s_x[s_whist[wid][dig[j]] + rank[j]] = k[j];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kItems; j++)
      if (j < rounds) k[j] = s_x[wid * per + j * kWave + lane];
    __syncthreads();
  }
  if (hb < 12) {  // already in order (one key' value): place the items by position
#pragma unroll
    for (int j = 0; j < kItems; j++)
      if (j < rounds) {
        const int q = wid * per + j * kWave + lane;
        if (q < tn) s_x[q] = k[j];
      }
    __syncthreads();
  }

  // 5. distinct-count events from sorted neighbours (reduce.h semantics + split flags).
  // Blocked: thread t owns sorted positions [16t, 16t + 16).  Records whose fragment key
  // equals a neighbour's gather (ref, strand, pos) all at once; the neighbour of the first /
  // last item comes from the adjacent lane or, at a wave edge, through LDS.
  const int q0 = t * kItems;
  uint32_t fr[kItems], fp[kItems];  // fragment identity: ref * 2 + strand, pos (~0: none)
  uint8_t fl[kItems];               // 1: equal key before, 2: equal key after, 4: mapped
#pragma unroll
  for (int j = 0; j < kItems; j++) {
    const int q = q0 + j;
    fr[j] = ~0u;
    fp[j] = ~0u;
    fl[j] = 0;
    if (q < tn) {
      const uint64_t sk = s_x[q];
      const uint64_t fk = sk >> 12;
      const uint32_t v = s_val[sk & 0xFFF];
      const bool mapped = !(v & kUnmappedValBit);
      const bool ep = q > 0 && (s_x[q - 1] >> 12) == fk;
      const bool en = q + 1 < tn && (s_x[q + 1] >> 12) == fk;
      fl[j] = (ep ? 1 : 0) | (en ? 2 : 0) | (mapped ? 4 : 0);
      if (mapped && (ep || en)) {
        const uint32_t i = v & ~kUnmappedValBit;
        fr[j] = (uint32_t)r.ref[i] * 2u + ((r.bits[i] & SCT_B_REVERSE) ? 1u : 0u);
        fp[j] = (uint32_t)r.pos[i];
      }
    }
  }
  uint32_t pfr = (uint32_t)__shfl_up((int)fr[kItems - 1], 1), pfp = (uint32_t)__shfl_up((int)fp[kItems - 1], 1);
  uint32_t nfr = (uint32_t)__shfl_down((int)fr[0], 1), nfp = (uint32_t)__shfl_down((int)fp[0], 1);
  if (lane == kWave - 1) {
    s_edge[0][wid] = fr[kItems - 1];
    s_edge[1][wid] = fp[kItems - 1];
  }
  if (lane == 0) {
    s_edge[2][wid] = fr[0];
    s_edge[3][wid] = fp[0];
  }
  __syncthreads();
  if (lane == 0 && wid > 0) {
    pfr = s_edge[0][wid - 1];
    pfp = s_edge[1][wid - 1];
  }
  if (lane == kWave - 1 && wid < kWaves - 1) {
    nfr = s_edge[2][wid + 1];
    nfp = s_edge[3][wid + 1];
  }

  const int sh1 = 12 + b.k2 + b.h;
  const int shm = 12 + b.h;
  const uint32_t k1m = b.k1_mask();
  int64_t acc[kDistinct];
#pragma unroll
  for (int i = 0; i < kDistinct; i++) acc[i] = 0;
  int64_t cur_e = -1;
  const auto slot = [](int i) { return distinct_slot(i); };
#pragma unroll
  for (int j = 0; j < kItems; j++) {
    const int q = q0 + j;
    const bool valid = q < tn;
    const uint64_t sk = valid ? s_x[q] : 0ull;
    const int bk = (int)(sk >> (KB + 12));
    const int64_t e = valid ? (int64_t)s_bent[bk] : cur_e;
    wave_flush<kDistinct>(acc, valid && e != cur_e && cur_e >= 0, cur_e, partials, slot);
    if (!valid) continue;
    cur_e = e;
    const uint64_t prev = q > 0 ? s_x[q - 1] : ~0ull;
    const uint64_t next = q + 1 < tn ? s_x[q + 1] : ~0ull;
    const uint32_t bd = s_bd[bk];
    const bool k1_head = (prev >> sh1) != (sk >> sh1) && !(bd & BD_K1_NOHEAD);
    const bool k1_multi = k1_head && ((bd & BD_K1_MULTI) || (next >> sh1) == (sk >> sh1));
    const bool mol_head = (prev >> shm) != (sk >> shm) && !(bd & BD_MOL_NOHEAD);
    const bool mol_single = mol_head && !(bd & BD_MOL_MULTI) && (next >> shm) != (sk >> shm);
    const uint32_t v = s_val[sk & 0xFFF];
    const uint32_t i = v & ~kUnmappedValBit;
    uint16_t f = (mol_head ? DF_MOL_HEAD : 0) | (mol_single ? DF_MOL_SINGLE : 0) | (k1_head ? DF_K1_HEAD : 0) |
                 (k1_multi ? DF_K1_MULTI : 0);
    acc[0] += mol_head;
    acc[1] += mol_single;
    acc[4] += k1_head;
    acc[5] += k1_multi;
    if constexpr (kCell) {
      if (k1_head) acc[6] += k1_is_mito[b.unscramble((uint32_t)(sk >> sh1) & k1m)];
    }
    if (fl[j] & 4) {
      const uint32_t pr = j > 0 ? fr[j - 1] : pfr, pp = j > 0 ? fp[j - 1] : pfp;
      const uint32_t nr = j + 1 < kItems ? fr[j + 1] : nfr, np = j + 1 < kItems ? fp[j + 1] : nfp;
      const uint64_t fk = sk >> 12;
      bool is_first = true, single = true;
      if (fl[j] & 1) {
        if (pr == fr[j] && pp == fp[j]) {
          is_first = false;
        } else {  // the neighbour holds another fragment under the same hash: scan the sub-run
          for (int pq = q - 2; pq >= 0; pq--) {
            const uint64_t kq = s_x[pq];
            if ((kq >> 12) != fk) break;
            const uint32_t vq = s_val[kq & 0xFFF];
            if (!(vq & kUnmappedValBit) && same_fragment(r, vq, i)) {
              is_first = false;
              break;
            }
          }
        }
      }
      if (is_first && (fl[j] & 2)) {
        if (nr == fr[j] && np == fp[j]) {
          single = false;
        } else {
          for (int pq = q + 2; pq < tn; pq++) {
            const uint64_t kq = s_x[pq];
            if ((kq >> 12) != fk) break;
            const uint32_t vq = s_val[kq & 0xFFF];
            if (!(vq & kUnmappedValBit) && same_fragment(r, vq, i)) {
              single = false;
              break;
            }
          }
        }
      }
      if (is_first) {
        acc[2] += 1;
        acc[3] += single;
        f |= DF_FRAG_FIRST | (single ? DF_FRAG_SINGLE : 0);
      }
    }
    if constexpr (kGene) dflags[i] = f;
  }
  wave_flush<kDistinct>(acc, cur_e >= 0, cur_e, partials, slot);
}

// A bucket whose whole key' is fixed and still holds > kBCap records: one piece of one
// molecule at one fragment hash.  One block; fragments resolved exactly by repeatedly taking
// the first unassigned mapped record as a representative.  `mark` is the other buffer's
// value array over the same range (dead: the parent segment was scattered out of it).
template <bool kCell, bool kGene>
__global__ void __launch_bounds__(kBlock) k_bucket_giant(const Seg* __restrict__ giants,
                                                         const uint64_t* __restrict__ keys_a,
                                                         uint32_t* __restrict__ vals_a,
                                                         const uint64_t* __restrict__ keys_b,
                                                         uint32_t* __restrict__ vals_b, RecCols r,
                                                         const uint8_t* __restrict__ k1_is_mito, Bits b,
                                                         int64_t* __restrict__ partials,
                                                         uint16_t* __restrict__ dflags) {
  __shared__ uint64_t s_red[kWaves];
  __shared__ uint32_t s_min[kWaves];
  const Seg g = giants[blockIdx.x];
  const bool pb = g.flags & BD_PARITY;
  const uint32_t* vals = pb ? vals_b : vals_a;
  uint32_t* mark = pb ? vals_a : vals_b;
  const int t = threadIdx.x;
  const int lane = t & (kWave - 1);
  const int wid = t / kWave;
  const bool k1_head = !(g.flags & BD_K1_NOHEAD);
  const bool mol_head = !(g.flags & BD_MOL_NOHEAD);
  for (uint32_t p = t; p < g.cnt; p += kBlock) {
    const uint32_t v = vals[g.start + p];
    mark[g.start + p] = (v & kUnmappedValBit) ? 1u : 0u;
    if constexpr (kGene) {
      uint16_t f = 0;
      if (p == 0) f = (k1_head ? (DF_K1_HEAD | DF_K1_MULTI) : 0) | (mol_head ? DF_MOL_HEAD : 0);
      dflags[v & ~kUnmappedValBit] = f;
    }
  }
  __syncthreads();
  int64_t n_frag = 0, n_single = 0;
  while (true) {
    uint32_t m = 0xFFFFFFFFu;
    for (uint32_t p = t; p < g.cnt; p += kBlock)
      if (!mark[g.start + p]) {
        m = p;
        break;
      }
    for (int o = kWave / 2; o > 0; o >>= 1) {
      const uint32_t y = (uint32_t)__shfl_xor((int)m, o);
      m = y < m ? y : m;
    }
    if (lane == 0) s_min[wid] = m;
    __syncthreads();
    uint32_t rep = 0xFFFFFFFFu;
#pragma unroll
    for (int w = 0; w < kWaves; w++) rep = s_min[w] < rep ? s_min[w] : rep;
    __syncthreads();
    if (rep == 0xFFFFFFFFu) break;  // block-uniform
    const uint32_t ir = vals[g.start + rep] & ~kUnmappedValBit;
    uint64_t c = 0;
    for (uint32_t p = rep + t; p < g.cnt; p += kBlock) {
      if (mark[g.start + p]) continue;
      const uint32_t ip = vals[g.start + p] & ~kUnmappedValBit;
      if (same_fragment(r, ip, ir)) {
        mark[g.start + p] = 1u;
        c++;
      }
    }
    c = wave_sum(c);
    if (lane == 0) s_red[wid] = c;
    __syncthreads();
    uint64_t tot = 0;
#pragma unroll
    for (int w = 0; w < kWaves; w++) tot += s_red[w];
    n_frag += 1;
    n_single += tot == 1;
    if (kGene && t == 0) dflags[ir] |= DF_FRAG_FIRST | (tot == 1 ? DF_FRAG_SINGLE : 0);
    __syncthreads();
  }
  if (t == 0) {
    int64_t* row = partials + (int64_t)g.ent * SCT_NP;
    const uint64_t key = (pb ? keys_b : keys_a)[g.start];
    const uint32_t k1 = b.unscramble((uint32_t)(key >> (b.k2 + b.h)) & b.k1_mask());
    const int64_t add[kDistinct] = {mol_head ? 1 : 0, 0, n_frag, n_single, k1_head ? 1 : 0, k1_head ? 1 : 0,
                                    (kCell && k1_head) ? (int64_t)k1_is_mito[k1] : 0};
    for (int i = 0; i < kDistinct; i++)
      if (add[i]) atomicAdd((unsigned long long*)&row[distinct_slot(i)], (unsigned long long)add[i]);
  }
}

}  // namespace sct
