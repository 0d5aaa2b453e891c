// bucket.h -- distinct counts without a device-wide sort.
//
// The reference's Counters (aggregator.py:264, 300-303, 530, 595) need, per entity, the
// number of distinct (k1, k2) molecule keys, (k1, k2, ref, pos, strand) fragment keys and k1
// values, and how many of each occur exactly once.  Records already arrive grouped by entity
// (cell-sorted input, iter_tag_groups, bam.py:492-540), so only a SEGMENTED grouping is
// needed, and only far enough to make every group small:
//
//   level 0   entities of <= kBCap records are terminal buckets as they stand;
//   level L   larger segments are split MSD-first on the next 8 bits of key' = [k1' | k2 |
//             fragment hash]: a per-segment digit histogram, a scan into cursors, and a
//             scatter that ranks each chunk in LDS and reserves one range per (chunk, digit)
//             with a single atomic; children of <= kBCap records become terminal buckets,
//             larger ones the next level's segments (records ping-pong between buffers A, B);
//   tile      one kWin-thread block per window of kWin record positions takes every terminal
//             bucket that starts in the window (<= kTileCap records) and inserts each record
//             into three LDS hash tables keyed by (bucket, k1), (bucket, k1, k2) and
//             (molecule slot, ref, strand, pos).  The inserting record of a key is its head,
//             the first record to find it present its "second": n_distinct = #heads and
//             n_single = #heads - #seconds, with no sort and no neighbour scan;
//   giant     a bucket whose whole key' is fixed but still > kBCap records (one molecule with
//             > kBCap reads under one fragment hash) is resolved by one block.
//
// A k1 group or molecule split across sibling buckets (only when a single k1 value or
// molecule has > kBCap records) carries flags so exactly one piece counts its head and the
// group's ">= 2 records" event.
//
// Records travel as a 16-byte payload (Pay: two u64 words side by side, one 16-byte load or store
// per record) so no pass gathers by index:
//   w0 = key' << 17 | ref (14 bits) << 3 | strand << 2 | mapped << 1 | k1 is mitochondrial
//   w1 = record index << 32 | pos (uint32)
// key' = [k1' | k2 | hash] with k1' = k1 * odd mod 2^k1 (Bits::scramble), so heavy genes with
// neighbouring ids do not pile into one top digit.  KB = k1 + k2 + h <= 47 (so a 10x-v3 shard,
// 2^24 UMIs and ~2^17 gene ids, stays on this path); a mapped ref id must be < 2^14.
#pragma once
#include <type_traits>

#include "radix.h"
#include "reduce.h"
#include "util.h"

namespace sct {

constexpr int kWin = 1024;                  // a tile owns the buckets starting in kWin positions
constexpr int kHTCap = 2040;                // hash-tile table slots (not a power of two: the three
                                            // tables fit 40 KB of LDS, 4 blocks per CU)
constexpr int kBCap = kHTCap - kWin - 1;    // records of a terminal bucket (1015)
constexpr int kTileCap = kWin + kBCap - 1;  // records per tile at most (2046)
constexpr int kChunk = 2048;                // records per partition work item (LDS-staged)
constexpr int kChunkItems = kChunk / kBlock;
constexpr int kMaxKeyBits = 47;             // KB <= 47: key' sits in w0 bits [63:17]
constexpr int kKeyShift = 17;
constexpr int kRefBits = 14;                // mapped reference ids must be < 2^14
constexpr int kFragBits = kRefBits + 1;     // (ref, strand) of a payload
constexpr uint64_t kW0Mapped = 1ull << 1;
constexpr uint64_t kW0Mito = 1ull << 0;
constexpr int kHBlock = 512;                // tile block: two window positions per thread
constexpr int kHWaves = kHBlock / kWave;
constexpr int kHTBits = 11;
constexpr int kHTSlots = 1 << kHTBits;      // hash table slots: > kTileCap, so probing ends
constexpr int kWinBits = 10;                // bucket ordinal (window offset) bits in the keys
constexpr int kNarrowK1Bits = 32 - 2 - kWinBits;  // k1 ids up to 20 bits use a 32-bit k1 table
// big buckets: kBCap < records <= kBigCap, one kBigBlock-thread block each with kBigSlots-slot
// tables (load factor <= 3/4).  Typically a hot gene's records in one cell: taking them here
// instead of splitting them further on the umi bits saves whole partition levels.
constexpr int kBigBlock = 1024;  // measured: 1024 threads 0.38 ms, 512 0.49, 256 0.76 at config 2
constexpr int kBigBits = 12;
constexpr int kBigSlots = 1 << kBigBits;
constexpr int kBigCap = 3 * kBigSlots / 4 - 1;  // 3071
static_assert(kTileCap < kHTSlots, "a tile's keys always fit its tables");
static_assert(kTileCap < kHTCap, "a tile's keys always fit its tables");
static_assert(kBigCap < kBigSlots && kBigSlots <= 4096, "big-bucket keys fit its tables; 12-bit slots");
static_assert(kWin == 2 * kHBlock && (1 << kWinBits) == kWin, "window layout");
static_assert(kBCap < (1 << 11), "count field");
static_assert(kHTSlots <= 4096, "molecule slots are 12 bits in the fragment key");
static_assert(12 + kFragBits + 32 + 2 <= 64, "fragment key: molecule slot, (ref, strand), pos, 2 state bits");
static_assert(kWinBits + kMaxKeyBits + 2 <= 64, "molecule key: window offset, key bits, 2 state bits");

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
struct alignas(16) Pay {
  uint64_t w0, w1;
};
__device__ __forceinline__ uint64_t pay_w0(const Pay* p, size_t i) {  // w0 alone: an 8-byte load
  return reinterpret_cast<const uint64_t*>(p)[2 * i];
}
struct alignas(16) Work {  // one chunk of a segment: its records [beg, beg + n), n <= kChunk
  uint32_t seg, beg, n, pad;
};
__device__ __forceinline__ Work make_work(uint32_t id, uint32_t start, uint32_t cnt, uint32_t k) {
  const uint32_t b = start + k * (uint32_t)kChunk;
  const uint32_t r = start + cnt - b;
  return Work{id, b, r < (uint32_t)kChunk ? r : (uint32_t)kChunk, 0u};
}
// Device counters of one level (n_giant and n_big accumulate over levels).  Round 5: no record
// counters (n_rec, n_big_rec) -- every classify block with a pushed or big child added to them, and
// those same-line atomics cost level 1's classification 0.09 of its 0.25 ms; the kernels that used
// them only for their profiling item counts now report none.
struct BucketCtl {
  uint32_t n_seg, n_work;  // the next level's segments and work items
  uint32_t n_giant, err;  // err: a mapped ref id >= 2^kRefBits (set by build_keys)
  uint32_t n_big;  // big buckets
};

__device__ __forceinline__ uint64_t payload_w0(uint64_t key, int32_t ref, bool reverse, bool mapped, bool mito) {
  return (key << kKeyShift) | ((uint64_t)((uint32_t)ref & ((1u << kRefBits) - 1)) << 3) |
         ((uint64_t)(reverse ? 1 : 0) << 2) | (mapped ? kW0Mapped : 0ull) | (mito ? kW0Mito : 0ull);
}
// fragment identity (ref, strand) of a payload: kFragBits bits
__device__ __forceinline__ uint32_t payload_frag(uint64_t w0) {
  return (uint32_t)(w0 >> 2) & ((1u << kFragBits) - 1);
}

// ctr: the level's (n_seg, n_work) counters
__device__ __forceinline__ void push_segment(const Seg& sg, Seg* __restrict__ seg, Work* __restrict__ work,
                                             uint32_t* ctr) {
  const uint32_t id = atomicAdd(&ctr[0], 1u);
  seg[id] = sg;
  const uint32_t nw = (sg.cnt + kChunk - 1) / kChunk;
  const uint32_t w0 = atomicAdd(&ctr[1], nw);
  for (uint32_t k = 0; k < nw; k++) work[w0 + k] = make_work(id, sg.start, sg.cnt, k);
}

// level 0: small entities are terminal buckets, mid-sized ones big buckets; larger ones segments,
// counted in seg_ctr (n_seg, n_work)
__global__ void k_bucket_level0(const int64_t* __restrict__ ent_start, int64_t n_ent, int64_t n,
                                uint16_t* __restrict__ bdesc, uint32_t* __restrict__ bent, Seg* __restrict__ seg,
                                Work* __restrict__ work, Seg* __restrict__ bigs, BucketCtl* ctl,
                                uint32_t* __restrict__ seg_ctr) {
  const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (e >= n_ent) return;
  const int64_t s0 = ent_start[e];
  const int64_t s1 = e + 1 < n_ent ? ent_start[e + 1] : n;
  const uint32_t c = (uint32_t)(s1 - s0);
  if (c <= (uint32_t)kBCap) {
    bdesc[s0] = (uint16_t)c;
    bent[s0] = (uint32_t)e;
    return;
  }
  if (c <= (uint32_t)kBigCap) {
    bigs[atomicAdd(&ctl->n_big, 1u)] = Seg{(uint32_t)s0, c, (uint32_t)e, 0u};
    return;
  }
  push_segment(Seg{(uint32_t)s0, c, (uint32_t)e, 0u}, seg, work, seg_ctr);
}

__global__ void __launch_bounds__(kBlock) k_bucket_hist(const Pay* __restrict__ pin, const Seg* __restrict__ seg,
                                                        const Work* __restrict__ work, int shift, int bits,
                                                        uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[kWaves][kRadix];
  const int wid = threadIdx.x / kWave;
  for (int i = threadIdx.x; i < kWaves * kRadix; i += kBlock) (&h[0][0])[i] = 0;
  const Work wk = work[xcd_tile(blockIdx.x, gridDim.x)];  // the chunk's range rides in the work item:
  const uint32_t beg = wk.beg;                             // no dependent segment load before the keys
  const uint32_t end = wk.beg + wk.n;
  const uint64_t mask = (1ull << bits) - 1;
  __syncthreads();
  for (uint32_t p = beg + threadIdx.x; p < end; p += kBlock) atomicAdd(&h[wid][(pay_w0(pin, p) >> shift) & mask], 1u);
  __syncthreads();
  const int d = threadIdx.x;
  uint32_t tot = 0;
#pragma unroll
  for (int w = 0; w < kWaves; w++) tot += h[w][d];
  if (tot) atomicAdd(&hist[(size_t)wk.seg * kRadix + d], tot);
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

// One level's scatter: rank a chunk in LDS on the level digit (an LDS atomic per record: the
// order inside a child bucket is irrelevant to the hash tiles), reserve one output range per
// present digit with one atomic on the segment's cursor, and write each digit's records as a
// contiguous run (LDS-staged, coalesced).  `shift` addresses w0 (key' bits + kKeyShift).
// kSBlock threads (4 records each): the 36 KB of staging allow 4 blocks per CU, so 512-thread
// blocks keep twice the waves in flight of 256-thread ones.
constexpr int kSBlock = 512;
constexpr int kSItems = kChunk / kSBlock;
static_assert(kRadix <= kSBlock, "one thread per digit");
__global__ void __launch_bounds__(kSBlock) k_bucket_scatter(const Pay* __restrict__ pin, Pay* __restrict__ pout,
                                                            const Seg* __restrict__ seg, const Work* __restrict__ work,
                                                            int shift, int bits, uint32_t* __restrict__ cur) {
  __shared__ Pay s_pay[kChunk];
  __shared__ uint32_t s_cnt[kRadix];
  __shared__ uint32_t s_start[kRadix];
  __shared__ uint32_t s_gbase[kRadix];
  __shared__ uint64_t s_scan[kSBlock / kWave + 1];
  const int t = threadIdx.x;
  const Work wk = work[xcd_tile(blockIdx.x, gridDim.x)];
  const uint32_t beg = wk.beg;
  const int tile_n = (int)wk.n;
  const uint32_t mask = (1u << bits) - 1;
  if (t < kRadix) s_cnt[t] = 0;
  __syncthreads();
  Pay k[kSItems];
  uint32_t rk[kSItems];
#pragma unroll
  for (int j = 0; j < kSItems; j++) {
    const int q = j * kSBlock + t;
    if (q < tile_n) k[j] = pin[beg + q];
  }
#pragma unroll
  for (int j = 0; j < kSItems; j++) {
    const int q = j * kSBlock + t;
    if (q < tile_n) rk[j] = atomicAdd(&s_cnt[(uint32_t)(k[j].w0 >> shift) & mask], 1u);
  }
  __syncthreads();
  {
    const uint32_t c = t < kRadix ? s_cnt[t] : 0u;
    uint64_t tot;
    const uint32_t st = (uint32_t)block_exclusive_scan_n<kSBlock, uint64_t>((uint64_t)c, &tot, s_scan);
    if (t < kRadix) {
      s_start[t] = st;
      if (c) s_gbase[t] = atomicAdd(&cur[(size_t)wk.seg * kRadix + t], c);
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kSItems; j++) {
    const int q = j * kSBlock + t;
    if (q < tile_n) s_pay[s_start[(uint32_t)(k[j].w0 >> shift) & mask] + rk[j]] = k[j];
  }
  __syncthreads();
  for (int q = t; q < tile_n; q += kSBlock) {
    const Pay kk = s_pay[q];
    const uint32_t d = (uint32_t)(kk.w0 >> shift) & mask;
    pout[s_gbase[d] + (uint32_t)(q - (int)s_start[d])] = kk;
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

// One block per segment, one thread per child digit: the children's record ranges (an exclusive
// scan of the digit counts; the scatter's cursors) and their classification -- terminal
// bucket, big bucket, giant, or next-level segment.  The block's new segments and work items are reserved
// with one atomic each.
// by_ent (level 1 planned before the key pass, segment.h k_level1_plan): the counts are per entity,
// hist[entity][digit], and each is replaced by its child's start | kL1SegMark for the key pass;
// the grid is an upper bound and *n_seg_dev the number of segments.
constexpr uint32_t kL1SegMark = 0x80000000u;
__global__ void __launch_bounds__(kBlock) k_bucket_classify(const Seg* __restrict__ seg,
                                                            uint32_t* __restrict__ hist,
                                                            uint32_t* __restrict__ cur, int depth, int bits,
                                                            int K1, int KM, int KB, int parity, int by_ent,
                                                            uint16_t* __restrict__ bdesc, uint32_t* __restrict__ bent,
                                                            Seg* __restrict__ nseg, Work* __restrict__ nwork,
                                                            Seg* __restrict__ giants, Seg* __restrict__ bigs,
                                                            BucketCtl* ctl, const uint32_t* __restrict__ n_seg_dev) {
  __shared__ uint32_t s_c[kRadix];
  __shared__ uint64_t s_scan[kWaves + 1];
  __shared__ uint32_t s_base[2];
  if (n_seg_dev && blockIdx.x >= *n_seg_dev) return;  // block-uniform
  const int d = threadIdx.x;
  const size_t i = (size_t)blockIdx.x * kRadix + d;
  const Seg sg = seg[blockIdx.x];
  const size_t hi = by_ent ? (size_t)sg.ent * kRadix + d : i;
  const uint32_t c = hist[hi];
  s_c[d] = c;
  uint64_t tot_c;
  const uint32_t start = sg.start + (uint32_t)block_exclusive_scan<uint64_t>((uint64_t)c, &tot_c, s_scan);
  cur[i] = start;
  if (by_ent) hist[hi] = start | kL1SegMark;
  const int depth1 = depth + bits;
  uint32_t fl = 0;
  if (c) {
    fl = split_flags(K1, depth, depth1, d, sg.flags, s_c, BD_K1_NOHEAD, BD_K1_MULTI);
    fl |= split_flags(KM, depth, depth1, d, sg.flags, s_c, BD_MOL_NOHEAD, BD_MOL_MULTI);
  }
  const uint32_t par = parity ? BD_PARITY : 0u;
  const bool terminal = c && c <= (uint32_t)kBCap;
  const bool big = c > (uint32_t)kBCap && c <= (uint32_t)kBigCap;
  const bool giant = c > (uint32_t)kBigCap && depth1 >= KB;
  const bool push = c > (uint32_t)kBigCap && !giant;
  if (terminal) {
    bdesc[start] = (uint16_t)(c | fl | par);
    bent[start] = sg.ent;
  } else if (giant) {
    const uint32_t id = atomicAdd(&ctl->n_giant, 1u);
    giants[id] = Seg{start, c, sg.ent, fl | par};
  } else if (big) {
    bigs[atomicAdd(&ctl->n_big, 1u)] = Seg{start, c, sg.ent, fl | par};
  }
  const uint32_t nw = push ? (c + kChunk - 1) / kChunk : 0u;
  // new segments and work items numbered by one scan of (segments << 32 | work items)
  uint64_t tot_sw;
  const uint64_t sw = block_exclusive_scan<uint64_t>(((uint64_t)(push ? 1 : 0) << 32) | nw, &tot_sw, s_scan);
  const uint32_t so = (uint32_t)(sw >> 32), wo = (uint32_t)sw;
  const uint64_t tot_s = tot_sw >> 32, tot_w = tot_sw & 0xffffffffull;
  if (d == 0 && tot_s) {
    s_base[0] = atomicAdd(&ctl->n_seg, (uint32_t)tot_s);
    s_base[1] = atomicAdd(&ctl->n_work, (uint32_t)tot_w);
  }
  __syncthreads();
  if (push) {
    const uint32_t id = s_base[0] + so;
    nseg[id] = Seg{start, c, sg.ent, fl};
    for (uint32_t k = 0; k < nw; k++) nwork[s_base[1] + wo + k] = make_work(id, start, c, k);
  }
}

// ---- LDS hash tables: entries key << 2 | state, state bit 0 = present, bit 1 = seen twice ----
__device__ __forceinline__ uint32_t ht_home(unsigned long long key, int tb) {
  return (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> (64 - tb));
}
__device__ __forceinline__ uint32_t ht_home(unsigned int key, int tb) { return (key * 0x9E3779B1u) >> (32 - tb); }

// Insert `key` (low two bits zero) into a table of 2^tb slots.  Returns the key's slot; ev = 1
// for the record that inserted the key (its head), 2 for the first record that found it
// present, else 0.  The table has more slots than the block has records, so the probe ends.
// The probe loop has one exit test (slot claimed or key found) and the state update follows it:
// a loop with nested exits compiled to ~25 scalar exec-mask operations per probe (round 4).
template <typename E>
__device__ __forceinline__ int ht_state(E* T, uint32_t h, E old) {
  if (old == 0) return 1;
  return (!(old & 2) && !(atomicOr(&T[h], (E)2) & 2)) ? 2 : 0;
}
template <typename E>
__device__ __forceinline__ uint32_t ht_insert(E* T, E key, int& ev, int tb = kHTBits) {
  const uint32_t mask = (1u << tb) - 1;
  uint32_t h = ht_home(key, tb);
  E old;
  while (true) {
    old = atomicCAS(&T[h], (E)0, (E)(key | 1));
    if (old == 0 || (old & ~(E)3) == key) break;
    h = (h + 1) & mask;
  }
  ev = ht_state(T, h, old);
  return h;
}

// ht_insert for a table of kHTCap slots: the home slot by multiply-shift range reduction of the
// hashed key, probing with wrap-around at kHTCap.
__device__ __forceinline__ uint32_t ht_home_cap(unsigned long long key) {
  return (uint32_t)(((key * 0x9E3779B97F4A7C15ull) >> 32) * (unsigned long long)kHTCap >> 32);
}
__device__ __forceinline__ uint32_t ht_home_cap(unsigned int key) {
  return (uint32_t)(((unsigned long long)(key * 0x9E3779B1u) * (unsigned long long)kHTCap) >> 32);
}
template <typename E>
__device__ __forceinline__ uint32_t ht_insert_cap(E* T, E key, int& ev) {
  uint32_t h = ht_home_cap(key);
  E old;
  while (true) {
    old = atomicCAS(&T[h], (E)0, (E)(key | 1));
    if (old == 0 || (old & ~(E)3) == key) break;
    h = h + 1 == (uint32_t)kHTCap ? 0u : h + 1;
  }
  ev = ht_state(T, h, old);
  return h;
}

// kWideK1: k1 ids need more than kNarrowK1Bits bits (64-bit k1 table entries)
template <bool kCell, bool kGene, bool kWideK1>
__global__ void __launch_bounds__(kHBlock) k_hash_tile(const uint16_t* __restrict__ bdesc,
                                                       const uint32_t* __restrict__ bent,
                                                       const Pay* __restrict__ pay_a,
                                                       const Pay* __restrict__ pay_b, int64_t n, Bits b,
                                                       int64_t* __restrict__ partials,
                                                       uint16_t* __restrict__ dflags) {
  using K1E = typename std::conditional<kWideK1, unsigned long long, unsigned int>::type;
  __shared__ K1E s_k1[kHTCap];                  // (bucket, k1)
  __shared__ unsigned long long s_mol[kHTCap];  // (bucket, k1, k2)
  __shared__ unsigned long long s_frg[kHTCap];  // (molecule slot, ref, strand, pos)
  __shared__ uint64_t s_red[kHWaves];
  __shared__ uint64_t s_lastp;
  static_assert(kHTCap % 2 == 0 && (kHTCap * sizeof(K1E)) % 16 == 0, "tables cleared with 16-byte stores");
  const int t = threadIdx.x;
  const unsigned wb = xcd_tile(blockIdx.x, gridDim.x);
  const int64_t w0 = (int64_t)wb * kWin;
  const int win_n = (int)((n - w0) < kWin ? (n - w0) : kWin);
  // descriptors of window offsets 2t, 2t+1 and their entities (meaningful at bucket starts only,
  // but loaded unconditionally so that no load waits for another); tables cleared meanwhile
  const int p0 = 2 * t;
  uint16_t dsc[2];
  uint32_t ent[2];
#pragma unroll
  for (int i = 0; i < 2; i++) {
    const bool in = p0 + i < win_n;
    dsc[i] = in ? bdesc[w0 + p0 + i] : (uint16_t)0;
    ent[i] = in ? bent[w0 + p0 + i] : 0u;
  }
  {
    uint4* z = reinterpret_cast<uint4*>(s_mol);
    for (int i = t; i < kHTCap / 2; i += kHBlock) z[i] = make_uint4(0, 0, 0, 0);
    z = reinterpret_cast<uint4*>(s_frg);
    for (int i = t; i < kHTCap / 2; i += kHBlock) z[i] = make_uint4(0, 0, 0, 0);
    z = reinterpret_cast<uint4*>(s_k1);
    for (int i = t; i < (int)(kHTCap * sizeof(K1E) / 16); i += kHBlock) z[i] = make_uint4(0, 0, 0, 0);
  }
  // The bucket of window offset x is the last start at or before x: a max-scan of the packed
  // (start + 1, descriptor, entity) of the starts carries the bucket's descriptor and entity to
  // every position, so no LDS array of descriptors is needed.
  const auto pack = [](int x, uint16_t d, uint32_t e) -> uint64_t {
    return ((uint64_t)(x + 1) << 48) | ((uint64_t)d << 32) | e;
  };
  const uint64_t m0 = dsc[0] ? pack(p0, dsc[0], ent[0]) : 0ull;
  const uint64_t m1 = dsc[1] ? pack(p0 + 1, dsc[1], ent[1]) : m0;
  uint64_t ex;
  {  // exclusive max-scan over the block (markers grow with the position: max = the latest start)
    const int lane = t & (kWave - 1), wid = t / kWave;
    uint64_t x = m1;
    for (int off = 1; off < kWave; off <<= 1) {
      const uint64_t y = __shfl_up(x, off);
      if (lane >= off) x = y > x ? y : x;
    }
    if (lane == kWave - 1) s_red[wid] = x;
    __syncthreads();
    uint64_t carry = 0;
    for (int w = 0; w < wid; w++) carry = s_red[w] > carry ? s_red[w] : carry;
    uint64_t e1 = __shfl_up(x, 1);
    if (lane == 0) e1 = 0;
    ex = e1 > carry ? e1 : carry;
  }
  uint64_t inc[2];
  inc[0] = m0 > ex ? m0 : ex;
  inc[1] = m1 > inc[0] ? m1 : inc[0];
  if (t == kHBlock - 1) s_lastp = inc[1];
  __syncthreads();
  const uint64_t lastp = s_lastp;
  if (lastp == 0) return;  // block-uniform: no bucket starts in this window
  const int last = (int)(lastp >> 48) - 1;
  const int end_off = last + (int)((lastp >> 32) & BD_COUNT);  // the last bucket may run past the window

  const int KB = b.k1 + b.k2 + b.h;
  const uint64_t kmask = (1ull << KB) - 1;
  const int sh_mol = b.h, sh_k1 = b.k2 + b.h;
  const int mol_bits = b.k1 + b.k2;
  int32_t acc[kDistinct];
#pragma unroll
  for (int i = 0; i < kDistinct; i++) acc[i] = 0;
  int64_t cur_e = -1;
  const auto slot = [](int i) { return distinct_slot(i); };
  // items 0, 1: window offsets 2t, 2t+1; items 2, 3: overflow offsets kWin + 2t, kWin + 2t + 1
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const int q = (j < 2 ? 0 : kWin) + p0 + (j & 1);  // offset from w0
    const uint64_t bp = j < 2 ? inc[j] : lastp;        // the bucket's (start + 1, descriptor, entity)
    const int bs = (int)(bp >> 48) - 1;                 // the bucket's start offset = its ordinal
    const uint32_t bd = (uint32_t)(bp >> 32) & 0xffffu;
    // inside the bucket's extent (a giant's range has no descriptor and follows some bucket)
    const bool valid = j < 2 ? (bs >= 0 && q < win_n && q < bs + (int)(bd & BD_COUNT)) : (q < end_off);
    const int64_t e = valid ? (int64_t)(uint32_t)bp : cur_e;
    wave_flush<kDistinct>(acc, valid && e != cur_e && cur_e >= 0, cur_e, partials, slot);
    if (!valid) continue;
    cur_e = e;
    const Pay x = ((bd & BD_PARITY) ? pay_b : pay_a)[w0 + q];
    const uint64_t x0 = x.w0, x1 = x.w1;
    const uint64_t key = (x0 >> kKeyShift) & kmask;  // ids >= the dictionary sizes stay inside KB bits
    int ek = 0, em, ef = 0;
    const uint32_t ms =
        ht_insert_cap<unsigned long long>(s_mol, (((uint64_t)bs << mol_bits) | (key >> sh_mol)) << 2, em);
    // A record whose molecule already had two records (em == 0) cannot change the (bucket, k1)
    // events: that group's inserter and first finder are among the molecule's first two records.
    if (em != 0) ht_insert_cap<K1E>(s_k1, (K1E)((((uint64_t)bs << b.k1) | (key >> sh_k1)) << 2), ek);
    if (x0 & kW0Mapped) {
      const uint64_t fk = ((((uint64_t)ms << kFragBits) | payload_frag(x0)) << 32) | (uint32_t)x1;
      ht_insert_cap<unsigned long long>(s_frg, fk << 2, ef);
    }
    // split groups: only the first piece counts the head, and it also carries the multi event
    const bool k1_head = ek == 1 && !(bd & BD_K1_NOHEAD);
    const bool k1_multi = (bd & BD_K1_MULTI) ? k1_head : ek == 2;
    const bool mol_head = em == 1 && !(bd & BD_MOL_NOHEAD);
    const bool mol_second = (bd & BD_MOL_MULTI) ? mol_head : em == 2;
    acc[0] += mol_head;
    acc[1] += (int32_t)mol_head - (int32_t)mol_second;
    acc[2] += ef == 1;
    acc[3] += (int32_t)(ef == 1) - (int32_t)(ef == 2);
    acc[4] += k1_head;
    acc[5] += k1_multi;
    if constexpr (kCell) acc[6] += (k1_head && (x0 & kW0Mito)) ? 1 : 0;
    if constexpr (kGene) {
      const uint16_t f = (mol_head ? (DF_MOL_HEAD | DF_MOL_SINGLE) : 0) | (mol_second ? DF_MOL_SECOND : 0) |
                         (ef == 1 ? (DF_FRAG_FIRST | DF_FRAG_SINGLE) : 0) | (ef == 2 ? DF_FRAG_SECOND : 0) |
                         (k1_head ? DF_K1_HEAD : 0) | (k1_multi ? DF_K1_MULTI : 0);
      dflags[x1 >> 32] = f;
    }
  }
  wave_flush<kDistinct>(acc, cur_e >= 0, cur_e, partials, slot);
}

// One big bucket (kBCap < records <= kBigCap, bucket.h header) per block: the hash tile's
// per-record logic with one bucket per block and kBigSlots-slot tables.
template <bool kCell, bool kGene, bool kWideK1>
__global__ void __launch_bounds__(kBigBlock) k_big_bucket(const Seg* __restrict__ bigs,
                                                          const Pay* __restrict__ pay_a,
                                                          const Pay* __restrict__ pay_b, Bits b,
                                                          int64_t* __restrict__ partials,
                                                          uint16_t* __restrict__ dflags) {
  using K1E = typename std::conditional<kWideK1, unsigned long long, unsigned int>::type;
  __shared__ K1E s_k1[kBigSlots];
  __shared__ unsigned long long s_mol[kBigSlots];
  __shared__ unsigned long long s_frg[kBigSlots];  // 80 KB in all: 2 blocks per CU
  const int t = threadIdx.x;
  const Seg g = bigs[blockIdx.x];
  int tb = kHTBits;  // tables sized to the bucket: load factor <= 3/4
  while ((1u << tb) * 3u < 4u * g.cnt + 4u) tb++;
  const int slots = 1 << tb;
  {
    uint4* z = reinterpret_cast<uint4*>(s_mol);
    for (int i = t; i < slots / 2; i += kBigBlock) z[i] = make_uint4(0, 0, 0, 0);
    z = reinterpret_cast<uint4*>(s_frg);
    for (int i = t; i < slots / 2; i += kBigBlock) z[i] = make_uint4(0, 0, 0, 0);
    z = reinterpret_cast<uint4*>(s_k1);
    for (int i = t; i < (int)(slots * sizeof(K1E) / 16); i += kBigBlock) z[i] = make_uint4(0, 0, 0, 0);
  }
  __syncthreads();
  const uint32_t bd = g.flags;
  const Pay* P = (bd & BD_PARITY) ? pay_b : pay_a;
  const int KB = b.k1 + b.k2 + b.h;
  const uint64_t kmask = (1ull << KB) - 1;
  const int sh_mol = b.h, sh_k1 = b.k2 + b.h;
  int32_t acc[kDistinct];
#pragma unroll
  for (int i = 0; i < kDistinct; i++) acc[i] = 0;
  for (uint32_t p = t; p < g.cnt; p += kBigBlock) {
    const Pay x = P[g.start + p];
    const uint64_t x0 = x.w0, x1 = x.w1;
    const uint64_t key = (x0 >> kKeyShift) & kmask;
    int ek = 0, em, ef = 0;
    const uint32_t ms = ht_insert<unsigned long long>(s_mol, (key >> sh_mol) << 2, em, tb);
    if (em != 0) ht_insert<K1E>(s_k1, (K1E)((key >> sh_k1) << 2), ek, tb);  // as in k_hash_tile
    if (x0 & kW0Mapped) {
      const uint64_t fk = ((((uint64_t)ms << kFragBits) | payload_frag(x0)) << 32) | (uint32_t)x1;
      ht_insert<unsigned long long>(s_frg, fk << 2, ef, tb);
    }
    const bool k1_head = ek == 1 && !(bd & BD_K1_NOHEAD);
    const bool k1_multi = (bd & BD_K1_MULTI) ? k1_head : ek == 2;
    const bool mol_head = em == 1 && !(bd & BD_MOL_NOHEAD);
    const bool mol_second = (bd & BD_MOL_MULTI) ? mol_head : em == 2;
    acc[0] += mol_head;
    acc[1] += (int32_t)mol_head - (int32_t)mol_second;
    acc[2] += ef == 1;
    acc[3] += (int32_t)(ef == 1) - (int32_t)(ef == 2);
    acc[4] += k1_head;
    acc[5] += k1_multi;
    if constexpr (kCell) acc[6] += (k1_head && (x0 & kW0Mito)) ? 1 : 0;
    if constexpr (kGene) {
      const uint16_t f = (mol_head ? (DF_MOL_HEAD | DF_MOL_SINGLE) : 0) | (mol_second ? DF_MOL_SECOND : 0) |
                         (ef == 1 ? (DF_FRAG_FIRST | DF_FRAG_SINGLE) : 0) | (ef == 2 ? DF_FRAG_SECOND : 0) |
                         (k1_head ? DF_K1_HEAD : 0) | (k1_multi ? DF_K1_MULTI : 0);
      dflags[x1 >> 32] = f;
    }
  }
  // one entity per block: wave sums, then one row atomic per wave and slot (no LDS, which keeps
  // the block at 80 KB)
  const int lane = t & (kWave - 1);
  int32_t mine = 0;
#pragma unroll
  for (int i = 0; i < kDistinct; i++) {
    const int32_t tot = wave_sum_dpp(acc[i]);
    mine = lane == i ? tot : mine;
  }
  if (lane < kDistinct && mine)
    atomicAdd((unsigned long long*)&partials[(int64_t)g.ent * SCT_NP + distinct_slot(lane)],
              (unsigned long long)(int64_t)mine);
}

// A bucket whose whole key' is fixed and still holds > kBCap records: one piece of one
// molecule at one fragment hash.  One block; fragments resolved exactly by repeatedly taking
// the first unassigned mapped record as a representative.  `mark` is the other buffer's w1
// words over the same range (dead: the parent segment was scattered out of it).
template <bool kCell, bool kGene>
__global__ void __launch_bounds__(kBlock) k_bucket_giant(const Seg* __restrict__ giants, Pay* __restrict__ pay_a,
                                                         Pay* __restrict__ pay_b, int64_t* __restrict__ partials,
                                                         uint16_t* __restrict__ dflags) {
  __shared__ uint64_t s_red[kWaves];
  __shared__ uint32_t s_min[kWaves];
  const Seg g = giants[blockIdx.x];
  const bool pb = g.flags & BD_PARITY;
  const Pay* P = pb ? pay_b : pay_a;
  Pay* other = pb ? pay_a : pay_b;
  struct W0 {
    const Pay* p;
    __device__ uint64_t operator[](size_t i) const { return p[i].w0; }
  } w0{P};
  struct W1 {
    const Pay* p;
    __device__ uint64_t operator[](size_t i) const { return p[i].w1; }
  } w1{P};
  struct Mark {
    Pay* p;
    __device__ uint64_t& operator[](size_t i) const { return p[i].w1; }
  } mark{other};
  const int t = threadIdx.x;
  const int lane = t & (kWave - 1);
  const int wid = t / kWave;
  const bool k1_head = !(g.flags & BD_K1_NOHEAD);
  const bool mol_head = !(g.flags & BD_MOL_NOHEAD);
  for (uint32_t p = t; p < g.cnt; p += kBlock) {
    mark[g.start + p] = (w0[g.start + p] & kW0Mapped) ? 0ull : 1ull;
    if constexpr (kGene) {
      uint16_t f = 0;
      if (p == 0) f = (k1_head ? (DF_K1_HEAD | DF_K1_MULTI) : 0) | (mol_head ? DF_MOL_HEAD : 0);
      dflags[w1[g.start + p] >> 32] = f;
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
    const uint32_t fr = payload_frag(w0[g.start + rep]);
    const uint32_t fp = (uint32_t)w1[g.start + rep];
    uint64_t c = 0;
    for (uint32_t p = rep + t; p < g.cnt; p += kBlock) {
      if (mark[g.start + p]) continue;
      if (payload_frag(w0[g.start + p]) == fr && (uint32_t)w1[g.start + p] == fp) {
        mark[g.start + p] = 1ull;
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
    if (kGene && t == 0) dflags[w1[g.start + rep] >> 32] |= DF_FRAG_FIRST | (tot == 1 ? DF_FRAG_SINGLE : 0);
    __syncthreads();
  }
  if (t == 0) {
    int64_t* row = partials + (int64_t)g.ent * SCT_NP;
    const bool mito = w0[g.start] & kW0Mito;
    const int64_t add[kDistinct] = {mol_head ? 1 : 0, 0, n_frag, n_single, k1_head ? 1 : 0, k1_head ? 1 : 0,
                                    (kCell && k1_head && mito) ? 1 : 0};
    for (int i = 0; i < kDistinct; i++)
      if (add[i]) atomicAdd((unsigned long long*)&row[distinct_slot(i)], (unsigned long long)add[i]);
  }
}

}  // namespace sct
