// sct_engine.hip -- MI355X (gfx950) per-cell / per-gene metric engine: host pipeline + C-ABI.
//
// Replaces the per-record Python loop of the reference
// (GatherCellMetrics / GatherGeneMetrics.extract_metrics, gatherer.py:116-232,
// driving MetricAggregator.parse_molecule, aggregator.py:236-334, and
// finalize, aggregator.py:342-387, 463-490, 571-578):
//
//   segment.h   entity runs (bam.iter_tag_groups, bam.py:492-540) and packed
//               64-bit keys [run | k1 | k2 | fragment hash], bits trimmed to the
//               dictionary sizes (cell: k1 = gene, k2 = umi; gene: k1 = cell)
//   bucket.h    distinct counts: per-entity MSD bucket partition of the keys
//               [k1 | k2 | fragment hash] until every bucket fits a tile, then an
//               LDS sort + neighbour pass per tile (the default path)
//   radix.h     device-wide LSD radix sort of (key, record index) -- the path for
//               keys too wide for bucket.h (k1 + k2 > 40 bits)
//   reduce.h    one pass over the globally sorted keys: Counter results from key runs
//   gene.h      gene buckets -> per-gene partial rows (LDS bins)
//   finalize.h  partial rows -> output rows; sequential Welford float path
//   tagsort.h   TagSortBam orders on the device; countmat.h  CountMatrix (CSR)
//   comm.h      RCCL all-reduce of gene partials (replaces MergeGeneMetrics, merge.py:74-191)
//
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -shared ... -lrccl.
// -ffp-contract=off keeps every Welford operation separately rounded, as Python does.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <vector>

#include "comm.h"
#include "common.h"
#include "countmat.h"
#include "exchange.h"
#include "finalize.h"
#include "fixedpt.h"
#include "bucket.h"
#include "gene.h"
#include "radix.h"
#include "reduce.h"
#include "segment.h"
#include "tagsort.h"
#include "util.h"

using namespace sct;

namespace {

constexpr int64_t kEntHistMax = 1 << 18;  // entities whose first partition level is planned (k_level1_plan)

struct Layout {
  size_t tile_cnt, scalars, scan_sums, pay_a, pay_b, half, counts, offsets, ent_start, partials;
  size_t gcounts, gcursor, gtoff, gwork, dflags, gpay, seen, zero_mito, ent_hist, l1_toff, l1_tslot;
  size_t bdesc, bent, seg_a, seg_b, work_a, work_b, seg_hist, seg_cur, giants, bigs, wctl, worder, wx, total;
  int64_t num_tiles, num_chunks, max_ent, max_gene_work, max_seg, max_work, count_cap;
  int n_buckets;
  bool gene;
};

Layout layout_for(const sct_plan_t* plan) {
  Layout L;
  const int64_t n = plan->n_records > 0 ? plan->n_records : 0;
  const int64_t n1 = n > 0 ? n : 1;
  L.num_tiles = cdiv(n1, kTile);
  const int64_t m = (int64_t)kRadix * cdiv(n1, kSortTile);  // radix counts of the global-sort path
  L.num_chunks = cdiv(m, kScanChunk);
  L.count_cap = m;
  L.max_ent = plan->max_entities > 0 ? plan->max_entities : n1;
  L.gene = plan->mode == SCT_MODE_GENE_GROUPED || (plan->flags & SCT_PLAN_GENE_PARTIALS);
  L.n_buckets = (int)cdiv(plan->n_gene_ids > 0 ? plan->n_gene_ids : 1, kGenesPerBucket);
  L.max_gene_work = L.n_buckets + cdiv(n1, kGeneChunk) + 1;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    size_t o = off;
    off += align_up(bytes);
    return o;
  };
  // the prefix [0, scalars + 256) is all sct_count_entities touches
  L.tile_cnt = take(sizeof(uint64_t) * (size_t)(L.num_tiles + 1));
  L.scalars = take(256);
  L.scan_sums = take(sizeof(uint64_t) * (size_t)(L.num_chunks + 1));
  // the bucket path's 16-byte payloads (Pay), ping-pong A / B; the global-sort path splits each
  // into its keys (u64) and values (u32): A = [keys a | values a], B = [keys b | values b]
  L.half = align_up(sizeof(uint64_t) * (size_t)n1);
  L.pay_a = take(2 * L.half);
  L.pay_b = take(2 * L.half);
  L.counts = take(sizeof(uint32_t) * (size_t)m);
  L.offsets = take(sizeof(uint32_t) * (size_t)m);
  L.ent_start = take(sizeof(int64_t) * (size_t)(L.max_ent + 1));
  L.partials = take(sizeof(int64_t) * SCT_NP * (size_t)L.max_ent);
  L.gcounts = take(L.gene ? sizeof(uint32_t) * (size_t)L.n_buckets : 0);  // records per gene bucket
  L.gcursor = take(L.gene ? sizeof(uint32_t) * (size_t)L.n_buckets : 0);
  L.gtoff = take(L.gene ? sizeof(uint32_t) * (size_t)L.n_buckets * (size_t)cdiv(n1, kEmitTile) : 0);
  L.gwork = take(L.gene ? sizeof(int64_t) * 3 * (size_t)L.max_gene_work : 0);
  L.dflags = take(L.gene ? sizeof(uint16_t) * (size_t)n1 : 0);
  L.gpay = take(L.gene ? sizeof(GenePayload) * (size_t)n1 : 0);
  L.seen = take(L.gene ? sizeof(uint32_t) * (size_t)(plan->n_cell_ids > 0 ? plan->n_cell_ids : 1) : 0);
  L.zero_mito = take(L.gene ? (size_t)(plan->n_gene_ids > 0 ? plan->n_gene_ids : 1) : 0);
  // the planned first partition level (segment.h k_level1_plan): digit counts per entity (1 KB each;
  // larger plans run level 1 as the other levels), each key-pass tile's offsets and slots
  const bool l1 = L.max_ent <= kEntHistMax;
  L.ent_hist = take(l1 ? sizeof(uint32_t) * kRadix * (size_t)L.max_ent : 0);
  L.l1_toff = take(l1 ? sizeof(uint32_t) * kL1Slots * kRadix * (size_t)cdiv(n1, kKTile) : 0);
  L.l1_tslot = take(l1 ? sizeof(uint2) * (size_t)cdiv(n1, kKTile) : 0);
  // bucket.h: segments have > kBCap records and are disjoint within a level (and giants overall)
  L.max_seg = n1 / (kBCap + 1) + 2;
  L.max_work = n1 / kChunk + L.max_seg + 2;
  L.bdesc = take(sizeof(uint16_t) * (size_t)n1);
  L.bent = take(sizeof(uint32_t) * (size_t)n1);
  L.seg_a = take(sizeof(Seg) * (size_t)L.max_seg);
  L.seg_b = take(sizeof(Seg) * (size_t)L.max_seg);
  L.work_a = take(sizeof(Work) * (size_t)L.max_work);
  L.work_b = take(sizeof(Work) * (size_t)L.max_work);
  L.seg_hist = take(sizeof(uint32_t) * kRadix * (size_t)L.max_seg);
  L.seg_cur = take(sizeof(uint32_t) * kRadix * (size_t)L.max_seg);
  L.giants = take(sizeof(Seg) * (size_t)L.max_seg);
  L.bigs = take(sizeof(Seg) * (size_t)L.max_seg);
  const bool welford = plan->float_mode == SCT_FLOAT_WELFORD;
  L.wctl = take(welford ? 2 * sizeof(WelfordCtl) : 0);  // the main queue and the head group's
  L.worder = take(welford ? sizeof(uint32_t) * (size_t)L.max_ent : 0);
  L.wx = take(welford ? sizeof(double) * 4 * (size_t)(n1 + kWfPad) : 0);  // every record's stream values
  L.total = off;
  return L;
}

size_t count_bytes(const Layout& L) { return L.scalars + 256; }

BucketCtl* bucket_ctl(void* ws, const Layout& L) {
  return reinterpret_cast<BucketCtl*>(at<uint64_t>(ws, L.scalars) + 8);
}
// level 0's (n_seg, n_work) when the first partition level is planned before the key pass
uint32_t* level0_ctr(void* ws, const Layout& L) { return reinterpret_cast<uint32_t*>(at<uint64_t>(ws, L.scalars) + 12); }
static_assert(sizeof(BucketCtl) <= 32, "BucketCtl at scalars + 64 B ends before the level-0 counters at + 96 B");

int check_plan(const sct_plan_t* plan, const sct_records_t* rec) {
  if (!plan) return fail(SCT_EINVAL, "plan is NULL");
  if (plan->mode < SCT_MODE_CELL || plan->mode > SCT_MODE_GENE_GROUPED)
    return fail(SCT_EINVAL, "unknown mode %d", plan->mode);
  if (plan->float_mode != SCT_FLOAT_EXACT_SUM && plan->float_mode != SCT_FLOAT_WELFORD)
    return fail(SCT_EINVAL, "unknown float_mode %d", plan->float_mode);
  if (plan->float_mode == SCT_FLOAT_WELFORD && plan->mode == SCT_MODE_GENE_GROUPED)
    return fail(SCT_EINVAL, "SCT_FLOAT_WELFORD needs a RUN mode (record order defines Welford order)");
  if ((plan->flags & SCT_PLAN_GENE_PARTIALS) && plan->mode != SCT_MODE_CELL)
    return fail(SCT_EINVAL, "SCT_PLAN_GENE_PARTIALS needs SCT_MODE_CELL");
  if (plan->n_records < 0 || plan->n_records > (int64_t)0x7FFFFFFF)
    return fail(SCT_EINVAL, "n_records %lld out of range [0, 2^31)", (long long)plan->n_records);
  if ((plan->mode == SCT_MODE_GENE_GROUPED || (plan->flags & SCT_PLAN_GENE_PARTIALS)) &&
      plan->float_mode != SCT_FLOAT_EXACT_SUM)
    return fail(SCT_EINVAL, "grouped gene partials need SCT_FLOAT_EXACT_SUM");
  if (plan->n_cell_ids <= 0 || plan->n_gene_ids <= 0 || plan->n_umi_ids <= 0)
    return fail(SCT_EINVAL, "dictionary sizes must be positive");
  if (cdiv(plan->n_gene_ids, kGenesPerBucket) > kMaxGeneBuckets)
    return fail(SCT_EINVAL, "n_gene_ids %d exceeds %d", plan->n_gene_ids, kGenesPerBucket * kMaxGeneBuckets);
  if (rec) {
    if (rec->n != plan->n_records) return fail(SCT_EINVAL, "records.n != plan.n_records");
    if (rec->n > 0 && (!rec->cell || !rec->umi || !rec->gene || !rec->ref || !rec->pos || !rec->gq_sum ||
                       !rec->gq_len || !rec->gq_gt30 || !rec->bits || !rec->xf || !rec->cy_gt30 ||
                       !rec->cy_len || !rec->uy_gt30 || !rec->uy_len))
      return fail(SCT_EINVAL, "a record column pointer is NULL");
  }
  return SCT_OK;
}

// heads + scan of the entity column; with `dup_check`, also flags cell ids seen in two runs.
// Copies (n_entities, dup flag) to the host and synchronizes.
// pre: a fill queued behind the count's copy (round 6: it runs while the host waits for the count)
int count_runs(const int32_t* ent, int64_t n, void* ws, const Layout& L, bool dup_check, int32_t n_ids,
               int64_t* n_ent, bool* dup, hipStream_t s, FillBatch* pre = nullptr) {
  const int64_t tiles = cdiv(n, kTile);
  uint64_t* tc = at<uint64_t>(ws, L.tile_cnt);
  uint64_t* sc = at<uint64_t>(ws, L.scalars);
  uint32_t* seen = nullptr;
  FillBatch fb;
  if (dup_check) {
    seen = at<uint32_t>(ws, L.seen);
    fb.add(seen, sizeof(uint32_t) * (size_t)n_ids);
  }
  fb.add(sc, 2 * sizeof(uint64_t));
  if (int rc = launch_fills(fb, s)) return rc;
  if (((uintptr_t)ent & 15) == 0) {
    LAUNCH_N("heads", n, k_heads4, dim3((unsigned)tiles), dim3(kBlock), s, ent, n, tc, seen, (uint32_t)n_ids, sc + 1);
  } else {
    LAUNCH_N("heads", n, k_heads, dim3((unsigned)tiles), dim3(kBlock), s, ent, n, tc, seen, (uint32_t)n_ids, sc + 1);
  }
  LAUNCH("scan", k_scan_wide, dim3(1), dim3(kScanWide), s, tc, tiles, sc);
  uint64_t host[2] = {0, 0};
  if (pre) {
    if (int rb = readback_start(sc, sizeof(host), s)) return rb;
    if (int rc = launch_fills(*pre, s)) return rc;
    if (int rb = readback_finish(host, sizeof(host))) return rb;
  } else {
    if (int rb = readback(host, sc, sizeof(host), s)) return rb;
  }
  *n_ent = (int64_t)host[0];
  if (dup) *dup = host[1] & 1;
  if (host[1] & 2) return fail(SCT_EINVAL, "an entity id lies outside [0, %d)", n_ids);
  return SCT_OK;
}

template <bool kWideK1>
int launch_hash_tile(bool cell, bool gene, dim3 grid, hipStream_t s, const uint16_t* bdesc, const uint32_t* bent,
                     const Pay* pa, const Pay* pb, int64_t n,
                     const Bits& b, int64_t* partials, uint16_t* dflags) {
  if (cell && gene) {
    LAUNCH_N("hash_tile", n, (k_hash_tile<true, true, kWideK1>), grid, dim3(kHBlock), s, bdesc, bent, pa, pb, n,
           b, partials, dflags);
  } else if (cell) {
    LAUNCH_N("hash_tile", n, (k_hash_tile<true, false, kWideK1>), grid, dim3(kHBlock), s, bdesc, bent, pa, pb, n,
           b, partials, dflags);
  } else {
    LAUNCH_N("hash_tile", n, (k_hash_tile<false, false, kWideK1>), grid, dim3(kHBlock), s, bdesc, bent, pa, pb,
           n, b, partials, dflags);
  }
  return SCT_OK;
}

// The first partition level planned before the key pass (segment.h k_level1_plan): run ids and
// per-entity digit counts, level 0, then level 1's classification with a grid sized for the most
// segments there can be (the device count bounds it): l1.hist then holds every segment child's start.
// No host wait.
// (its buffers -- bdesc, the level-0 counters, l1.hist -- are zeroed by the caller: level1_fills)
void level1_fills(const Layout& L, void* ws, int64_t n, int64_t n_ent, const L1Plan& l1, FillBatch& fb,
                  bool bdesc_done) {
  if (!bdesc_done) fb.add(at<uint16_t>(ws, L.bdesc), sizeof(uint16_t) * (size_t)n);
  fb.add(level0_ctr(ws, L), 3 * sizeof(uint32_t));
  fb.add(l1.hist, sizeof(uint32_t) * kRadix * (size_t)n_ent);
}

int bucket_level1_plan(const Layout& L, void* ws, const KeyCols& kc, int64_t n, int64_t n_ent, const Bits& b,
                       int64_t* ent_start, const L1Plan& l1, hipStream_t s) {
  uint16_t* bdesc = at<uint16_t>(ws, L.bdesc);
  uint32_t* bent = at<uint32_t>(ws, L.bent);
  BucketCtl* ctl = bucket_ctl(ws, L);
  uint32_t* ctr0 = level0_ctr(ws, L);
  const int KB = b.k1 + b.k2 + b.h;
  LAUNCH_N("level1_plan", n, k_level1_plan, dim3((unsigned)cdiv(n, kKTile)), dim3(kBlock), s, kc.ent, kc.k1, kc.n_k1, n,
         (const uint64_t*)at<uint64_t>(ws, L.tile_cnt), b, b.k1 - kRadixBits, ent_start, l1);
  LAUNCH("bucket_level0", k_bucket_level0, dim3((unsigned)cdiv(n_ent, kBlock)), dim3(kBlock), s, ent_start, n_ent, n,
         bdesc, bent, at<Seg>(ws, L.seg_a), at<Work>(ws, L.work_a), at<Seg>(ws, L.bigs), ctl, ctr0);
  const int64_t max_seg = n_ent < n / (kBigCap + 1) + 1 ? n_ent : n / (kBigCap + 1) + 1;
  if (max_seg > L.max_seg) return fail(SCT_ENOMEM, "level 1: %lld segments exceed the workspace", (long long)max_seg);
  LAUNCH("bucket_classify", k_bucket_classify, dim3((unsigned)max_seg), dim3(kBlock), s,
         (const Seg*)at<Seg>(ws, L.seg_a), l1.hist, at<uint32_t>(ws, L.seg_cur), 0, kRadixBits, b.k1, b.k1 + b.k2, KB,
         1, 1, bdesc, bent, at<Seg>(ws, L.seg_b), at<Work>(ws, L.work_b), at<Seg>(ws, L.giants), at<Seg>(ws, L.bigs),
         ctl, (const uint32_t*)ctr0);
  return SCT_OK;
}

// One stream of the device's side-stream pool (below) for work beside the caller's stream (round 6):
// from_caller() makes it wait for the work queued on the caller's stream so far, to_caller() the
// reverse; use() hands out the stream for a launch.
hipError_t side_streams(int dev, hipStream_t* s2, hipStream_t* s3, bool* alone);
void side_streams_release(int dev, hipStream_t s2, hipStream_t s3);
struct SideStream {
  int dev = -1;
  hipStream_t s = nullptr, s_pair = nullptr;
  std::vector<hipEvent_t> evs;
  bool synced = true;  // the caller's stream waits for everything queued here so far
  bool is_open() const { return s != nullptr; }
  hipError_t open(hipStream_t caller) {
    if (s) return from_caller(caller);
    int prev = 0;
    hipError_t e = hipStreamGetDevice(caller, &dev);
    if (e == hipSuccess) e = hipGetDevice(&prev);
    if (e != hipSuccess) return e;
    if (prev != dev && (e = hipSetDevice(dev)) != hipSuccess) return e;
    bool alone = true;
    e = side_streams(dev, &s, &s_pair, &alone);
    if (e != hipSuccess) s = nullptr;
    if (prev != dev) (void)hipSetDevice(prev);
    return e == hipSuccess ? from_caller(caller) : e;
  }
  hipStream_t use() {
    synced = false;
    return s;
  }
  hipError_t event(hipEvent_t* ev) {
    hipError_t e = hipEventCreateWithFlags(ev, hipEventDisableTiming);
    if (e == hipSuccess) evs.push_back(*ev);
    return e;
  }
  hipError_t from_caller(hipStream_t caller) {
    hipEvent_t ev = nullptr;
    hipError_t e = event(&ev);
    if (e == hipSuccess) e = hipEventRecord(ev, caller);
    if (e == hipSuccess) e = hipStreamWaitEvent(s, ev, 0);
    return e;
  }
  hipError_t to_caller(hipStream_t caller) {
    hipEvent_t ev = nullptr;
    hipError_t e = event(&ev);
    if (e == hipSuccess) e = hipEventRecord(ev, s);
    if (e == hipSuccess) e = hipStreamWaitEvent(caller, ev, 0);
    if (e == hipSuccess) synced = true;
    return e;
  }
  ~SideStream() {
    // an early return (an error, or the global-sort redo that reuses the workspace): nothing may
    // still write into the workspace once the call is left
    if (s && !synced) (void)hipStreamSynchronize(s);
    for (hipEvent_t ev : evs) (void)hipEventDestroy(ev);
    if (s) side_streams_release(dev, s, s_pair);
  }
};

// bucket.h driver: level 0 classification, MSD levels until no segment exceeds kBCap, then
// the hash-tile pass (+ giants).  One host wait per level to size the next level's launches,
// for a copy queued right after the classification: the level's scatter runs meanwhile.
// planned: level 0 and level 1 ran before the key pass (bucket_level1_plan), and the key pass wrote
// the level-1 children: the loop starts at level 2.
// Returns 1 (not an error code) when build_keys saw a mapped ref id the payload cannot hold:
// the caller then reruns on the global-sort path.
int bucket_distinct(const Layout& L, void* ws, int64_t n, int64_t n_ent, const int64_t* ent_start,
                    const uint8_t* mito, const Bits& b, bool cell, bool gene, int64_t* partials, uint16_t* dflags,
                    bool planned, hipStream_t s, SideStream& side) {
  if (n == 0) return SCT_OK;
  Pay* pa = at<Pay>(ws, L.pay_a);
  Pay* pb = at<Pay>(ws, L.pay_b);
  uint16_t* bdesc = at<uint16_t>(ws, L.bdesc);
  uint32_t* bent = at<uint32_t>(ws, L.bent);
  Seg* seg[2] = {at<Seg>(ws, L.seg_a), at<Seg>(ws, L.seg_b)};
  Work* work[2] = {at<Work>(ws, L.work_a), at<Work>(ws, L.work_b)};
  uint32_t* hist = at<uint32_t>(ws, L.seg_hist);
  uint32_t* cur = at<uint32_t>(ws, L.seg_cur);
  Seg* giants = at<Seg>(ws, L.giants);
  BucketCtl* ctl = bucket_ctl(ws, L);
  const int KB = b.k1 + b.k2 + b.h;
  Seg* bigs = at<Seg>(ws, L.bigs);
  int depth = 0, level = 1, c = 0;
  if (planned) {
    depth = KB < kRadixBits ? KB : kRadixBits;
    level = 2;
    c = 1;
  } else {
    HIPCHK(hipMemsetAsync(bdesc, 0, sizeof(uint16_t) * (size_t)n, s));
    HIPCHK(hipMemsetAsync(ctl, 0, offsetof(BucketCtl, err), s));  // keeps ctl->err from build_keys
    HIPCHK(hipMemsetAsync(&ctl->n_big, 0, sizeof(uint32_t), s));
    LAUNCH("bucket_level0", k_bucket_level0, dim3((unsigned)cdiv(n_ent, kBlock)), dim3(kBlock), s, ent_start, n_ent,
           n, bdesc, bent, seg[0], work[0], bigs, ctl, &ctl->n_seg);
  }
  BucketCtl h{};
  // planned: the level-1 counts were read back early (pipeline: queued before the key pass), so the
  // host sizes level 2 while the key pass still runs; the key pass's error flag is read with the next
  // level's counts (kernels before that stay in bounds: ids are clamped, ref ids masked)
  bool err_pending = false;
  if (planned) {
    if (int rb = readback_finish(&h, sizeof(h))) return rb;
    err_pending = true;
  }
  if (!planned || h.n_seg == 0) {
    if (int rb = readback(&h, ctl, sizeof(h), s)) return rb;
    err_pending = false;
  }
  const auto err_check = [&]() -> int {
    if (h.err & 2) return fail(SCT_EINVAL, "a gene / cell / umi id lies outside its dictionary size");
    return h.err ? 1 : SCT_OK;
  };
  if (!err_pending)
    if (int e = err_check()) return e;
  // Round 6: the big buckets of levels 0 and 1 (their records are final once the key pass has run)
  // start on a side stream right away, beside levels >= 2, whose small partition kernels leave most
  // CUs idle; the caller's stream waits for them after the hash-tile launch.  Big buckets, level
  // segments and terminal buckets are disjoint record ranges, and the partial rows are summed
  // with atomics, so the order between the streams does not matter.
  const auto launch_big = [&](uint32_t cnt, const Seg* bg, hipStream_t st) -> int {
    const dim3 bgrid(cnt);
    const bool wide = b.k1 > kNarrowK1Bits;
#define SCT_BIG(C, G, W) \
  LAUNCH("big_bucket", (k_big_bucket<C, G, W>), bgrid, dim3(kBigBlock), st, bg, pa, pb, b, partials, dflags)
    if (cell && gene) {
      if (wide) { SCT_BIG(true, true, true); } else { SCT_BIG(true, true, false); }
    } else if (cell) {
      if (wide) { SCT_BIG(true, false, true); } else { SCT_BIG(true, false, false); }
    } else {
      if (wide) { SCT_BIG(false, false, true); } else { SCT_BIG(false, false, false); }
    }
#undef SCT_BIG
    return SCT_OK;
  };
  const char* no_early = getenv("SCT_NO_EARLY_BIG");
  const bool side_big = side.is_open() && !(no_early && no_early[0] == '1');
  const bool early_big = side_big && h.n_big > 0 && h.n_seg > 0;
  const char* no_late = getenv("SCT_NO_LEVEL_BIG");
  uint32_t big_done = 0;
  if (early_big) {
    if (int r = launch_big(h.n_big, bigs, side.use())) return r;
    big_done = h.n_big;
  }
  while (h.n_seg > 0) {
    if ((int64_t)h.n_seg > L.max_seg || (int64_t)h.n_work > L.max_work)
      return fail(SCT_ENOMEM, "bucket level %d: %u segments / %u work items exceed the workspace", level, h.n_seg,
                  h.n_work);
    const int bits = KB - depth < kRadixBits ? KB - depth : kRadixBits;
    const int shift = KB - depth - bits + kKeyShift;
    const int src = (level - 1) & 1;
    const Pay* pin = src ? pb : pa;
    Pay* pout = src ? pa : pb;
    HIPCHK(hipMemsetAsync(hist, 0, sizeof(uint32_t) * kRadix * (size_t)h.n_seg, s));
    LAUNCH("bucket_hist", k_bucket_hist, dim3(h.n_work), dim3(kBlock), s, pin, (const Seg*)seg[c],
           (const Work*)work[c], shift, bits, hist);
    HIPCHK(hipMemsetAsync(ctl, 0, 2 * sizeof(uint32_t), s));  // next level's n_seg, n_work
    LAUNCH("bucket_classify", k_bucket_classify, dim3(h.n_seg), dim3(kBlock), s, (const Seg*)seg[c], hist, cur, depth,
           bits, b.k1, b.k1 + b.k2, KB, level & 1, 0, bdesc, bent, seg[c ^ 1], work[c ^ 1], giants, bigs, ctl,
           (const uint32_t*)nullptr);
    // the next level's counts are final after classify: read them while the scatter runs
    if (int rb = readback_start(ctl, sizeof(h), s)) return rb;
    const uint32_t n_work = h.n_work;
    LAUNCH("bucket_scatter", k_bucket_scatter, dim3(n_work), dim3(kSBlock), s, pin, pout,
           (const Seg*)seg[c], (const Work*)work[c], shift, bits, cur);
    if (int rb = readback_finish(&h, sizeof(h))) return rb;
    if (err_pending) {
      err_pending = false;
      if (int e = err_check()) return e;
    }
    // this level's big buckets (written by its scatter) join the side stream when another level follows
    if (side_big && h.n_seg > 0 && h.n_big > big_done && !(no_late && no_late[0] == '1')) {
      HIPCHK(side.from_caller(s));
      if (int r = launch_big(h.n_big - big_done, bigs + big_done, side.use())) return r;
      big_done = h.n_big;
    }
    c ^= 1;
    depth += bits;
    level++;
  }
  const dim3 tgrid((unsigned)cdiv(n, kWin));
  // the early big buckets finish before the hash tiles start (SCT_BIG_BESIDE_HASH=1: they may run into
  // them; the hash tiles' 40 KB blocks then hold every CU's LDS and the big buckets' 80 KB blocks wait)
  const char* beside = getenv("SCT_BIG_BESIDE_HASH");
  const bool join_first = big_done > 0 && !(beside && beside[0] == '1');
  if (join_first) HIPCHK(side.to_caller(s));
  int rc;
  if (b.k1 > kNarrowK1Bits) {
    rc = launch_hash_tile<true>(cell, gene, tgrid, s, bdesc, bent, pa, pb, n, b, partials, dflags);
  } else {
    rc = launch_hash_tile<false>(cell, gene, tgrid, s, bdesc, bent, pa, pb, n, b, partials, dflags);
  }
  if (rc) return rc;
  // (round 4: the big buckets on a side stream beside the hash tiles measured the same step time,
  // 5.26 ms either way, profiles/r04/e_l1fast_gbam_dicts/var/); round 6: those of levels 0-1 already
  // run beside levels >= 2 (above), so only the later levels' big buckets are launched here
  if (big_done > 0 && !join_first) HIPCHK(side.to_caller(s));
  if (h.n_big > big_done) {
    rc = launch_big(h.n_big - big_done, bigs + big_done, s);
    if (rc) return rc;
  }
  if (h.n_giant > 0) {
    const dim3 ggrid(h.n_giant);
    if (cell && gene) {
      LAUNCH("bucket_giant", (k_bucket_giant<true, true>), ggrid, dim3(kBlock), s, (const Seg*)giants, pa, pb,
             partials, dflags);
    } else if (cell) {
      LAUNCH("bucket_giant", (k_bucket_giant<true, false>), ggrid, dim3(kBlock), s, (const Seg*)giants, pa, pb,
             partials, dflags);
    } else {
      LAUNCH("bucket_giant", (k_bucket_giant<false, false>), ggrid, dim3(kBlock), s, (const Seg*)giants, pa, pb,
             partials, dflags);
    }
  }
  return SCT_OK;
}

// The RUN-mode pipeline (entity = runs of the cell column, or of the gene column in gene
// mode; GROUPED runs the cell view).  Writes partial rows into the workspace, output rows
// if out_i / out_f are set, and grouped gene partials (cell view) if gene_partials is set.
template <bool kBucket, bool kStreams>
int launch_build_keys(bool cell, bool gene, dim3 grid, hipStream_t s, const KeyCols& kc, const RecCols& rc2,
                      const uint8_t* mito, int64_t n, const uint64_t* toff, const Bits& b, uint64_t* keys,
                      void* vals, int64_t* ent_start, int64_t* partials, uint32_t* gcounts, int n_buckets,
                      uint32_t* err, uint32_t* gwide, uint32_t* gtoff, const L1Plan& l1) {
  if (cell && gene) {
    LAUNCH_SHM_N("build_keys", n, (k_build_keys_run<true, true, kBucket, kStreams>), grid, dim3(kBlock),
               sizeof(uint32_t) * (size_t)n_buckets, s, kc, rc2, mito, n, toff, b, keys, vals, ent_start, partials,
               gcounts, n_buckets, err, gwide, gtoff, l1);
  } else if (cell) {
    LAUNCH_N("build_keys", n, (k_build_keys_run<true, false, kBucket, kStreams>), grid, dim3(kBlock), s, kc, rc2, mito, n,
           toff, b, keys, vals, ent_start, partials, gcounts, n_buckets, err, gwide, gtoff, l1);
  } else {
    LAUNCH_N("build_keys", n, (k_build_keys_run<false, false, kBucket, kStreams>), grid, dim3(kBlock), s, kc, rc2, mito,
           n, toff, b, keys, vals, ent_start, partials, gcounts, n_buckets, err, gwide, gtoff, l1);
  }
  return SCT_OK;
}

// Sequential Welford (SCT_FLOAT_WELFORD): big entities one wave each (largest first), small ones a
// lane each.  It needs only the entity starts, the input columns and its own workspace, and writes
// only the mean / variance slots of the output rows (k_finalize writes the others), so it runs on a
// side stream from the moment the entity starts exist, beside the key pass' successors (bucket
// partition, hash tiles) on the caller's stream.
// The side streams come from a per-device pool of (s2, s3) pairs created once and reused (round 4:
// creating them per call cost ~0.6 ms of host time before the first Welford launch).  A call holds
// its pair until it returns, so concurrent pipelines on one device get pairs of their own (round 5:
// a shared pair queued one pipeline's head kernel behind another's, and the start gate then held
// the second pipeline's key pass for its whole time-out).
constexpr int kMaxSideDevices = 64;
struct SidePool {
  std::mutex mu;
  std::vector<std::pair<hipStream_t, hipStream_t>> free[kMaxSideDevices];
  int in_use[kMaxSideDevices] = {};  // pairs held by running calls, per device
};
SidePool& side_pool() {
  static SidePool p;
  return p;
}
// *alone: no other call on this device holds a pair (so no other pipeline's Welford kernels can
// share a hardware queue with this one's)
hipError_t side_streams(int dev, hipStream_t* s2, hipStream_t* s3, bool* alone) {  // (`dev` is current)
  if (dev < 0 || dev >= kMaxSideDevices) return hipErrorInvalidDevice;
  SidePool& p = side_pool();
  {
    std::lock_guard<std::mutex> g(p.mu);
    *alone = p.in_use[dev] == 0;
    if (!p.free[dev].empty()) {
      *s2 = p.free[dev].back().first;
      *s3 = p.free[dev].back().second;
      p.free[dev].pop_back();
      p.in_use[dev]++;
      return hipSuccess;
    }
  }
  hipStream_t a = nullptr, b = nullptr;
  hipError_t e = hipStreamCreateWithFlags(&a, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&b, hipStreamNonBlocking);
  if (e != hipSuccess) {
    if (a) (void)hipStreamDestroy(a);
    return e;
  }
  *s2 = a;
  *s3 = b;
  std::lock_guard<std::mutex> g(p.mu);
  p.in_use[dev]++;
  return hipSuccess;
}
void side_streams_release(int dev, hipStream_t s2, hipStream_t s3) {
  SidePool& p = side_pool();
  std::lock_guard<std::mutex> g(p.mu);
  p.free[dev].emplace_back(s2, s3);
  p.in_use[dev]--;
}
struct WelfordSide {
  int dev = -1;
  hipStream_t s2 = nullptr, s3 = nullptr;
  hipEvent_t fork = nullptr, join = nullptr, fork3 = nullptr, join3 = nullptr;
  ~WelfordSide() {  // the caller's stream waits on `join` and `join3` before anything after the pipeline
    if (fork) (void)hipEventDestroy(fork);
    if (join) (void)hipEventDestroy(join);
    if (fork3) (void)hipEventDestroy(fork3);
    if (join3) (void)hipEventDestroy(join3);
    if (s2) side_streams_release(dev, s2, s3);  // (work still queued on them stays in order)
  }
};

int welford_stage(const Layout& L, void* ws, bool cell, int64_t n, int64_t n_ent, const RecCols& rc2,
                  const int64_t* ent_start, double* out_f, hipStream_t s, WelfordSide& wf) {
  // the side stream lives on the caller's stream's device (the calling thread's current device
  // may be another one)
  int dev = 0, prev = 0;
  HIPCHK(hipStreamGetDevice(s, &dev));
  HIPCHK(hipGetDevice(&prev));
  if (prev != dev) HIPCHK(hipSetDevice(dev));
  bool alone = true;
  hipError_t ce = side_streams(dev, &wf.s2, &wf.s3, &alone);
  if (ce == hipSuccess) wf.dev = dev;
  if (ce == hipSuccess) ce = hipEventCreateWithFlags(&wf.fork, hipEventDisableTiming);
  if (ce == hipSuccess) ce = hipEventCreateWithFlags(&wf.join, hipEventDisableTiming);
  if (ce == hipSuccess) ce = hipEventCreateWithFlags(&wf.fork3, hipEventDisableTiming);
  if (ce == hipSuccess) ce = hipEventCreateWithFlags(&wf.join3, hipEventDisableTiming);
  if (prev != dev) HIPCHK(hipSetDevice(prev));
  HIPCHK(ce);
  HIPCHK(hipEventRecord(wf.fork, s));
  HIPCHK(hipStreamWaitEvent(wf.s2, wf.fork, 0));
  hipStream_t s2 = wf.s2, s3 = wf.s3;
  const dim3 egrid((unsigned)cdiv(n_ent, kBlock));
  if (n >= kWfWave) {
    WelfordCtl* wc = at<WelfordCtl>(ws, L.wctl);
    WelfordCtl* wch = wc + 1;  // the head group's queue
    uint32_t* worder = at<uint32_t>(ws, L.worder);
    HIPCHK(hipMemsetAsync(wc, 0, 2 * sizeof(WelfordCtl), s2));
    LAUNCH("welford_bins", k_welford_bins, egrid, dim3(kBlock), s2, ent_start, n_ent, n, wc);
    LAUNCH("welford_order", k_welford_order, egrid, dim3(kBlock), s2, ent_start, n_ent, n, wc, worder);
    LAUNCH("welford_split", k_welford_split, dim3(1), dim3(kWave), s2, wc, wch);
    // the rest on s3: every record's samples, then the other groups' chains and the small entities
    HIPCHK(hipEventRecord(wf.fork3, s2));
    HIPCHK(hipStreamWaitEvent(s3, wf.fork3, 0));
    double* xs = at<double>(ws, L.wx);
    const dim3 xgrid((unsigned)cdiv(n, kBlock));
    const dim3 hgrid((unsigned)kWfBlocks);
    // Round 5: the head kernel's blocks each need a whole CU (k_welford_head2), which a flood of
    // other blocks keeps from them: inside the pipeline its blocks started ~1.4 ms after the launch
    // (config 2).  The key pass (the caller's stream) and the sample pass (s3) first wait on the
    // device, boundedly, for the head blocks to be resident (k_wf_gate).  A scheduling aid only: on
    // the time-out they go on, and nothing waits on them.
    // Round 6: the head kernels are submitted before the gates, so a gate that lands on
    // the head stream's hardware queue (4 per process) sits behind them instead of holding them up
    // for its whole time-out; and the gates are left out when another call on this device holds a
    // side-stream pair (concurrent pipelines: their head blocks compete for the same CUs, so one
    // pipeline's gate could wait on CUs another pipeline holds).
    const uint32_t* started = &wch->started;
    constexpr unsigned kHeadBlocks = (unsigned)(kWfHeadEnts / kW2Ents);
    const char* nogate = getenv("SCT_NO_WF_GATE");
    const bool gate = alone && !(nogate && nogate[0] == '1');
    if (cell) {
      LAUNCH("welford_x_head", k_welford_x_ents<true>, hgrid, dim3(kBlock), s2, rc2, ent_start, n_ent, n,
             (const uint32_t*)worder, (const WelfordCtl*)wch, xs);
      LAUNCH_N("welford_head", n, k_welford_head2<true>, dim3(kHeadBlocks), dim3(kW2Waves * kWave), s2, ent_start,
               n_ent, n, (const uint32_t*)worder, wch, (const double*)xs, out_f);
    } else {
      LAUNCH("welford_x_head", k_welford_x_ents<false>, hgrid, dim3(kBlock), s2, rc2, ent_start, n_ent, n,
             (const uint32_t*)worder, (const WelfordCtl*)wch, xs);
      LAUNCH_N("welford_head", n, k_welford_head2<false>, dim3(kHeadBlocks), dim3(kW2Waves * kWave), s2, ent_start,
               n_ent, n, (const uint32_t*)worder, wch, (const double*)xs, out_f);
    }
    if (gate) {
      HIPCHK(hipStreamWaitEvent(s, wf.fork3, 0));
      LAUNCH("welford_gate", k_wf_gate, dim3(1), dim3(kWave), s, started, kHeadBlocks, kWfGateTicks);
      LAUNCH("welford_gate", k_wf_gate, dim3(1), dim3(kWave), s3, started, kHeadBlocks, kWfGateTicks);
    }
    if (cell) {
      LAUNCH_N("welford_x", n, k_welford_x<true>, xgrid, dim3(kBlock), s3, rc2, n, xs, ent_start, n_ent,
               (const uint32_t*)worder, (const uint32_t*)&wch->n_big);
      LAUNCH_N("welford_chains", n, k_welford_chains<true>, dim3(kWfBlocks), dim3(kBlock), s3, ent_start, n_ent, n,
               (const uint32_t*)worder, wc, (const double*)xs, out_f);
    } else {
      LAUNCH_N("welford_x", n, k_welford_x<false>, xgrid, dim3(kBlock), s3, rc2, n, xs, ent_start, n_ent,
               (const uint32_t*)worder, (const uint32_t*)&wch->n_big);
      LAUNCH_N("welford_chains", n, k_welford_chains<false>, dim3(kWfBlocks), dim3(kBlock), s3, ent_start, n_ent, n,
               (const uint32_t*)worder, wc, (const double*)xs, out_f);
    }
  } else {
    HIPCHK(hipEventRecord(wf.fork3, s2));
    HIPCHK(hipStreamWaitEvent(s3, wf.fork3, 0));
  }
  if (cell) {
    LAUNCH("welford", k_welford<true>, egrid, dim3(kBlock), s3, rc2, ent_start, n_ent, n, out_f);
  } else {
    LAUNCH("welford", k_welford<false>, egrid, dim3(kBlock), s3, rc2, ent_start, n_ent, n, out_f);
  }
  return SCT_OK;
}

int pipeline(const sct_plan_t* plan, const sct_records_t* rec, const uint8_t* gene_is_mito, void* ws,
             size_t ws_bytes, int64_t* out_i, double* out_f, int64_t capacity, int64_t* n_rows,
             int64_t* gene_partials, hipStream_t s, bool allow_bucket = true) {
  const Layout L = layout_for(plan);
  if (!ws || ws_bytes < L.total) return fail(SCT_ENOMEM, "workspace too small (%zu < %zu)", ws_bytes, L.total);
  const int64_t n = rec->n;
  const bool cell = plan->mode != SCT_MODE_GENE;
  const bool gene = gene_partials != nullptr;
  const bool exact = plan->float_mode == SCT_FLOAT_EXACT_SUM;
  const int32_t* ent_col = cell ? rec->cell : rec->gene;

  int64_t n_ent = 0;
  bool dup = false;
  // the bucket descriptors (2 bytes per record, the step's largest fill) are zeroed while the host
  // waits for the entity count, when the first partition level will be planned (below)
  const char* nol1 = getenv("SCT_NO_L1_PLAN");
  const char* force = getenv("SCT_FORCE_GLOBAL_SORT");
  const char* nopre = getenv("SCT_NO_PREFILL");
  const int k1_bits = bitlen((uint64_t)(cell ? plan->n_gene_ids : plan->n_cell_ids));
  const bool may_plan = allow_bucket && k1_bits + bitlen((uint64_t)plan->n_umi_ids) <= kMaxKeyBits &&
                        !(force && force[0] == '1') && L.max_ent <= kEntHistMax && k1_bits >= kRadixBits &&
                        !(nol1 && nol1[0] == '1') && !(nopre && nopre[0] == '1') && n > 0;
  FillBatch pre;
  if (may_plan) pre.add(at<uint16_t>(ws, L.bdesc), sizeof(uint16_t) * (size_t)n);
  int rc = count_runs(ent_col, n, ws, L, gene, plan->n_cell_ids, &n_ent, &dup, s, may_plan ? &pre : nullptr);
  if (rc) return rc;
  if (dup) return fail(SCT_EINVAL, "grouped gene partials need cell-sorted records (a cell id forms two runs)");
  if (n_ent > L.max_ent)
    return fail(SCT_ENOMEM, "%lld entities exceed plan.max_entities %lld", (long long)n_ent, (long long)L.max_ent);
  if (out_i && n_ent > capacity)
    return fail(SCT_EINVAL, "%lld entities exceed output capacity %lld", (long long)n_ent, (long long)capacity);

  // key bits.  Bucket path (default): [k1' | k2 | hash], KB <= kMaxKeyBits, entities implied by
  // the record ranges.  Global-sort path: [run | k1' | k2 | hash], padded to whole radix digits.
  Bits b;
  b.k1 = bitlen((uint64_t)(cell ? plan->n_gene_ids : plan->n_cell_ids));
  b.k2 = bitlen((uint64_t)plan->n_umi_ids);
  const bool bucket = allow_bucket && b.k1 + b.k2 <= kMaxKeyBits && !(force && force[0] == '1');
  int used;
  if (bucket) {
    b.e = 0;
    used = b.k1 + b.k2;
    b.h = kMaxKeyBits - used < 8 ? kMaxKeyBits - used : 8;
  } else {
    b.e = bitlen((uint64_t)n_ent);
    used = b.e + b.k1 + b.k2;
    if (used > 63) return fail(SCT_EINVAL, "packed key needs %d bits (> 63)", used);
    // fill the last radix digit with fragment-hash bits (same pass count), every shift < 64
    const int padded = ((used + kRadixBits - 1) / kRadixBits) * kRadixBits;
    b.h = (padded > 63 ? 63 : padded) - used;
    if (b.h > 32) b.h = 32;
  }
  if (b.k1 > 0) {  // spread neighbouring k1 ids over the top key digits (odd multiplier, bijective)
    b.mul = 0x9E3779B1u & b.k1_mask();
    b.mul |= 1u;
    uint32_t inv = b.mul;  // Newton: inverse mod 2^32, then mod 2^k1
    for (int it = 0; it < 5; it++) inv *= 2u - b.mul * inv;
    b.inv = inv & b.k1_mask();
  }

  KeyCols kc{ent_col, cell ? rec->gene : rec->cell, rec->umi, (uint32_t)(cell ? plan->n_gene_ids : plan->n_cell_ids),
             (uint32_t)plan->n_umi_ids};
  RecCols rc2{rec->ref, rec->pos, rec->gq_sum, rec->gq_len, rec->gq_gt30, rec->bits, rec->xf,
              rec->cy_gt30, rec->cy_len, rec->uy_gt30, rec->uy_len};
  SortBuffers B{at<uint64_t>(ws, L.pay_a), at<uint64_t>(ws, L.pay_b), at<uint32_t>(ws, L.pay_a + L.half),
                at<uint32_t>(ws, L.pay_b + L.half), at<uint32_t>(ws, L.counts), at<uint32_t>(ws, L.offsets),
                at<uint64_t>(ws, L.scan_sums), L.count_cap};
  int64_t* ent_start = at<int64_t>(ws, L.ent_start);
  int64_t* partials = at<int64_t>(ws, L.partials);
  uint32_t* gcounts = gene ? at<uint32_t>(ws, L.gcounts) : nullptr;
  uint32_t* gtoff = gene ? at<uint32_t>(ws, L.gtoff) : nullptr;
  // bucket path: the first partition level planned before the key pass when its digit comes from
  // k1 alone (segment.h k_level1_plan), so the key pass writes the level-1 children itself
  const bool planned = bucket && L.max_ent <= kEntHistMax && n_ent > 0 && b.k1 >= kRadixBits &&
                       !(nol1 && nol1[0] == '1');
  L1Plan l1{};
  if (planned)
    l1 = L1Plan{at<uint32_t>(ws, L.ent_hist), at<uint32_t>(ws, L.l1_toff), at<uint2>(ws, L.l1_tslot),
                at<Pay>(ws, L.pay_b)};
  const uint8_t* mito = gene_is_mito;
  // every buffer the step zeroes before its first kernel, in one launch
  FillBatch fb;
  if (cell && !mito) {
    uint8_t* z = at<uint8_t>(ws, L.zero_mito);
    fb.add(z, (size_t)plan->n_gene_ids);
    mito = z;
  }
  fb.add(partials, sizeof(int64_t) * SCT_NP * (size_t)n_ent);
  if (gene) {
    fb.add(gcounts, sizeof(uint32_t) * (size_t)L.n_buckets);
    fb.add(gene_partials, sizeof(int64_t) * SCT_NP * (size_t)plan->n_gene_ids);  // (written by gene_reduce only)
  }

  // 1. input order: runs, keys, additive metrics (+ gene-bucket counts per tile)
  const dim3 tgrid((unsigned)cdiv(n, kKTile));  // key-pass blocks (tile offsets are per kTile)
  const uint64_t* toff = at<uint64_t>(ws, L.tile_cnt);
  // exact mean / variance lanes of the output rows ride along in the same launch
  const bool streams = exact && out_i;
  BucketCtl* ctl = bucket_ctl(ws, L);
  fb.add(ctl, sizeof(BucketCtl));
  // gene payload format: narrow (8 B) unless an operand does not fit (checked by the exact-stream
  // pass; without it the wide format is used)
  uint32_t* gwide = reinterpret_cast<uint32_t*>(at<uint64_t>(ws, L.scalars) + 16);
  fb.add(gwide, sizeof(uint32_t), streams ? 0 : 1);
  if (planned) level1_fills(L, ws, n, n_ent, l1, fb, may_plan);
  rc = launch_fills(fb, s);
  if (rc) return rc;
  if (planned) {
    rc = bucket_level1_plan(L, ws, kc, n, n_ent, b, ent_start, l1, s);
    if (rc) return rc;
    // level 1's counts, final after its classification: copied now, read by bucket_distinct while
    // the key pass runs (no host wait between the key pass and level 2)
    if (int rb = readback_start(bucket_ctl(ws, L), sizeof(BucketCtl), s)) return rb;
  }
  // Welford (the drop-in default): forked as soon as the entity starts exist -- after the level-1
  // plan when there is one (round 4: the head group's chains then start before the key pass),
  // else after the key pass
  WelfordSide wf;
  const bool wf_fork_early = planned && !exact && out_i;
  if (wf_fork_early) {
    rc = welford_stage(L, ws, cell, n, n_ent, rc2, ent_start, out_f, s, wf);
    if (rc) return rc;
  }

  if (bucket) {
    uint64_t* pay = at<uint64_t>(ws, L.pay_a);  // (the bucket path writes Pay records through `keys`)
    rc = streams ? launch_build_keys<true, true>(cell, gene, tgrid, s, kc, rc2, mito, n, toff, b, pay, nullptr, ent_start,
                                                 partials, gcounts, L.n_buckets, &ctl->err, gwide, gtoff, l1)
                 : launch_build_keys<true, false>(cell, gene, tgrid, s, kc, rc2, mito, n, toff, b, pay, nullptr, ent_start,
                                                  partials, gcounts, L.n_buckets, &ctl->err, gwide, gtoff, l1);
  } else {
    rc = streams ? launch_build_keys<false, true>(cell, gene, tgrid, s, kc, rc2, mito, n, toff, b, B.ka, B.va,
                                                  ent_start, partials, gcounts, L.n_buckets, &ctl->err, gwide, gtoff,
                                                  l1)
                 : launch_build_keys<false, false>(cell, gene, tgrid, s, kc, rc2, mito, n, toff, b, B.ka, B.va,
                                                   ent_start, partials, gcounts, L.n_buckets, &ctl->err, gwide, gtoff,
                                                   l1);
    if (rc) return rc;
    uint32_t err = 0;  // the bucket path reads the flag at its first level sync
    if (int rb = readback(&err, &ctl->err, sizeof(err), s)) return rb;
    if (err & 2) return fail(SCT_EINVAL, "a gene / cell / umi id lies outside its dictionary size");
  }
  if (rc) return rc;
  if (!wf_fork_early && !exact && out_i) {  // the entity starts exist now (the key pass wrote them)
    rc = welford_stage(L, ws, cell, n, n_ent, rc2, ent_start, out_f, s, wf);
    if (rc) return rc;
  }

  // Round 6: a side stream forked after the key pass (planned bucket path, exact floats) runs the
  // gene view's plan and the big buckets of levels 0-1 beside the partition levels >= 2 and the
  // hash tiles, and the cell rows' finalize beside the gene view
  SideStream side;
  hipEvent_t plan_done = nullptr;
  const char* no_side = getenv("SCT_NO_SIDE");
  const bool use_side = bucket && planned && exact && !(no_side && no_side[0] == '1');
  uint32_t* gcur = gene ? at<uint32_t>(ws, L.gcursor) : nullptr;
  int64_t* gwork = gene ? at<int64_t>(ws, L.gwork) : nullptr;
  int64_t* n_gwork = at<int64_t>(ws, L.scalars) + 4;
  if (use_side) {
    HIPCHK(side.open(s));
    if (gene) {
      LAUNCH_SHM("gene_plan", k_gene_plan, dim3(1), dim3(kBlock), 2 * sizeof(uint32_t) * (size_t)(L.n_buckets + 1),
                 side.use(), (const uint32_t*)gcounts, L.n_buckets, gcur, gwork, n_gwork);
      HIPCHK(side.event(&plan_done));
      HIPCHK(hipEventRecord(plan_done, side.s));
    }
  }

  // 2-3. distinct counts (+ per-record distinct events for the gene view)
  uint16_t* dflags = gene ? at<uint16_t>(ws, L.dflags) : nullptr;
  if (bucket) {
    rc = bucket_distinct(L, ws, n, n_ent, ent_start, mito, b, cell, gene, partials, dflags, planned, s, side);
    if (rc == 1) {  // a mapped ref id does not fit the bucket payload: redo on the global-sort path
      if (wf.s2) HIPCHK(hipStreamSynchronize(wf.s2));  // (its workspace is reused by the redo)
      if (wf.s3) HIPCHK(hipStreamSynchronize(wf.s3));
      if (side.is_open()) HIPCHK(hipStreamSynchronize(side.s));
      return pipeline(plan, rec, gene_is_mito, ws, ws_bytes, out_i, out_f, capacity, n_rows, gene_partials, s,
                      false);
    }
    if (rc) return rc;
  } else {
    int which = 0;
    rc = radix_sort(B, n, used + b.h, &which, s);
    if (rc) return rc;
    const uint64_t* keys = which ? B.kb : B.ka;
    const uint32_t* vals = which ? B.vb : B.va;
    const dim3 rgrid((unsigned)cdiv(n, kReduceTile));
    if (cell && gene) {
      LAUNCH_N("reduce_sorted", n, (k_reduce_sorted<true, true>), rgrid, dim3(kBlock), s, keys, vals, n, rc2, mito, b,
             partials, dflags);
    } else if (cell) {
      LAUNCH_N("reduce_sorted", n, (k_reduce_sorted<true, false>), rgrid, dim3(kBlock), s, keys, vals, n, rc2, mito, b,
             partials, dflags);
    } else {
      LAUNCH_N("reduce_sorted", n, (k_reduce_sorted<false, false>), rgrid, dim3(kBlock), s, keys, vals, n, rc2, mito, b,
             partials, dflags);
    }
  }

  if (out_i) {
    const char* no_sfin = getenv("SCT_NO_SIDE_FIN");
    const bool side_fin = side.is_open() && gene && !(no_sfin && no_sfin[0] == '1');
    if (side_fin) HIPCHK(side.from_caller(s));
    hipStream_t fs = side_fin ? side.use() : s;
    LAUNCH("finalize", k_finalize, dim3((unsigned)cdiv(n_ent * kFinThreads, kBlock)), dim3(kBlock), fs, (const int64_t*)partials,
           n_ent, cell ? SCT_MODE_CELL : SCT_MODE_GENE, exact ? 1 : 0, (const int64_t*)ent_start, out_i, out_f);
    if (!exact) {  // launched on the side streams after the key pass (welford_stage): joined here
      HIPCHK(hipEventRecord(wf.join, wf.s2));
      HIPCHK(hipStreamWaitEvent(s, wf.join, 0));
      HIPCHK(hipEventRecord(wf.join3, wf.s3));
      HIPCHK(hipStreamWaitEvent(s, wf.join3, 0));
    }
  }
  if (gene) {
    // 4. gene view: bucket starts, payload emission (input order), bucket reduction
    void* gpay = at<GenePayload>(ws, L.gpay);
    if (plan_done) {
      HIPCHK(hipStreamWaitEvent(s, plan_done, 0));
    } else {
      LAUNCH_SHM("gene_plan", k_gene_plan, dim3(1), dim3(kBlock), 2 * sizeof(uint32_t) * (size_t)(L.n_buckets + 1), s,
                 (const uint32_t*)gcounts, L.n_buckets, gcur, gwork, n_gwork);
    }
    static_assert(kEmitTile == kKTile, "gene_emit tiles are the key pass's tiles (gtoff)");
    const int staged = L.n_buckets <= kEmitStagedBuckets ? 1 : 0;
    LAUNCH_SHM_N("gene_emit", n, k_gene_emit, dim3((unsigned)cdiv(n, kEmitTile)), dim3(kBlock),
               (staged ? 3 : 2) * sizeof(uint32_t) * (size_t)L.n_buckets, s, rec->gene, rc2, (const uint16_t*)dflags,
               n, (const uint32_t*)gcur, (const uint32_t*)gtoff, L.n_buckets, (const uint32_t*)gwide, staged, gpay);
    LAUNCH_N("gene_reduce", n, k_gene_reduce, dim3((unsigned)L.max_gene_work), dim3(kBlock), s, (const void*)gpay,
           (const int64_t*)gwork, (const int64_t*)n_gwork, plan->n_gene_ids, (const uint32_t*)gwide, gene_partials);
  }
  if (side.is_open()) HIPCHK(side.to_caller(s));
  if (n_rows) *n_rows = n_ent;
  return SCT_OK;
}

// ---- tag sort ----
struct SortLayout {
  size_t recs, recs2, ka, kb, va, vb, counts, offsets, sums, bad, lka, lkb, lva, lvb, longs, tctl, gseg, total;
  int64_t count_cap;
};

struct CountLayout {
  size_t ka, kb, va, vb, counts, offsets, sums, flags_a, offs_a, flags_b, offs_b, pair_cell, pair_col, pair_tri;
  size_t cell_first, cell_npairs, cell_pstart, row_of, row_pairs, scalars, total;
  int64_t count_cap;
};

CountLayout count_layout(const sct_count_input_t* in) {
  CountLayout L;
  const int64_t n1 = in->n > 0 ? in->n : 1;
  const int64_t c1 = in->n_cell_ids > 0 ? in->n_cell_ids : 1;
  const int64_t m = n1 > c1 ? n1 : c1;  // the record sort and the cell-order sort share buffers
  const int64_t cm = (int64_t)kRadix * cdiv(m, kSortTile);
  L.count_cap = cm;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    size_t o = off;
    off += align_up(bytes);
    return o;
  };
  L.ka = take(8 * (size_t)m);
  L.kb = take(8 * (size_t)m);
  L.va = take(4 * (size_t)m);
  L.vb = take(4 * (size_t)m);
  L.counts = take(4 * (size_t)cm);
  L.offsets = take(4 * (size_t)cm);
  L.sums = take(8 * (size_t)(cdiv(cm > m ? cm : m, kScanChunk) + 1));
  L.flags_a = take(4 * (size_t)n1);
  L.offs_a = take(4 * (size_t)n1);
  L.flags_b = take(4 * (size_t)n1);
  L.offs_b = take(4 * (size_t)n1);
  L.pair_cell = take(4 * (size_t)n1);
  L.pair_col = take(4 * (size_t)n1);
  L.pair_tri = take(4 * (size_t)n1);
  L.cell_first = take(4 * (size_t)c1);
  L.cell_npairs = take(4 * (size_t)c1);
  L.cell_pstart = take(4 * (size_t)c1);
  L.row_of = take(4 * (size_t)c1);
  L.row_pairs = take(4 * (size_t)c1);
  L.scalars = take(6 * sizeof(uint64_t));
  L.total = off;
  return L;
}

SortLayout sort_layout(int64_t n) {
  SortLayout L;
  const int64_t n1 = n > 0 ? n : 1;
  // The digit counts serve two tilings: the row passes (kRowTile) and radix_sort (kSortTile, the
  // tiebreak and multi-round paths).  Round 3 sized them by kRowTile alone, which only held while
  // both tiles were 2048 items: a 1024-item kSortTile overflowed `counts` into `offsets`, the scan
  // then read its own output, and the downsweep wrote through garbage offsets (the illegal memory
  // access of the SCT_SORT_ITEMS=4 build).  radix_sort now also checks its capacity.
  const int64_t row_tiles = cdiv(n1, kRowTile), sort_tiles = cdiv(n1, kSortTile);
  int64_t tiles = row_tiles > sort_tiles ? row_tiles : sort_tiles;
  const int64_t seg_tiles = cdiv(n1, kSegTile) + kMsdRadix;  // the group sort's segmented passes (tagsort.h)
  tiles = tiles > seg_tiles ? tiles : seg_tiles;
  const int64_t msd_tiles = cdiv(n1, kMsdTile) * (kMsdRadix / kRadix);  // and its MSD pass (kMsdRadix digits)
  tiles = tiles > msd_tiles ? tiles : msd_tiles;
  const int64_t m = (int64_t)kRadix * tiles;
  L.count_cap = m;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    size_t o = off;
    off += align_up(bytes);
    return o;
  };
  L.recs = take(sizeof(PackedRec) * (size_t)n1);
  L.recs2 = take(sizeof(PackedRec) * (size_t)n1);
  L.ka = take(sizeof(uint64_t) * (size_t)n1);
  L.kb = take(sizeof(uint64_t) * (size_t)n1);
  L.va = take(sizeof(uint32_t) * (size_t)n1);
  L.vb = take(sizeof(uint32_t) * (size_t)n1);
  L.counts = take(sizeof(uint32_t) * (size_t)m);
  L.offsets = take(sizeof(uint32_t) * (size_t)m);
  L.sums = take(sizeof(uint64_t) * (size_t)(cdiv(m, kScanChunk) + 1));
  L.bad = take(sizeof(uint64_t));
  // tiebreak fix-up of runs longer than kTieShort (tagsort.h): compact keys / values, run list
  L.lka = take(sizeof(uint64_t) * (size_t)n1);
  L.lkb = take(sizeof(uint64_t) * (size_t)n1);
  L.lva = take(sizeof(uint32_t) * (size_t)n1);
  L.lvb = take(sizeof(uint32_t) * (size_t)n1);
  L.longs = take(sizeof(uint4) * (size_t)(n1 / (kTieShort + 1) + 1));
  L.tctl = take(4 * sizeof(uint32_t));
  L.gseg = take((3 * kMsdRadix + 1) * sizeof(uint32_t));
  L.total = off;
  return L;
}

// the order's fields, most significant first (+ the tiebreak, least significant)
int order_fields(int32_t order, const sct_plan_t* plan, bool tie, int32_t n_tie, KeyField* f, int* nf) {
  const KeyField cell{0, bitlen((uint64_t)plan->n_cell_ids)}, umi{1, bitlen((uint64_t)plan->n_umi_ids)},
      gene{2, bitlen((uint64_t)plan->n_gene_ids)};
  int k = 0;
  if (order == SCT_ORDER_CELL) {
    f[k++] = cell;
  } else if (order == SCT_ORDER_CELL_UMI_GENE) {
    f[k++] = cell, f[k++] = umi, f[k++] = gene;
  } else if (order == SCT_ORDER_GENE_CELL_UMI) {
    f[k++] = gene, f[k++] = cell, f[k++] = umi;
  } else {
    return fail(SCT_EINVAL, "unknown sort order %d", order);
  }
  if (tie) {
    if (n_tie <= 0) return fail(SCT_EINVAL, "n_tiebreak_ids must be positive");
    f[k++] = KeyField{3, bitlen((uint64_t)n_tie)};
  }
  *nf = k;
  return SCT_OK;
}

int check_sort_args(const sct_plan_t* plan, const sct_records_t* rec) {
  if (!plan || !rec) return fail(SCT_EINVAL, "NULL plan or records");
  if (plan->n_records < 0 || plan->n_records > (int64_t)0x7FFFFFFF)
    return fail(SCT_EINVAL, "n_records %lld out of range [0, 2^31)", (long long)plan->n_records);
  if (rec->n != plan->n_records) return fail(SCT_EINVAL, "records.n != plan.n_records");
  if (plan->n_cell_ids <= 0 || plan->n_gene_ids <= 0 || plan->n_umi_ids <= 0)
    return fail(SCT_EINVAL, "dictionary sizes must be positive");
  return SCT_OK;
}

}  // namespace

// ======================================================================================
// C-ABI
// ======================================================================================

extern "C" {

int sct_abi_version(void) { return SCT_ABI_VERSION; }

const char* sct_last_error(void) { return last_error().c_str(); }

int sct_profile_enable(int on) {
  prof_on() = on != 0;
  return SCT_OK;
}

int sct_profile_only(const char* kernel_name) {
  prof_only() = kernel_name ? kernel_name : "";
  return SCT_OK;
}

int sct_profile_read_items(const char** names, double* ms, int64_t* launches, int64_t* items, int max_kernels) {
  // waits for the recorded events, returns per-kernel totals, and resets the counters
  static thread_local std::vector<std::string> held;
  held.clear();
  int k = 0;
  for (auto& e : prof_entries()) {
    double tot = 0.0;
    for (auto& pr : e.ev) {
      float t = 0.f;
      if (hipEventSynchronize(pr.second) == hipSuccess && hipEventElapsedTime(&t, pr.first, pr.second) == hipSuccess)
        tot += t;
      (void)hipEventDestroy(pr.first);
      (void)hipEventDestroy(pr.second);
    }
    held.push_back(e.name);
    if (k < max_kernels) {
      if (ms) ms[k] = tot;
      if (launches) launches[k] = (int64_t)e.ev.size();
      if (items) items[k] = e.items;
    }
    k++;
  }
  for (int i = 0; i < k && i < max_kernels; i++)
    if (names) names[i] = held[i].c_str();
  prof_entries().clear();
  return k;
}

int sct_profile_read(const char** names, double* ms, int64_t* launches, int max_kernels) {
  return sct_profile_read_items(names, ms, launches, nullptr, max_kernels);
}

int sct_workspace_size(const sct_plan_t* plan, size_t* bytes) {
  int rc = check_plan(plan, nullptr);
  if (rc) return rc;
  if (!bytes) return fail(SCT_EINVAL, "bytes is NULL");
  *bytes = layout_for(plan).total;
  return SCT_OK;
}

int sct_count_entities(const sct_plan_t* plan, const sct_records_t* rec, void* workspace, size_t workspace_bytes,
                       int64_t* n_entities, void* stream) {
  last_error().clear();
  int rc = check_plan(plan, rec);
  if (rc) return rc;
  if (!n_entities) return fail(SCT_EINVAL, "n_entities is NULL");
  if (plan->mode == SCT_MODE_GENE_GROUPED) {
    *n_entities = plan->n_gene_ids;
    return SCT_OK;
  }
  if (rec->n == 0) {
    *n_entities = 0;
    return SCT_OK;
  }
  sct_plan_t p1 = *plan;
  p1.max_entities = 1;
  p1.flags = 0;
  const Layout L = layout_for(&p1);
  if (!workspace || workspace_bytes < count_bytes(L))
    return fail(SCT_ENOMEM, "workspace too small for counting (%zu < %zu)", workspace_bytes, count_bytes(L));
  return count_runs(plan->mode == SCT_MODE_CELL ? rec->cell : rec->gene, rec->n, workspace, L, false, 0, n_entities,
                    nullptr, (hipStream_t)stream);
}

int sct_compute_metrics(const sct_plan_t* plan, const sct_records_t* rec, const uint8_t* gene_is_mito,
                        const uint8_t* gene_is_multi, void* workspace, size_t workspace_bytes, int64_t* out_ints,
                        double* out_floats, int64_t capacity, int64_t* n_rows, void* stream) {
  (void)gene_is_multi;  // multi-gene rows are dropped by the caller (gatherer.py:210-212)
  last_error().clear();
  int rc = check_plan(plan, rec);
  if (rc) return rc;
  if (plan->mode == SCT_MODE_GENE_GROUPED)
    return fail(SCT_EINVAL, "sct_compute_metrics handles RUN modes; use sct_gene_partials for GROUPED");
  if (!n_rows || !out_ints || !out_floats) return fail(SCT_EINVAL, "NULL output");
  if (plan->mode == SCT_MODE_CELL && !gene_is_mito) return fail(SCT_EINVAL, "gene_is_mito is NULL");
  if (rec->n == 0) {
    *n_rows = 0;
    return SCT_OK;
  }
  return pipeline(plan, rec, gene_is_mito, workspace, workspace_bytes, out_ints, out_floats, capacity, n_rows,
                  nullptr, (hipStream_t)stream);
}

int sct_gene_partials(const sct_plan_t* plan, const sct_records_t* rec, void* workspace, size_t workspace_bytes,
                      int64_t* partials, void* stream) {
  last_error().clear();
  int rc = check_plan(plan, rec);
  if (rc) return rc;
  if (plan->mode != SCT_MODE_GENE_GROUPED) return fail(SCT_EINVAL, "sct_gene_partials needs SCT_MODE_GENE_GROUPED");
  if (plan->float_mode != SCT_FLOAT_EXACT_SUM) return fail(SCT_EINVAL, "GROUPED partials need SCT_FLOAT_EXACT_SUM");
  if (!partials) return fail(SCT_EINVAL, "partials is NULL");
  hipStream_t s = (hipStream_t)stream;
  if (rec->n == 0) {
    HIPCHK(hipMemsetAsync(partials, 0, sizeof(int64_t) * SCT_NP * (size_t)plan->n_gene_ids, s));
    return SCT_OK;
  }
  return pipeline(plan, rec, nullptr, workspace, workspace_bytes, nullptr, nullptr, 0, nullptr, partials, s);
}

int sct_cell_metrics_gene_partials(const sct_plan_t* plan, const sct_records_t* rec, const uint8_t* gene_is_mito,
                                   void* workspace, size_t workspace_bytes, int64_t* out_ints, double* out_floats,
                                   int64_t capacity, int64_t* n_rows, int64_t* gene_partials, void* stream) {
  last_error().clear();
  int rc = check_plan(plan, rec);
  if (rc) return rc;
  if (plan->mode != SCT_MODE_CELL || !(plan->flags & SCT_PLAN_GENE_PARTIALS))
    return fail(SCT_EINVAL, "needs SCT_MODE_CELL with SCT_PLAN_GENE_PARTIALS");
  if (!n_rows || !out_ints || !out_floats || !gene_partials || !gene_is_mito) return fail(SCT_EINVAL, "NULL argument");
  hipStream_t s = (hipStream_t)stream;
  if (rec->n == 0) {
    *n_rows = 0;
    HIPCHK(hipMemsetAsync(gene_partials, 0, sizeof(int64_t) * SCT_NP * (size_t)plan->n_gene_ids, s));
    return SCT_OK;
  }
  return pipeline(plan, rec, gene_is_mito, workspace, workspace_bytes, out_ints, out_floats, capacity, n_rows,
                  gene_partials, s);
}

int sct_tag_sort_workspace_size(const sct_plan_t* plan, size_t* bytes) {
  if (!plan || !bytes) return fail(SCT_EINVAL, "NULL argument");
  *bytes = sort_layout(plan->n_records).total;
  return SCT_OK;
}

int sct_tag_sort(const sct_plan_t* plan, const sct_records_t* in, const int32_t* tiebreak, int32_t n_tiebreak_ids,
                 int32_t order, const sct_records_t* out, void* workspace, size_t workspace_bytes, void* stream) {
  last_error().clear();
  int rc = check_sort_args(plan, in);
  if (rc) return rc;
  if (!out || out->n != in->n) return fail(SCT_EINVAL, "out must hold records.n records");
  KeyField f[4];
  int nf = 0;
  rc = order_fields(order, plan, tiebreak != nullptr, n_tiebreak_ids, f, &nf);
  if (rc) return rc;
  const int64_t n = in->n;
  if (n == 0) return SCT_OK;
  const SortLayout L = sort_layout(n);
  if (!workspace || workspace_bytes < L.total)
    return fail(SCT_ENOMEM, "workspace too small (%zu < %zu)", workspace_bytes, L.total);
  hipStream_t s = (hipStream_t)stream;
  uint4* recs = at<uint4>(workspace, L.recs);
  if (order == SCT_ORDER_CELL && !tiebreak) {  // whole rows through 8-bit LSD passes, no gathers
    const int bits = f[0].bits;
    const int passes = bits > kRadixBits ? (bits + kRadixBits - 1) / kRadixBits : 1;
    const int64_t tiles = cdiv(n, kRowTile);
    uint32_t* counts = at<uint32_t>(workspace, L.counts);
    uint32_t* offsets = at<uint32_t>(workspace, L.offsets);
    uint64_t* sums = at<uint64_t>(workspace, L.sums);
    uint4* rows[2] = {recs, at<uint4>(workspace, L.recs2)};
    int32_t* keys[2] = {at<int32_t>(workspace, L.ka), at<int32_t>(workspace, L.kb)};
    for (int ps = 0; ps < passes; ps++) {
      const int shift = ps * kRadixBits;
      const bool first = ps == 0, last = ps == passes - 1;
      const int32_t* hkey = first ? in->cell : keys[(ps - 1) & 1];
      LAUNCH_N("tag_row_hist", n, k_row_hist, dim3((unsigned)tiles), dim3(kBlock), s, hkey, n, shift, tiles, counts);
      rc = scan_counts(counts, (int64_t)kRadix * tiles, offsets, sums, s);
      if (rc) return rc;
      const uint4* rin = first ? nullptr : rows[(ps - 1) & 1];
      uint4* rout = rows[ps & 1];
      int32_t* kout = keys[ps & 1];
#define SCT_ROWS(A, Z)                                                                                              \
  LAUNCH_N("tag_row_scatter", n, (k_row_scatter<A, Z>), dim3((unsigned)tiles), dim3(kBlock), s, *in, rin, rout, kout, \
         *out, n, shift, tiles, (const uint32_t*)offsets)
      if (first && last) {
        SCT_ROWS(true, true);
      } else if (first) {
        SCT_ROWS(true, false);
      } else if (last) {
        SCT_ROWS(false, true);
      } else {
        SCT_ROWS(false, false);
      }
#undef SCT_ROWS
    }
    return SCT_OK;
  }
  SortBuffers B{at<uint64_t>(workspace, L.ka), at<uint64_t>(workspace, L.kb), at<uint32_t>(workspace, L.va),
                at<uint32_t>(workspace, L.vb), at<uint32_t>(workspace, L.counts), at<uint32_t>(workspace, L.offsets),
                at<uint64_t>(workspace, L.sums), L.count_cap};
  const dim3 grid((unsigned)cdiv(n, kBlock));
  // (CB, UB, GE[, query name]) by groups (tagsort.h, round 6): an LSD sort of (cell, top umi bits) only,
  // then every group sorted inside its own positions
  const char* grp_env = getenv("SCT_TAG_GROUP_SORT");
  if (order == SCT_ORDER_CELL_UMI_GENE && !(grp_env && grp_env[0] == '0')) {
    GroupBits gb{};
    gb.c = f[0].bits, gb.u = f[1].bits, gb.g = f[2].bits, gb.t = tiebreak ? f[3].bits : 0;
    const int ub_min = gb.u + gb.g + gb.t - 52 > 0 ? gb.u + gb.g + gb.t - 52 : 0;  // W fits 52 bits
    const int passes = (gb.c + ub_min + kRadixBits - 1) / kRadixBits;
    if (ub_min <= gb.u && passes <= 4) {
      const char* msd_env = getenv("SCT_TAG_GROUP_MSD");
      const bool msd = gb.c + ub_min > kRadixBits && !(msd_env && msd_env[0] == '0');
      // K1 is filled to the width its passes sort anyway (smaller groups for free): LSD, whole 8-bit
      // digits; MSD, the kMsdBits-bit top digit plus the fewest 8-bit segmented passes (<= 32 bits)
      int kw = kRadixBits * passes;
      if (msd) {
        const int segp = gb.c + ub_min > kMsdBits ? (gb.c + ub_min - kMsdBits + kRadixBits - 1) / kRadixBits : 0;
        kw = kMsdBits + kRadixBits * segp < 32 ? kMsdBits + kRadixBits * segp : 32;
      }
      gb.ub = kw - gb.c < gb.u ? kw - gb.c : gb.u;
      gb.ul = gb.u - gb.ub;
      uint4* longs = at<uint4>(workspace, L.longs);
      uint32_t* tctl = at<uint32_t>(workspace, L.tctl);
      HIPCHK(hipMemsetAsync(tctl, 0, 4 * sizeof(uint32_t), s));
      int which = 0;
      const int kbits = gb.c + gb.ub;
      const uint32_t* keys = nullptr;
      const uint32_t* perm = nullptr;
      if (msd) {
        // rows written once in the order of K1's top digit, then the rest of K1 inside those buckets
        const int sh_top = kbits > kMsdBits ? kbits - kMsdBits : 0;
        const int64_t mt = cdiv(n, kMsdTile);
        const int64_t tmax = cdiv(n, kSegTile) + kMsdRadix;
        if ((int64_t)kMsdRadix * mt > L.count_cap || (int64_t)kRadix * tmax > L.count_cap)
          return fail(SCT_EINVAL, "group sort: digit counts exceed the workspace");
        uint32_t* ka32 = reinterpret_cast<uint32_t*>(B.ka);
        uint32_t* kb32 = reinterpret_cast<uint32_t*>(B.kb);
        uint32_t* gseg = at<uint32_t>(workspace, L.gseg);
        LAUNCH_N("tag_group_hist", n, k_gmsd_hist, dim3((unsigned)mt), dim3(kBlock), s, in->cell, in->umi, n, gb,
                 sh_top, mt, B.counts, tctl);
        rc = scan_counts(B.counts, (int64_t)kMsdRadix * mt, B.offsets, B.sums, s);
        if (rc) return rc;
        LAUNCH_N("tag_group_msd", n, k_gmsd_scatter, dim3((unsigned)mt), dim3(kBlock), s, *in, tiebreak, n, gb, sh_top,
                 mt, (const uint32_t*)B.offsets, recs, ka32);
        LAUNCH("tag_group_plan", k_gseg_plan, dim3(1), dim3(kBlock), s, (const uint32_t*)B.offsets, mt, n, gseg);
        const int passes = (sh_top + kRadixBits - 1) / kRadixBits;
        int cur = 0;
        for (int ps = 0; ps < passes; ps++) {
          const uint32_t* kin = cur ? kb32 : ka32;
          const uint32_t* vin = cur ? B.vb : B.va;
          uint32_t* kout = cur ? ka32 : kb32;
          uint32_t* vout = cur ? B.va : B.vb;
          LAUNCH_N("radix_upsweep", n, k_gseg_upsweep, dim3((unsigned)tmax), dim3(kBlock), s, kin, ps * kRadixBits,
                   (const uint32_t*)gseg, B.counts);
          rc = scan_counts(B.counts, (int64_t)kRadix * tmax, B.offsets, B.sums, s);
          if (rc) return rc;
          if (ps == 0) {
            LAUNCH_N("radix_downsweep", n, k_gseg_downsweep<true>, dim3((unsigned)tmax), dim3(kBlock), s, kin, vin,
                     kout, vout, ps * kRadixBits, (const uint32_t*)gseg, (const uint32_t*)B.offsets);
          } else {
            LAUNCH_N("radix_downsweep", n, k_gseg_downsweep<false>, dim3((unsigned)tmax), dim3(kBlock), s, kin, vin,
                     kout, vout, ps * kRadixBits, (const uint32_t*)gseg, (const uint32_t*)B.offsets);
          }
          cur ^= 1;
        }
        keys = cur ? kb32 : ka32;
        perm = cur ? B.vb : B.va;
        if (passes == 0)  // the top digit was all of K1: the rows are in K1 order already
          LAUNCH("tag_group_iota", k_iota, dim3((unsigned)cdiv(n, kBlock)), dim3(kBlock), s, B.va, n);
      } else {
        LAUNCH_N("tag_group_keys", n, k_pack_group_keys, grid, dim3(kBlock), s, *in, n, gb, tiebreak, recs,
                 reinterpret_cast<uint32_t*>(B.ka), tctl);
        if (kbits > 0) {
          rc = radix_sort32(B, n, kbits, &which, s, true);
        } else {  // one group: the values are the positions
          LAUNCH("tag_group_iota", k_iota, dim3((unsigned)cdiv(n, kBlock)), dim3(kBlock), s, B.va, n);
        }
        if (rc) return rc;
        keys = reinterpret_cast<const uint32_t*>(which ? B.kb : B.ka);
        perm = which ? B.vb : B.va;
      }
      uint2* glong = reinterpret_cast<uint2*>(longs);
      LAUNCH_N("tag_group_wave", n, k_group_wave, grid, dim3(kBlock), s, keys, perm, (const uint4*)recs, n, gb, *out,
               glong, tctl);
      uint32_t h[3] = {0, 0, 0};
      if (int rb = readback(h, tctl, sizeof(h), s)) return rb;
      if (!h[1] && !h[2]) {
        if (h[0])
          LAUNCH("tag_group_long", k_group_long, dim3(h[0]), dim3(kBlock), s, keys, perm, (const uint4*)recs, gb,
                 (const uint2*)glong, *out);
        return SCT_OK;
      }
      // a group past kGroupCap records or a cell id the key cannot hold: the general path below
    }
  }
  int field_bits = 0;
  for (int i = 0; i < nf - (tiebreak ? 1 : 0); i++) field_bits += f[i].bits;
  if (!(tiebreak && field_bits <= 64)) LAUNCH_N("tag_pack", n, k_pack, grid, dim3(kBlock), s, *in, recs);
  if (tiebreak && field_bits <= 64) {
    // one radix sort on the tag fields, then the query-name order inside runs of equal fields
    RoundKey rk{};
    rk.nf = nf - 1;
    rk.bits = field_bits;
    for (int i = 0; i < rk.nf; i++) rk.f[i] = f[i];
    const int tie_top = f[nf - 1].bits;  // the tiebreak's width
    int th = (field_bits + kRadixBits - 1) / kRadixBits * kRadixBits - field_bits;  // free bits of the last digit
    if (th > tie_top) th = tie_top;
    if (field_bits + th > 64) th = 64 - field_bits;
    LAUNCH_N("tag_pack_keys", n, k_pack_field_keys, grid, dim3(kBlock), s, *in, n, rk, tiebreak, tie_top, th, recs,
             B.ka, B.va);
    int which = 0;
    rc = radix_sort(B, n, field_bits + th, &which, s);
    if (rc) return rc;
    const uint64_t* keys = which ? B.kb : B.ka;
    uint32_t* perm = which ? B.vb : B.va;
    uint4* longs = at<uint4>(workspace, L.longs);
    uint32_t* tctl = at<uint32_t>(workspace, L.tctl);
    HIPCHK(hipMemsetAsync(tctl, 0, 2 * sizeof(uint32_t), s));
    uint32_t* pos_of = at<uint32_t>(workspace, L.recs2);  // the row buffer is free on this path
    if (SCT_TIE_V2) {
      LAUNCH("tag_ties", k_tie_wave2, grid, dim3(kBlock), s, keys, perm, tiebreak, n, longs, tctl);
    } else {
      LAUNCH("tag_ties", k_tie_wave, grid, dim3(kBlock), s, keys, perm, tiebreak, n, longs, tctl);
    }
    uint32_t h[2] = {0, 0};
    if (int rb = readback(h, tctl, sizeof(h), s)) return rb;
    if (h[0] > 0) {  // runs longer than kTieShort: (run, tiebreak) radix sort of their records
      const int tie_bits = bitlen((uint64_t)n_tiebreak_ids);
      SortBuffers LB{at<uint64_t>(workspace, L.lka), at<uint64_t>(workspace, L.lkb), at<uint32_t>(workspace, L.lva),
                     at<uint32_t>(workspace, L.lvb), B.counts, B.offsets, B.sums, B.count_cap};
      LAUNCH("tag_long_keys", k_long_keys, dim3(h[0]), dim3(kBlock), s, (const uint4*)longs, (const uint32_t*)perm,
             tiebreak, tie_bits, LB.ka, LB.va, pos_of);
      int w2 = 0;
      rc = radix_sort(LB, (int64_t)h[1], bitlen((uint64_t)h[1]) + tie_bits, &w2, s);
      if (rc) return rc;
      LAUNCH("tag_long_scatter", k_long_scatter, dim3((unsigned)cdiv(h[1], kBlock)), dim3(kBlock), s,
             (const uint32_t*)pos_of, (const uint32_t*)(w2 ? LB.vb : LB.va), (int64_t)h[1], perm);
    }
    LAUNCH_N("tag_unpack", n, k_unpack, grid, dim3(kBlock), s, (const uint4*)recs, (const uint32_t*)perm, n, *out);
    return SCT_OK;
  }
  // rounds: fields from the least significant end, packed greedily into <= 64-bit keys
  const uint32_t* perm = nullptr;
  int hi = nf;  // fields [lo, hi) of the next round (most significant first)
  while (hi > 0) {
    int lo = hi, bits = 0;
    while (lo > 0 && bits + f[lo - 1].bits <= 64) bits += f[--lo].bits;
    RoundKey rk{};
    rk.nf = hi - lo;
    rk.bits = bits;
    for (int i = 0; i < rk.nf; i++) rk.f[i] = f[lo + i];
    LAUNCH_N("tag_keys", n, k_round_keys, grid, dim3(kBlock), s, (const uint4*)recs, tiebreak, perm, n, rk, B.ka, B.va);
    int which = 0;
    rc = radix_sort(B, n, bits, &which, s);
    if (rc) return rc;
    perm = which ? B.vb : B.va;
    hi = lo;
  }
  LAUNCH_N("tag_unpack", n, k_unpack, grid, dim3(kBlock), s, (const uint4*)recs, perm, n, *out);
  return SCT_OK;
}

// ---- cell bins for the exchange between devices (exchange.h; SplitBam's bins, bam.py:439-480) ----

int sct_bin_workspace_size(const sct_plan_t* plan, int32_t n_bins, size_t* bytes) {
  last_error().clear();
  if (!plan || !bytes) return fail(SCT_EINVAL, "NULL argument");
  if (n_bins < 1 || n_bins > SCT_MAX_BINS) return fail(SCT_EINVAL, "n_bins %d outside [1, %d]", n_bins, SCT_MAX_BINS);
  const int64_t tiles = cdiv(plan->n_records > 0 ? plan->n_records : 1, kBinTile);
  const int64_t m = (int64_t)n_bins * tiles;
  *bytes = 2 * align_up(sizeof(uint32_t) * (size_t)m) + align_up(sizeof(uint64_t) * (size_t)(cdiv(m, kScanChunk) + 1));
  return SCT_OK;
}

int sct_bin_records(const sct_plan_t* plan, const sct_records_t* in, const int32_t* tiebreak,
                    const uint8_t* bin_of_cell, int32_t n_bins, const sct_records_t* out, int32_t* tiebreak_out,
                    int64_t* bin_counts, void* workspace, size_t workspace_bytes, void* stream) {
  last_error().clear();
  int rc = check_sort_args(plan, in);
  if (rc) return rc;
  if (!out || out->n != in->n) return fail(SCT_EINVAL, "out must hold records.n records");
  if (n_bins < 1 || n_bins > SCT_MAX_BINS) return fail(SCT_EINVAL, "n_bins %d outside [1, %d]", n_bins, SCT_MAX_BINS);
  if (!bin_counts) return fail(SCT_EINVAL, "bin_counts is NULL");
  if ((tiebreak == nullptr) != (tiebreak_out == nullptr))
    return fail(SCT_EINVAL, "tiebreak and tiebreak_out: both or neither");
  hipStream_t s = (hipStream_t)stream;
  const int64_t n = in->n;
  if (n == 0) {
    HIPCHK(hipMemsetAsync(bin_counts, 0, sizeof(int64_t) * (size_t)n_bins, s));
    return SCT_OK;
  }
  size_t need = 0;
  rc = sct_bin_workspace_size(plan, n_bins, &need);
  if (rc) return rc;
  if (!workspace || workspace_bytes < need) return fail(SCT_ENOMEM, "workspace too small (%zu < %zu)", workspace_bytes, need);
  const int64_t tiles = cdiv(n, kBinTile);
  const int64_t m = (int64_t)n_bins * tiles;
  uint32_t* counts = (uint32_t*)workspace;
  uint32_t* offsets = (uint32_t*)((uint8_t*)workspace + align_up(sizeof(uint32_t) * (size_t)m));
  uint64_t* sums = (uint64_t*)((uint8_t*)workspace + 2 * align_up(sizeof(uint32_t) * (size_t)m));
  const uint32_t nb = (uint32_t)n_bins, nc = (uint32_t)plan->n_cell_ids;
  const int bin_bits = bitlen((uint64_t)n_bins);  // bits of the bin values 0 .. n_bins - 1
  LAUNCH_N("bin_hist", n, k_bin_hist, dim3((unsigned)tiles), dim3(kBlock), s, in->cell, n, bin_of_cell, nb, nc, tiles,
           counts);
  rc = scan_counts(counts, m, offsets, sums, s);
  if (rc) return rc;
  if (tiebreak) {
    LAUNCH_N("bin_scatter", n, k_bin_scatter<true>, dim3((unsigned)tiles), dim3(kBlock), s, *in, tiebreak, *out,
             tiebreak_out, n, bin_of_cell, nb, nc, bin_bits, tiles, (const uint32_t*)offsets);
  } else {
    LAUNCH_N("bin_scatter", n, k_bin_scatter<false>, dim3((unsigned)tiles), dim3(kBlock), s, *in, tiebreak, *out,
             tiebreak_out, n, bin_of_cell, nb, nc, bin_bits, tiles, (const uint32_t*)offsets);
  }
  LAUNCH("bin_totals", k_bin_totals, dim3(1), dim3(kBlock), s, (const uint32_t*)offsets, tiles, nb, n, bin_counts);
  return SCT_OK;
}

int sct_verify_sort(const sct_plan_t* plan, const sct_records_t* rec, const int32_t* tiebreak, int32_t order,
                    void* workspace, size_t workspace_bytes, int64_t* first_violation, void* stream) {
  last_error().clear();
  int rc = check_sort_args(plan, rec);
  if (rc) return rc;
  if (!first_violation) return fail(SCT_EINVAL, "first_violation is NULL");
  KeyField f[4];
  int nf = 0;
  rc = order_fields(order, plan, false, 0, f, &nf);
  if (rc) return rc;
  *first_violation = -1;
  if (rec->n < 2) return SCT_OK;
  const SortLayout L = sort_layout(rec->n);
  if (!workspace || workspace_bytes < L.total)
    return fail(SCT_ENOMEM, "workspace too small (%zu < %zu)", workspace_bytes, L.total);
  hipStream_t s = (hipStream_t)stream;
  unsigned long long* bad = at<unsigned long long>(workspace, L.bad);
  const unsigned long long none = (unsigned long long)rec->n;
  HIPCHK(hipMemsetAsync(bad, 0xFF, sizeof(unsigned long long), s));  // no violation: ~0
  for (int i = nf; i < 3; i++) f[i] = KeyField{0, 0};
  LAUNCH("tag_verify", k_verify_order, dim3((unsigned)cdiv(rec->n - 1, kBlock)), dim3(kBlock), s, *rec, tiebreak,
         f[0], f[1], f[2], nf, bad);
  unsigned long long h = 0;
  if (int rb = readback(&h, bad, sizeof(h), s)) return rb;
  *first_violation = h >= none ? -1 : (int64_t)h;
  return SCT_OK;
}

int sct_count_matrix_workspace_size(const sct_count_input_t* in, size_t* bytes) {
  last_error().clear();
  if (!in || !bytes) return fail(SCT_EINVAL, "NULL argument");
  *bytes = count_layout(in).total;
  return SCT_OK;
}

int sct_count_matrix(const sct_count_input_t* in, sct_count_output_t* out, void* workspace, size_t workspace_bytes,
                     void* stream) {
  last_error().clear();
  if (!in || !out) return fail(SCT_EINVAL, "NULL argument");
  out->n_rows = out->nnz = out->n_sorted = 0;
  out->unknown_record = -1;
  const int64_t n = in->n;
  if (n < 0 || n >= (int64_t)0x7FFFFFFF) return fail(SCT_EINVAL, "records must be in [0, 2^31 - 1)");
  if (in->n_cell_ids < 0 || in->n_umi_ids < 0 || in->n_gene_ids < 0 || in->n_cols < 0)
    return fail(SCT_EINVAL, "negative dictionary size");
  if (!out->indptr) return fail(SCT_EINVAL, "indptr is NULL");
  hipStream_t s = (hipStream_t)stream;
  if (n == 0) {
    HIPCHK(hipMemsetAsync(out->indptr, 0, sizeof(int32_t), s));
    HIPCHK(hipStreamSynchronize(s));
    return SCT_OK;
  }
  if (!in->cell || !in->umi || !in->gene || !in->xf || !in->qhead || !in->gene_col || !out->row_cell ||
      !out->indices || !out->data)
    return fail(SCT_EINVAL, "NULL column");
  CountKey K;
  K.cbits = bitlen((uint64_t)in->n_cell_ids);
  K.colbits = bitlen((uint64_t)(in->n_cols > 0 ? in->n_cols : 1));
  K.ubits = bitlen((uint64_t)in->n_umi_ids);
  K.total = K.cbits + K.colbits + K.ubits;
  if (K.total > 63)
    return fail(SCT_EINVAL, "cell (%d) + column (%d) + molecule (%d) id bits exceed 63", K.cbits, K.colbits, K.ubits);
  const CountLayout L = count_layout(in);
  if (!workspace || workspace_bytes < L.total)
    return fail(SCT_ENOMEM, "workspace too small (%zu < %zu)", workspace_bytes, L.total);
  const int64_t nc = in->n_cell_ids;
  SortBuffers B{at<uint64_t>(workspace, L.ka), at<uint64_t>(workspace, L.kb), at<uint32_t>(workspace, L.va),
                at<uint32_t>(workspace, L.vb), at<uint32_t>(workspace, L.counts), at<uint32_t>(workspace, L.offsets),
                at<uint64_t>(workspace, L.sums), L.count_cap};
  uint32_t* fa = at<uint32_t>(workspace, L.flags_a);
  uint32_t* oa = at<uint32_t>(workspace, L.offs_a);
  uint32_t* fb = at<uint32_t>(workspace, L.flags_b);
  uint32_t* ob = at<uint32_t>(workspace, L.offs_b);
  int32_t* pair_cell = at<int32_t>(workspace, L.pair_cell);
  int32_t* pair_col = at<int32_t>(workspace, L.pair_col);
  uint32_t* pair_tri = at<uint32_t>(workspace, L.pair_tri);
  uint32_t* cell_first = at<uint32_t>(workspace, L.cell_first);
  uint32_t* cell_npairs = at<uint32_t>(workspace, L.cell_npairs);
  uint32_t* cell_pstart = at<uint32_t>(workspace, L.cell_pstart);
  uint32_t* row_of = at<uint32_t>(workspace, L.row_of);
  uint32_t* row_pairs = at<uint32_t>(workspace, L.row_pairs);
  // scalars: [0] unknown record, [1] kept groups, [2] pairs, [3] triples, [4] rows, [5] err
  uint64_t* sc = at<uint64_t>(workspace, L.scalars);
  HIPCHK(hipMemsetAsync(cell_first, 0xFF, sizeof(uint32_t) * (size_t)(nc ? nc : 1), s));
  HIPCHK(hipMemsetAsync(sc, 0xFF, sizeof(uint64_t), s));
  HIPCHK(hipMemsetAsync(sc + 1, 0, 5 * sizeof(uint64_t), s));
  CountCols c{in->cell, in->umi,     in->gene,       in->xf,         in->qhead,      in->gene_col, n,
              in->n_cell_ids, in->n_umi_ids, in->n_gene_ids, in->cell_none, in->umi_none, in->n_cols};
  // 1. molecule keys of the counted groups, compacted
  LAUNCH("count_groups", k_cm_groups, dim3((unsigned)cdiv(n, kBlock)), dim3(kBlock), s, c, K, B.kb, fa, cell_first,
         (unsigned long long*)sc, (uint32_t*)(sc + 5));
  int rc = scan_counts(fa, n, oa, B.sums, s);
  if (rc) return rc;
  LAUNCH("count_compact", k_cm_compact, dim3((unsigned)cdiv(n, kBlock)), dim3(kBlock), s, (const uint64_t*)B.kb,
         (const uint32_t*)fa, (const uint32_t*)oa, n, B.ka, B.va, sc + 1);
  uint64_t h[6];
  if (int rb = readback(h, sc, sizeof(h), s)) return rb;
  if (h[5]) return fail(SCT_EINVAL, "a dictionary id is outside its dictionary");
  if (h[0] != ~0ull) {
    out->unknown_record = (int64_t)h[0];
    return SCT_OK;
  }
  const int64_t m = (int64_t)h[1];
  out->n_sorted = m;
  int64_t nnz = 0, n_rows = 0;
  uint64_t n_triples = 0;
  if (m > 0) {
    // 2. sort; triples and (cell, column) pairs numbered by scans
    int which = 0;
    rc = radix_sort(B, m, K.total, &which, s);
    if (rc) return rc;
    const uint64_t* sorted = which ? B.kb : B.ka;
    const dim3 grid((unsigned)cdiv(m, kBlock));
    LAUNCH("count_heads", k_cm_heads, grid, dim3(kBlock), s, sorted, m, K, fa, fb);
    rc = scan_counts(fa, m, oa, B.sums, s);
    if (rc) return rc;
    rc = scan_counts(fb, m, ob, B.sums, s);
    if (rc) return rc;
    LAUNCH("count_emit", k_cm_emit, grid, dim3(kBlock), s, sorted, m, K, (const uint32_t*)fb, (const uint32_t*)ob,
           (const uint32_t*)fa, (const uint32_t*)oa, pair_cell, pair_col, pair_tri, cell_pstart, sc + 2);
    // 3. row order: counted cells by the record index of their first counted molecule
    LAUNCH("count_rowkeys", k_cm_rowkeys, dim3((unsigned)cdiv(nc, kBlock)), dim3(kBlock), s,
           (const uint32_t*)cell_first, (int32_t)nc, B.ka, B.va, sc + 4);
    if (int rb = readback(h, sc, sizeof(h), s)) return rb;
    nnz = (int64_t)h[2];
    n_triples = h[3];
    n_rows = (int64_t)h[4];
    LAUNCH("count_cells", k_cm_cells, dim3((unsigned)cdiv(nnz, kBlock)), dim3(kBlock), s, (const int32_t*)pair_cell,
           nnz, (const uint32_t*)cell_pstart, cell_npairs);
    rc = radix_sort(B, nc, 32, &which, s);
    if (rc) return rc;
    const uint32_t* cells = which ? B.vb : B.va;
    LAUNCH("count_rows", k_cm_rows, dim3((unsigned)cdiv(n_rows, kBlock)), dim3(kBlock), s, cells, n_rows,
           (const uint32_t*)cell_npairs, out->row_cell, row_of, row_pairs);
    rc = scan_counts(row_pairs, n_rows, (uint32_t*)out->indptr, B.sums, s);
    if (rc) return rc;
    LAUNCH("count_scatter", k_cm_scatter, dim3((unsigned)cdiv(nnz, kBlock)), dim3(kBlock), s, nnz, n_triples,
           (const int32_t*)pair_cell, (const int32_t*)pair_col, (const uint32_t*)pair_tri,
           (const uint32_t*)cell_pstart, (const uint32_t*)row_of, (const int32_t*)out->indptr, out->indices,
           out->data);
  }
  LAUNCH("count_tail", k_cm_set_tail, dim3(1), dim3(kWave), s, out->indptr, n_rows, nnz);
  HIPCHK(hipStreamSynchronize(s));
  out->n_rows = n_rows;
  out->nnz = nnz;
  return SCT_OK;
}

int sct_finalize_partials(int32_t mode, const int64_t* partials, int64_t rows, int64_t* out_ints, double* out_floats,
                          void* stream) {
  last_error().clear();
  if (mode < SCT_MODE_CELL || mode > SCT_MODE_GENE_GROUPED) return fail(SCT_EINVAL, "unknown mode %d", mode);
  if (rows < 0 || (rows > 0 && (!partials || !out_ints || !out_floats)))
    return fail(SCT_EINVAL, "bad finalize arguments");
  if (rows == 0) return SCT_OK;
  hipStream_t s = (hipStream_t)stream;
  LAUNCH("finalize", k_finalize, dim3((unsigned)cdiv(rows * kFinThreads, kBlock)), dim3(kBlock), s, partials, rows, (int)mode, 1,
         (const int64_t*)nullptr, out_ints, out_floats);
  return SCT_OK;
}

#ifdef SCT_W2_PROF  // experiments only: the Welford head kernel's per-wave barrier ticks (finalize.h)
int sct_debug_w2_prof(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(sct_w2_prof), sizeof(sct_w2_prof)) == hipSuccess ? 0 : -1;
}
#endif

}  // extern "C"
