// util.h -- host error/profiling plumbing and device helpers shared by the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <utility>
#include <vector>

#include "common.h"

namespace sct {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / kWave;

// ---------------- host: thread-local error string ----------------
inline std::string& last_error() {
  static thread_local std::string e;
  return e;
}

inline int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
inline int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  last_error() = buf;
  return code;
}

#define HIPCHK(expr)                                                                           \
  do {                                                                                         \
    hipError_t _e = (expr);                                                                    \
    if (_e != hipSuccess)                                                                      \
      return ::sct::fail(SCT_EHIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__, \
                         __LINE__);                                                            \
  } while (0)

#define LAUNCHCHK() HIPCHK(hipGetLastError())

// Small device -> host readbacks (run counts, level counters, error flags) between launches:
// copied through a pinned per-thread buffer, since a copy into pageable memory is staged by
// the runtime; then the stream is synchronized.
// The buffer belongs to the calling host thread and is freed when the thread exits.
struct PinnedReadback {
  static constexpr size_t kCap = 256;
  void* buf = nullptr;
  ~PinnedReadback() {
    if (buf) (void)hipHostFree(buf);
  }
};
inline int readback(void* dst, const void* src, size_t bytes, hipStream_t s) {
  static thread_local PinnedReadback rb;
  if (bytes > PinnedReadback::kCap)
    return fail(SCT_EINVAL, "readback of %zu bytes exceeds %zu", bytes, PinnedReadback::kCap);
  if (!rb.buf) HIPCHK(hipHostMalloc(&rb.buf, PinnedReadback::kCap, hipHostMallocPortable));
  HIPCHK(hipMemcpyAsync(rb.buf, src, bytes, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  memcpy(dst, rb.buf, bytes);
  return SCT_OK;
}

// The same readback split in two: the copy is queued (readback_start) and waited for later
// (readback_finish), so the kernels queued in between keep the device busy while the host
// waits for the copy.  One outstanding early readback per host thread.
struct EarlyReadback {
  void* buf = nullptr;
  hipEvent_t ev = nullptr;
  ~EarlyReadback() {
    if (buf) (void)hipHostFree(buf);
    if (ev) (void)hipEventDestroy(ev);
  }
};
inline EarlyReadback& early_readback() {
  static thread_local EarlyReadback rb;
  return rb;
}
inline int readback_start(const void* src, size_t bytes, hipStream_t s) {
  EarlyReadback& rb = early_readback();
  if (bytes > PinnedReadback::kCap)
    return fail(SCT_EINVAL, "readback of %zu bytes exceeds %zu", bytes, PinnedReadback::kCap);
  if (!rb.buf) HIPCHK(hipHostMalloc(&rb.buf, PinnedReadback::kCap, hipHostMallocPortable));
  if (!rb.ev) HIPCHK(hipEventCreateWithFlags(&rb.ev, hipEventDisableTiming));
  HIPCHK(hipMemcpyAsync(rb.buf, src, bytes, hipMemcpyDeviceToHost, s));
  HIPCHK(hipEventRecord(rb.ev, s));
  return SCT_OK;
}
inline int readback_finish(void* dst, size_t bytes) {
  EarlyReadback& rb = early_readback();
  HIPCHK(hipEventSynchronize(rb.ev));
  memcpy(dst, rb.buf, bytes);
  return SCT_OK;
}

// ---------------- host: optional per-kernel timing with HIP events ----------------
struct ProfEntry {
  std::string name;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;
  int64_t items = 0;  // items processed over the timed launches; -1 once a launch did not say
};
inline bool& prof_on() {
  static thread_local bool on = false;
  return on;
}
inline std::string& prof_only() {  // "" = every kernel
  static thread_local std::string name;
  return name;
}
inline bool prof_wants(const char* n) { return prof_on() && (prof_only().empty() || prof_only() == n); }
inline std::vector<ProfEntry>& prof_entries() {
  static thread_local std::vector<ProfEntry> v;
  return v;
}

// items: what the launch processes (records, payloads, sort items), for the algorithmic bytes per
// launch of the roofline; -1 when the launch does not say
struct ProfScope {
  hipEvent_t a = nullptr, b = nullptr;
  hipStream_t s;
  const char* name;
  int64_t items;
  ProfScope(const char* n, hipStream_t st, int64_t it = -1) : s(st), name(n), items(it) {
    if (prof_wants(n) && hipEventCreate(&a) == hipSuccess && hipEventCreate(&b) == hipSuccess)
      (void)hipEventRecord(a, s);
  }
  ~ProfScope() {
    if (!a || !b) return;
    (void)hipEventRecord(b, s);
    for (auto& e : prof_entries())
      if (e.name == name) {
        e.ev.emplace_back(a, b);
        e.items = (e.items < 0 || items < 0) ? -1 : e.items + items;
        return;
      }
    ProfEntry e{name, {{a, b}}};
    e.items = items;
    prof_entries().push_back(e);
  }
};

#define LAUNCH(name, kern, grid, block, strm, ...)               \
  do {                                                           \
    ::sct::ProfScope _ps(name, strm);                            \
    hipLaunchKernelGGL(kern, grid, block, 0, strm, __VA_ARGS__); \
  } while (0);                                                   \
  LAUNCHCHK()

// LAUNCH that records the items the launch processes (ProfScope)
#define LAUNCH_N(name, items, kern, grid, block, strm, ...)      \
  do {                                                           \
    ::sct::ProfScope _ps(name, strm, (int64_t)(items));          \
    hipLaunchKernelGGL(kern, grid, block, 0, strm, __VA_ARGS__); \
  } while (0);                                                   \
  LAUNCHCHK()

// Several small fills in one launch (round 5: the step issued ~10 hipMemsetAsync calls, each its
// own ~5 us kernel).  Span k gets the byte value val[k] (memset semantics); blockIdx.y picks the span,
// 16-byte stores where the span allows them.
constexpr int kFillSpans = 12;
struct FillSpans {
  uint8_t* p[kFillSpans];
  uint64_t bytes[kFillSpans];
  uint32_t val[kFillSpans];
  int n;
};
__global__ void __launch_bounds__(256) k_fill_spans(FillSpans f) {
  const int k = blockIdx.y;
  uint8_t* p = f.p[k];
  const uint64_t nb = f.bytes[k];
  const uint32_t v8 = f.val[k] & 0xffu;
  const uint32_t v = v8 * 0x01010101u;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t head = ((16 - ((uintptr_t)p & 15)) & 15) < nb ? ((16 - ((uintptr_t)p & 15)) & 15) : nb;
  if (i0 < head) p[i0] = (uint8_t)v8;
  const uint64_t nw = (nb - head) / 16;
  uint4* q = reinterpret_cast<uint4*>(p + head);
  for (uint64_t i = i0; i < nw; i += stride) q[i] = make_uint4(v, v, v, v);
  const uint64_t tail0 = head + nw * 16;
  if (i0 < nb - tail0) p[tail0 + i0] = (uint8_t)v8;
}
struct FillBatch {
  FillSpans f{};
  uint64_t most = 0;
  bool overflow = false;  // a span past kFillSpans: launch_fills fails instead of dropping it
  void add(void* p, size_t bytes, uint8_t val = 0) {
    if (!bytes) return;
    if (f.n >= kFillSpans) {
      overflow = true;
      return;
    }
    f.p[f.n] = static_cast<uint8_t*>(p);
    f.bytes[f.n] = bytes;
    f.val[f.n] = val;
    f.n++;
    most = bytes > most ? bytes : most;
  }
  bool full() const { return f.n == kFillSpans; }
};

// with `shm` bytes of dynamic LDS (sct_dyn_lds)
#define LAUNCH_SHM(name, kern, grid, block, shm, strm, ...)        \
  do {                                                             \
    ::sct::ProfScope _ps(name, strm);                              \
    hipLaunchKernelGGL(kern, grid, block, shm, strm, __VA_ARGS__); \
  } while (0);                                                     \
  LAUNCHCHK()

#define LAUNCH_SHM_N(name, items, kern, grid, block, shm, strm, ...) \
  do {                                                               \
    ::sct::ProfScope _ps(name, strm, (int64_t)(items));              \
    hipLaunchKernelGGL(kern, grid, block, shm, strm, __VA_ARGS__);   \
  } while (0);                                                       \
  LAUNCHCHK()

inline int bitlen(uint64_t v) {  // bits for ids 0..v-1; 0 when v <= 1
  return v <= 1 ? 0 : 64 - __builtin_clzll(v - 1);
}
inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

template <typename T>
inline T* at(void* ws, size_t off) {
  return reinterpret_cast<T*>(static_cast<char*>(ws) + off);
}

// ---------------- device helpers ----------------
// dynamic LDS of a launch (sized per launch: gene-bucket arrays follow the dictionary size)
extern __shared__ uint32_t sct_dyn_lds[];
constexpr unsigned kXcds = 8;  // MI355X: 8 XCDs, each with its own (non-coherent) 4 MiB L2

// Workgroups are dispatched round-robin over the XCDs (block b -> XCD b % 8).  Map them to
// logical tiles so that each XCD owns one contiguous range of tiles: neighbouring tiles
// (same entity, same record-index window) then share an L2, so scattered writes and
// gathers into that window combine there instead of leaving partial lines in 8 L2s.
__device__ __forceinline__ unsigned xcd_tile(unsigned b, unsigned n) {
  const unsigned x = b % kXcds, i = b / kXcds;
  const unsigned per = n / kXcds, rem = n % kXcds;
  return x * per + (x < rem ? x : rem) + i;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
  for (int off = kWave / 2; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

// exclusive scan over the kBlock threads of the block; *total gets the block sum.
// `lds` needs kWaves + 1 entries.  Contains barriers: call from every thread.
template <typename T>
__device__ __forceinline__ T block_exclusive_scan(T v, T* total, T* lds) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  T x = v;
  for (int off = 1; off < kWave; off <<= 1) {
    T y = __shfl_up(x, off);
    if (lane >= off) x += y;
  }
  if (lane == kWave - 1) lds[wid] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    T run = 0;
    for (int w = 0; w < kWaves; w++) {
      T t = lds[w];
      lds[w] = run;
      run += t;
    }
    lds[kWaves] = run;
  }
  __syncthreads();
  T res = lds[wid] + x - v;
  *total = lds[kWaves];
  __syncthreads();
  return res;
}

// block_exclusive_scan for a block of NT threads; `lds` needs NT / 64 + 1 entries.
template <int NT, typename T>
__device__ __forceinline__ T block_exclusive_scan_n(T v, T* total, T* lds) {
  constexpr int W = NT / kWave;
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  T x = v;
  for (int off = 1; off < kWave; off <<= 1) {
    T y = __shfl_up(x, off);
    if (lane >= off) x += y;
  }
  if (lane == kWave - 1) lds[wid] = x;
  __syncthreads();
  if (threadIdx.x < kWave) {  // wave 0 scans the W wave totals
    T w = threadIdx.x < W ? lds[threadIdx.x] : (T)0;
    T s = w;
    for (int off = 1; off < W; off <<= 1) {
      T y = __shfl_up(s, off);
      if ((int)threadIdx.x >= off) s += y;
    }
    if (threadIdx.x < W) lds[threadIdx.x] = s - w;
    if (threadIdx.x == W - 1) lds[W] = s;
  }
  __syncthreads();
  T res = lds[wid] + x - v;
  *total = lds[W];
  __syncthreads();
  return res;
}

// exclusive max-scan (values >= 0) for a block of NT threads; `lds` needs NT / 64 entries
template <int NT>
__device__ __forceinline__ uint32_t block_exclusive_max_n(uint32_t v, uint32_t* lds) {
  constexpr int W = NT / kWave;
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
  (void)W;
  return ex > carry ? ex : carry;
}

// a / b of two small non-negative integers, correctly rounded (Python int / int);
// 0 for b == 0 (only reached by records the reference never aggregates)
__device__ __forceinline__ double ratio(uint32_t a, uint32_t b) { return b ? (double)a / (double)b : 0.0; }

// The same RN(a / b) without a division instruction sequence (the f64 divide is ~10 dependent
// ops including v_rcp_f64 / v_div_scale / v_div_fixup, and dominated the quality streams):
// with y = RN(1/b) from a table, q0 = RN(a*y), the residual r = a - q0*b is exact (one FMA),
// and q = RN(q0 + r*y) is the correctly rounded quotient.  Checked bit-identical to IEEE a / b
// for every a, b < 2^16 (tests/native/divcheck.c), which covers all uint8 / uint16 columns.
constexpr int kRcpN = 256;  // table of 1/b for b < kRcpN (LDS); larger b divide once
__device__ __forceinline__ void fill_rcp(double* s_rcp) {
  for (int i = threadIdx.x; i < kRcpN; i += blockDim.x) s_rcp[i] = i ? 1.0 / (double)i : 0.0;
}
__device__ __forceinline__ double rcp_of(uint32_t b, const double* s_rcp) {  // RN(1 / b); 0 for b == 0
  return b < (uint32_t)kRcpN ? s_rcp[b] : 1.0 / (double)b;
}
// RN(a / b) from y = RN(1 / b); 0 when y == 0 (b == 0: the table's entry 0)
__device__ __forceinline__ double ratio_y(uint32_t a, uint32_t b, double y) {
  const double da = (double)a, db = (double)b;
  const double q0 = da * y;
  const double r = __fma_rn(-q0, db, da);
  return __fma_rn(r, y, q0);
}
__device__ __forceinline__ double ratio_rcp(uint32_t a, uint32_t b, const double* s_rcp) {
  if (b == 0) return 0.0;
  return ratio_y(a, b, rcp_of(b, s_rcp));
}

__device__ __forceinline__ uint32_t frag_hash(int32_t ref, int32_t pos, uint32_t strand) {
  uint32_t h = (uint32_t)ref * 0x9E3779B1u ^ ((uint32_t)pos * 0x85EBCA77u) ^ (strand * 0xC2B2AE3Du);
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  h *= 0x297A2D39u;
  h ^= h >> 15;
  return h;
}

}  // namespace sct

namespace sct {

// Wave-cooperative flush of per-lane partial sums into int64 rows.
//
// Lanes with `member` set hold partial sums v[0..K) for entity `e` (per lane).  For every
// distinct entity among the members (a wave-uniform loop; one iteration when the wave
// is inside one entity), the members' values are summed across the wave and lanes
// 0..K-1 add slot SlotOf(i) of that entity's row with ONE atomic instruction (K
// contiguous-ish int64 adds) instead of K single-lane instructions per lane.
// Members' v[] are cleared.  Every lane of the wave must call it.
// DPP wave reduction (GFX9 quad_perm / row_shr / row_bcast): the sum of all 64 lanes, returned
// uniformly.  Every lane must be active.  No LDS traffic, unlike __shfl_xor (ds_bpermute).
template <int kCtrl, int kRowMask>
__device__ __forceinline__ int32_t dpp_i32(int32_t v) {
  return __builtin_amdgcn_update_dpp(0, v, kCtrl, kRowMask, 0xf, false);
}
__device__ __forceinline__ int32_t wave_sum_dpp(int32_t v) {
  v += dpp_i32<0xb1, 0xf>(v);   // quad_perm [1,0,3,2]
  v += dpp_i32<0x4e, 0xf>(v);   // quad_perm [2,3,0,1]
  v += dpp_i32<0x114, 0xf>(v);  // row_shr:4
  v += dpp_i32<0x118, 0xf>(v);  // row_shr:8  -> lane 15 of each row holds the row sum
  v += dpp_i32<0x142, 0xa>(v);  // row_bcast:15 -> lanes 31 / 63 hold two-row sums
  v += dpp_i32<0x143, 0xc>(v);  // row_bcast:31 -> lane 63 holds the wave sum
  return __builtin_amdgcn_readlane(v, 63);
}
template <int kCtrl, int kRowMask>
__device__ __forceinline__ int64_t dpp_i64(int64_t v) {
  const uint32_t lo = (uint32_t)dpp_i32<kCtrl, kRowMask>((int32_t)(uint32_t)v);
  const uint32_t hi = (uint32_t)dpp_i32<kCtrl, kRowMask>((int32_t)(uint32_t)((uint64_t)v >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
template <int kCtrl, int kRowMask, typename T>
__device__ __forceinline__ T dpp_val(T v) {
  if constexpr (sizeof(T) == 8) return (T)dpp_i64<kCtrl, kRowMask>((int64_t)v);
  else return (T)dpp_i32<kCtrl, kRowMask>((int32_t)v);
}
__device__ __forceinline__ int64_t wave_sum_dpp(int64_t v) {
  v += dpp_i64<0xb1, 0xf>(v);
  v += dpp_i64<0x4e, 0xf>(v);
  v += dpp_i64<0x114, 0xf>(v);
  v += dpp_i64<0x118, 0xf>(v);
  v += dpp_i64<0x142, 0xa>(v);
  v += dpp_i64<0x143, 0xc>(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int32_t)(uint32_t)v, 63);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int32_t)(uint32_t)((uint64_t)v >> 32), 63);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

// Sum over the wave of an int64 value with |v| < 2^49 on every lane: the low 24 bits and the
// (arithmetic) rest are summed as two int32 DPP reductions, which cannot overflow (64 lanes:
// < 2^30 and < 2^31), instead of a carry-propagating 64-bit DPP add per step.
__device__ __forceinline__ int64_t wave_sum_dpp_split(int64_t v) {
  const int32_t lo = (int32_t)(v & 0xFFFFFF);
  const int32_t hi = (int32_t)(v >> 24);
  return (int64_t)wave_sum_dpp(lo) + ((int64_t)wave_sum_dpp(hi) << 24);
}

// Wave-cooperative flush of per-lane partial sums into int64 rows.
//
// Lanes with `member` set hold partial sums v[0..K) for entity `e` (per lane).  For every
// distinct entity among the members (a wave-uniform loop; one iteration when the wave
// is inside one entity), the members' values are summed across the wave (DPP) and lanes
// 0..K-1 add slot SlotOf(i) of that entity's row with ONE atomic instruction instead of K
// single-lane instructions per lane.  Members' v[] are cleared.  Every lane of the wave must
// call it with all lanes active.  T = int32_t, or int64_t with |v| < 2^49 per lane (the key
// pass's fixed-point lanes: < 2^45 for 32 records).
template <int K, typename T, typename SlotOf>
__device__ __forceinline__ void wave_flush(T (&v)[K], bool member, int64_t e, int64_t* __restrict__ rows,
                                           SlotOf slot_of) {
  static_assert(K <= kWave, "one lane per slot");
  const int lane = threadIdx.x & (kWave - 1);
  uint64_t pending = __ballot(member);
  while (pending) {
    const int lead = __ffsll((unsigned long long)pending) - 1;
    const int64_t el = __shfl(e, lead);
    const bool in = member && e == el;
    int64_t mine = 0;
#pragma unroll
    for (int i = 0; i < K; i++) {
      T tot;
      if constexpr (sizeof(T) == 8) tot = (T)wave_sum_dpp_split(in ? (int64_t)v[i] : 0);
      else tot = wave_sum_dpp(in ? v[i] : (T)0);
      mine = (lane == i) ? (int64_t)tot : mine;
    }
    if (lane < K && mine) atomicAdd((unsigned long long*)&rows[el * SCT_NP + slot_of(lane)], (unsigned long long)mine);
    if (in) {
#pragma unroll
      for (int i = 0; i < K; i++) v[i] = 0;
    }
    pending &= ~__ballot(in);
  }
}


// wave_flush for small non-negative int32 counters (every lane's v[i] < 2^10, so a field's wave sum
// stays below 2^16): two counters per 32-bit word, one DPP reduction per word -- half the
// reductions of wave_flush (the key pass's 13 record counters, flushed at every run boundary).
template <int K, typename SlotOf>
__device__ __forceinline__ void wave_flush_packed16(int32_t (&v)[K], bool member, int64_t e,
                                                    int64_t* __restrict__ rows, SlotOf slot_of) {
  static_assert(K <= kWave, "one lane per slot");
  constexpr int W = (K + 1) / 2;
  const int lane = threadIdx.x & (kWave - 1);
  uint64_t pending = __ballot(member);
  while (pending) {
    const int lead = __ffsll((unsigned long long)pending) - 1;
    const int64_t el = __shfl(e, lead);
    const bool in = member && e == el;
    int32_t tot[W];
#pragma unroll
    for (int w = 0; w < W; w++) {
      const uint32_t lo = in ? (uint32_t)v[2 * w] : 0u;
      const uint32_t hi = (in && 2 * w + 1 < K) ? (uint32_t)v[2 * w + 1] : 0u;
      tot[w] = wave_sum_dpp((int32_t)(lo | (hi << 16)));
    }
    int64_t mine = 0;
#pragma unroll
    for (int i = 0; i < K; i++) mine = (lane == i) ? (int64_t)(((uint32_t)tot[i / 2] >> (16 * (i % 2))) & 0xffffu) : mine;
    if (lane < K && mine) atomicAdd((unsigned long long*)&rows[el * SCT_NP + slot_of(lane)], (unsigned long long)mine);
    if (in) {
#pragma unroll
      for (int i = 0; i < K; i++) v[i] = 0;
    }
    pending &= ~__ballot(in);
  }
}

}  // namespace sct

namespace sct {
inline int launch_fills(FillBatch& fb, hipStream_t s) {
  if (fb.overflow) return fail(SCT_EINVAL, "internal: more than %d fill spans in one batch", kFillSpans);
  if (!fb.f.n) return SCT_OK;
  uint64_t blocks = (fb.most / 16 + 255) / 256;
  blocks = blocks < 1 ? 1 : (blocks > 2048 ? 2048 : blocks);
  LAUNCH("fill", k_fill_spans, dim3((unsigned)blocks, (unsigned)fb.f.n), dim3(256), s, fb.f);
  fb = FillBatch{};
  return SCT_OK;
}
}  // namespace sct
