// gbam.hip -- BAM -> columnar decode on the device (include/sct_gbam.h): libsct_gbam.so.
//
//   1. host: map the file, hop the BGZF member headers (bgzf.h scan_blocks), inflate the first
//      member(s) with zlib only far enough to find where the header ends (H);
//   2. copy the compressed file to HBM once; k_inflate (inflate.h): one wave per member, every
//      payload lands at its prefix-sum offset in one contiguous buffer U;
//   3. record starts: k_guess picks, per member, the first offset from which four records chain
//      plausibly; k_walk follows block_size from each member's start to the first start in the
//      next member; a guess that disagrees with the previous member's landing is replaced by it
//      and the walk repeats (the member holding H starts exactly, so agreement everywhere proves
//      every start by induction); a second walk writes the record offsets;
//   4. k_parse: one lane per record -- the validation and fields of bamdec.cpp parse_record
//      (sct_bam.h), and CB / UB / GE interned in open-addressing tables (one 64-bit CAS per
//      insert: the string's offset in U, its length and 16 hash bits); k_parse_count: the
//      count-matrix mode (three named tags, XF, the query-name group head);
//   5. per dictionary the occupied slots are compacted, the distinct strings packed and copied to
//      the host, sorted there (Python's sorted() order, the missing tag first) and the rank of
//      every slot copied back; k_remap turns slot ids into ranks.
// Anything the device path does not reproduce exactly returns SCT_GBAM_HOST (the caller decodes
// with sct_bam_decode, whose first-offending-record error is the reference's exception).
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <hipcub/hipcub.hpp>
#include <memory>
#include <string>
#include <string_view>
#include <thread>
#include <vector>

#include "../../include/sct_bam.h"
#include "../../include/sct_gbam.h"
#include "bgzf.h"
#include "inflate.h"

namespace gb {

constexpr uint64_t kUnknown = ~0ull, kBadWalk = ~0ull - 1;
constexpr uint32_t kScan = 1u << 18;  // bytes a member's start guess looks through
constexpr int kStartRounds = 512;      // record-start repair rounds before the file goes to the host decoder
constexpr uint64_t kPad = 1u << 16;   // readable bytes after the file image and after U

__device__ __forceinline__ uint32_t u16(const uint8_t* U, uint64_t p) { return U[p] | (uint32_t)U[p + 1] << 8; }
__device__ __forceinline__ uint32_t u32(const uint8_t* U, uint64_t p) {
  return U[p] | (uint32_t)U[p + 1] << 8 | (uint32_t)U[p + 2] << 16 | (uint32_t)U[p + 3] << 24;
}

// four records chain from p the way alignment records do (SAM/BAM spec 4.2): a hint only --
// k_walk's agreement check decides
// open_end: U ends inside a record that continues in the next window (a chain reaching the end
// cannot be disproved)
// (every field is checked before a record running past U is accepted, so an arbitrary offset whose
// first four bytes read as a huge block_size does not pass for a start at an open end; U has kPad
// readable bytes past ulen)
__device__ bool plausible(const uint8_t* U, uint64_t ulen, uint64_t p, bool open_end) {
  for (int j = 0; j < 4; j++) {
    if (p == ulen) return true;
    if (p + 36 > ulen) return open_end && j > 0;
    const uint32_t bs = u32(U, p);
    if (bs < 33 || bs > (1u << 28)) return false;
    const uint64_t d = p + 4;
    if ((int32_t)u32(U, d) < -1 || (int32_t)u32(U, d + 4) < -1) return false;
    const uint32_t lrn = U[d + 8];
    if (lrn == 0 || 32 + lrn > bs) return false;
    if (d + 32 + lrn > ulen) return open_end && j > 0;
    if (U[d + 32 + lrn - 1] != 0) return false;
    for (uint32_t q = 0; q + 1 < lrn; q++) {
      const uint32_t c = U[d + 32 + q];
      if (c < 33 || c > 126) return false;
    }
    const uint64_t need = 32ull + lrn + 4ull * u16(U, d + 12) + (u32(U, d + 16) + 1ull) / 2 + u32(U, d + 16);
    if (need > bs) return false;
    if (p + 4 + bs > ulen) return open_end;  // the rest of this record is in the next window
    p = d + bs;
  }
  return true;
}

// S[m] for members mH < m < n_mem: the first plausible record start at or after O[m] (member mH
// too when H is kUnknown: a part's first record, proven later against the previous part's walk).
// check_end: the walk must land exactly on ulen (S[n_mem]); else the end is found, not checked.
// open_end: U ends inside a record that continues in the next window.
__global__ void k_guess(const uint8_t* __restrict__ U, uint64_t ulen, const uint64_t* __restrict__ O, uint32_t mH,
                        uint32_t n_mem, uint64_t H, uint64_t* __restrict__ S, uint32_t open_end, uint32_t check_end) {
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m == 0) S[n_mem] = check_end ? ulen : kUnknown;
  if (m < mH || m >= n_mem) return;
  if (m == mH && H != kUnknown) {
    S[m] = H;
    return;
  }
  const uint64_t p0 = O[m];
  uint64_t s = p0 >= ulen ? ulen : kUnknown;
  const uint64_t e = min(ulen, p0 + kScan);
  for (uint64_t p = p0; p < e; p++)
    if (plausible(U, ulen, p, open_end != 0)) {
      s = p;
      break;
    }
  S[m] = s;
}

// Walk member m's records from S[m] up to the first start at or after O[m+1]: cnt[m] records,
// land[m+1] the landing (kBadWalk: a record runs past U), last[m] the start of its last record.
// With `starts`, write the offsets.  open_end: a walk stops at a record running past U (it continues
// in the next window) and lands on its start.
__global__ void k_walk(const uint8_t* __restrict__ U, uint64_t ulen, const uint64_t* __restrict__ O, uint32_t mH,
                       uint32_t n_mem, const uint64_t* __restrict__ S, uint32_t* __restrict__ cnt,
                       uint64_t* __restrict__ land, uint64_t* __restrict__ starts, const uint64_t* __restrict__ base,
                       uint64_t* __restrict__ last, uint32_t open_end) {
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= n_mem) return;
  if (m < mH) {
    cnt[m] = 0;
    land[m + 1] = kUnknown;
    if (last) last[m] = kUnknown;
    return;
  }
  uint64_t p = S[m];
  if (p == kUnknown) {
    cnt[m] = 0;
    land[m + 1] = kUnknown;
    if (last) last[m] = kUnknown;
    return;
  }
  const uint64_t end = O[m + 1];
  const bool open = open_end != 0;  // (a long record may cut through several members)
  uint32_t n = 0;
  uint64_t lp = kUnknown;
  uint64_t* out = starts ? starts + base[m] : nullptr;
  while (p < end) {
    if (p + 4 > ulen) {
      p = open ? p : kBadWalk;
      break;
    }
    const uint64_t bs = u32(U, p);
    if (p + 4 + bs > ulen) {
      p = open ? p : kBadWalk;
      break;
    }
    if (out) out[n] = p;
    lp = p;
    n++;
    p += 4 + bs;
  }
  cnt[m] = n;
  land[m + 1] = p;
  if (last) last[m] = lp;
}

// ag[m]: member m's start agrees with its predecessor's landing this round (mH: exact by
// construction).  Computed before k_fix rewrites any start.
__global__ void k_agree(uint32_t mH, uint32_t n_mem, const uint64_t* __restrict__ S,
                        const uint64_t* __restrict__ land, uint8_t* __restrict__ ag) {
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m > n_mem) return;
  ag[m] = m < mH ? 0 : (m == mH || land[m] == S[m]) ? 1 : 0;
}

// Replace a start that disagrees with its predecessor's landing -- only when the predecessor's own
// start agreed (a landing walked from a wrong start would carry the error forward one member per
// round); count the disagreements (S[n_mem] = ulen is fixed: a landing elsewhere stays one).
// Each round the agreeing prefix from mH grows past at least one more member, and a run of k
// wrong guesses takes k rounds.
__global__ void k_fix(uint32_t mH, uint32_t n_mem, uint64_t* __restrict__ S, const uint64_t* __restrict__ land,
                      const uint8_t* __restrict__ ag, uint32_t* __restrict__ n_bad) {
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m <= mH || m > n_mem) return;
  const uint64_t l = land[m];
  if (l == S[m]) return;
  if (m == n_mem && S[m] == kUnknown) return;  // an open end (the record continues in the next window)
  if (m < n_mem && ag[m - 1] && l != kUnknown && l != kBadWalk) S[m] = l;
  atomicAdd(n_bad, 1u);
}

__global__ void k_u32_to_u64(const uint32_t* __restrict__ a, uint64_t* __restrict__ b, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) b[i] = a[i];
}

__global__ void k_any(const uint32_t* __restrict__ st, uint32_t n, uint32_t* __restrict__ flag) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && st[i] != ST_OK) atomicOr(flag, 1u << (st[i] & 15));
}

// ---------------- record parse ----------------
// bits / xf codes: include/sctools_gpu.h, sctools_amd/columnar.py
enum : uint32_t {
  B_UNMAPPED = 1u << 0, B_REVERSE = 1u << 1, B_DUPLICATE = 1u << 2, B_SPLICED = 1u << 3, B_NH1 = 1u << 4,
  B_PERFECT_UMI = 1u << 5, B_HAS_CB = 1u << 6, B_PERFECT_CB = 1u << 7
};
enum : uint32_t { XF_ABSENT = 0, XF_CODING, XF_INTRONIC, XF_UTR, XF_INTERGENIC, XF_OTHER };
enum : uint32_t { TV_NONE = 0, TV_STR = 1, TV_INT = 2, TV_RAW = 3 };

struct Cols {
  int32_t *cell, *umi, *gene, *ref, *pos;
  uint16_t *gq_sum, *gq_len, *gq_gt30;
  uint8_t *bits, *xf, *cy_gt30, *cy_len, *uy_gt30, *uy_len;
};

// Interning tables.  An entry is (off << 28) | (len << 16) | 16 hash bits, off 35 bits, bit 63
// set when the string lies in the window payload U (else in the arena A, where k_promote moves the
// strings a window inserted before its payload is replaced).  Inserts of a window are listed in
// newl[k] (newc[2k] entries, newc[2k + 1] bytes) for k_promote; newl null: no list (one window).
struct Dicts {
  unsigned long long* table[3];
  uint64_t mask[3];
  const uint8_t* A;
  uint32_t* newl[3];
  unsigned long long* newc;
};
constexpr unsigned long long kInU = 1ull << 63;
__device__ __forceinline__ uint64_t ent_off(unsigned long long e) { return (e & ~kInU) >> 28; }
__device__ __forceinline__ uint32_t ent_len(unsigned long long e) { return (uint32_t)(e >> 16) & 0xfff; }
__device__ __forceinline__ const uint8_t* ent_src(unsigned long long e, const uint8_t* U, const uint8_t* A) {
  return (e & kInU) ? U : A;
}

struct DTag {
  uint32_t kind;  // TV_*
  uint64_t off;   // value bytes in U (strings)
  uint32_t n;     // string length
  int64_t i;      // integer value
};

__device__ __forceinline__ bool str_eq(const uint8_t* U, uint64_t a, uint64_t b, uint32_t n) {
  for (uint32_t k = 0; k < n; k++)
    if (U[a + k] != U[b + k]) return false;
  return true;
}
// Python == of two present tag values where at least one is a string
__device__ __forceinline__ bool val_eq_str(const uint8_t* U, const DTag& a, const DTag& b) {
  return a.kind == TV_STR && b.kind == TV_STR && a.n == b.n && str_eq(U, a.off, b.off, a.n);
}
__device__ __forceinline__ bool lit_eq(const uint8_t* U, const DTag& v, const char* s, uint32_t n) {
  if (v.n != n) return false;
  for (uint32_t k = 0; k < n; k++)
    if (U[v.off + k] != (uint8_t)s[k]) return false;
  return true;
}

// bytes of a tag value of type t at U[p..end) (bgzf.h read_tag), 0 = unknown type or truncated
__device__ uint32_t tag_value(const uint8_t* U, uint64_t p, uint64_t end, uint32_t t, DTag* v) {
  const uint64_t room = end > p ? end - p : 0;
  uint32_t w = 0;
  switch (t) {
    case 'Z':
    case 'H': {
      uint64_t q = p;
      while (q < end && U[q]) q++;
      if (q >= end) return 0;
      if (v) v->kind = TV_STR, v->off = p, v->n = (uint32_t)(q - p);
      return (uint32_t)(q - p + 1);
    }
    case 'A':
      if (room < 1) return 0;
      if (v) v->kind = TV_STR, v->off = p, v->n = 1;
      return 1;
    case 'c': case 'C': w = 1; break;
    case 's': case 'S': w = 2; break;
    case 'i': case 'I': case 'f': w = 4; break;
    case 'd': w = 8; break;
    case 'B': {
      if (room < 5) return 0;
      const uint32_t sub = U[p];
      const uint32_t ew = (sub == 'c' || sub == 'C') ? 1 : (sub == 's' || sub == 'S') ? 2
                        : (sub == 'i' || sub == 'I' || sub == 'f') ? 4 : 0;
      if (!ew) return 0;
      const uint64_t len = 5 + (uint64_t)u32(U, p + 1) * ew;
      if (len > room) return 0;
      if (v) v->kind = TV_RAW, v->off = p, v->n = 0;
      return (uint32_t)len;
    }
    default:
      return 0;
  }
  if (w > room) return 0;
  if (v) {
    v->off = p, v->n = 0;
    switch (t) {
      case 'c': v->kind = TV_INT, v->i = (int8_t)U[p]; break;
      case 'C': v->kind = TV_INT, v->i = U[p]; break;
      case 's': v->kind = TV_INT, v->i = (int16_t)u16(U, p); break;
      case 'S': v->kind = TV_INT, v->i = u16(U, p); break;
      case 'i': v->kind = TV_INT, v->i = (int32_t)u32(U, p); break;
      case 'I': v->kind = TV_INT, v->i = u32(U, p); break;
      default: v->kind = TV_RAW; break;
    }
  }
  return w;
}

__device__ __forceinline__ uint64_t hash_str(const uint8_t* U, uint64_t off, uint32_t n) {
  uint64_t h = 1469598103934665603ull;
  for (uint32_t k = 0; k < n; k++) h = (h ^ U[off + k]) * 1099511628211ull;
  h ^= h >> 29;
  h *= 0xBF58476D1CE4E5B9ull;
  h ^= h >> 32;
  return h;
}

__device__ __forceinline__ bool str_eq2(const uint8_t* X, uint64_t a, const uint8_t* U, uint64_t b, uint32_t n) {
  for (uint32_t k = 0; k < n; k++)
    if (X[a + k] != U[b + k]) return false;
  return true;
}

// slot id of the string U[off, off+n) (inserted if new); -1: not internable here (host)
__device__ int32_t intern(const Dicts& D, int k, const uint8_t* U, uint64_t off, uint32_t n) {
  unsigned long long* __restrict__ table = D.table[k];
  const uint64_t mask = D.mask[k];
  if (n > 4095 || off >= (1ull << 35)) return -1;
  for (uint32_t j = 0; j < n; j++)
    if (U[off + j] >= 0x80) return -1;  // "replace"-decoded bytes: ranked on the host path
  const uint64_t h = hash_str(U, off, n);
  const uint64_t tag = (h >> 48) | 1;  // never 0 with off, n -- the empty slot is 0
  const unsigned long long mine = kInU | (off << 28) | ((uint64_t)n << 16) | tag;
  uint64_t slot = h & mask;
  while (true) {
    unsigned long long cur = __hip_atomic_load(&table[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == 0) {
      const unsigned long long prev = atomicCAS(&table[slot], 0ull, mine);
      if (prev == 0) {
        if (D.newl[k]) {  // listed for k_promote
          D.newl[k][atomicAdd(&D.newc[2 * k], 1ull)] = (uint32_t)slot;
          atomicAdd(&D.newc[2 * k + 1], (unsigned long long)n);
        }
        return (int32_t)slot;
      }
      cur = prev;
    }
    if ((cur & 0xffff) == tag && ent_len(cur) == n && str_eq2(ent_src(cur, U, D.A), ent_off(cur), U, off, n))
      return (int32_t)slot;
    slot = (slot + 1) & mask;
  }
}

// The strings a window inserted move to the arena (its payload is about to be replaced): entry i of
// the list gets arena bytes at *cursor (any order) and its table entry is rewritten to point there.
__global__ void k_promote(unsigned long long* __restrict__ table, const uint32_t* __restrict__ list, uint64_t n_new,
                          const uint8_t* __restrict__ U, uint8_t* __restrict__ A,
                          unsigned long long* __restrict__ cursor) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_new) return;
  const uint32_t slot = list[i];
  const unsigned long long e = table[slot];
  const uint32_t n = ent_len(e);
  const uint64_t src = ent_off(e);
  const uint64_t dst = atomicAdd(cursor, (unsigned long long)n);
  for (uint32_t k = 0; k < n; k++) A[dst + k] = U[src + k];
  table[slot] = (dst << 28) | (e & 0xfffffffull);
}

// A table grown to twice (or more) its capacity: every entry re-inserted (its hash recomputed from
// its bytes), map[old slot] = new slot, for k_remap_slots over the columns already written.
__global__ void k_rehash(const unsigned long long* __restrict__ old, uint64_t old_cap,
                         unsigned long long* __restrict__ tab, uint64_t mask, const uint8_t* __restrict__ U,
                         const uint8_t* __restrict__ A, int32_t* __restrict__ map) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= old_cap) return;
  const unsigned long long e = old[i];
  if (!e) return;
  const uint64_t h = hash_str(ent_src(e, U, A), ent_off(e), ent_len(e));
  uint64_t slot = h & mask;
  while (atomicCAS(&tab[slot], 0ull, e) != 0ull) slot = (slot + 1) & mask;  // every entry is distinct
  map[i] = (int32_t)slot;
}
__global__ void k_apply_map(int32_t* __restrict__ col, uint64_t n, const int32_t* __restrict__ map) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) col[i] = map[col[i]];
}
__global__ void k_remap_slots(int32_t* __restrict__ col, uint64_t n, const int32_t* __restrict__ map) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t v = col[i];
  if (v >= 0) col[i] = map[v];
}

// One lane per record: bamdec.cpp parse_record (same checks, same order of outcomes); any
// record the host would reject or key differently sets *host.
__global__ void k_parse(const uint8_t* __restrict__ U, const uint64_t* __restrict__ starts, uint64_t n,
                        uint32_t is_cell, Cols C, Dicts D, uint32_t* __restrict__ flags) {
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const uint64_t p = starts[r];
  const uint32_t bs = u32(U, p);
  const uint64_t d = p + 4;
  bool host = false;
  do {
    if (bs < 32) { host = true; break; }
    const int32_t ref = (int32_t)u32(U, d), pos = (int32_t)u32(U, d + 4);
    const uint32_t lrn = U[d + 8];
    const uint32_t n_cigar = u16(U, d + 12), flag = u16(U, d + 14);
    const uint32_t l_seq = u32(U, d + 16);
    const uint64_t cig = d + 32 + lrn;
    const uint64_t qual = cig + 4ull * n_cigar + (l_seq + 1ull) / 2;
    const uint64_t tag0 = qual + l_seq;
    const uint64_t end = d + bs;
    if (tag0 > end) { host = true; break; }
    DTag cb{}, cr{}, cy{}, ub{}, ur{}, uy{}, ge{}, xf{}, nh{};
    uint64_t q = tag0;
    while (q + 3 <= end) {
      const uint32_t a = U[q], b = U[q + 1], t = U[q + 2];
      q += 3;
      DTag v{};
      const uint32_t used = tag_value(U, q, end, t, &v);
      if (!used) { host = true; break; }
      q += used;
      const uint32_t ab = a << 8 | b;
      if (ab == ('C' << 8 | 'B')) cb = v;
      else if (ab == ('C' << 8 | 'R')) cr = v;
      else if (ab == ('C' << 8 | 'Y')) cy = v;
      else if (ab == ('U' << 8 | 'B')) ub = v;
      else if (ab == ('U' << 8 | 'R')) ur = v;
      else if (ab == ('U' << 8 | 'Y')) uy = v;
      else if (ab == ('G' << 8 | 'E')) ge = v;
      else if (ab == ('X' << 8 | 'F')) xf = v;
      else if (ab == ('N' << 8 | 'H')) nh = v;
    }
    if (host) break;
    // dictionary values other than strings are keyed by the host path
    if ((cb.kind && cb.kind != TV_STR) || (ub.kind && ub.kind != TV_STR) || (ge.kind && ge.kind != TV_STR)) {
      host = true;
      break;
    }
    bool validate = is_cell;
    if (!is_cell) {
      bool comma = false;
      for (uint32_t k = 0; k < ge.n && ge.kind; k++) comma |= U[ge.off + k] == ',';
      validate = !comma;
    }
    uint32_t bits = 0, cg = 0, cl = 0, ug = 0, ul = 0;
    if (is_cell) {
      if (cy.kind != TV_STR || cy.n == 0) { host = true; break; }
      for (uint32_t k = 0; k < cy.n; k++) cg += U[cy.off + k] > 63;
      cl = cy.n;
      if (cb.kind) {
        bits |= B_HAS_CB;
        if (!cr.kind) { host = true; break; }
        if (val_eq_str(U, cr, cb)) bits |= B_PERFECT_CB;
      }
    } else if (cb.kind) {
      bits |= B_HAS_CB;
    }
    bool do_uy = validate;
    if (!validate && uy.kind) {
      if (uy.kind == TV_STR) do_uy = uy.n > 0;
      else if (uy.kind == TV_INT && uy.i != 0) { host = true; break; }
    }
    if (do_uy) {
      if (uy.kind != TV_STR || uy.n == 0) { host = true; break; }
      for (uint32_t k = 0; k < uy.n; k++) ug += U[uy.off + k] > 63;
      ul = uy.n;
    }
    if (ur.kind && ub.kind && val_eq_str(U, ur, ub)) bits |= B_PERFECT_UMI;
    const bool aq_none = l_seq == 0 || U[qual] == 0xff;
    uint32_t q0 = 0, q1 = 0;
    if (!aq_none) {
      uint32_t start = 0;
      for (uint32_t k = 0; k < n_cigar; k++) {
        const uint32_t c = u32(U, cig + 4ull * k), op = c & 0xf, len = c >> 4;
        if (op == 5) {
          if (start != 0 && start != l_seq) { host = true; break; }
        } else if (op == 4) {
          start += len;
        } else {
          break;
        }
      }
      if (host) break;
      uint32_t qend = l_seq;
      for (int k = (int)n_cigar - 1; k > 0; k--) {
        const uint32_t c = u32(U, cig + 4ull * k), op = c & 0xf, len = c >> 4;
        if (op == 5) {
          if (qend != l_seq) { host = true; break; }
        } else if (op == 4) {
          qend -= len;
        } else {
          break;
        }
      }
      if (host) break;
      q0 = start;
      q1 = qend < start ? start : qend;
    }
    if (validate && (aq_none || q1 == q0)) { host = true; break; }
    uint32_t x = XF_ABSENT;
    if (xf.kind) {
      x = XF_OTHER;
      if (xf.kind == TV_STR) {
        if (lit_eq(U, xf, "CODING", 6)) x = XF_CODING;
        else if (lit_eq(U, xf, "INTRONIC", 8)) x = XF_INTRONIC;
        else if (lit_eq(U, xf, "UTR", 3)) x = XF_UTR;
        else if (lit_eq(U, xf, "INTERGENIC", 10)) x = XF_INTERGENIC;
      }
    }
    if (flag & 0x4) {
      bits |= B_UNMAPPED;
    } else {
      if (validate && (!xf.kind || !nh.kind)) { host = true; break; }
      if (nh.kind == TV_INT && nh.i == 1) bits |= B_NH1;
      uint64_t n_len = 0;
      for (uint32_t k = 0; k < n_cigar; k++) {
        const uint32_t c = u32(U, cig + 4ull * k);
        if ((c & 0xf) == 3) n_len += c >> 4;
      }
      if (n_len) bits |= B_SPLICED;
    }
    if (flag & 0x10) bits |= B_REVERSE;
    if (flag & 0x400) bits |= B_DUPLICATE;
    uint32_t s = 0, g = 0;
    for (uint32_t k = q0; k < q1; k++) {
      const uint32_t v = U[qual + k];
      s += v;
      g += v > 30;
    }
    if (q1 - q0 > 0xffff || s > 0xffff || cl > 0xff || ul > 0xff) { host = true; break; }
    int32_t id0 = -1, id1 = -1, id2 = -1;
    if (cb.kind) host |= (id0 = intern(D, 0, U, cb.off, cb.n)) < 0;
    else atomicOr(&flags[1], 1u);
    if (ub.kind) host |= (id1 = intern(D, 1, U, ub.off, ub.n)) < 0;
    else atomicOr(&flags[2], 1u);
    if (ge.kind) host |= (id2 = intern(D, 2, U, ge.off, ge.n)) < 0;
    else atomicOr(&flags[3], 1u);
    if (host) break;
    C.cell[r] = id0, C.umi[r] = id1, C.gene[r] = id2;
    C.ref[r] = ref, C.pos[r] = pos;
    C.gq_sum[r] = (uint16_t)s, C.gq_len[r] = (uint16_t)(q1 - q0), C.gq_gt30[r] = (uint16_t)g;
    C.bits[r] = (uint8_t)bits, C.xf[r] = (uint8_t)x;
    C.cy_gt30[r] = (uint8_t)cg, C.cy_len[r] = (uint8_t)cl, C.uy_gt30[r] = (uint8_t)ug, C.uy_len[r] = (uint8_t)ul;
  } while (false);
  if (host) atomicOr(&flags[0], 1u);
}

// One lane per record: bamdec.cpp parse_count_record (count.py:222-270 reads the three named
// dictionary tags, XF and the query name; no validation) plus the itertools.groupby head flag of
// count.py:83-86 -- the record's query name differs from the previous record's.  tags: the
// three tag names as (a << 8 | b).
struct CountCols {
  int32_t *cell, *umi, *gene;
  uint8_t *xf, *qhead;
};
// has_prev: starts[-1] is the previous window's last record (the query-name comparison of record 0)
__global__ void k_parse_count(const uint8_t* __restrict__ U, const uint64_t* __restrict__ starts, uint64_t n,
                              uint32_t tcb, uint32_t tub, uint32_t tge, CountCols C, Dicts D,
                              uint32_t* __restrict__ flags, uint32_t has_prev) {
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const uint64_t p = starts[r];
  const uint32_t bs = u32(U, p);
  const uint64_t d = p + 4;
  bool host = false;
  do {
    if (bs < 32) { host = true; break; }
    const uint32_t lrn = U[d + 8];
    const uint32_t n_cigar = u16(U, d + 12);
    const uint32_t l_seq = u32(U, d + 16);
    const uint64_t tag0 = 32ull + lrn + 4ull * n_cigar + (l_seq + 1ull) / 2 + l_seq;
    if (tag0 > bs || lrn == 0) { host = true; break; }
    const uint64_t end = d + bs;
    DTag cb{}, ub{}, ge{}, xf{};
    uint64_t q = d + tag0;
    while (q + 3 <= end) {
      const uint32_t a = U[q], b = U[q + 1], t = U[q + 2];
      q += 3;
      DTag v{};
      const uint32_t used = tag_value(U, q, end, t, &v);
      if (!used) { host = true; break; }
      q += used;
      const uint32_t ab = a << 8 | b;
      if (ab == tcb) cb = v;  // (not else-if: a tag name may be given twice, as on the host)
      if (ab == tub) ub = v;
      if (ab == tge) ge = v;
      if (ab == ('X' << 8 | 'F')) xf = v;
    }
    if (host) break;
    if ((cb.kind && cb.kind != TV_STR) || (ub.kind && ub.kind != TV_STR) || (ge.kind && ge.kind != TV_STR)) {
      host = true;  // integer / float / array values: the host's str() of them, or its ETYPED
      break;
    }
    uint32_t x = XF_ABSENT;
    if (xf.kind) x = xf.kind == TV_STR && lit_eq(U, xf, "INTERGENIC", 10) ? XF_INTERGENIC : XF_OTHER;
    uint32_t head = 1;
    if (r || has_prev) {
      const uint64_t pp = starts[r - 1] + 4;
      // the previous record's name lies before this record (a malformed previous record sets
      // *host on its own lane, and then head is not used)
      if (U[pp + 8] == lrn && pp + 32 + lrn <= p) head = !str_eq(U, pp + 32, d + 32, lrn - 1);
    }
    int32_t id0 = -1, id1 = -1, id2 = -1;
    if (cb.kind) host |= (id0 = intern(D, 0, U, cb.off, cb.n)) < 0;
    else atomicOr(&flags[1], 1u);
    if (ub.kind) host |= (id1 = intern(D, 1, U, ub.off, ub.n)) < 0;
    else atomicOr(&flags[2], 1u);
    if (ge.kind) host |= (id2 = intern(D, 2, U, ge.off, ge.n)) < 0;
    else atomicOr(&flags[3], 1u);
    if (host) break;
    C.cell[r] = id0, C.umi[r] = id1, C.gene[r] = id2;
    C.xf[r] = (uint8_t)x, C.qhead[r] = (uint8_t)head;
  } while (false);
  if (host) atomicOr(&flags[0], 1u);
}

// ---------------- dictionaries ----------------
__global__ void k_occupied(const unsigned long long* __restrict__ table, uint64_t cap, uint32_t* __restrict__ occ) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < cap) occ[i] = table[i] != 0;
}
__global__ void k_compact(const unsigned long long* __restrict__ table, uint64_t cap,
                          const uint32_t* __restrict__ dense, uint64_t* __restrict__ uent,
                          uint32_t* __restrict__ ulen) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cap) return;
  const unsigned long long v = table[i];
  if (!v) return;
  uent[dense[i]] = v;
  ulen[dense[i]] = ent_len(v);
}
__global__ void k_pack(const uint8_t* __restrict__ U, const uint8_t* __restrict__ A, const uint64_t* __restrict__ uent,
                       const uint64_t* __restrict__ boff, uint32_t n, uint8_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const unsigned long long e = uent[i];
  const uint8_t* src = ent_src(e, U, A);
  const uint64_t s = ent_off(e), o = boff[i];
  for (uint32_t k = 0; k < ent_len(e); k++) out[o + k] = src[s + k];
}
// Dictionaries ranked on the device (round 4): a string of <= 16 bytes compares in Python's order
// (code points = bytes for the ASCII the device path admits) exactly as its big-endian, zero-padded
// 16-byte key (no dictionary string holds a NUL), so two stable 64-bit radix sorts (low word, then
// high) give the ranks.  *too_long: some string is longer (the host sort ranks that dictionary).
__global__ void k_strkey(const uint8_t* __restrict__ U, const uint8_t* __restrict__ A,
                         const uint64_t* __restrict__ uent, uint32_t n, uint64_t* __restrict__ khi,
                         uint64_t* __restrict__ klo, uint32_t* __restrict__ idx, uint32_t* __restrict__ too_long) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const unsigned long long e = uent[i];
  const uint32_t len = ent_len(e);
  if (len > 16) atomicOr(too_long, 1u);
  const uint8_t* src = ent_src(e, U, A) + ent_off(e);
  uint64_t hi = 0, lo = 0;
  for (uint32_t k = 0; k < 16 && k < len; k++) {
    const uint64_t b = src[k];
    if (k < 8)
      hi |= b << (56 - 8 * k);
    else
      lo |= b << (56 - 8 * (k - 8));
  }
  khi[i] = hi;
  klo[i] = lo;
  idx[i] = i;
}
__global__ void k_gather_key(const uint64_t* __restrict__ key, const uint32_t* __restrict__ idx, uint32_t n,
                             uint64_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = key[idx[i]];
}
// ranked order -> rank of every dense id, and the entries / lengths in ranked order
__global__ void k_rank_order(const uint32_t* __restrict__ order, const uint64_t* __restrict__ uent, uint32_t n,
                             int32_t hn, int32_t* __restrict__ rank, uint64_t* __restrict__ uent2,
                             uint32_t* __restrict__ ulen2) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const uint32_t i = order[r];
  rank[i] = (int32_t)r + hn;
  const unsigned long long e = uent[i];
  uent2[r] = e;
  ulen2[r] = ent_len(e);
}

__global__ void k_remap(int32_t* __restrict__ col, uint64_t n, const uint32_t* __restrict__ dense,
                        const int32_t* __restrict__ rank) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t v = col[i];
  col[i] = v < 0 ? 0 : rank[dense[v]];
}

}  // namespace gb

// ---------------- host ----------------
namespace {
using namespace gb;

double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

thread_local std::string g_gerr;
int gfail(int code, const char* msg) {
  g_gerr = msg;
  return code;
}

// A device allocation that fails declines the file to the host decoder (SCT_GBAM_HOST) instead of
// failing the decode: a BAM too large for the device's memory is still a valid input.
#define HIPOK(x)                                                                            \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ == hipErrorOutOfMemory) {                                                        \
      (void)hipGetLastError();                                                              \
      return gfail(SCT_GBAM_HOST, "device memory exhausted: the host decoder takes the file"); \
    }                                                                                       \
    if (e_ != hipSuccess) return gfail(SCT_BAM_EIO, hipGetErrorString(e_));                 \
  } while (0)

// SCT_GBAM_MAX_DEVICE_BYTES (tests): a cap on the device bytes the process's decodes hold at once;
// an allocation past it fails as hipMalloc does when HBM is exhausted.
uint64_t device_cap() {  // read per allocation (a few per decode): tests change it between calls
  const char* v = getenv("SCT_GBAM_MAX_DEVICE_BYTES");
  return v && *v ? (uint64_t)strtoull(v, nullptr, 10) : ~0ull;
}
std::atomic<uint64_t> g_held{0};  // device bytes held by DevBufs

template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  size_t bytes = 0;
  hipError_t alloc(size_t count) {
    free();
    const size_t b = std::max<size_t>(count, 1) * sizeof(T);
    if (g_held + b > device_cap()) return hipErrorOutOfMemory;
    const hipError_t e = hipMalloc(&p, b);
    if (e != hipSuccess) {
      p = nullptr;
      return e;
    }
    n = count;
    bytes = b;
    g_held += b;
    return hipSuccess;
  }
  void free() {
    if (p) {
      (void)hipFree(p);
      g_held -= bytes;
    }
    p = nullptr;
    n = 0;
    bytes = 0;
  }
  ~DevBuf() { free(); }
};

// the caller thread's current device, restored when an entry point returns (the library switches to
// the handle's device; the caller's own work must not move with it)
struct DeviceGuard {
  int prev = -1;
  DeviceGuard() {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

// the byte offset where the alignments start: magic, l_text, text, n_ref, references
// (SAM/BAM spec 4.2); the leading members are inflated on the host until it is known.
// false: not a BAM header (the host path reports it).
bool header_end(const uint8_t* f, const std::vector<Block>& blocks, uint64_t* H) {
  std::vector<uint8_t> buf;
  z_stream z;
  memset(&z, 0, sizeof(z));
  if (inflateInit2(&z, -15) != Z_OK) return false;
  bool ok = false;
  for (size_t k = 0; k < blocks.size(); k++) {
    const size_t at = buf.size();
    buf.resize(at + blocks[k].isize);
    if (blocks[k].isize && !inflate_block(f, blocks[k], buf.data() + at, z)) break;
    const size_t len = buf.size();
    if (len < 12) continue;
    if (memcmp(buf.data(), "BAM\1", 4) != 0) break;
    uint64_t off = 8 + (uint64_t)rd32(buf.data() + 4);
    if (off + 4 > len) continue;
    const uint32_t n_ref = rd32(buf.data() + off);
    off += 4;
    bool done = true;
    for (uint32_t r = 0; r < n_ref && done; r++) {
      if (off + 4 > len) done = false;
      else off += 4 + (uint64_t)rd32(buf.data() + off) + 4;
    }
    if (!done || off > len) continue;
    *H = off;
    ok = true;
    break;
  }
  inflateEnd(&z);
  return ok;
}

// Python's sorted() on the strings, the missing value first: rank of each distinct string
// The mapping's page-table entries made in parallel (a large file in the page cache): the member
// scan below and the copies to the device then run without a page fault every few members.
void prefault(const uint8_t* f, uint64_t fsize) {
  constexpr uint64_t kPage = 4096, kMin = 64ull << 20;
  if (fsize < kMin) return;
  const unsigned T = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  std::vector<std::thread> th;
  std::atomic<uint64_t> sink{0};
  for (unsigned t = 0; t < T; t++)
    th.emplace_back([&, t] {
      const uint64_t lo = fsize * t / T / kPage * kPage, hi = fsize * (t + 1) / T;
      uint64_t acc = 0;
      for (uint64_t o = lo; o < hi; o += kPage) acc += ((const volatile uint8_t*)f)[o];
      sink += acc;
    });
  for (auto& x : th) x.join();
}

void rank_strings(const std::string& bytes, const std::vector<uint64_t>& off, int32_t has_none,
                  std::vector<int32_t>& rank, std::vector<uint32_t>& order) {
  const size_t n = off.size() - 1;
  order.resize(n);
  for (size_t i = 0; i < n; i++) order[i] = (uint32_t)i;
  auto sv = [&](uint32_t i) { return std::string_view(bytes.data() + off[i], off[i + 1] - off[i]); };
  auto less = [&](uint32_t a, uint32_t b) { return sv(a) < sv(b); };
  const size_t T = std::min<size_t>(16, std::max<size_t>(1, n / 65536));
  if (T <= 1) {
    std::sort(order.begin(), order.end(), less);
  } else {  // sorted chunks, merged pairwise
    std::vector<size_t> cut(T + 1);
    for (size_t t = 0; t <= T; t++) cut[t] = n * t / T;
    std::vector<std::thread> th;
    for (size_t t = 0; t < T; t++)
      th.emplace_back([&, t] { std::sort(order.begin() + cut[t], order.begin() + cut[t + 1], less); });
    for (auto& x : th) x.join();
    for (size_t w = 1; w < T; w *= 2) {
      th.clear();
      for (size_t t = 0; t + w < T; t += 2 * w) {
        const size_t a = cut[t], m = cut[t + w], b = cut[std::min(T, t + 2 * w)];
        th.emplace_back([&, a, m, b] {
          std::inplace_merge(order.begin() + a, order.begin() + m, order.begin() + b, less);
        });
      }
      for (auto& x : th) x.join();
    }
  }
  rank.resize(n);
  for (size_t r = 0; r < n; r++) rank[order[r]] = (int32_t)r + has_none;
}

}  // namespace

// One window: a range of BGZF members inflated together into U, after `carry` -- the bytes of the
// previous window from its last complete record on (that record, already parsed, gives the next
// record's query-name comparison in count mode; the rest is the record the window boundary cut).
// A file that fits the device is one window, inflated once (pass 1 keeps its payload and record
// starts for the parse); a larger one is inflated window by window twice: pass 1 (sct_gbam_open)
// proves every member's first record start and counts the records, pass 2 (sct_gbam_parse) inflates
// each window again, walks from the proven starts and parses -- the device holds one window's
// compressed bytes and payload, the columns and the dictionaries, never the whole file.
struct WinInfo {
  uint32_t m_lo = 0, m_hi = 0;  // members [m_lo, m_hi)
  uint32_t mH = 0;              // first walk member whose start is known (window 0: the header's member)
  uint64_t H = 0;               // that start (window 0: the header end; later windows: 0, the carry)
  uint64_t ulen = 0;            // carry + the members' payload
  bool has_prev = false;        // the carry begins with the previous window's last record
  bool last = false;            // the part's last window: no carry, records complete in U
  bool check = false;           // ... and the file's: its last record must end exactly at ulen
  uint32_t m_look = 0;          // members [m_hi, m_look) inflated after the window's own: a part's last
                                // window reads on into the next part for its records cut at the end
  uint64_t n_rec = 0;           // records this window parses (a carried record excluded)
  uint64_t base = 0;            // global index of its first parsed record
  std::vector<uint64_t> S;      // proven walk-member starts (pass 2 walks from them)
  std::string carry;            // the carry bytes (host copy)
};

struct sct_gbam {
  int device = 0;
  hipStream_t st = nullptr;
  int32_t part = 0, n_parts = 1;
  uint32_t pm_lo = 0, pm_hi = 0;  // the part's members
  int64_t first_abs = -1, land_abs = -1;  // payload offsets: its first record, the first record after it
  const uint8_t* f = nullptr;  // the mapped file (kept for pass 2)
  uint64_t fsize = 0;
  std::vector<Block> blocks;
  std::vector<uint64_t> O;  // payload offset of every member (n_mem + 1)
  std::vector<WinInfo> win;
  DevBuf<uint8_t> in, u;    // a window's compressed bytes and payload
  DevBuf<uint64_t> starts;  // one window: pass 1's record starts
  bool kept = false;        // one window: u and starts already hold the file
  uint64_t ulen = 0, H = 0;
  int64_t n = 0;
  std::string dict_bytes[3];
  std::vector<int64_t> dict_off[3];
  int32_t has_none[3] = {0, 0, 0};
  double t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  ~sct_gbam() {
    if (f) munmap((void*)f, fsize);
  }
};

namespace {

template <class I, class O>
hipError_t exclusive_sum(I* in, O* out, uint64_t n, hipStream_t st, DevBuf<uint8_t>& tmp) {
  size_t bytes = 0;
  // 64-bit item counts (rocPRIM scans size_t items): parse_begin admits tables of 2^31 slots
  hipError_t e = hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, in, out, (size_t)n, st);
  if (e != hipSuccess) return e;
  if (tmp.n < bytes) {
    e = tmp.alloc(bytes);
    if (e != hipSuccess) return e;
  }
  return hipcub::DeviceScan::ExclusiveSum(tmp.p, bytes, in, out, (size_t)n, st);
}

inline unsigned grid(uint64_t n, unsigned b) { return (unsigned)((n + b - 1) / b); }

constexpr int kCopyChunks = 8;
struct CopyStream {  // a non-blocking copy stream and one event per piece
  hipStream_t s = nullptr;
  hipEvent_t ev[kCopyChunks] = {};
  hipError_t init(hipStream_t) {
    hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    for (int k = 0; k < kCopyChunks && e == hipSuccess; k++) e = hipEventCreateWithFlags(&ev[k], hipEventDisableTiming);
    return e;
  }
  ~CopyStream() {  // (the consumer stream's waits are enqueued; destruction is deferred past them)
    for (auto& e : ev)
      if (e) (void)hipEventDestroy(e);
    if (s) (void)hipStreamDestroy(s);
  }
};

// Payload bytes per window: SCT_GBAM_WINDOW_BYTES, else a quarter of the device's free memory (the
// payload plus its compressed image then stay well inside it; a file under that is one window).
uint64_t window_bytes() {
  const char* v = getenv("SCT_GBAM_WINDOW_BYTES");
  if (v && *v) return std::max<uint64_t>(1, strtoull(v, nullptr, 10));
  size_t fr = 0, tot = 0;
  if (hipMemGetInfo(&fr, &tot) != hipSuccess || fr == 0) return 1ull << 30;
  return std::max<uint64_t>(64ull << 20, std::min<uint64_t>(fr / 4, 16ull << 30));
}

// Windows of whole members of the part [pm_lo, pm_hi), each at most `wb` payload bytes (at least
// one member); window 0 reaches at least one member past mH (the header's).  The last window of a
// part that is not the file's last reads on kLookahead payload bytes into the next part's members.
constexpr uint64_t kLookahead = 1u << 18;
void plan_windows(sct_gbam* G, uint32_t mH, uint64_t H, uint64_t wb) {
  const uint32_t n_mem = (uint32_t)G->blocks.size(), hi = G->pm_hi;
  G->win.clear();
  uint32_t m = G->pm_lo;
  while (m < hi) {
    WinInfo w;
    w.m_lo = m;
    uint64_t sz = 0;
    const uint32_t min_hi = G->win.empty() ? std::min(hi, G->pm_lo + mH + 2) : m + 1;
    while (m < hi && (m < min_hi || sz + G->blocks[m].isize <= wb)) sz += G->blocks[m++].isize;
    w.m_hi = w.m_look = m;
    G->win.push_back(std::move(w));
  }
  if (G->win.empty()) return;
  WinInfo& l = G->win.back();
  l.last = true;
  l.check = hi == n_mem;
  for (uint64_t sz = 0; l.m_look < n_mem && sz < kLookahead; l.m_look++) sz += G->blocks[l.m_look].isize;
  G->win[0].mH = mH;
  G->win[0].H = H;
}

// Inflate window w into G->u: the carry, then its members (copied in pieces on a copy stream while
// the members of the pieces already there inflate on st).  false: a member did not inflate (host).
int inflate_window(sct_gbam* G, WinInfo& w, bool timed) {
  hipStream_t st = G->st;
  const uint32_t nm = w.m_look - w.m_lo;  // the window's members and its lookahead
  const uint64_t c = w.carry.size();
  const uint64_t b0 = G->blocks[w.m_lo].off;
  const uint64_t b1 = w.m_look < G->blocks.size() ? G->blocks[w.m_look].off : G->fsize;
  w.ulen = c + (G->O[w.m_look] - G->O[w.m_lo]);
  double t1 = now();
  if (G->in.n < b1 - b0 + kPad) HIPOK(G->in.alloc(b1 - b0 + kPad));
  HIPOK(hipMemsetAsync(G->in.p + (b1 - b0), 0, kPad, st));
  if (G->u.n < w.ulen + kPad) HIPOK(G->u.alloc(w.ulen + kPad));
  HIPOK(hipMemsetAsync(G->u.p + w.ulen, 0, kPad, st));
  if (c) HIPOK(hipMemcpyAsync(G->u.p, w.carry.data(), c, hipMemcpyHostToDevice, st));
  std::vector<Member> mem(nm);
  for (uint32_t k = 0; k < nm; k++) {
    const Block& b = G->blocks[w.m_lo + k];
    const uint16_t xlen = rd16(G->f + b.off + 10);
    mem[k].in_off = b.off + 12 + xlen - b0;
    mem[k].clen = b.csize - 12 - xlen - 8;
    mem[k].isize = b.isize;
    mem[k].out_off = c + G->O[w.m_lo + k] - G->O[w.m_lo];
  }
  DevBuf<Member> d_mem;
  DevBuf<uint32_t> d_stat, d_flag;
  HIPOK(d_mem.alloc(nm));
  HIPOK(d_stat.alloc(nm));
  HIPOK(d_flag.alloc(1));
  HIPOK(hipMemcpyAsync(d_mem.p, mem.data(), nm * sizeof(Member), hipMemcpyHostToDevice, st));
  HIPOK(hipMemsetAsync(d_flag.p, 0, sizeof(uint32_t), st));
  CopyStream cs;
  HIPOK(cs.init(st));
  uint32_t m0 = 0;
  for (int k = 0; k < kCopyChunks && m0 < nm; k++) {
    // members [m0, m1): about 1 / kCopyChunks of the window each; a member's read-ahead past its own
    // bytes may see the next piece unwritten (never consumed: the stream ends inside the member)
    const uint64_t want = b0 + (b1 - b0) * (uint64_t)(k + 1) / kCopyChunks;
    uint32_t m1 = m0 + 1;
    while (m1 < nm && G->blocks[w.m_lo + m1].off < want) m1++;
    if (k == kCopyChunks - 1) m1 = nm;
    const uint64_t p0 = G->blocks[w.m_lo + m0].off - b0;
    const uint64_t p1 = (m1 < nm ? G->blocks[w.m_lo + m1].off : b1) - b0;
    HIPOK(hipMemcpyAsync(G->in.p + p0, G->f + b0 + p0, p1 - p0, hipMemcpyHostToDevice, cs.s));
    HIPOK(hipEventRecord(cs.ev[k], cs.s));
    HIPOK(hipStreamWaitEvent(st, cs.ev[k], 0));
    hipLaunchKernelGGL(k_inflate, dim3(m1 - m0), dim3(64), 0, st, G->in.p, d_mem.p + m0, G->u.p, d_stat.p + m0);
    HIPOK(hipGetLastError());
    m0 = m1;
  }
  if (timed) G->t[1] += now() - t1;  // the copy (this thread waits for the pageable pieces)
  t1 = now();
  hipLaunchKernelGGL(k_any, dim3(grid(nm, 256)), dim3(256), 0, st, d_stat.p, nm, d_flag.p);
  uint32_t bad = 0;
  HIPOK(hipMemcpyAsync(&bad, d_flag.p, sizeof(bad), hipMemcpyDeviceToHost, st));
  HIPOK(hipStreamSynchronize(st));
  if (timed) G->t[2] += now() - t1;  // the inflate left after the last piece arrived
  if (bad) {
    char msg[96];
    snprintf(msg, sizeof(msg), "a BGZF member did not inflate on the device (status mask 0x%x)", bad);
    return gfail(SCT_GBAM_HOST, msg);
  }
  return SCT_BAM_OK;
}

// The walk members' offsets in window w's payload: member 0 begins at 0 (its carry), the others
// where their payload lands; the end is where the window's own members end (the lookahead holds no
// record of the window's, only the rest of one cut at the end).
std::vector<uint64_t> walk_offsets(const sct_gbam* G, const WinInfo& w) {
  const uint32_t nm = w.m_hi - w.m_lo;
  std::vector<uint64_t> o(nm + 1);
  for (uint32_t k = 0; k <= nm; k++) o[k] = k == 0 ? 0 : w.carry.size() + G->O[w.m_lo + k] - G->O[w.m_lo];
  return o;
}
inline uint64_t abs_of(const sct_gbam* G, const WinInfo& w, uint64_t x) { return G->O[w.m_lo] - w.carry.size() + x; }

// Pass 1 on the inflated window: prove the members' record starts (guess, walk, repair rounds),
// count the records, and take the carry for the next window.  With `starts` (one window), also
// write every record start.
int prove_window(sct_gbam* G, WinInfo& w, WinInfo* next, DevBuf<uint64_t>* starts) {
  hipStream_t st = G->st;
  const uint32_t nm = w.m_hi - w.m_lo;
  const uint32_t open = w.last ? 0u : 1u, check = w.check ? 1u : 0u;
  const std::vector<uint64_t> Oh = walk_offsets(G, w);
  DevBuf<uint64_t> d_O, d_S, d_land, d_base, d_last;
  DevBuf<uint32_t> d_cnt, d_flag;
  DevBuf<uint8_t> d_ag;
  HIPOK(d_O.alloc(nm + 1));
  HIPOK(d_S.alloc(nm + 1));
  HIPOK(d_land.alloc(nm + 1));
  HIPOK(d_last.alloc(nm));
  HIPOK(d_cnt.alloc(nm));
  HIPOK(d_base.alloc(nm + 1));
  HIPOK(d_ag.alloc(nm + 1));
  HIPOK(d_flag.alloc(1));
  HIPOK(hipMemcpyAsync(d_O.p, Oh.data(), (nm + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(k_guess, dim3(grid(nm, 64)), dim3(64), 0, st, G->u.p, w.ulen, d_O.p, w.mH, nm, w.H, d_S.p, open,
                     check);
  int rounds = 0;
  for (;; rounds++) {
    if (rounds == kStartRounds) return gfail(SCT_GBAM_HOST, "record starts did not converge");
    hipLaunchKernelGGL(k_walk, dim3(grid(nm, 64)), dim3(64), 0, st, G->u.p, w.ulen, d_O.p, w.mH, nm, d_S.p, d_cnt.p,
                       d_land.p, (uint64_t*)nullptr, (const uint64_t*)nullptr, d_last.p, open);
    HIPOK(hipMemsetAsync(d_flag.p, 0, sizeof(uint32_t), st));
    hipLaunchKernelGGL(k_agree, dim3(grid(nm + 1, 256)), dim3(256), 0, st, w.mH, nm, (const uint64_t*)d_S.p,
                       (const uint64_t*)d_land.p, d_ag.p);
    hipLaunchKernelGGL(k_fix, dim3(grid(nm + 1, 256)), dim3(256), 0, st, w.mH, nm, d_S.p, d_land.p,
                       (const uint8_t*)d_ag.p, d_flag.p);
    uint32_t nbad = 0;
    HIPOK(hipMemcpyAsync(&nbad, d_flag.p, sizeof(nbad), hipMemcpyDeviceToHost, st));
    HIPOK(hipStreamSynchronize(st));
    if (nbad == 0) break;
    uint64_t lastland = 0;
    HIPOK(hipMemcpy(&lastland, d_land.p + nm, sizeof(lastland), hipMemcpyDeviceToHost));
    // only the final landing disagrees and every start before it is proven: a truncated record
    if (w.check && nbad == 1 && lastland != w.ulen && rounds > 0) {
      uint64_t s_last = 0;
      HIPOK(hipMemcpy(&s_last, d_S.p + nm - 1, sizeof(s_last), hipMemcpyDeviceToHost));
      if (s_last != kUnknown) return gfail(SCT_GBAM_HOST, "truncated BAM record");
    }
  }
  G->t[7] += rounds;
  std::vector<uint32_t> cnt(nm);
  std::vector<uint64_t> last(nm);
  w.S.resize(nm + 1);
  uint64_t land_end = 0;
  HIPOK(hipMemcpyAsync(cnt.data(), d_cnt.p, nm * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  HIPOK(hipMemcpyAsync(last.data(), d_last.p, nm * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
  HIPOK(hipMemcpyAsync(w.S.data(), d_S.p, (nm + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
  HIPOK(hipMemcpyAsync(&land_end, d_land.p + nm, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
  HIPOK(hipStreamSynchronize(st));
  uint64_t total = 0, lastrec = kUnknown;
  for (uint32_t k = 0; k < nm; k++) {
    total += cnt[k];
    if (cnt[k]) lastrec = last[k];
  }
  if (w.has_prev && total == 0) return gfail(SCT_GBAM_HOST, "record starts did not converge");
  w.n_rec = total - (w.has_prev ? 1 : 0);
  if (&w == &G->win.front()) G->first_abs = w.S[w.mH] == kUnknown ? -1 : (int64_t)abs_of(G, w, w.S[w.mH]);
  if (w.last) {
    if (land_end == kUnknown || land_end == kBadWalk) return gfail(SCT_GBAM_HOST, "a part's last record runs past its lookahead");
    G->land_abs = (int64_t)abs_of(G, w, land_end);
  }
  if (next) {  // the carry: from the last complete record (or the cut record alone) to the end
    if (lastrec == kUnknown) return gfail(SCT_GBAM_HOST, "a BAM record longer than a decode window");
    const uint64_t from = lastrec;
    next->carry.resize(w.ulen - from);
    if (!next->carry.empty())
      HIPOK(hipMemcpy(&next->carry[0], G->u.p + from, w.ulen - from, hipMemcpyDeviceToHost));
    next->has_prev = true;
    next->mH = 0;
    next->H = 0;
  }
  if (starts) {
    std::vector<uint64_t> base(nm + 1, 0);
    for (uint32_t k = 0; k < nm; k++) base[k + 1] = base[k] + cnt[k];
    HIPOK(starts->alloc(total));
    HIPOK(hipMemcpyAsync(d_base.p, base.data(), (nm + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_walk, dim3(grid(nm, 64)), dim3(64), 0, st, G->u.p, w.ulen, d_O.p, w.mH, nm, d_S.p, d_cnt.p,
                       d_land.p, starts->p, (const uint64_t*)d_base.p, (uint64_t*)nullptr, open);
    HIPOK(hipStreamSynchronize(st));
  }
  return SCT_BAM_OK;
}

// Pass 2 of a window that pass 1 did not keep: inflate it again and write its record starts from the
// proven member starts (no guesses).  *total: records in the window's payload (a carried one included).
int restart_window(sct_gbam* G, WinInfo& w, DevBuf<uint64_t>& starts, uint64_t* total) {
  int rc = inflate_window(G, w, true);
  if (rc) return rc;
  const double t1 = now();
  hipStream_t st = G->st;
  const uint32_t nm = w.m_hi - w.m_lo;
  const uint32_t open = w.last ? 0u : 1u;
  const std::vector<uint64_t> Oh = walk_offsets(G, w);
  DevBuf<uint64_t> d_O, d_S, d_land, d_base, d_cnt64;
  DevBuf<uint32_t> d_cnt;
  DevBuf<uint8_t> tmp;
  HIPOK(d_O.alloc(nm + 1));
  HIPOK(d_S.alloc(nm + 1));
  HIPOK(d_land.alloc(nm + 1));
  HIPOK(d_cnt.alloc(nm));
  HIPOK(d_cnt64.alloc(nm + 1));
  HIPOK(d_base.alloc(nm + 1));
  HIPOK(hipMemcpyAsync(d_O.p, Oh.data(), (nm + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, st));
  HIPOK(hipMemcpyAsync(d_S.p, w.S.data(), (nm + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(k_walk, dim3(grid(nm, 64)), dim3(64), 0, st, G->u.p, w.ulen, d_O.p, w.mH, nm, d_S.p, d_cnt.p,
                     d_land.p, (uint64_t*)nullptr, (const uint64_t*)nullptr, (uint64_t*)nullptr, open);
  HIPOK(hipMemsetAsync(d_cnt64.p + nm, 0, sizeof(uint64_t), st));
  hipLaunchKernelGGL(k_u32_to_u64, dim3(grid(nm, 256)), dim3(256), 0, st, d_cnt.p, d_cnt64.p, nm);
  HIPOK(exclusive_sum(d_cnt64.p, d_base.p, nm + 1, st, tmp));
  uint64_t n = 0;
  HIPOK(hipMemcpyAsync(&n, d_base.p + nm, sizeof(n), hipMemcpyDeviceToHost, st));
  HIPOK(hipStreamSynchronize(st));
  if (n != w.n_rec + (w.has_prev ? 1 : 0)) return gfail(SCT_BAM_EIO, "a window's record count changed between passes");
  if (starts.n < n) HIPOK(starts.alloc(n));
  hipLaunchKernelGGL(k_walk, dim3(grid(nm, 64)), dim3(64), 0, st, G->u.p, w.ulen, d_O.p, w.mH, nm, d_S.p, d_cnt.p,
                     d_land.p, starts.p, (const uint64_t*)d_base.p, (uint64_t*)nullptr, open);
  HIPOK(hipGetLastError());
  *total = n;
  G->t[3] += now() - t1;
  return SCT_BAM_OK;
}

// Part `part` of `n_parts`: the members from the first one starting at or after part/n_parts of the
// file's bytes to the next part's first (part 0 also takes the header's members).  Its records are
// those starting in its members' payload; the first one at first_start (a payload offset), or, when
// first_start < 0, where a start is guessed and proven from inside the part -- the caller checks it
// against the previous part's landing (sct_gbam_part_bounds) and reopens the part on a mismatch.
int open_impl(const char* path, int32_t part, int32_t n_parts, int64_t first_start, int32_t device, void* stream,
              sct_gbam_t** out, int64_t* n_records) {
  const double t0 = now();
  std::unique_ptr<sct_gbam> G(new sct_gbam());
  G->device = device;
  G->st = (hipStream_t)stream;
  G->part = part;
  G->n_parts = n_parts;
  HIPOK(hipSetDevice(device));
  const int fd = open(path, O_RDONLY);
  if (fd < 0) return gfail(SCT_GBAM_HOST, "cannot open");
  struct stat sb;
  if (fstat(fd, &sb) != 0 || sb.st_size == 0) {
    close(fd);
    return gfail(SCT_GBAM_HOST, "empty file");
  }
  const uint64_t fsize = (uint64_t)sb.st_size;
  const uint8_t* f = (const uint8_t*)mmap(nullptr, fsize, PROT_READ, MAP_PRIVATE, fd, 0);
  close(fd);
  if (f == MAP_FAILED) return gfail(SCT_GBAM_HOST, "cannot map");
  G->f = f;
  G->fsize = fsize;
  prefault(f, fsize);
  std::vector<Block>& blocks = G->blocks;
  if (scan_blocks(f, fsize, blocks) != SCT_BAM_OK) return gfail(SCT_GBAM_HOST, "not BGZF");
  uint64_t H = 0;
  if (!header_end(f, blocks, &H)) return gfail(SCT_GBAM_HOST, "no BAM header");
  const uint32_t n_mem = (uint32_t)blocks.size();
  G->O.assign(n_mem + 1, 0);
  uint64_t ulen = 0;
  for (uint32_t k = 0; k < n_mem; k++) {
    const Block& b = blocks[k];
    const uint16_t xlen = rd16(f + b.off + 10);
    if (b.csize < 12u + xlen + 8u) return gfail(SCT_GBAM_HOST, "short member");
    if (b.isize > 65536) return gfail(SCT_GBAM_HOST, "member larger than 64 KB");
    G->O[k] = ulen;
    ulen += b.isize;
  }
  G->O[n_mem] = ulen;
  G->ulen = ulen;
  G->H = H;
  if (H >= ulen) return gfail(SCT_GBAM_HOST, "no records");  // the host path's empty-file error
  uint32_t mH = 0;
  while (mH + 1 < n_mem && G->O[mH + 1] <= H) mH++;
  // the part's members (byte-balanced; part 0 keeps the header's)
  auto cut = [&](int32_t p) -> uint32_t {
    if (p <= 0) return 0;
    if (p >= n_parts) return n_mem;
    const uint64_t want = fsize * (uint64_t)p / (uint64_t)n_parts;
    uint32_t m = (uint32_t)(std::lower_bound(blocks.begin(), blocks.end(), want,
                                             [](const Block& b, uint64_t v) { return b.off < v; }) -
                            blocks.begin());
    return std::max<uint32_t>(m, std::min<uint32_t>(n_mem, mH + 1));
  };
  G->pm_lo = cut(part);
  G->pm_hi = std::max(G->pm_lo, cut(part + 1));
  if (G->pm_lo == G->pm_hi) {
    // an empty part (more parts than members, or a header longer than the part's share): no
    // records, and transparent to the landing chain -- it starts and lands where it is told to
    // (the previous part's landing may lie past its member boundary), else at that boundary
    G->first_abs = G->land_abs = first_start >= 0 ? first_start : (int64_t)G->O[G->pm_lo];
    G->t[0] = now() - t0;
    *n_records = 0;
    *out = G.release();
    return SCT_BAM_OK;
  }
  uint32_t wmH = 0;
  uint64_t wH = kUnknown;
  if (part == 0) {
    wmH = mH;
    wH = H;
  } else if (first_start >= 0) {
    if ((uint64_t)first_start < G->O[G->pm_lo] || (uint64_t)first_start > G->O[G->pm_hi])
      return gfail(SCT_BAM_EIO, "first_start outside the part");
    wH = (uint64_t)first_start - G->O[G->pm_lo];
  }
  plan_windows(G.get(), wmH, wH, window_bytes());
  G->t[0] = now() - t0;
  G->t[6] = G->pm_hi - G->pm_lo;

  // pass 1: every window inflated, its member starts proven, its records counted
  const bool one = G->win.size() == 1;
  uint64_t n = 0;
  for (size_t k = 0; k < G->win.size(); k++) {
    WinInfo& w = G->win[k];
    int rc = inflate_window(G.get(), w, true);
    if (rc) return rc;
    const double t1 = now();
    rc = prove_window(G.get(), w, k + 1 < G->win.size() ? &G->win[k + 1] : nullptr, one ? &G->starts : nullptr);
    if (rc) return rc;
    w.base = n;
    n += w.n_rec;
    G->t[3] += now() - t1;
  }
  G->kept = one;
  if (one) G->in.free();
  if (n == 0 && n_parts == 1) return gfail(SCT_GBAM_HOST, "no records");
  G->n = (int64_t)n;
  *n_records = (int64_t)n;
  *out = G.release();
  return SCT_BAM_OK;
}

// The three device hash tables (2^k slots each) and the parse flags: [0] a record needs the host
// decoder, [1..3] some record lacks CB / UB / GE.  Several windows: tables grown before a window
// that could fill them past half (k_rehash), new strings listed and moved to the arena after each
// window (k_promote).
struct ParseState {
  uint64_t cap[3] = {1024, 1024, 1024};
  uint64_t used[3] = {0, 0, 0};  // entries
  DevBuf<unsigned long long> tab[3];
  DevBuf<uint8_t> arena;
  uint64_t arena_used = 0;
  DevBuf<uint32_t> newl[3];
  DevBuf<unsigned long long> newc;
  Dicts D{};
  DevBuf<uint32_t> flags;
  uint32_t fl[4] = {0, 0, 0, 0};
};

int parse_begin(sct_gbam* G, ParseState& P) {
  HIPOK(hipSetDevice(G->device));
  uint64_t biggest = 0;
  for (const WinInfo& w : G->win) biggest = std::max<uint64_t>(biggest, w.n_rec);
  const uint64_t first = G->kept ? (uint64_t)G->n : biggest;
  for (int k = 0; k < 3; k++) {
    while (P.cap[k] < 2 * first) P.cap[k] <<= 1;
    if (P.cap[k] > (1ull << 31)) return gfail(SCT_GBAM_HOST, "too many records for the device tables");
    HIPOK(P.tab[k].alloc(P.cap[k]));
    HIPOK(hipMemsetAsync(P.tab[k].p, 0, P.cap[k] * sizeof(unsigned long long), G->st));
    P.D.table[k] = P.tab[k].p;
    P.D.mask[k] = P.cap[k] - 1;
    if (!G->kept) {
      HIPOK(P.newl[k].alloc(biggest + 1));
      P.D.newl[k] = P.newl[k].p;
    }
  }
  if (!G->kept) {
    HIPOK(P.newc.alloc(6));
    HIPOK(hipMemsetAsync(P.newc.p, 0, 6 * sizeof(unsigned long long), G->st));
    P.D.newc = P.newc.p;
    HIPOK(P.arena.alloc(1 << 20));
  }
  P.D.A = P.arena.p;
  HIPOK(P.flags.alloc(4));
  HIPOK(hipMemsetAsync(P.flags.p, 0, 4 * sizeof(uint32_t), G->st));
  return SCT_BAM_OK;
}

// Before a window of `n_rec` records: every table keeps at most half its slots filled even if all
// the window's strings are new; a grown table renumbers its slots in the columns already written.
int ensure_tables(sct_gbam* G, ParseState& P, int32_t* const colk[3], uint64_t written, uint64_t n_rec) {
  hipStream_t st = G->st;
  for (int k = 0; k < 3; k++) {
    uint64_t cap = P.cap[k];
    while (cap < 2 * (P.used[k] + n_rec)) cap <<= 1;
    if (cap == P.cap[k]) continue;
    if (cap > (1ull << 31)) return gfail(SCT_GBAM_HOST, "too many distinct strings for the device tables");
    DevBuf<unsigned long long> nt;
    DevBuf<int32_t> map;
    HIPOK(nt.alloc(cap));
    HIPOK(map.alloc(P.cap[k]));
    HIPOK(hipMemsetAsync(nt.p, 0, cap * sizeof(unsigned long long), st));
    hipLaunchKernelGGL(k_rehash, dim3(grid(P.cap[k], 256)), dim3(256), 0, st, P.tab[k].p, P.cap[k], nt.p, cap - 1,
                       G->u.p, P.arena.p, map.p);
    if (written)
      hipLaunchKernelGGL(k_remap_slots, dim3(grid(written, 256)), dim3(256), 0, st, colk[k], written, map.p);
    HIPOK(hipGetLastError());
    HIPOK(hipStreamSynchronize(st));
    std::swap(P.tab[k].p, nt.p);
    std::swap(P.tab[k].n, nt.n);
    std::swap(P.tab[k].bytes, nt.bytes);
    P.cap[k] = cap;
    P.D.table[k] = P.tab[k].p;
    P.D.mask[k] = cap - 1;
  }
  return SCT_BAM_OK;
}

// After a window's parse: its new strings move from the payload to the arena.
int promote(sct_gbam* G, ParseState& P) {
  hipStream_t st = G->st;
  unsigned long long c[6];
  HIPOK(hipMemcpyAsync(c, P.newc.p, sizeof(c), hipMemcpyDeviceToHost, st));
  HIPOK(hipStreamSynchronize(st));
  const uint64_t bytes = c[1] + c[3] + c[5];
  if (P.arena_used + bytes > P.arena.n) {
    DevBuf<uint8_t> na;
    HIPOK(na.alloc(std::max<uint64_t>(2 * P.arena.n, P.arena_used + bytes)));
    if (P.arena_used) HIPOK(hipMemcpyAsync(na.p, P.arena.p, P.arena_used, hipMemcpyDeviceToDevice, st));
    HIPOK(hipStreamSynchronize(st));
    std::swap(P.arena.p, na.p);
    std::swap(P.arena.n, na.n);
    std::swap(P.arena.bytes, na.bytes);
    P.D.A = P.arena.p;
  }
  if (P.arena_used + bytes >= (1ull << 35)) return gfail(SCT_GBAM_HOST, "dictionary strings past 32 GB");
  DevBuf<unsigned long long> cursor;
  HIPOK(cursor.alloc(1));
  unsigned long long cur = P.arena_used;
  HIPOK(hipMemcpyAsync(cursor.p, &cur, sizeof(cur), hipMemcpyHostToDevice, st));
  for (int k = 0; k < 3; k++)
    if (c[2 * k])
      hipLaunchKernelGGL(k_promote, dim3(grid(c[2 * k], 256)), dim3(256), 0, st, P.tab[k].p, P.newl[k].p,
                         (uint64_t)c[2 * k], G->u.p, P.arena.p, cursor.p);
  HIPOK(hipGetLastError());
  HIPOK(hipMemsetAsync(P.newc.p, 0, 6 * sizeof(unsigned long long), st));
  HIPOK(hipStreamSynchronize(st));
  for (int k = 0; k < 3; k++) P.used[k] += c[2 * k];
  P.arena_used += bytes;
  return SCT_BAM_OK;
}

int parse_flags(sct_gbam* G, ParseState& P) {
  HIPOK(hipGetLastError());
  HIPOK(hipMemcpyAsync(P.fl, P.flags.p, sizeof(P.fl), hipMemcpyDeviceToHost, G->st));
  HIPOK(hipStreamSynchronize(G->st));
  if (P.fl[0]) return gfail(SCT_GBAM_HOST, "a record needs the host decoder");
  return SCT_BAM_OK;
}

// Dictionary k ranked on the device (gb::k_strkey): false if a string is longer than 16 bytes
// (the caller ranks it on the host); else true, with *rc the result (the ranked strings and offsets
// copied to G->dict_bytes / dict_off, column colk remapped to ranks).
bool rank_on_device(sct_gbam* G, ParseState& P, int k, int32_t hn, DevBuf<uint64_t>& uent, DevBuf<uint32_t>& ulen,
                    DevBuf<uint64_t>& boff, DevBuf<uint32_t>& dense, int32_t* col, DevBuf<uint8_t>& tmp, int* rc) {
  hipStream_t st = G->st;
  const uint32_t nu = (uint32_t)uent.n;
  const uint64_t n = (uint64_t)G->n;
  *rc = SCT_BAM_OK;
  auto err = [&](hipError_t e) {
    *rc = e == hipErrorOutOfMemory ? gfail(SCT_GBAM_HOST, "device memory exhausted: the host decoder takes the file")
                                   : gfail(SCT_BAM_EIO, hipGetErrorString(e));
    return true;
  };
#define DOK(x)                              \
  do {                                      \
    const hipError_t e_ = (x);              \
    if (e_ != hipSuccess) return err(e_);   \
  } while (0)
  DevBuf<uint64_t> khi, klo, kt;
  DevBuf<uint32_t> ia, ib, flag;
  DOK(khi.alloc(nu));
  DOK(klo.alloc(nu));
  DOK(kt.alloc(nu));
  DOK(ia.alloc(nu));
  DOK(ib.alloc(nu));
  DOK(flag.alloc(1));
  DOK(hipMemsetAsync(flag.p, 0, sizeof(uint32_t), st));
  hipLaunchKernelGGL(gb::k_strkey, dim3(grid(nu, 256)), dim3(256), 0, st, G->u.p, P.arena.p, uent.p, nu, khi.p,
                     klo.p, ia.p, flag.p);
  uint32_t too_long = 0;
  DOK(hipMemcpyAsync(&too_long, flag.p, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  DOK(hipStreamSynchronize(st));
  if (too_long) return false;
  // stable LSD: by the low word, then by the high word
  size_t tb = 0;
  DOK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, klo.p, kt.p, ia.p, ib.p, (int)nu, 0, 64, st));
  if (tmp.n < tb) DOK(tmp.alloc(tb));
  DOK(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb, klo.p, kt.p, ia.p, ib.p, (int)nu, 0, 64, st));
  hipLaunchKernelGGL(gb::k_gather_key, dim3(grid(nu, 256)), dim3(256), 0, st, khi.p, ib.p, nu, klo.p);
  DOK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, klo.p, kt.p, ib.p, ia.p, (int)nu, 0, 64, st));
  if (tmp.n < tb) DOK(tmp.alloc(tb));
  DOK(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb, klo.p, kt.p, ib.p, ia.p, (int)nu, 0, 64, st));
  // ia = the ranked order; ranks, entries and lengths in ranked order, their byte offsets
  DevBuf<int32_t> rank_d;
  DevBuf<uint64_t> uent2;
  DOK(rank_d.alloc(nu));
  DOK(uent2.alloc(nu));
  hipLaunchKernelGGL(gb::k_rank_order, dim3(grid(nu, 256)), dim3(256), 0, st, ia.p, uent.p, nu, hn, rank_d.p,
                     uent2.p, ulen.p);
  DOK(exclusive_sum(ulen.p, boff.p, (uint64_t)nu + 1, st, tmp));
  uint64_t total = 0;
  DOK(hipMemcpyAsync(&total, boff.p + nu, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
  DOK(hipStreamSynchronize(st));
  DevBuf<uint8_t> packed;
  DOK(packed.alloc(total));
  hipLaunchKernelGGL(gb::k_pack, dim3(grid(nu, 256)), dim3(256), 0, st, G->u.p, P.arena.p, uent2.p, boff.p, nu,
                     packed.p);
  std::string& db = G->dict_bytes[k];
  std::vector<int64_t>& dof = G->dict_off[k];
  db.assign(total, '\0');
  dof.assign((size_t)nu + 1 + (hn ? 1 : 0), 0);
  if (total) DOK(hipMemcpyAsync(&db[0], packed.p, total, hipMemcpyDeviceToHost, st));
  static_assert(sizeof(int64_t) == sizeof(uint64_t), "offsets copied as they are");
  DOK(hipMemcpyAsync(dof.data() + (hn ? 1 : 0), boff.p, ((size_t)nu + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost,
                     st));
  if (n) hipLaunchKernelGGL(gb::k_remap, dim3(grid(n, 256)), dim3(256), 0, st, col, n, dense.p, rank_d.p);
  DOK(hipGetLastError());
  DOK(hipStreamSynchronize(st));
#undef DOK
  return true;
}

// The interned ids -> ranks in Python's sorted() order (None first), and the ranked strings.
int dictionaries_impl(sct_gbam* G, ParseState& P, int32_t* const colk[3]) {
  const double t1 = now();
  hipStream_t st = G->st;
  const uint64_t n = (uint64_t)G->n;
  const uint32_t* fl = P.fl;
  DevBuf<unsigned long long>* tab = P.tab;
  DevBuf<uint32_t> occ, dense;
  DevBuf<uint8_t> tmp;
  for (int k = 0; k < 3; k++) {
    const uint64_t cap = P.cap[k];
    HIPOK(occ.alloc(cap));
    HIPOK(dense.alloc(cap));
    const int32_t hn = fl[1 + k] ? 1 : 0;
    G->has_none[k] = hn;
    hipLaunchKernelGGL(k_occupied, dim3(grid(cap, 256)), dim3(256), 0, st, tab[k].p, cap, occ.p);
    HIPOK(exclusive_sum(occ.p, dense.p, cap, st, tmp));
    uint32_t last[2] = {0, 0};
    HIPOK(hipMemcpyAsync(&last[0], dense.p + cap - 1, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIPOK(hipMemcpyAsync(&last[1], occ.p + cap - 1, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIPOK(hipStreamSynchronize(st));
    const uint64_t nu = (uint64_t)last[0] + last[1];
    DevBuf<uint64_t> uent, boff;
    DevBuf<uint32_t> ulen;
    DevBuf<int32_t> rank_d;
    HIPOK(uent.alloc(nu));
    HIPOK(ulen.alloc(nu + 1));
    HIPOK(boff.alloc(nu + 1));
    HIPOK(hipMemsetAsync(ulen.p + nu, 0, sizeof(uint32_t), st));
    hipLaunchKernelGGL(k_compact, dim3(grid(cap, 256)), dim3(256), 0, st, tab[k].p, cap, dense.p, uent.p, ulen.p);
    HIPOK(exclusive_sum(ulen.p, boff.p, nu + 1, st, tmp));
    if (nu > 0 && nu < (1ull << 31)) {  // ranked on the device unless a string is longer than 16 bytes
      int rc = 0;
      if (rank_on_device(G, P, k, hn, uent, ulen, boff, dense, colk[k], tmp, &rc)) {
        if (rc) return rc;
        continue;
      }
    }
    std::vector<uint64_t> hoff(nu + 1);
    HIPOK(hipMemcpyAsync(hoff.data(), boff.p, (nu + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    HIPOK(hipStreamSynchronize(st));
    const uint64_t total = hoff[nu];
    DevBuf<uint8_t> packed;
    HIPOK(packed.alloc(total));
    if (nu)
      hipLaunchKernelGGL(k_pack, dim3(grid(nu, 256)), dim3(256), 0, st, G->u.p, P.arena.p, uent.p, boff.p,
                         (uint32_t)nu, packed.p);
    std::string bytes(total, '\0');
    if (total) HIPOK(hipMemcpyAsync(&bytes[0], packed.p, total, hipMemcpyDeviceToHost, st));
    HIPOK(hipStreamSynchronize(st));
    std::vector<int32_t> rank;
    std::vector<uint32_t> order;
    rank_strings(bytes, hoff, hn, rank, order);
    std::string& db = G->dict_bytes[k];
    std::vector<int64_t>& dof = G->dict_off[k];
    db.clear();
    db.reserve(total);
    dof.clear();
    dof.reserve(nu + 2);
    dof.push_back(0);
    if (hn) dof.push_back(0);
    for (uint64_t r = 0; r < nu; r++) {
      const uint32_t i = order[r];
      db.append(bytes.data() + hoff[i], hoff[i + 1] - hoff[i]);
      dof.push_back((int64_t)db.size());
    }
    HIPOK(rank_d.alloc(nu));
    if (nu) HIPOK(hipMemcpyAsync(rank_d.p, rank.data(), nu * sizeof(int32_t), hipMemcpyHostToDevice, st));
    if (n) hipLaunchKernelGGL(k_remap, dim3(grid(n, 256)), dim3(256), 0, st, colk[k], n, dense.p, rank_d.p);
    HIPOK(hipStreamSynchronize(st));
  }
  G->t[5] = now() - t1;
  return SCT_BAM_OK;
}

// Pass 2 over the windows: `launch(w, starts of its parsed records, count, has_prev)` parses one
// window's records into the columns at w.base.
template <class Launch>
int parse_windows(sct_gbam* G, ParseState& P, int32_t* const colk[3], Launch launch) {
  if (G->kept) {
    const double t0 = now();
    launch(G->win[0], G->starts.p, (uint64_t)G->n, false);
    const int rc = parse_flags(G, P);
    G->t[4] = now() - t0;
    return rc;
  }
  DevBuf<uint64_t> starts;
  for (WinInfo& w : G->win) {
    uint64_t total = 0;
    int rc = restart_window(G, w, starts, &total);
    if (rc) return rc;
    const double t0 = now();
    rc = ensure_tables(G, P, colk, w.base, w.n_rec);
    if (rc) return rc;
    const uint64_t skip = w.has_prev ? 1 : 0;
    if (w.n_rec) launch(w, starts.p + skip, w.n_rec, w.has_prev);
    rc = parse_flags(G, P);
    if (rc) return rc;
    rc = promote(G, P);
    if (rc) return rc;
    G->t[4] += now() - t0;
  }
  G->in.free();
  return SCT_BAM_OK;
}

int parse_impl(sct_gbam* G, int32_t metric_mode, void* const* cols) {
  ParseState P;
  int rc = parse_begin(G, P);
  if (rc) return rc;
  Cols C;
  C.cell = (int32_t*)cols[0], C.umi = (int32_t*)cols[1], C.gene = (int32_t*)cols[2];
  C.ref = (int32_t*)cols[3], C.pos = (int32_t*)cols[4];
  C.gq_sum = (uint16_t*)cols[5], C.gq_len = (uint16_t*)cols[6], C.gq_gt30 = (uint16_t*)cols[7];
  C.bits = (uint8_t*)cols[8], C.xf = (uint8_t*)cols[9], C.cy_gt30 = (uint8_t*)cols[10];
  C.cy_len = (uint8_t*)cols[11], C.uy_gt30 = (uint8_t*)cols[12], C.uy_len = (uint8_t*)cols[13];
  int32_t* const colk[3] = {C.cell, C.umi, C.gene};
  const uint32_t is_cell = metric_mode == SCT_BAM_CELL_METRICS ? 1u : 0u;
  rc = parse_windows(G, P, colk, [&](const WinInfo& w, const uint64_t* starts, uint64_t n, bool) {
    Cols Cw = C;
    const uint64_t b = w.base;
    Cw.cell += b, Cw.umi += b, Cw.gene += b, Cw.ref += b, Cw.pos += b;
    Cw.gq_sum += b, Cw.gq_len += b, Cw.gq_gt30 += b, Cw.bits += b, Cw.xf += b;
    Cw.cy_gt30 += b, Cw.cy_len += b, Cw.uy_gt30 += b, Cw.uy_len += b;
    hipLaunchKernelGGL(k_parse, dim3(grid(n, 256)), dim3(256), 0, G->st, G->u.p, starts, n, is_cell, Cw, P.D,
                       P.flags.p);
  });
  if (rc) return rc;
  return dictionaries_impl(G, P, colk);
}

int parse_count_impl(sct_gbam* G, const char* tags, void* const* cols) {
  ParseState P;
  int rc = parse_begin(G, P);
  if (rc) return rc;
  CountCols C;
  C.cell = (int32_t*)cols[0], C.umi = (int32_t*)cols[1], C.gene = (int32_t*)cols[2];
  C.xf = (uint8_t*)cols[3], C.qhead = (uint8_t*)cols[4];
  auto tag = [&](int k) { return (uint32_t)(uint8_t)tags[2 * k] << 8 | (uint8_t)tags[2 * k + 1]; };
  int32_t* const colk[3] = {C.cell, C.umi, C.gene};
  rc = parse_windows(G, P, colk, [&](const WinInfo& w, const uint64_t* starts, uint64_t n, bool has_prev) {
    CountCols Cw = C;
    const uint64_t b = w.base;
    Cw.cell += b, Cw.umi += b, Cw.gene += b, Cw.xf += b, Cw.qhead += b;
    hipLaunchKernelGGL(k_parse_count, dim3(grid(n, 256)), dim3(256), 0, G->st, G->u.p, starts, n, tag(0), tag(1),
                       tag(2), Cw, P.D, P.flags.p, has_prev ? 1u : 0u);
  });
  if (rc) return rc;
  return dictionaries_impl(G, P, colk);
}

}  // namespace

extern "C" {

const char* sct_gbam_last_error(void) { return g_gerr.c_str(); }

int sct_gbam_open(const char* path, int32_t device, void* stream, sct_gbam_t** out, int64_t* n_records) {
  return sct_gbam_open_part(path, 0, 1, -1, device, stream, out, n_records);
}

int sct_gbam_open_part(const char* path, int32_t part, int32_t n_parts, int64_t first_start, int32_t device,
                       void* stream, sct_gbam_t** out, int64_t* n_records) {
  g_gerr.clear();
  if (out) *out = nullptr;
  if (n_records) *n_records = 0;
  if (!path || !out || !n_records) return gfail(SCT_BAM_EIO, "NULL argument");
  if (n_parts < 1 || part < 0 || part >= n_parts) return gfail(SCT_BAM_EIO, "part outside [0, n_parts)");
  DeviceGuard guard;
  return open_impl(path, part, n_parts, first_start, device, stream, out, n_records);
}

int sct_gbam_part_bounds(const sct_gbam_t* h, int64_t* first_start, int64_t* end_landing) {
  if (!h || !first_start || !end_landing) return gfail(SCT_BAM_EIO, "NULL argument");
  *first_start = h->first_abs;
  *end_landing = h->land_abs;
  return SCT_BAM_OK;
}

// The parts' ranked dictionaries `which` merged (sorted union, the missing tag first if any part
// has it): parts[0] then holds the merged one, remap[p][i] = the merged id of part p's id i.
int sct_gbam_merge_dictionaries(sct_gbam_t* const* parts, int32_t n_parts, int32_t which, int32_t* const* remap) {
  if (!parts || n_parts < 1 || which < 0 || which > 2 || !remap) return gfail(SCT_BAM_EIO, "bad arguments");
  for (int32_t p = 0; p < n_parts; p++)
    if (!parts[p] || !remap[p]) return gfail(SCT_BAM_EIO, "NULL part or remap");
  int32_t hn = 0;
  for (int32_t p = 0; p < n_parts; p++) hn |= parts[p]->has_none[which];
  using SV = std::string_view;
  struct Cur {
    int32_t p;
    int64_t i, n;
  };
  auto name = [&](int32_t p, int64_t i) {
    const sct_gbam* h = parts[p];
    const std::vector<int64_t>& o = h->dict_off[which];
    return SV(h->dict_bytes[which].data() + o[i], (size_t)(o[i + 1] - o[i]));
  };
  std::vector<Cur> cur;
  for (int32_t p = 0; p < n_parts; p++) {
    const sct_gbam* h = parts[p];
    const int64_t n = h->dict_off[which].empty() ? 0 : (int64_t)h->dict_off[which].size() - 1;
    int64_t i = 0;
    if (h->has_none[which] && n > 0) remap[p][i++] = 0;  // the missing tag: merged id 0
    cur.push_back(Cur{p, i, n});
  }
  std::string bytes;
  std::vector<int64_t> off{0};
  if (hn) off.push_back(0);
  // k-way merge (the parts' lists are sorted and duplicate-free)
  auto greater = [&](const Cur& a, const Cur& b) { return name(b.p, b.i) < name(a.p, a.i); };
  std::vector<Cur> heap;
  for (const Cur& c : cur)
    if (c.i < c.n) heap.push_back(c);
  std::make_heap(heap.begin(), heap.end(), greater);
  int32_t id = hn ? 0 : -1;
  std::string last;
  bool have = false;
  while (!heap.empty()) {
    std::pop_heap(heap.begin(), heap.end(), greater);
    Cur c = heap.back();
    heap.pop_back();
    const SV v = name(c.p, c.i);
    if (!have || v != SV(last)) {
      bytes.append(v.data(), v.size());
      off.push_back((int64_t)bytes.size());
      last.assign(v.data(), v.size());
      have = true;
      id++;
    }
    remap[c.p][c.i] = id;
    if (++c.i < c.n) {
      heap.push_back(c);
      std::push_heap(heap.begin(), heap.end(), greater);
    }
  }
  parts[0]->dict_bytes[which] = std::move(bytes);
  parts[0]->dict_off[which] = std::move(off);
  parts[0]->has_none[which] = hn;
  return SCT_BAM_OK;
}

// column[i] = remap[column[i]] on the part's device and stream (n_ids entries of host `remap`).
int sct_gbam_remap(sct_gbam_t* h, const int32_t* remap, int64_t n_ids, void* column, int64_t n) {
  g_gerr.clear();
  if (!h || (!remap && n_ids) || (!column && n)) return gfail(SCT_BAM_EIO, "NULL argument");
  if (n == 0) return SCT_BAM_OK;
  DeviceGuard guard;
  HIPOK(hipSetDevice(h->device));
  DevBuf<int32_t> d;
  HIPOK(d.alloc((size_t)std::max<int64_t>(n_ids, 1)));
  if (n_ids) HIPOK(hipMemcpyAsync(d.p, remap, (size_t)n_ids * sizeof(int32_t), hipMemcpyHostToDevice, h->st));
  hipLaunchKernelGGL(k_apply_map, dim3(grid((uint64_t)n, 256)), dim3(256), 0, h->st, (int32_t*)column, (uint64_t)n,
                     (const int32_t*)d.p);
  HIPOK(hipGetLastError());
  HIPOK(hipStreamSynchronize(h->st));
  return SCT_BAM_OK;
}

int sct_gbam_parse(sct_gbam_t* h, int32_t metric_mode, void* const* columns) {
  g_gerr.clear();
  if (!h || !columns) return gfail(SCT_BAM_EIO, "NULL argument");
  if (metric_mode != SCT_BAM_CELL_METRICS && metric_mode != SCT_BAM_GENE_METRICS)
    return gfail(SCT_BAM_EIO, "the device decode reads the cell and gene metric modes");
  for (int k = 0; k < 14; k++)
    if (!columns[k]) return gfail(SCT_BAM_EIO, "NULL column");
  DeviceGuard guard;
  return parse_impl(h, metric_mode, columns);
}

int sct_gbam_parse_count(sct_gbam_t* h, const char* tags, void* const* columns) {
  g_gerr.clear();
  if (!h || !tags || !columns) return gfail(SCT_BAM_EIO, "NULL argument");
  for (int k = 0; k < 6; k++)
    if (!tags[k]) return gfail(SCT_BAM_EIO, "tags: six characters (cell, molecule, gene tag names)");
  for (int k = 0; k < 5; k++)
    if (!columns[k]) return gfail(SCT_BAM_EIO, "NULL column");
  DeviceGuard guard;
  return parse_count_impl(h, tags, columns);
}

int sct_gbam_dictionary(const sct_gbam_t* h, int32_t which, int64_t* n, const char** bytes, const int64_t** offsets,
                        int32_t* has_none) {
  if (!h || which < 0 || which > 2 || !n || !bytes || !offsets || !has_none) return gfail(SCT_BAM_EIO, "bad arguments");
  *n = h->dict_off[which].empty() ? 0 : (int64_t)h->dict_off[which].size() - 1;
  *bytes = h->dict_bytes[which].data();
  *offsets = h->dict_off[which].data();
  *has_none = h->has_none[which];
  return SCT_BAM_OK;
}

int sct_gbam_read_inflated(const sct_gbam_t* h, uint64_t off, uint64_t n, void* dst, uint64_t* total) {
  if (!h) return gfail(SCT_BAM_EIO, "NULL handle");
  if (total) *total = h->ulen;
  if (!n) return SCT_BAM_OK;
  if (!dst || off > h->ulen || n > h->ulen - off) return gfail(SCT_BAM_EIO, "range outside the payload");
  if (!h->kept) return gfail(SCT_BAM_EIO, "the payload is decoded window by window: not resident");
  DeviceGuard guard;
  HIPOK(hipSetDevice(h->device));
  HIPOK(hipMemcpy(dst, h->u.p + off, n, hipMemcpyDeviceToHost));
  return SCT_BAM_OK;
}

int sct_gbam_timing(const sct_gbam_t* h, double* t8) {
  if (!h || !t8) return gfail(SCT_BAM_EIO, "NULL argument");
  for (int k = 0; k < 8; k++) t8[k] = h->t[k];
  return SCT_BAM_OK;
}

int64_t sct_gbam_windows(const sct_gbam_t* h) { return h ? (int64_t)h->win.size() : 0; }

void sct_gbam_close(sct_gbam_t* h) {
  if (!h) return;
  DeviceGuard guard;
  (void)hipSetDevice(h->device);
  delete h;
}

}  // extern "C"
