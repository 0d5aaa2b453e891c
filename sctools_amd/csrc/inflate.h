// inflate.h -- raw-deflate (RFC 1951) decode of BGZF members on gfx950, one wavefront per member.
//
// The member's Huffman decode is sequential, so the wave decodes one symbol at a time with
// every value wave-uniform (readfirstlane'd into SGPRs: the bit buffer, the table entry, the
// output position), and spends its 64 lanes where the work is parallel: building the decode
// tables (a ballot per code length, one table entry per lane), copying a match (one byte per
// lane, the overlapping case as src = pos - dist + i mod dist), refilling the compressed-input
// ring and flushing the window to HBM.
//
// LDS per wave (~11 KB at the default 4 KB window, 14 waves per CU): the window (a ring of the
// newest output bytes; older ones are flushed to HBM and read back from there by far matches), a
// 1024-entry literal/length table (10-bit root), a 256-entry distance
// table (8-bit root), the canonical code data for codes longer than the root (decoded by the
// counting method of zlib's puff.c), and a 1 KB ring of compressed words refilled 512 bytes at
// a time from registers loaded one refill ahead (so the ring never waits on HBM).
//
// Validation follows zlib's inflate (inflate.c / inftrees.c, zlib 1.2.x): the block type, the
// stored-block length check, HLIT <= 286 and HDIST <= 30, over-subscribed and incomplete code
// sets (a single one-bit code excepted), a missing end-of-block code, invalid symbols, a
// distance before the member's start; on top, the member must produce exactly ISIZE bytes
// without reading past its compressed length.  Any failure sets the member's status and the
// host decodes the file instead.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gb {

// (round 4: a 9-bit literal / length root table -- 2 KB of LDS instead of 4 KB, so 20 waves per CU
// instead of 17; longer codes take the slow path: inflate 0.141 -> 0.122 s on a 20M-record
// config-2-shaped BAM; then an 8-bit one, 1 KB: 0.122 -> 0.112 s; a 7-bit distance table gained
// nothing (0.123 s); profiles/r04/h_inflate_window/)
constexpr uint32_t kLitBits = 8, kDistBits = 8, kClBits = 7;
// The LDS window holds the newest kWin output bytes; older ones are read back from the member's
// output in HBM, already flushed there (pos - flushed <= kFlush + 258 < kWin at every copy), so a
// smaller window costs only those far matches and buys waves per CU (24M-record BAM: inflate
// 0.459 s with a 32 KB window at 4 waves per CU, 0.347 s at 16 KB, 0.246 s at 8 KB, 0.180 s at 4 KB;
// round 4, 20M-record config-2-shaped BAM: 0.147 s at 4 KB, 0.139 s at 2 KB, profiles/r04/h_inflate_window/).
#ifndef SCT_INFL_WIN
#define SCT_INFL_WIN 2048
#endif
constexpr uint32_t kWin = SCT_INFL_WIN, kWinMask = kWin - 1, kFlush = kWin / 4;
static_assert((kWin & (kWin - 1)) == 0 && kWin >= 2048 && kWin <= 32768, "a power-of-two window");
static_assert(kFlush + 2 * 258 < kWin, "unflushed bytes always sit in the window, clear of a far copy");
constexpr uint32_t kRingW = 256, kRingMask = kRingW - 1, kRingHalf = 128;

// table entry: bits 0..3 code length, 4..6 kind, 8..12 extra bits, 16..31 value
enum : uint32_t { E_LIT = 0, E_LEN = 1, E_EOB = 2, E_LONG = 3, E_BAD = 4 };
enum : uint32_t { T_LIT = 0, T_DIST = 1, T_CL = 2 };

// member status codes
enum : uint32_t {
  ST_OK = 0, ST_BTYPE = 1, ST_STORED = 2, ST_COUNTS = 3, ST_CODES = 4, ST_LENS = 5, ST_SYMBOL = 6,
  ST_DIST = 7, ST_SIZE = 8, ST_OVERRUN = 9
};

struct Member {
  uint64_t in_off;   // first byte of the raw deflate data in the device file image
  uint64_t out_off;  // first byte of the member's payload in the inflated buffer
  uint32_t clen;     // deflate bytes
  uint32_t isize;    // payload bytes
};

struct InflateLds {
  uint32_t lit[1u << kLitBits];
  uint32_t dist[1u << kDistBits];  // also the code-length code table (kClBits root)
  uint16_t lsort[288];
  uint16_t dsort[32];
  uint16_t lcnt[16], loff[16], dcnt[16], doff[16];
  uint8_t lens[320 + 16];
  uint32_t ring[kRingW];
  uint8_t win[kWin];
};

__constant__ uint16_t kLenBase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                      31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2,
                                      2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t kDistBase[30] = {1,    2,    3,    4,    5,    7,     9,     13,    17,  25,
                                       33,   49,   65,   97,   129,  193,   257,   385,   513, 769,
                                       1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6,
                                       6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

__device__ __forceinline__ uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ uint32_t ent(uint32_t len, uint32_t kind, uint32_t extra, uint32_t val) {
  return len | (kind << 4) | (extra << 8) | (val << 16);
}

// entry of symbol `sym` with code length `len` in table `t`
__device__ __forceinline__ uint32_t sym_entry(uint32_t t, uint32_t sym, uint32_t len) {
  if (t == T_LIT) {
    if (sym < 256) return ent(len, E_LIT, 0, sym);
    if (sym == 256) return ent(len, E_EOB, 0, 0);
    if (sym <= 285) return ent(len, E_LEN, kLenExtra[sym - 257], kLenBase[sym - 257]);
    return ent(len, E_BAD, 0, 0);
  }
  if (t == T_DIST) return sym < 30 ? ent(len, E_LIT, kDistExtra[sym], kDistBase[sym]) : ent(len, E_BAD, 0, 0);
  return ent(len, E_LIT, 0, sym);
}

// Canonical Huffman decode table for lens[0..n) (RFC 1951 3.2.2), built by the whole wave.
// Entries of a root-bit prefix of a longer code are E_LONG (decoded by slow_decode).  Returns
// false for an over-subscribed set, or an incomplete one other than a single one-bit code
// (inftrees.c); an empty set gives an all-E_BAD table.  Per-length data lives in lane L (VGPRs)
// and in cnt_out / off_out (LDS), so the build holds no SGPR arrays next to the decode state.
__device__ bool build_table(const uint8_t* lens, uint32_t n, uint32_t root, uint32_t t, uint32_t* table,
                            uint16_t* sorted, uint16_t* cnt_out, uint16_t* off_out, uint32_t lane) {
  uint32_t mine = 0;  // lane L: #codes of length L
  for (uint32_t c = 0; c < n; c += 64) {
    const uint32_t s = c + lane;
    const uint32_t l = s < n ? lens[s] : 0;
    for (uint32_t L = 1; L < 16; L++) {
      const uint32_t k = (uint32_t)__popcll(__ballot(l == L));
      if (lane == L) mine += k;
    }
  }
  if (lane < 16) cnt_out[lane] = lane ? (uint16_t)mine : 0;
  // Kraft sum in units of 2^-15, the longest length, offsets of each length in sorted[]
  uint32_t kraft = 0, maxl = 0, off = 0;
  for (uint32_t L = 1; L < 16; L++) {
    const uint32_t k = uni(__builtin_amdgcn_readlane((int)mine, (int)L));
    kraft += k << (15 - L);
    if (k) maxl = L;
    if (lane == L) off_out[L] = (uint16_t)off;
    off += k;
  }
  if (lane == 0) off_out[0] = 0;
  if (maxl == 0) {
    for (uint32_t i = lane; i < (1u << root); i += 64) table[i] = ent(0, E_BAD, 0, 0);
    return true;
  }
  if (kraft > (1u << 15)) return false;
  if (kraft < (1u << 15) && (t == T_CL || maxl != 1)) return false;
  // symbols sorted by (length, symbol); lane L holds the running position of length L
  uint32_t run = lane < 16 ? off_out[lane] : 0;
  const uint64_t lt = (1ull << lane) - 1;
  for (uint32_t c = 0; c < n; c += 64) {
    const uint32_t s = c + lane;
    const uint32_t l = s < n ? lens[s] : 0;
    for (uint32_t L = 1; L < 16; L++) {
      const uint64_t m = __ballot(l == L);
      if (!m) continue;
      const uint32_t base = uni(__builtin_amdgcn_readlane((int)run, (int)L));
      if (l == L) sorted[base + (uint32_t)__popcll(m & lt)] = (uint16_t)s;
      if (lane == L) run += (uint32_t)__popcll(m);
    }
  }
  // per-lane copies of the per-length data for the table fill (first code: RFC next_code)
  uint32_t vcnt[11], voff[11], vfirst[11];
  uint32_t code = 0;
  vcnt[0] = voff[0] = vfirst[0] = 0;
#pragma unroll
  for (uint32_t L = 1; L <= 10; L++) {
    vcnt[L] = cnt_out[L];
    voff[L] = off_out[L];
    code = (code + vcnt[L - 1]) << 1;
    vfirst[L] = code;
  }
  const uint32_t none = maxl > root ? ent(0, E_LONG, 0, 0) : ent(0, E_BAD, 0, 0);
  for (uint32_t i = lane; i < (1u << root); i += 64) {
    uint32_t e = none;
#pragma unroll
    for (uint32_t L = 1; L <= 10; L++) {
      if (L <= root) {
        const uint32_t c = __builtin_bitreverse32(i & ((1u << L) - 1)) >> (32 - L);
        const uint32_t k = c - vfirst[L];
        if (k < vcnt[L]) e = sym_entry(t, sorted[voff[L] + k], L);
      }
    }
    table[i] = e;
  }
  return true;
}

// A code longer than the table root, bit by bit (puff.c decode()): the entry, E_BAD if none.
__device__ uint32_t slow_decode(uint64_t buf, const uint16_t* cnt, const uint16_t* sorted, uint32_t t) {
  int code = 0, first = 0, index = 0;
  for (uint32_t len = 1; len < 16; len++) {
    code |= (int)((buf >> (len - 1)) & 1);
    const int count = cnt[len];
    if (code - count < first) return sym_entry(t, sorted[index + (code - first)], len);
    index += count;
    first += count;
    first <<= 1;
    code <<= 1;
  }
  return ent(0, E_BAD, 0, 0);
}

// the wave-uniform bit reader over the LDS ring of compressed words
struct Bits {
  uint64_t buf;     // unconsumed bits, LSB first
  uint32_t cnt;     // bits in buf
  uint32_t rw;      // next word to append to buf (word index from the member's first word)
  uint32_t nw;      // ring word rw, loaded ahead
  uint32_t rfill;   // the ring holds words [rfill - kRingW, rfill)
  uint32_t px, py;  // this lane's words rfill + 2*lane, +1, loaded one refill ahead
};

__device__ __forceinline__ void ring_push(Bits& b, InflateLds& S, const uint32_t* src, uint32_t lane) {
  S.ring[(b.rfill + 2 * lane) & kRingMask] = b.px;
  S.ring[(b.rfill + 2 * lane + 1) & kRingMask] = b.py;
  b.rfill += kRingHalf;
  b.px = src[b.rfill + 2 * lane];
  b.py = src[b.rfill + 2 * lane + 1];
}

// (re)start reading at byte `q` from src
__device__ void bits_init(Bits& b, InflateLds& S, const uint32_t* src, uint32_t q, uint32_t lane) {
  const uint32_t w = q >> 2;
  b.rfill = w;
  b.px = src[w + 2 * lane];
  b.py = src[w + 2 * lane + 1];
  ring_push(b, S, src, lane);
  ring_push(b, S, src, lane);
  b.rw = w;
  b.buf = 0;
  b.cnt = 0;
  b.nw = S.ring[w & kRingMask];
}

__device__ __forceinline__ void need(Bits& b, InflateLds& S, uint32_t n) {
  if (b.cnt < n) {
    b.buf |= (uint64_t)uni(b.nw) << b.cnt;
    b.cnt += 32;
    b.rw++;
    b.nw = S.ring[b.rw & kRingMask];
  }
}
__device__ __forceinline__ void drop(Bits& b, uint32_t n) {
  b.buf >>= n;
  b.cnt -= n;
}

__device__ __forceinline__ void flush_to(InflateLds& S, uint8_t* out, uint32_t& flushed, uint32_t upto,
                                         uint32_t lane) {
  for (uint32_t j = flushed + lane; j < upto; j += 64) out[j] = S.win[j & kWinMask];
  flushed = upto;
  // far matches read flushed bytes back from HBM, other lanes' stores: a workgroup-scope
  // release / acquire pair (the wave is the workgroup) makes them visible to every lane
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// One wave per member.  status[m]: ST_* (0 = the member's payload is in out[out_off, +isize)).
__global__ __launch_bounds__(64) void k_inflate(const uint8_t* __restrict__ in, const Member* __restrict__ mem,
                                                 uint8_t* __restrict__ outbuf, uint32_t* __restrict__ status) {
  __shared__ InflateLds S;
  const uint32_t lane = threadIdx.x;
  const Member M = mem[blockIdx.x];
  if (M.isize == 0) {
    if (lane == 0) status[blockIdx.x] = ST_OK;
    return;
  }
  const uint64_t a = M.in_off;
  const uint32_t* src = reinterpret_cast<const uint32_t*>(in) + (a >> 2);
  const uint32_t skip = (uint32_t)(a & 3);
  const uint32_t limit_bits = (skip + M.clen) * 8;  // stream bits available from src word 0
  uint8_t* out = outbuf + M.out_off;
  const uint32_t isize = M.isize;
  Bits b;
  bits_init(b, S, src, 0, lane);
  need(b, S, 32);
  drop(b, skip * 8);
  uint32_t pos = 0, flushed = 0, st = ST_OK;
  bool last = false;
  while (!last && st == ST_OK) {
    need(b, S, 32);
    last = (b.buf & 1) != 0;
    const uint32_t type = (uint32_t)(b.buf >> 1) & 3;
    drop(b, 3);
    if (type == 0) {  // stored
      drop(b, b.cnt & 7);
      need(b, S, 32);
      const uint32_t len = (uint32_t)b.buf & 0xffff, nlen = (uint32_t)(b.buf >> 16) & 0xffff;
      drop(b, 32);
      if (len != (~nlen & 0xffff)) { st = ST_STORED; break; }
      const uint32_t q = (b.rw * 32 - b.cnt) >> 3;  // byte position of the stored data
      if (pos + len > isize || (q + len) * 8 > limit_bits) { st = ST_SIZE; break; }
      const uint8_t* sb = reinterpret_cast<const uint8_t*>(src) + q;
      for (uint32_t done = 0; done < len;) {
        if (pos - flushed >= kFlush) flush_to(S, out, flushed, flushed + kFlush, lane);
        const uint32_t c = min(len - done, kFlush);
        for (uint32_t j = lane; j < c; j += 64) S.win[(pos + j) & kWinMask] = sb[done + j];
        pos += c;
        done += c;
      }
      bits_init(b, S, src, q + len, lane);
      need(b, S, 32);
      drop(b, ((q + len) & 3) * 8);
      continue;
    }
    if (type == 3) { st = ST_BTYPE; break; }
    if (type == 1) {  // fixed codes
      for (uint32_t i = lane; i < 320; i += 64)
        S.lens[i] = i < 144 ? 8 : i < 256 ? 9 : i < 280 ? 7 : i < 288 ? 8 : 5;
      build_table(S.lens, 288, kLitBits, T_LIT, S.lit, S.lsort, S.lcnt, S.loff, lane);
      build_table(S.lens + 288, 32, kDistBits, T_DIST, S.dist, S.dsort, S.dcnt, S.doff, lane);
    } else {  // dynamic codes
      const uint32_t hlit = ((uint32_t)b.buf & 31) + 257, hdist = ((uint32_t)(b.buf >> 5) & 31) + 1;
      const uint32_t hclen = ((uint32_t)(b.buf >> 10) & 15) + 4;
      drop(b, 14);
      if (hlit > 286 || hdist > 30) { st = ST_COUNTS; break; }
      if (lane < 19) S.lens[lane] = 0;
      need(b, S, 32);
      const uint32_t k1 = hclen < 10 ? hclen : 10;
      if (lane < k1) S.lens[kClOrder[lane]] = (uint8_t)((b.buf >> (3 * lane)) & 7);
      drop(b, 3 * k1);
      if (hclen > 10) {
        need(b, S, 32);
        if (lane < hclen - 10) S.lens[kClOrder[10 + lane]] = (uint8_t)((b.buf >> (3 * lane)) & 7);
        drop(b, 3 * (hclen - 10));
      }
      if (!uni(build_table(S.lens, 19, kClBits, T_CL, S.dist, S.dsort, S.dcnt, S.doff, lane))) { st = ST_CODES; break; }
      const uint32_t nl = hlit + hdist;
      uint32_t i = 0, prev = 0;
      while (i < nl) {
        if (b.rfill - b.rw < kRingHalf) ring_push(b, S, src, lane);
        need(b, S, 32);
        const uint32_t e = uni(S.dist[(uint32_t)b.buf & ((1u << kClBits) - 1)]);
        if (((e >> 4) & 7) != E_LIT) { st = ST_LENS; break; }
        drop(b, e & 15);
        const uint32_t sym = e >> 16;
        if (sym < 16) {
          if (lane == 0) S.lens[i] = (uint8_t)sym;
          prev = sym;
          i++;
          continue;
        }
        uint32_t rep, val = 0;
        if (sym == 16) {
          if (i == 0) { st = ST_LENS; break; }
          rep = 3 + ((uint32_t)b.buf & 3), val = prev;
          drop(b, 2);
        } else if (sym == 17) {
          rep = 3 + ((uint32_t)b.buf & 7);
          drop(b, 3);
        } else {
          rep = 11 + ((uint32_t)b.buf & 127);
          drop(b, 7);
        }
        if (i + rep > nl) { st = ST_LENS; break; }
        for (uint32_t j = lane; j < rep; j += 64) S.lens[i + j] = (uint8_t)val;
        prev = val;
        i += rep;
      }
      if (st != ST_OK) break;
      if (uni(S.lens[256]) == 0) { st = ST_LENS; break; }
      const uint32_t ok1 = uni(build_table(S.lens, hlit, kLitBits, T_LIT, S.lit, S.lsort, S.lcnt, S.loff, lane));
      const uint32_t ok2 = uni(build_table(S.lens + hlit, hdist, kDistBits, T_DIST, S.dist, S.dsort, S.dcnt, S.doff, lane));
      if (!ok1 || !ok2) {
        st = ST_CODES;
        break;
      }
    }
    // the block's symbols
    while (true) {
      if (pos - flushed >= kFlush) flush_to(S, out, flushed, flushed + kFlush, lane);
      if (b.rfill - b.rw < kRingHalf) ring_push(b, S, src, lane);
      if (b.rw * 32 > limit_bits + 64) { st = ST_OVERRUN; break; }
      need(b, S, 32);
      uint32_t e = uni(S.lit[(uint32_t)b.buf & ((1u << kLitBits) - 1)]);
      uint32_t kind = (e >> 4) & 7;
      if (kind == E_LONG) {
        e = uni(slow_decode(b.buf, S.lcnt, S.lsort, T_LIT));
        kind = (e >> 4) & 7;
      }
      drop(b, e & 15);
      if (kind == E_LIT) {
        if (pos >= isize) { st = ST_SIZE; break; }
        if (lane == 0) S.win[pos & kWinMask] = (uint8_t)(e >> 16);
        pos++;
        continue;
      }
      if (kind == E_EOB) break;
      if (kind != E_LEN) { st = ST_SYMBOL; break; }
      const uint32_t lx = (e >> 8) & 31;
      const uint32_t len = (e >> 16) + ((uint32_t)b.buf & ((1u << lx) - 1));
      drop(b, lx);
      need(b, S, 28);
      uint32_t de = uni(S.dist[(uint32_t)b.buf & ((1u << kDistBits) - 1)]);
      uint32_t dk = (de >> 4) & 7;
      if (dk == E_LONG) {
        de = uni(slow_decode(b.buf, S.dcnt, S.dsort, T_DIST));
        dk = (de >> 4) & 7;
      }
      if (dk != E_LIT) { st = ST_DIST; break; }
      drop(b, de & 15);
      const uint32_t dx = (de >> 8) & 31;
      const uint32_t dist = (de >> 16) + ((uint32_t)b.buf & ((1u << dx) - 1));
      drop(b, dx);
      if (dist > pos) { st = ST_DIST; break; }
      if (pos + len > isize) { st = ST_SIZE; break; }
      if (dist <= kWin) {  // wave-uniform: every source byte is in the window
        for (uint32_t j = lane; j < len; j += 64) {
          uint32_t r = j;
          if (dist < len) {  // overlapping: the last `dist` bytes repeat
            r = j - (uint32_t)((float)j * __frcp_rn((float)dist)) * dist;
            r = (int)r < 0 ? r + dist : r;
            r = r >= dist ? r - dist : r;
          }
          S.win[(pos + j) & kWinMask] = S.win[(pos - dist + r) & kWinMask];
        }
      } else {  // a far match (len <= 258 < dist): its older bytes come from the flushed output
        // a source byte is read from the window only if no destination of this copy shares its
        // slot (p >= pos + len - kWin: an earlier 64-byte round could have overwritten it); the
        // others were flushed (flushed > pos - kFlush - 258 > pos + len - kWin)
        for (uint32_t j = lane; j < len; j += 64) {
          const uint32_t p = pos - dist + j;
          S.win[(pos + j) & kWinMask] = dist - j + len <= kWin ? S.win[p & kWinMask] : out[p];
        }
      }
      pos += len;
    }
  }
  if (st == ST_OK && (pos != isize || b.rw * 32 - b.cnt > limit_bits)) st = pos != isize ? ST_SIZE : ST_OVERRUN;
  if (st == ST_OK) flush_to(S, out, flushed, pos, lane);
  if (lane == 0) status[blockIdx.x] = st;
}

}  // namespace gb
