// fixedpt.h -- exact, order-free mean / variance for the metric streams.
//
// The reference updates a Welford accumulator per record
// (OnlineGaussianSufficientStatistic.update, src/sctools/stats.py:82-87), which
// is sequential and order dependent.  SCT_FLOAT_EXACT_SUM replaces it with
// exact integer sums that any number of threads, tiles or GPUs can add in any
// order:
//
//   every stream value x is a double RN(a/b) with 1 <= b < 2^16 (a quality
//   fraction or a mean quality), so x == 0 or x >= 2^-16, hence X = x * 2^68
//   is an integer (< 2^75 for Phred <= 93).  Per entity we keep
//     S = sum X     as 3 lanes of 32-bit limb sums,
//     Q = sum X^2   as 5 lanes of 32-bit limb sums,
//   each lane a plain int64 sum (headroom: < 2^31 records per entity).
//   mean = RN(S / (n 2^68)),  var = RN((n Q - S^2) / (n (n-1) 2^136)),
//   both correctly rounded from the exact rationals.
//
// Used by the HIP kernels (device) and compiled on the host by the tests.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define SCT_HD __host__ __device__ __forceinline__
#else
#define SCT_HD static inline
#endif

namespace sct {

constexpr int kStreamLanes = 8;  // 3 lanes of sum X + 5 lanes of sum X^2

SCT_HD uint64_t umulhi64(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umul64hi(a, b);
#else
  return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}

SCT_HD int clz64(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return x ? __clzll((long long)x) : 64;
#else
  return x ? __builtin_clzll(x) : 64;
#endif
}

SCT_HD uint64_t dbits(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return (uint64_t)__double_as_longlong(x);
#else
  union {
    double d;
    uint64_t u;
  } v;
  v.d = x;
  return v.u;
#endif
}

// The 8 lane increments of one sample x (fx_accumulate adds exactly these): X = x*2^68 and X^2
// as 32-bit limb pieces.  x must be 0 or in [2^-16, 2^16).  inc[7] (bits >= 128 of X^2) is
// returned as 64 bits: it exceeds 32 bits only for x >= 2^12.
// The 53-bit significand is split as m = mh 2^32 + ml (mh < 2^21), so m^2 takes three 32x32
// products instead of a general 64x64 multiply, and the shifts by s and 2s use the
// (v >> 1) >> (63 - k) form, which needs no select for k == 0.
SCT_HD void fx_increments(double x, uint32_t (&inc)[kStreamLanes - 1], uint64_t& inc7) {
  const uint64_t b = dbits(x);
  const uint32_t bhi = (uint32_t)(b >> 32);
  const int ex = (int)((bhi >> 20) & 0x7ff);
  // x == 0 adds zeros (branch-free: m = 0, s = 0)
  const uint32_t mh = ex ? ((bhi & 0xFFFFFu) | 0x100000u) : 0u;
  const uint32_t ml = ex ? (uint32_t)b : 0u;
  const int s = ex ? ex - 1007 : 0;  // X = m << s, 0 <= s <= 31
  const uint64_t m = ((uint64_t)mh << 32) | ml;
  const uint64_t lo = m << s;
  const uint32_t hi = (uint32_t)(((uint64_t)mh << s) >> 32);
  inc[0] = (uint32_t)lo;
  inc[1] = (uint32_t)(lo >> 32);
  inc[2] = hi;
  // m^2 = A + 2B 2^32 + C 2^64
  const uint64_t A = (uint64_t)ml * ml;
  const uint64_t B2 = ((uint64_t)ml * mh) << 1;  // < 2^54
  const uint64_t C = (uint64_t)mh * mh;          // < 2^42
  const uint64_t plo = A + (B2 << 32);
  const uint64_t phi = C + (B2 >> 32) + (plo < A ? 1u : 0u);
  const int t = 2 * s;  // < 64
  const uint64_t w0 = plo << t;
  const uint64_t w1 = (phi << t) | ((plo >> 1) >> (63 - t));
  const uint64_t w2 = (phi >> 1) >> (63 - t);
  inc[3] = (uint32_t)w0;
  inc[4] = (uint32_t)(w0 >> 32);
  inc[5] = (uint32_t)w1;
  inc[6] = (uint32_t)(w1 >> 32);
  inc7 = w2;
}

// Add X = x*2^68 and X^2 into 8 lanes (limb sums).  x must be 0 or in [2^-16, 2^16).
SCT_HD void fx_accumulate(int64_t* lanes, double x) {
  uint32_t inc[kStreamLanes - 1];
  uint64_t inc7;
  fx_increments(x, inc, inc7);
  for (int k = 0; k < kStreamLanes - 1; k++) lanes[k] += (int64_t)inc[k];
  lanes[kStreamLanes - 1] += (int64_t)inc7;
}

// ---- small fixed-size unsigned big integers (little-endian 64-bit limbs) ----
constexpr int kW = 6;  // 384 bits
struct Big {
  uint64_t w[kW];
};

SCT_HD void big_zero(Big& a) {
  for (int i = 0; i < kW; i++) a.w[i] = 0;
}

// a += v * 2^(32*k)  (v < 2^63)
SCT_HD void big_add_shifted32(Big& a, uint64_t v, int k) {
  const int word = k / 2;
  const int sh = (k & 1) * 32;
  uint64_t lo = v << sh;
  uint64_t hi = sh ? (v >> (64 - sh)) : 0;
  uint64_t carry = 0;
  for (int i = word; i < kW; i++) {
    uint64_t add = (i == word) ? lo : (i == word + 1 ? hi : 0);
    uint64_t s1 = a.w[i] + add;
    uint64_t c1 = s1 < add;
    uint64_t s2 = s1 + carry;
    uint64_t c2 = s2 < carry;
    a.w[i] = s2;
    carry = c1 + c2;
    if (i > word + 1 && carry == 0) break;
  }
}

SCT_HD int big_bitlen(const Big& a) {
  for (int i = kW - 1; i >= 0; i--)
    if (a.w[i]) return 64 * i + (64 - clz64(a.w[i]));
  return 0;
}

SCT_HD void big_shl(Big& a, int k) {
  const int ws = k / 64, bs = k % 64;
  for (int i = kW - 1; i >= 0; i--) {
    uint64_t v = 0;
    const int src = i - ws;
    if (src >= 0) {
      v = a.w[src] << bs;
      if (bs && src - 1 >= 0) v |= a.w[src - 1] >> (64 - bs);
    }
    a.w[i] = v;
  }
}

// a * v (v < 2^64), truncated to kW words
SCT_HD void big_mul_small(Big& a, uint64_t v) {
  uint64_t carry = 0;
  for (int i = 0; i < kW; i++) {
    const uint64_t lo = a.w[i] * v;
    const uint64_t hi = umulhi64(a.w[i], v);
    const uint64_t s = lo + carry;
    carry = hi + (s < lo);
    a.w[i] = s;
  }
}

// r = a * b truncated to kW words
SCT_HD void big_mul(const Big& a, const Big& b, Big& r) {
  big_zero(r);
  for (int i = 0; i < kW; i++) {
    if (!a.w[i]) continue;
    uint64_t carry = 0;
    for (int j = 0; i + j < kW; j++) {
      const uint64_t lo = a.w[i] * b.w[j];
      const uint64_t hi = umulhi64(a.w[i], b.w[j]);
      uint64_t s = r.w[i + j] + lo;
      uint64_t c = s < lo;
      s += carry;
      c += s < carry;
      r.w[i + j] = s;
      carry = hi + c;
    }
  }
}

// a -= b (requires a >= b)
SCT_HD void big_sub(Big& a, const Big& b) {
  uint64_t borrow = 0;
  for (int i = 0; i < kW; i++) {
    const uint64_t bi = b.w[i] + borrow;
    const uint64_t nb = (bi < borrow) || (a.w[i] < bi);
    a.w[i] -= bi;
    borrow = nb;
  }
}

// floor((u1:u0) / v) with u1 < v (Hacker's Delight divlu, 32-bit digits)
SCT_HD uint64_t divlu(uint64_t u1, uint64_t u0, uint64_t v, uint64_t* rem) {
  const uint64_t b = 1ull << 32;
  const int s = clz64(v);
  v <<= s;
  const uint64_t vn1 = v >> 32, vn0 = v & 0xffffffffu;
  const uint64_t un32 = (u1 << s) | (s ? (u0 >> (64 - s)) : 0);
  const uint64_t un10 = u0 << s;
  const uint64_t un1 = un10 >> 32, un0 = un10 & 0xffffffffu;
  uint64_t q1 = un32 / vn1;
  uint64_t rhat = un32 - q1 * vn1;
  while (q1 >= b || q1 * vn0 > b * rhat + un1) {
    q1--;
    rhat += vn1;
    if (rhat >= b) break;
  }
  const uint64_t un21 = un32 * b + un1 - q1 * v;
  uint64_t q0 = un21 / vn1;
  rhat = un21 - q0 * vn1;
  while (q0 >= b || q0 * vn0 > b * rhat + un0) {
    q0--;
    rhat += vn1;
    if (rhat >= b) break;
  }
  if (rem) *rem = (un21 * b + un0 - q0 * v) >> s;
  return q1 * b + q0;
}

// q = a / v, returns remainder
SCT_HD uint64_t big_div_small(const Big& a, uint64_t v, Big& q) {
  uint64_t r = 0;
  for (int i = kW - 1; i >= 0; i--) q.w[i] = divlu(r, a.w[i], v, &r);
  return r;
}

SCT_HD int big_bit(const Big& a, int i) { return (int)((a.w[i / 64] >> (i % 64)) & 1u); }

SCT_HD int big_any_below(const Big& a, int nbits) {
  for (int i = 0; i < nbits / 64; i++)
    if (a.w[i]) return 1;
  const int r = nbits % 64;
  if (r && (a.w[nbits / 64] & ((1ull << r) - 1))) return 1;
  return 0;
}

// bits [lo, lo+53) of a as an integer
SCT_HD uint64_t big_extract53(const Big& a, int lo) {
  const int w = lo / 64, b = lo % 64;
  uint64_t v = a.w[w] >> b;
  if (b && w + 1 < kW) v |= a.w[w + 1] << (64 - b);
  return v & ((1ull << 53) - 1);
}

SCT_HD double sct_ldexp(double x, int e) {
  // exact scaling by 2^e for results in the normal range
  while (e > 1000) {
    x *= 0x1p1000;
    e -= 1000;
  }
  while (e < -1000) {
    x *= 0x1p-1000;
    e += 1000;
  }
  const uint64_t bits = (uint64_t)(e + 1023) << 52;
#if defined(__HIP_DEVICE_COMPILE__)
  return x * __longlong_as_double((long long)bits);
#else
  union {
    uint64_t u;
    double d;
  } v;
  v.u = bits;
  return x * v.d;
#endif
}

// RN(num / d * 2^e2), num >= 0, d >= 1, result assumed normal.
SCT_HD double big_div_to_double(Big num, uint64_t d, int e2) {
  const int nb = big_bitlen(num);
  if (nb == 0) return 0.0;
  const int db = 64 - clz64(d);
  int k = 0;
  const int want = db + 66;  // quotient >= 2^65
  if (nb < want) {
    k = want - nb;
    big_shl(num, k);
  }
  Big q;
  const uint64_t rem = big_div_small(num, d, q);
  const int qb = big_bitlen(q);
  int drop = qb - 53;
  uint64_t mant = big_extract53(q, drop) | (1ull << 52);
  const int round = big_bit(q, drop - 1);
  const int sticky = (rem != 0) || big_any_below(q, drop - 1);
  if (round && (sticky || (mant & 1))) {
    mant += 1;
    if (mant == (1ull << 53)) {
      mant >>= 1;
      drop += 1;
    }
  }
  return sct_ldexp((double)mant, drop - k + e2);
}

// mean and variance of one stream from its 8 lanes and the record count n
SCT_HD void fx_finalize(const int64_t* lanes, int64_t n, double* mean, double* var) {
  if (n <= 0) {
    *mean = 0.0;
    *var = __builtin_nan("");
    return;
  }
  Big s;
  big_zero(s);
  for (int k = 0; k < 3; k++) big_add_shifted32(s, (uint64_t)lanes[k], k);
  *mean = big_div_to_double(s, (uint64_t)n, -68);
  if (n < 2) {
    *var = __builtin_nan("");
    return;
  }
  Big q;
  big_zero(q);
  for (int k = 0; k < 5; k++) big_add_shifted32(q, (uint64_t)lanes[3 + k], k);
  big_mul_small(q, (uint64_t)n);
  Big s2;
  big_mul(s, s, s2);
  big_sub(q, s2);
  *var = big_div_to_double(q, (uint64_t)n * (uint64_t)(n - 1), -136);
}

}  // namespace sct
