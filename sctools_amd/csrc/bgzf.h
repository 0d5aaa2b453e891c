// bgzf.h -- BGZF / BAM helpers shared by the native decoder (bamdec.cpp) and splitter
// (bamsplit.cpp): little-endian reads, the lock-striped string interner, BGZF member scan
// (SAM/BAM spec 4.1) and inflate, and the BGZF writer's deflate of one block.  Host C++ (zlib).
#pragma once
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <zlib.h>

#include <atomic>
#include <mutex>
#include <string>
#include <vector>

// the calling thread's last error, shared by every entry point of libsct_bam.so
namespace sctbam {
inline thread_local std::string g_err;
inline int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
inline int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}
}  // namespace sctbam

namespace {
using sctbam::fail;
using sctbam::g_err;

inline uint16_t rd16(const uint8_t* p) {
  uint16_t v;
  memcpy(&v, p, 2);
  return v;
}
inline uint32_t rd32(const uint8_t* p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}


// ---------------- string interning ----------------
inline uint64_t hash_bytes(const char* p, size_t n) {
  uint64_t h = 1469598103934665603ull;  // FNV-1a, then a mix
  for (size_t i = 0; i < n; i++) h = (h ^ (uint8_t)p[i]) * 1099511628211ull;
  h ^= h >> 29;
  h *= 0xBF58476D1CE4E5B9ull;
  h ^= h >> 32;
  return h;
}

class Interner {
 public:
  static constexpr int kStripes = 256;
  Interner() : next_(1) {}
  // provisional id >= 1 of the string
  int32_t intern(const char* p, size_t n) { return intern(p, n, hash_bytes(p, n)); }
  int32_t intern(const char* p, size_t n, uint64_t h) {
    Stripe& s = stripes_[h & (kStripes - 1)];
    std::lock_guard<std::mutex> lk(s.m);
    if (s.slots.empty()) s.slots.assign(64, Slot{0, 0, 0, 0});
    size_t mask = s.slots.size() - 1;
    size_t i = (h >> 8) & mask;
    while (true) {
      Slot& e = s.slots[i];
      if (e.pid == 0) break;
      if (e.hash == h && e.len == n && memcmp(s.arena.data() + e.off, p, n) == 0) return e.pid;
      i = (i + 1) & mask;
    }
    const int32_t pid = next_.fetch_add(1);
    Slot ne{h, (uint32_t)s.arena.size(), (uint32_t)n, pid};
    s.arena.append(p, n);
    s.slots[i] = ne;
    if (++s.used * 2 > s.slots.size()) grow(s);
    return pid;
  }
  int32_t count() const { return next_.load() - 1; }
  // all (string, provisional id)
  void collect(std::vector<std::pair<std::string, int32_t>>& out) const {
    for (const Stripe& s : stripes_)
      for (const Slot& e : s.slots)
        if (e.pid) out.emplace_back(std::string(s.arena.data() + e.off, e.len), e.pid);
  }

 private:
  struct Slot {
    uint64_t hash;
    uint32_t off, len;
    int32_t pid;
  };
  struct Stripe {
    std::mutex m;
    std::vector<Slot> slots;
    std::string arena;
    size_t used = 0;
  };
  static void grow(Stripe& s) {
    std::vector<Slot> old;
    old.swap(s.slots);
    s.slots.assign(old.size() * 2, Slot{0, 0, 0, 0});
    const size_t mask = s.slots.size() - 1;
    for (const Slot& e : old) {
      if (!e.pid) continue;
      size_t i = (e.hash >> 8) & mask;
      while (s.slots[i].pid) i = (i + 1) & mask;
      s.slots[i] = e;
    }
  }
  Stripe stripes_[kStripes];
  std::atomic<int32_t> next_;
};

// a tag's value as the Python reader sees it: a string (Z, H, A; integers printed in decimal
// for the string tags) or an integer; float and array values (f, d, B) keep their raw bytes
// (`raw`: s, n), so that distinct values stay distinct where a value is only a key
struct TagVal {
  bool present = false, is_str = false, raw = false;
  char type = 0;
  const char* s = nullptr;
  size_t n = 0;
  int64_t i = 0;
  char num[24];
};

// Z/H/A/integer/float/array value at p (type t) within [p, end); returns the bytes the value
// occupies, or 0 for an unknown type or a value running past `end` (a malformed record)
inline size_t read_tag(const uint8_t* p, const uint8_t* end, char t, TagVal* v) {
  const size_t room = end > p ? (size_t)(end - p) : 0;
  size_t w = 0;
  switch (t) {
    case 'Z':
    case 'H': {
      const uint8_t* z = room ? (const uint8_t*)memchr(p, 0, room) : nullptr;
      if (!z) return 0;
      if (v) v->present = true, v->is_str = true, v->s = (const char*)p, v->n = z - p;
      if (v) v->type = t;
      return z - p + 1;
    }
    case 'A':
      if (room < 1) return 0;
      if (v) v->present = true, v->is_str = true, v->s = (const char*)p, v->n = 1, v->type = t;
      return 1;
    case 'c': case 'C': w = 1; break;
    case 's': case 'S': w = 2; break;
    case 'i': case 'I': case 'f': w = 4; break;
    case 'd': w = 8; break;
    case 'B': {
      if (room < 5) return 0;
      const char sub = (char)p[0];
      const size_t ew = (sub == 'c' || sub == 'C') ? 1 : (sub == 's' || sub == 'S') ? 2
                      : (sub == 'i' || sub == 'I' || sub == 'f') ? 4 : 0;
      if (!ew) return 0;
      const uint64_t len = 5 + (uint64_t)rd32(p + 1) * ew;
      if (len > room) return 0;
      if (v) v->present = true, v->raw = true, v->type = t, v->s = (const char*)p, v->n = (size_t)len;
      return (size_t)len;
    }
    default:
      return 0;
  }
  if (w > room) return 0;
  if (v) {
    v->present = true;
    v->type = t;
    switch (t) {
      case 'c': v->i = (int8_t)p[0]; break;
      case 'C': v->i = p[0]; break;
      case 's': v->i = (int16_t)rd16(p); break;
      case 'S': v->i = rd16(p); break;
      case 'i': v->i = (int32_t)rd32(p); break;
      case 'I': v->i = rd32(p); break;
      default: v->raw = true, v->s = (const char*)p, v->n = w; break;  // f, d
    }
  }
  return w;
}

// the string form of an integer value (the Python tag value passed through str()); string and
// raw values are left as they are
inline void as_str(TagVal& v) {
  if (!v.present || v.is_str || v.raw) return;
  snprintf(v.num, sizeof(v.num), "%lld", (long long)v.i);
  v.s = v.num;
  v.n = strlen(v.num);
  v.is_str = true;
}

// ---------------- BGZF ----------------
struct Block {
  uint64_t off;
  uint32_t csize, isize;
};

inline int scan_blocks(const uint8_t* f, uint64_t size, std::vector<Block>& blocks) {
  uint64_t off = 0;
  while (off < size) {
    if (size - off < 18 || f[off] != 31 || f[off + 1] != 139 || f[off + 2] != 8 || !(f[off + 3] & 4))
      return fail(SCT_BAM_EFORMAT, "not a BGZF block at byte %llu", (unsigned long long)off);
    const uint16_t xlen = rd16(f + off + 10);
    uint64_t p = off + 12, end = off + 12 + xlen;
    int64_t bsize = -1;
    while (p + 4 <= end) {
      const uint16_t slen = rd16(f + p + 2);
      if (f[p] == 66 && f[p + 1] == 67 && slen == 2) bsize = rd16(f + p + 4);
      p += 4 + slen;
    }
    if (bsize < 0 || off + (uint64_t)bsize + 1 > size)
      return fail(SCT_BAM_EFORMAT, "bad BGZF block size at byte %llu", (unsigned long long)off);
    const uint32_t csize = (uint32_t)bsize + 1;
    const uint32_t isize = rd32(f + off + csize - 4);
    blocks.push_back(Block{off, csize, isize});
    off += csize;
  }
  return SCT_BAM_OK;
}

inline bool inflate_block(const uint8_t* f, const Block& b, uint8_t* out, z_stream& z) {
  const uint16_t xlen = rd16(f + b.off + 10);
  const uint64_t data = b.off + 12 + xlen;
  const uint32_t clen = b.csize - 12 - xlen - 8;
  if (inflateReset(&z) != Z_OK) return false;
  z.next_in = const_cast<Bytef*>(f + data);
  z.avail_in = clen;
  z.next_out = out;
  z.avail_out = b.isize;
  const int rc = inflate(&z, Z_FINISH);
  return rc == Z_STREAM_END && z.avail_out == 0;
}

// ---------------- BGZF writer ----------------
constexpr size_t kBgzfMaxInput = 0xff00;  // uncompressed bytes per block (as htslib writes them)

// One BGZF member holding `n` <= kBgzfMaxInput bytes, appended to `out`.  `z` is a raw-deflate
// stream (deflateInit2(..., -15, ...)) reused across calls.  Returns false on a zlib error.
inline bool bgzf_block(const uint8_t* in, size_t n, int level, z_stream& z, std::vector<uint8_t>& out) {
  const size_t h = out.size();
  out.resize(h + 18 + deflateBound(&z, n) + 8 + 64);
  uint8_t* o = out.data() + h;
  static const uint8_t head[16] = {31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 66, 67, 2, 0};
  memcpy(o, head, 16);
  if (deflateReset(&z) != Z_OK || deflateParams(&z, level, Z_DEFAULT_STRATEGY) != Z_OK) return false;
  z.next_in = const_cast<Bytef*>(in);
  z.avail_in = (uInt)n;
  z.next_out = o + 18;
  z.avail_out = (uInt)(out.size() - h - 18 - 8);
  if (deflate(&z, Z_FINISH) != Z_STREAM_END) return false;
  size_t clen = z.total_out;
  if (18 + clen + 8 > 65536) {  // incompressible: store
    if (deflateReset(&z) != Z_OK || deflateParams(&z, 0, Z_DEFAULT_STRATEGY) != Z_OK) return false;
    z.next_in = const_cast<Bytef*>(in);
    z.avail_in = (uInt)n;
    z.next_out = o + 18;
    z.avail_out = (uInt)(out.size() - h - 18 - 8);
    if (deflate(&z, Z_FINISH) != Z_STREAM_END) return false;
    clen = z.total_out;
  }
  const uint32_t bsize = (uint32_t)(18 + clen + 8 - 1);
  o[16] = (uint8_t)(bsize & 0xff);
  o[17] = (uint8_t)(bsize >> 8);
  const uint32_t crc = (uint32_t)crc32(crc32(0L, Z_NULL, 0), in, (uInt)n);
  const uint32_t isz = (uint32_t)n;
  memcpy(o + 18 + clen, &crc, 4);
  memcpy(o + 18 + clen + 4, &isz, 4);
  out.resize(h + 18 + clen + 8);
  return true;
}

// the empty member that ends a BGZF file (SAM/BAM spec 4.1.2)
const uint8_t kBgzfEof[28] = {31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 66, 67, 2, 0,
                              27, 0, 3, 0, 0, 0, 0, 0, 0, 0, 0, 0};

}  // namespace
