// bgzf.h -- BGZF / BAM helpers shared by the native decoder (bamdec.cpp) and splitter
// (bamsplit.cpp): little-endian reads, BGZF member scan (SAM/BAM spec 4.1) and inflate, and
// the BGZF writer's deflate of one block.  Host C++ (zlib).
#pragma once
#include <stdint.h>
#include <string.h>
#include <zlib.h>

#include <vector>

namespace {

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


// ---------------- BGZF ----------------
struct Block {
  uint64_t off;
  uint32_t csize, isize;
};

int fail(int code, const char* fmt, ...);

int scan_blocks(const uint8_t* f, uint64_t size, std::vector<Block>& blocks) {
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

bool inflate_block(const uint8_t* f, const Block& b, uint8_t* out, z_stream& z) {
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
bool bgzf_block(const uint8_t* in, size_t n, int level, z_stream& z, std::vector<uint8_t>& out) {
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
