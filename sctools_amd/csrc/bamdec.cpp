// bamdec.cpp -- native BAM -> 32-byte SoA columns (include/sct_bam.h).
//
// Host code: zlib for the BGZF members, OpenMP for parallel inflate / parse / intern.
//   1. The file is memory-mapped; BGZF block boundaries are found by hopping the BSIZE
//      fields (SAM/BAM spec 4.1).
//   2. Windows of ~256 MB of uncompressed data: blocks inflated concurrently into one buffer
//      (a record cut by the window end is carried into the next window), record starts
//      found by hopping block_size, records parsed concurrently.
//   3. Per record, the fields the reference's aggregation reads (aggregator.py:251-334,
//      507-530) with the same validation order and exception classes as
//      sctools_amd.columnar.record_fields: CY, CR (cell metrics), UY, the aligned qualities
//      (pysam 0.16 getQueryStart / getQueryEnd soft-clip trimming, None when absent), XF and
//      NH on mapped reads, then the 32-byte limits.
//   4. CB / UB / GE strings are interned in lock-striped open-addressing tables to provisional
//      ids, then ranked: ids are positions in the sorted string list, a missing tag first --
//      the order of Python's sorted() on the decoded strings (bytes >= 0x80 decode to U+FFFD,
//      as the Python reader's "ascii"/"replace" does).
#include <fcntl.h>
#include <omp.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/sct_bam.h"
#include "bgzf.h"

namespace {

// bits / xf codes: sctools_amd/columnar.py, include/sctools_gpu.h
enum : uint8_t {
  B_UNMAPPED = 1u << 0,
  B_REVERSE = 1u << 1,
  B_DUPLICATE = 1u << 2,
  B_SPLICED = 1u << 3,
  B_NH1 = 1u << 4,
  B_PERFECT_UMI = 1u << 5,
  B_HAS_CB = 1u << 6,
  B_PERFECT_CB = 1u << 7,
};
enum : uint8_t { XF_ABSENT = 0, XF_CODING, XF_INTRONIC, XF_UTR, XF_INTERGENIC, XF_OTHER };

// ---------------- records ----------------
struct Columns {
  std::vector<int32_t> cell, umi, gene, ref, pos;
  std::vector<uint16_t> gq_sum, gq_len, gq_gt30;
  std::vector<uint8_t> bits, xf, cy_gt30, cy_len, uy_gt30, uy_len;
  std::vector<uint8_t> qhead;   // count-matrix mode only
  std::vector<int32_t> qname;   // sort-key mode only
  void resize(size_t n) {
    cell.resize(n), umi.resize(n), gene.resize(n), ref.resize(n), pos.resize(n);
    gq_sum.resize(n), gq_len.resize(n), gq_gt30.resize(n);
    bits.resize(n), xf.resize(n), cy_gt30.resize(n), cy_len.resize(n), uy_gt30.resize(n), uy_len.resize(n);
  }
};

bool str_eq(const TagVal& a, const TagVal& b) { return a.n == b.n && memcmp(a.s, b.s, a.n) == 0; }
// Python == of two present tag values of the kinds read_tag distinguishes
bool val_eq(const TagVal& a, const TagVal& b) {
  if (a.is_str || b.is_str) return a.is_str && b.is_str && str_eq(a, b);
  if (a.raw || b.raw) return a.raw && b.raw && a.type == b.type && str_eq(a, b);
  return a.i == b.i;
}

struct RecErr {
  int code = 0;
  std::string msg;
};

// #chars with Phred (char - 33) > 30, and the length: _quality_string_to_numeric +
// _quality_above_threshold (aggregator.py:191-231)
int frac_counts(const TagVal& v, uint32_t* gt, uint32_t* len, RecErr& e) {
  if (!v.is_str) {
    e.code = SCT_BAM_TYPEERROR;
    e.msg = "object of type 'int' has no len()";
    return -1;
  }
  if (v.n == 0) {
    e.code = SCT_BAM_ZERODIV;
    e.msg = "division by zero";
    return -1;
  }
  uint32_t g = 0;
  for (size_t i = 0; i < v.n; i++) g += ((uint8_t)v.s[i] > 63) ? 1u : 0u;
  *gt = g;
  *len = (uint32_t)v.n;
  return 0;
}

struct Parsed {
  int32_t ref, pos;
  uint32_t gq_sum, gq_len, gq_gt30, cy_gt30, cy_len, uy_gt30, uy_len;
  uint8_t bits, xf;
  TagVal cb, ub, ge;
};

// A dictionary tag whose value the native path cannot key as the Python reader does: a float or
// an array (any mode), or an integer where the order of the values matters (sort keys: Python
// compares ints numerically, and an int with a str raises TypeError, bam.py:660-668).  The
// caller then decodes with the Python reader (SCT_BAM_ETYPED).
int typed_keys(const Parsed& o, bool ints, RecErr& e) {
  for (const TagVal* v : {&o.cb, &o.ub, &o.ge})
    if (v->present && (v->raw || (ints && !v->is_str))) {
      e.code = SCT_BAM_ETYPED;
      e.msg = std::string("a dictionary tag holds a value of type ") + v->type;
      return -1;
    }
  return 0;
}

// One record (bytes after block_size).  Mirrors sctools_amd.columnar.record_fields.
int parse_record(const uint8_t* d, uint32_t bs, bool is_cell, Parsed& o, RecErr& e) {
  if (bs < 32) {
    e.code = SCT_BAM_EFORMAT;
    e.msg = "truncated BAM record";
    return -1;
  }
  const int32_t ref = (int32_t)rd32(d), pos = (int32_t)rd32(d + 4);
  const uint32_t l_read_name = d[8];
  const uint32_t n_cigar = rd16(d + 12), flag = rd16(d + 14);
  const uint32_t l_seq = rd32(d + 16);
  const uint64_t cig_off = 32 + (uint64_t)l_read_name;
  const uint64_t qual_off = cig_off + 4ull * n_cigar + (l_seq + 1) / 2;
  const uint64_t tag_off = qual_off + l_seq;
  if (tag_off > bs) {
    e.code = SCT_BAM_EFORMAT;
    e.msg = "truncated BAM record";
    return -1;
  }
  const uint8_t* cig = d + cig_off;
  const uint8_t* qual = d + qual_off;
  // tags of interest
  TagVal cb, cr, cy, ub, ur, uy, ge, xf, nh;
  const uint8_t* p = d + tag_off;
  const uint8_t* end = d + bs;
  while (p + 3 <= end) {
    const char a = (char)p[0], b = (char)p[1], t = (char)p[2];
    p += 3;
    TagVal* v = nullptr;
    if (a == 'C' && b == 'B') v = &cb;
    else if (a == 'C' && b == 'R') v = &cr;
    else if (a == 'C' && b == 'Y') v = &cy;
    else if (a == 'U' && b == 'B') v = &ub;
    else if (a == 'U' && b == 'R') v = &ur;
    else if (a == 'U' && b == 'Y') v = &uy;
    else if (a == 'G' && b == 'E') v = &ge;
    else if (a == 'X' && b == 'F') v = &xf;
    else if (a == 'N' && b == 'H') v = &nh;
    const size_t used = read_tag(p, end, t, v);
    if (!used || p + used > end) {
      e.code = SCT_BAM_EFORMAT;
      e.msg = std::string("unsupported or truncated BAM tag type ") + t;
      return -1;
    }
    p += used;
  }
  // gene metrics skip validation for multi-gene runs (gatherer.py:210-212)
  bool validate = is_cell;
  if (!is_cell) {
    TagVal g = ge;  // str(ge) without touching ge (its string form may point into g.num)
    as_str(g);
    validate = !(g.present && g.n > 0 && memchr(g.s, ',', g.n));
  }
  uint8_t bits = 0;
  uint32_t cg = 0, cl = 0, ug = 0, ul = 0;
  if (is_cell) {
    if (!cy.present) {
      e.code = SCT_BAM_KEYERROR;
      e.msg = "CY";
      return -1;
    }
    if (frac_counts(cy, &cg, &cl, e)) return -1;
    if (cb.present) {
      bits |= B_HAS_CB;
      if (!cr.present) {
        e.code = SCT_BAM_KEYERROR;
        e.msg = "CR";
        return -1;
      }
      // CR == CB compares the Python values: equal only for equal types and contents
      if (val_eq(cr, cb)) bits |= B_PERFECT_CB;
    }
  } else if (cb.present) {
    bits |= B_HAS_CB;
  }
  if (validate) {
    if (!uy.present) {
      e.code = SCT_BAM_KEYERROR;
      e.msg = "UY";
      return -1;
    }
    if (frac_counts(uy, &ug, &ul, e)) return -1;
  } else if (uy.present && (uy.is_str ? uy.n > 0 : uy.i != 0)) {  // `if uyq:` on the default-"" value
    if (frac_counts(uy, &ug, &ul, e)) return -1;
  }
  if (ur.present && ub.present && val_eq(ur, ub))
    bits |= B_PERFECT_UMI;
  // query_alignment_qualities (pysam 0.16)
  bool aq_none = l_seq == 0 || qual[0] == 0xFF;
  uint32_t q0 = 0, q1 = 0;
  if (!aq_none) {
    uint32_t start = 0;
    for (uint32_t k = 0; k < n_cigar; k++) {
      const uint32_t c = rd32(cig + 4 * k), op = c & 0xF, len = c >> 4;
      if (op == 5) {  // H
        if (start != 0 && start != l_seq) {
          e.code = SCT_BAM_VALUEERROR;
          e.msg = "Invalid clipping in CIGAR string";
          return -1;
        }
      } else if (op == 4) {  // S
        start += len;
      } else {
        break;
      }
    }
    uint32_t qend = l_seq;
    for (int k = (int)n_cigar - 1; k > 0; k--) {
      const uint32_t c = rd32(cig + 4 * k), op = c & 0xF, len = c >> 4;
      if (op == 5) {
        if (qend != l_seq) {
          e.code = SCT_BAM_VALUEERROR;
          e.msg = "Invalid clipping in CIGAR string";
          return -1;
        }
      } else if (op == 4) {
        qend -= len;
      } else {
        break;
      }
    }
    q0 = start;
    q1 = qend < start ? start : qend;
  }
  if (aq_none && validate) {
    e.code = SCT_BAM_TYPEERROR;
    e.msg = "'NoneType' object is not iterable";
    return -1;
  }
  if (q1 == q0 && validate) {
    e.code = SCT_BAM_ZERODIV;
    e.msg = "division by zero";
    return -1;
  }
  uint8_t x = XF_ABSENT;
  if (xf.present) {
    x = XF_OTHER;
    if (xf.is_str) {
      const std::string s(xf.s, xf.n);
      if (s == "CODING") x = XF_CODING;
      else if (s == "INTRONIC") x = XF_INTRONIC;
      else if (s == "UTR") x = XF_UTR;
      else if (s == "INTERGENIC") x = XF_INTERGENIC;
    }
  }
  if (flag & 0x4) {
    bits |= B_UNMAPPED;
  } else {
    int64_t nh_v = 0;
    bool nh_int = false;
    if (validate) {
      if (!xf.present) {
        e.code = SCT_BAM_KEYERROR;
        e.msg = "XF";
        return -1;
      }
      if (!nh.present) {
        e.code = SCT_BAM_KEYERROR;
        e.msg = "NH";
        return -1;
      }
    }
    if (nh.present && !nh.is_str && !nh.raw) nh_v = nh.i, nh_int = true;
    if (nh_int && nh_v == 1) bits |= B_NH1;
    uint64_t n_len = 0;
    for (uint32_t k = 0; k < n_cigar; k++) {
      const uint32_t c = rd32(cig + 4 * k);
      if ((c & 0xF) == 3) n_len += c >> 4;
    }
    if (n_len) bits |= B_SPLICED;
  }
  if (flag & 0x10) bits |= B_REVERSE;
  if (flag & 0x400) bits |= B_DUPLICATE;
  uint32_t s = 0, g = 0;
  for (uint32_t k = q0; k < q1; k++) {
    s += qual[k];
    g += qual[k] > 30 ? 1u : 0u;
  }
  if (q1 - q0 > 0xFFFF || s > 0xFFFF || cl > 0xFF || ul > 0xFF) {
    e.code = SCT_BAM_VALUEERROR;
    e.msg = "record exceeds the 32-byte columnar limits";
    return -1;
  }
  o.ref = ref, o.pos = pos, o.gq_sum = s, o.gq_len = q1 - q0, o.gq_gt30 = g;
  o.cy_gt30 = cg, o.cy_len = cl, o.uy_gt30 = ug, o.uy_len = ul, o.bits = bits, o.xf = x;
  o.cb = cb, o.ub = ub, o.ge = ge;
  return typed_keys(o, false, e);
}

// Count-matrix mode: the three dictionary tags (names in `tags`), XF and the query name; no
// validation (count.py:222-270 reads only these, through has_tag / get_tag_or_default).
// sortkeys: the TagSortBam / VerifyBamSort keys, where an integer value also counts as typed.
int parse_count_record(const uint8_t* d, uint32_t bs, const char* tags, bool sortkeys, Parsed& o, const char** qname,
                       uint32_t* qlen, RecErr& e) {
  if (bs < 32) {
    e.code = SCT_BAM_EFORMAT;
    e.msg = "truncated BAM record";
    return -1;
  }
  const uint32_t l_read_name = d[8];
  const uint32_t n_cigar = rd16(d + 12);
  const uint32_t l_seq = rd32(d + 16);
  const uint64_t tag_off = 32ull + l_read_name + 4ull * n_cigar + (l_seq + 1) / 2 + l_seq;
  if (tag_off > bs || l_read_name == 0) {
    e.code = SCT_BAM_EFORMAT;
    e.msg = "truncated BAM record";
    return -1;
  }
  *qname = (const char*)d + 32;
  *qlen = l_read_name - 1;  // without the NUL
  TagVal xf;
  o.cb = TagVal(), o.ub = TagVal(), o.ge = TagVal();
  const uint8_t* p = d + tag_off;
  const uint8_t* end = d + bs;
  while (p + 3 <= end) {
    const char a = (char)p[0], b = (char)p[1], t = (char)p[2];
    p += 3;
    TagVal v;
    const size_t used = read_tag(p, end, t, &v);
    if (!used || p + used > end) {
      e.code = SCT_BAM_EFORMAT;
      e.msg = std::string("unsupported or truncated BAM tag type ") + t;
      return -1;
    }
    if (a == tags[0] && b == tags[1]) o.cb = v;
    if (a == tags[2] && b == tags[3]) o.ub = v;
    if (a == tags[4] && b == tags[5]) o.ge = v;
    if (a == 'X' && b == 'F') xf = v;
    p += used;
  }
  uint8_t x = XF_ABSENT;
  if (xf.present) {
    x = XF_OTHER;
    if (xf.is_str && xf.n == 10 && memcmp(xf.s, "INTERGENIC", 10) == 0) x = XF_INTERGENIC;
  }
  o.ref = (int32_t)rd32(d), o.pos = (int32_t)rd32(d + 4);
  o.gq_sum = o.gq_len = o.gq_gt30 = o.cy_gt30 = o.cy_len = o.uy_gt30 = o.uy_len = 0;
  o.bits = 0, o.xf = x;
  return typed_keys(o, sortkeys, e);
}

// Per-thread direct-mapped cache in front of the shared tables: cell-sorted input repeats
// the CB of the previous record and hot genes repeat constantly, so most lookups never take
// a stripe lock.
struct TagCache {
  static constexpr int kSlots = 1024, kMaxLen = 40;
  struct Entry {
    uint64_t hash = 0;
    int32_t pid = 0;
    uint8_t len = 0;
    char bytes[kMaxLen];
  };
  Entry e[kSlots];
};

int32_t intern_bytes(Interner& in, TagCache& c, const char* p, size_t n) {
  const uint64_t h = hash_bytes(p, n);
  TagCache::Entry& x = c.e[h & (TagCache::kSlots - 1)];
  if (x.pid && x.hash == h && x.len == n && memcmp(x.bytes, p, n) == 0) return x.pid;
  const int32_t pid = in.intern(p, n, h);
  if (n <= (size_t)TagCache::kMaxLen) {
    x.hash = h, x.pid = pid, x.len = (uint8_t)n;
    memcpy(x.bytes, p, n);
  }
  return pid;
}

// intern a tag value's string form; 0 = missing.  Bytes >= 0x80 become U+FFFD (the Python
// reader decodes with "ascii"/"replace").
int32_t intern_tag(Interner& in, TagCache& c, TagVal& v, std::string& tmp) {
  if (!v.present) return 0;
  as_str(v);
  bool ascii = true;
  for (size_t i = 0; i < v.n; i++)
    if ((uint8_t)v.s[i] >= 0x80) {
      ascii = false;
      break;
    }
  if (ascii) return intern_bytes(in, c, v.s, v.n);
  tmp.clear();
  for (size_t i = 0; i < v.n; i++) {
    if ((uint8_t)v.s[i] < 0x80) tmp.push_back(v.s[i]);
    else tmp.append("\xEF\xBF\xBD");
  }
  return intern_bytes(in, c, tmp.data(), tmp.size());
}

}  // namespace

struct sct_bam {
  Columns c;
  int64_t n = 0;
  std::string dict_bytes[4];  // CB, UB, GE (or the three named tags), query names (sort-key mode)
  std::vector<int64_t> dict_off[4];
  int32_t has_none[4] = {0, 0, 0, 0};
};

extern "C" {

const char* sct_bam_last_error(void) { return g_err.c_str(); }

int sct_bam_decode(const char* path, int32_t metric_mode, int32_t n_threads, sct_bam_t** out, int64_t* bad_record) {
  return sct_bam_decode_tags(path, metric_mode, "CBUBGE", n_threads, out, bad_record);
}

int sct_bam_decode_tags(const char* path, int32_t metric_mode, const char* tags, int32_t n_threads, sct_bam_t** out,
                        int64_t* bad_record) {
  g_err.clear();
  if (out) *out = nullptr;
  if (bad_record) *bad_record = -1;
  if (!path || !out || !tags) return fail(SCT_BAM_EIO, "NULL argument");
  if (metric_mode < SCT_BAM_CELL_METRICS || metric_mode > SCT_BAM_SORT_KEYS)
    return fail(SCT_BAM_EIO, "unknown decode mode %d", metric_mode);
  if (strlen(tags) != 6) return fail(SCT_BAM_EIO, "tags must name three two-character tags");
  const bool sortkeys = metric_mode == SCT_BAM_SORT_KEYS;
  const bool counting = metric_mode == SCT_BAM_COUNT_MATRIX;
  const bool generic = counting || sortkeys;  // named tags, no validation
  if (!generic && memcmp(tags, "CBUBGE", 6) != 0) return fail(SCT_BAM_EIO, "the metric modes read CB / UB / GE");
  const bool is_cell = metric_mode == SCT_BAM_CELL_METRICS;
  if (n_threads <= 0) n_threads = omp_get_max_threads();
  const int fd = open(path, O_RDONLY);
  if (fd < 0) return fail(SCT_BAM_EIO, "cannot open %s", path);
  struct stat st;
  if (fstat(fd, &st) != 0 || st.st_size == 0) {
    close(fd);
    return fail(SCT_BAM_EFORMAT, "%s is empty", path);
  }
  const uint64_t fsize = (uint64_t)st.st_size;
  const uint8_t* f = (const uint8_t*)mmap(nullptr, fsize, PROT_READ, MAP_PRIVATE, fd, 0);
  close(fd);
  if (f == MAP_FAILED) return fail(SCT_BAM_EIO, "cannot map %s", path);
  struct Unmap {
    const uint8_t* f;
    uint64_t n;
    ~Unmap() { munmap((void*)f, n); }
  } unmap{f, fsize};

  const bool timing = getenv("SCT_BAM_TIMING") != nullptr;
  double t_inflate = 0, t_parse = 0;
  auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
  double t0 = now();
  std::vector<Block> blocks;
  int rc = scan_blocks(f, fsize, blocks);
  if (rc) return rc;
  const double t_scan = now() - t0;

  sct_bam* B = new sct_bam();
  std::unique_ptr<sct_bam> guard(B);
  Interner dicts[4];
  std::atomic<int32_t> has_none[4];
  for (auto& h : has_none) h = 0;

  // carry + this window's inflated bytes; grown without zero-filling (inflate writes every byte)
  struct Buf {
    std::unique_ptr<uint8_t[]> p;
    size_t n = 0, cap = 0;
    uint8_t* data() { return p.get(); }
    size_t size() const { return n; }
    void resize(size_t m) {
      if (m > cap) {
        const size_t c = m + m / 4;
        std::unique_ptr<uint8_t[]> q(new uint8_t[c]);
        if (n) memcpy(q.get(), p.get(), n < m ? n : m);
        p.swap(q);
        cap = c;
      }
      n = m;
    }
  } buf;
  size_t carry = 0;          // bytes at the front of buf left from the previous window
  bool header_done = false;
  size_t bi = 0;
  uint64_t kWindow = 256ull << 20;  // SCT_BAM_WINDOW (bytes) shrinks it: tests of the carry path
  if (const char* w = getenv("SCT_BAM_WINDOW")) kWindow = strtoull(w, nullptr, 10) ? strtoull(w, nullptr, 10) : kWindow;
  std::vector<z_stream> zs(n_threads);
  for (auto& z : zs) {
    memset(&z, 0, sizeof(z));
    inflateInit2(&z, -15);
  }
  struct ZEnd {
    std::vector<z_stream>& zs;
    ~ZEnd() {
      for (auto& z : zs) inflateEnd(&z);
    }
  } zend{zs};

  std::vector<uint64_t> starts;
  int64_t base = 0;
  std::string prev_qname;  // the last record's query name of the previous window (count mode)
  bool have_prev = false;
  while (bi < blocks.size() || carry) {
    // 1. inflate the next window of blocks behind the carried bytes
    size_t bj = bi;
    uint64_t isz = 0;
    while (bj < blocks.size() && (isz < kWindow || bj == bi)) isz += blocks[bj++].isize;
    if (bj == bi && carry) return fail(SCT_BAM_EFORMAT, "truncated BAM record at the end of %s", path);
    std::vector<uint64_t> dst(bj - bi + 1);
    dst[0] = carry;
    for (size_t k = bi; k < bj; k++) dst[k - bi + 1] = dst[k - bi] + blocks[k].isize;
    buf.resize(dst.back());
    double ti = now();
    std::atomic<int> bad{0};
#pragma omp parallel for num_threads(n_threads) schedule(dynamic, 4)
    for (long k = (long)bi; k < (long)bj; k++) {
      if (blocks[k].isize && !inflate_block(f, blocks[k], buf.data() + dst[k - bi], zs[omp_get_thread_num()]))
        bad = 1;
    }
    if (bad) return fail(SCT_BAM_EIO, "cannot inflate a BGZF block of %s", path);
    t_inflate += now() - ti;
    ti = now();
    bi = bj;
    size_t off = 0;
    const size_t len = buf.size();
    if (!header_done) {  // magic, text, references (the header is small: in the first window)
      if (len < 12 || memcmp(buf.data(), "BAM\1", 4) != 0) return fail(SCT_BAM_EFORMAT, "%s is not a BAM file", path);
      off = 8 + (size_t)rd32(buf.data() + 4);
      if (off + 4 > len) return fail(SCT_BAM_EFORMAT, "BAM header of %s exceeds the first window", path);
      const uint32_t n_ref = rd32(buf.data() + off);
      off += 4;
      for (uint32_t r = 0; r < n_ref; r++) {
        if (off + 4 > len) return fail(SCT_BAM_EFORMAT, "BAM header of %s exceeds the first window", path);
        off += 4 + (size_t)rd32(buf.data() + off) + 4;
      }
      header_done = true;
    }
    // 2. record starts
    starts.clear();
    while (off + 4 <= len) {
      const uint32_t bs = rd32(buf.data() + off);
      if (off + 4 + bs > len) break;
      starts.push_back(off);
      off += 4 + bs;
    }
    if (bi == blocks.size() && off != len) return fail(SCT_BAM_EFORMAT, "truncated BAM record at the end of %s", path);
    // 3. parse + intern
    const int64_t nw = (int64_t)starts.size();
    B->c.resize((size_t)(base + nw));
    if (counting) B->c.qhead.resize((size_t)(base + nw));
    if (sortkeys) B->c.qname.resize((size_t)(base + nw));
    std::atomic<int64_t> first_bad{INT64_MAX};
    std::mutex err_m;
    RecErr first_err;
    Columns& C = B->c;
#pragma omp parallel num_threads(n_threads)
    {
      std::string tmp;
      Parsed o;
      RecErr e;
      std::unique_ptr<TagCache[]> cache(new TagCache[4]);
#pragma omp for schedule(dynamic, 4096)
      for (int64_t i = 0; i < nw; i++) {
        const uint8_t* d = buf.data() + starts[i] + 4;
        const uint32_t bs = rd32(buf.data() + starts[i]);
        const char* qn = nullptr;
        uint32_t qlen = 0;
        if (generic ? parse_count_record(d, bs, tags, sortkeys, o, &qn, &qlen, e) : parse_record(d, bs, is_cell, o, e)) {
          std::lock_guard<std::mutex> lk(err_m);
          if (base + i < first_bad.load()) {
            first_bad = base + i;
            first_err = e;
          }
          continue;
        }
        const int64_t j = base + i;
        if (counting) {
          // groupby(query_name): a new group where the name differs from the previous record's
          const uint8_t* pd = i ? buf.data() + starts[i - 1] + 4 : nullptr;
          bool head;
          if (pd) head = pd[8] != qlen + 1 || memcmp(pd + 32, qn, qlen) != 0;
          else head = !have_prev || prev_qname.size() != qlen || memcmp(prev_qname.data(), qn, qlen) != 0;
          C.qhead[j] = head ? 1 : 0;
        }
        C.ref[j] = o.ref, C.pos[j] = o.pos;
        C.gq_sum[j] = (uint16_t)o.gq_sum, C.gq_len[j] = (uint16_t)o.gq_len, C.gq_gt30[j] = (uint16_t)o.gq_gt30;
        C.bits[j] = o.bits, C.xf[j] = o.xf;
        C.cy_gt30[j] = (uint8_t)o.cy_gt30, C.cy_len[j] = (uint8_t)o.cy_len;
        C.uy_gt30[j] = (uint8_t)o.uy_gt30, C.uy_len[j] = (uint8_t)o.uy_len;
        if (sortkeys) {  // get_tag_or_default(record, key, ""): an empty value sorts as a missing one
          C.qname[j] = intern_bytes(dicts[3], cache[3], qn, qlen);
          for (TagVal* v : {&o.cb, &o.ub, &o.ge}) {
            as_str(*v);
            if (v->present && v->n == 0) v->present = false;
          }
        }
        C.cell[j] = intern_tag(dicts[0], cache[0], o.cb, tmp);
        C.umi[j] = intern_tag(dicts[1], cache[1], o.ub, tmp);
        C.gene[j] = intern_tag(dicts[2], cache[2], o.ge, tmp);
        if (!o.cb.present) has_none[0] = 1;
        if (!o.ub.present) has_none[1] = 1;
        if (!o.ge.present) has_none[2] = 1;
      }
    }
    t_parse += now() - ti;
    if (first_bad.load() != INT64_MAX) {
      if (bad_record) *bad_record = first_bad.load();
      return fail(first_err.code, "%s", first_err.msg.c_str());
    }
    if (counting && nw) {
      const uint8_t* ld = buf.data() + starts[nw - 1] + 4;
      prev_qname.assign((const char*)ld + 32, ld[8] ? ld[8] - 1 : 0);
      have_prev = true;
    }
    base += nw;
    // 4. carry the cut record
    carry = len - off;
    if (carry) memmove(buf.data(), buf.data() + off, carry);
    buf.resize(carry);
    if (bi == blocks.size() && carry == 0) break;
  }
  B->n = base;
  if (base == 0 && !generic) return fail(SCT_BAM_EMPTY, "generator raised StopIteration");
  // 5. rank the dictionaries: sorted strings, the missing value first
  for (int t = 0; t < (sortkeys ? 4 : 3); t++) {
    std::vector<std::pair<std::string, int32_t>> all;
    dicts[t].collect(all);
    std::sort(all.begin(), all.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
    const int32_t hn = has_none[t].load();
    std::vector<int32_t> rank((size_t)dicts[t].count() + 1, 0);
    B->has_none[t] = hn;
    B->dict_off[t].push_back(0);
    if (hn) B->dict_off[t].push_back(0);
    for (size_t r = 0; r < all.size(); r++) {
      rank[all[r].second] = (int32_t)r + hn;
      B->dict_bytes[t] += all[r].first;
      B->dict_off[t].push_back((int64_t)B->dict_bytes[t].size());
    }
    std::vector<int32_t>& col = t == 0 ? B->c.cell : t == 1 ? B->c.umi : t == 2 ? B->c.gene : B->c.qname;
#pragma omp parallel for num_threads(n_threads) schedule(static)
    for (int64_t i = 0; i < base; i++) col[i] = rank[col[i]];
  }
  if (timing)
    fprintf(stderr, "sct_bam: %lld records, scan %.3fs, inflate %.3fs, parse+intern %.3fs, rank %.3fs (%d threads)\n",
            (long long)base, t_scan, t_inflate, t_parse, now() - t0 - t_scan - t_inflate - t_parse, n_threads);
  *out = guard.release();
  return SCT_BAM_OK;
}

int64_t sct_bam_n(const sct_bam_t* b) { return b ? b->n : 0; }

const void* sct_bam_column(const sct_bam_t* b, const char* name) {
  if (!b || !name) return nullptr;
  const Columns& c = b->c;
  const std::string s(name);
  if (s == "cell") return c.cell.data();
  if (s == "umi") return c.umi.data();
  if (s == "gene") return c.gene.data();
  if (s == "ref") return c.ref.data();
  if (s == "pos") return c.pos.data();
  if (s == "gq_sum") return c.gq_sum.data();
  if (s == "gq_len") return c.gq_len.data();
  if (s == "gq_gt30") return c.gq_gt30.data();
  if (s == "bits") return c.bits.data();
  if (s == "xf") return c.xf.data();
  if (s == "cy_gt30") return c.cy_gt30.data();
  if (s == "cy_len") return c.cy_len.data();
  if (s == "uy_gt30") return c.uy_gt30.data();
  if (s == "uy_len") return c.uy_len.data();
  if (s == "qhead") return c.qhead.empty() && b->n ? nullptr : c.qhead.data();
  if (s == "qname") return c.qname.empty() && b->n ? nullptr : c.qname.data();
  return nullptr;
}

int sct_bam_dictionary(const sct_bam_t* b, int32_t which, int64_t* n, const char** bytes, const int64_t** offsets,
                       int32_t* has_none) {
  if (!b || which < 0 || which > 3 || !n || !bytes || !offsets || !has_none)
    return fail(SCT_BAM_EIO, "bad sct_bam_dictionary arguments");
  *n = b->dict_off[which].empty() ? 0 : (int64_t)b->dict_off[which].size() - 1;
  *bytes = b->dict_bytes[which].data();
  *offsets = b->dict_off[which].data();
  *has_none = b->has_none[which];
  return SCT_BAM_OK;
}

void sct_bam_close(sct_bam_t* b) { delete b; }

}  // extern "C"
