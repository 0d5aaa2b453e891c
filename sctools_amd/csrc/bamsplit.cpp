// bamsplit.cpp -- SplitBam: cell-disjoint BAM chunks (include/sct_bam.h, sct_bam_split).
//
// The reference (bam.split, bam.py:361-488; CLI SplitBam, platform.py:153-223) reads every
// input BAM twice in a multiprocessing pool: once to collect the barcodes (the first of `tags`
// present on a record, get_barcode_for_alignment, bam.py:263-290), then to write each record to
// the chunk of its barcode through pysam, and finally merges each chunk's per-input pieces with
// samtools.  Every barcode lands in exactly one chunk: the cell-sharding invariant the
// multi-GPU metric path relies on.
//
// Here, host C++ over the same BGZF machinery as the decoder (bgzf.h):
//   pass 1  windows of inflated blocks (parallel inflate), records found by hopping block_size,
//           each record's barcode (first tag of the priority list present) interned in parallel;
//   bins    barcodes ranked in string order (deterministic; the reference iterates a Python set),
//           rank -> chunk (rank when there are no more barcodes than chunks, else rank % chunks),
//           as bam.py:439-448 assigns its list;
//   pass 2  the same windows again: records copied byte for byte, in file order, to their
//           chunk's staging buffer (a parallel stable partition), full 0xff00-byte pieces
//           deflated in parallel into BGZF members and appended to the chunk file, which starts
//           with the input's header and ends with the BGZF EOF member.
// Several inputs are concatenated in input order (they must share the reference list); the
// reference merges its per-input pieces with samtools merge instead.
#include <fcntl.h>
#include <omp.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <memory>
#include <string>
#include <vector>

#include "../../include/sct_bam.h"
#include "bgzf.h"

namespace {

struct Mapped {
  const uint8_t* f = nullptr;
  uint64_t n = 0;
  std::vector<Block> blocks;
  ~Mapped() {
    if (f) munmap((void*)f, n);
  }
};

int map_bam(const char* path, Mapped& m) {
  const int fd = open(path, O_RDONLY);
  if (fd < 0) return fail(SCT_BAM_EIO, "cannot open %s", path);
  struct stat st;
  if (fstat(fd, &st) != 0 || st.st_size == 0) {
    close(fd);
    return fail(SCT_BAM_EFORMAT, "%s is empty", path);
  }
  m.n = (uint64_t)st.st_size;
  const void* p = mmap(nullptr, m.n, PROT_READ, MAP_PRIVATE, fd, 0);
  close(fd);
  if (p == MAP_FAILED) return fail(SCT_BAM_EIO, "cannot map %s", path);
  m.f = (const uint8_t*)p;
  return scan_blocks(m.f, m.n, m.blocks);
}

// Walks an input window by window: inflates blocks in parallel, hands the caller the header
// bytes once and every window's complete records (record starts into `buf`).
class Walker {
 public:
  Walker(const Mapped& m, int threads) : m_(m), threads_(threads), zs_(threads) {
    for (auto& z : zs_) {
      memset(&z, 0, sizeof(z));
      inflateInit2(&z, -15);
    }
    if (const char* w = getenv("SCT_BAM_WINDOW")) window_ = strtoull(w, nullptr, 10) ? strtoull(w, nullptr, 10) : window_;
  }
  ~Walker() {
    for (auto& z : zs_) inflateEnd(&z);
  }
  std::string header;  // magic .. references, uncompressed
  std::vector<uint8_t> buf;
  std::vector<uint64_t> starts;

  // next window; returns 1 with records in (buf, starts), 0 at the end, < 0 on error
  int next(const char* path) {
    if (bi_ == m_.blocks.size() && carry_ == 0) return 0;
    size_t bj = bi_;
    uint64_t isz = 0;
    while (bj < m_.blocks.size() && (isz < window_ || bj == bi_)) isz += m_.blocks[bj++].isize;
    if (bj == bi_) return fail(SCT_BAM_EFORMAT, "truncated BAM record at the end of %s", path);
    std::vector<uint64_t> dst(bj - bi_ + 1);
    dst[0] = carry_;
    for (size_t k = bi_; k < bj; k++) dst[k - bi_ + 1] = dst[k - bi_] + m_.blocks[k].isize;
    buf.resize(dst.back());
    int bad = 0;
#pragma omp parallel for num_threads(threads_) schedule(dynamic, 4) reduction(| : bad)
    for (long k = (long)bi_; k < (long)bj; k++)
      if (m_.blocks[k].isize && !inflate_block(m_.f, m_.blocks[k], buf.data() + dst[k - bi_], zs_[omp_get_thread_num()]))
        bad = 1;
    if (bad) return fail(SCT_BAM_EIO, "cannot inflate a BGZF block of %s", path);
    bi_ = bj;
    size_t off = 0;
    const size_t len = buf.size();
    if (!header_done_) {
      if (len < 12 || memcmp(buf.data(), "BAM\1", 4) != 0) return fail(SCT_BAM_EFORMAT, "%s is not a BAM file", path);
      off = 8 + (size_t)rd32(buf.data() + 4);
      if (off + 4 > len) return fail(SCT_BAM_EFORMAT, "BAM header of %s exceeds the first window", path);
      const uint32_t n_ref = rd32(buf.data() + off);
      off += 4;
      for (uint32_t r = 0; r < n_ref; r++) {
        if (off + 4 > len) return fail(SCT_BAM_EFORMAT, "BAM header of %s exceeds the first window", path);
        off += 4 + (size_t)rd32(buf.data() + off) + 4;
      }
      header.assign((const char*)buf.data(), off);
      header_done_ = true;
    }
    starts.clear();
    while (off + 4 <= len) {
      const uint32_t bs = rd32(buf.data() + off);
      if (off + 4 + bs > len) break;
      starts.push_back(off);
      off += 4 + bs;
    }
    if (bi_ == m_.blocks.size() && off != len) return fail(SCT_BAM_EFORMAT, "truncated BAM record at the end of %s", path);
    pending_ = off;
    return 1;
  }
  // after the caller is done with this window: keep the cut record for the next one
  void advance() {
    const size_t len = buf.size();
    carry_ = len - pending_;
    if (carry_) memmove(buf.data(), buf.data() + pending_, carry_);
    buf.resize(carry_);
  }

 private:
  const Mapped& m_;
  int threads_;
  std::vector<z_stream> zs_;
  size_t bi_ = 0, carry_ = 0, pending_ = 0;
  bool header_done_ = false;
  uint64_t window_ = 256ull << 20;
};

// the barcode of a record: the first of `tags` (priority order) present, as (type, bytes):
// strings as themselves, integers in decimal with a distinct type byte (a Python int and a str
// are different barcodes)
bool record_barcode(const uint8_t* d, uint32_t bs, const char* tags, int n_tags, std::string& out, bool& bad) {
  bad = false;
  if (bs < 32) {
    bad = true;
    return false;
  }
  const uint32_t l_read_name = d[8];
  const uint32_t n_cigar = rd16(d + 12);
  const uint32_t l_seq = rd32(d + 16);
  uint64_t p = 32 + (uint64_t)l_read_name + 4ull * n_cigar + (l_seq + 1) / 2 + l_seq;
  if (p > bs) {
    bad = true;
    return false;
  }
  const uint8_t* end = d + bs;
  int best = n_tags;
  TagVal bestv;
  char bestt = 0;
  const uint8_t* q = d + p;
  while (q + 3 <= end) {
    const char t = (char)q[2];
    TagVal v;
    const size_t w = read_tag(q + 3, end, t, &v);
    if (!w) {
      bad = true;
      return false;
    }
    for (int k = 0; k < best; k++)
      if (q[0] == (uint8_t)tags[2 * k] && q[1] == (uint8_t)tags[2 * k + 1]) {
        best = k;
        bestv = v;
        bestt = t;
        break;
      }
    q += 3 + w;
  }
  if (best == n_tags) return false;
  if (bestv.is_str) {
    out.assign(1, 'Z');
    out.append(bestv.s, bestv.n);
  } else {
    as_str(bestv);
    out.assign(1, (bestt == 'f' || bestt == 'd' || bestt == 'B') ? bestt : 'i');
    out.append(bestv.s, bestv.n);
  }
  return true;
}

}  // namespace

extern "C" {

int sct_bam_split(const char* const* in_paths, int32_t n_in, const char* out_prefix, const char* tags, int32_t n_tags,
                  int32_t n_subfiles, int32_t raise_missing, int32_t level, int32_t n_threads, int32_t* n_out,
                  int64_t* bad_record) {
  g_err.clear();
  if (n_out) *n_out = 0;
  if (bad_record) *bad_record = -1;
  if (!in_paths || n_in < 1 || !out_prefix || !tags || !n_out) return fail(SCT_BAM_EIO, "NULL argument");
  if (n_tags < 1 || (int)strlen(tags) != 2 * n_tags) return fail(SCT_BAM_VALUEERROR, "At least one tag must be passed");
  if (n_subfiles < 1) return fail(SCT_BAM_VALUEERROR, "n_subfiles must be >= 1");
  if (level < 0 || level > 9) level = 6;
  if (n_threads <= 0) n_threads = omp_get_max_threads();

  // pass 1: every record's barcode (provisional interned id, 0 = none)
  Interner dict;
  std::vector<std::vector<int32_t>> rec_bc(n_in);
  std::string header0;
  int64_t base = 0;
  for (int in = 0; in < n_in; in++) {
    Mapped m;
    int rc = map_bam(in_paths[in], m);
    if (rc) return rc;
    Walker w(m, n_threads);
    std::vector<int32_t>& ids = rec_bc[in];
    while ((rc = w.next(in_paths[in])) == 1) {
      const int64_t nw = (int64_t)w.starts.size();
      const size_t at = ids.size();
      ids.resize(at + (size_t)nw);
      int64_t first_missing = INT64_MAX, first_bad = INT64_MAX;
#pragma omp parallel num_threads(n_threads)
      {
        std::string bc;
        int64_t miss = INT64_MAX, badr = INT64_MAX;
#pragma omp for schedule(dynamic, 4096)
        for (int64_t i = 0; i < nw; i++) {
          const uint8_t* d = w.buf.data() + w.starts[i] + 4;
          const uint32_t bs = rd32(w.buf.data() + w.starts[i]);
          bool bad;
          if (record_barcode(d, bs, tags, n_tags, bc, bad)) {
            ids[at + i] = dict.intern(bc.data(), bc.size());
          } else {
            ids[at + i] = 0;
            if (bad) badr = std::min(badr, i);
            else miss = std::min(miss, i);
          }
        }
#pragma omp critical
        {
          first_missing = std::min(first_missing, miss);
          first_bad = std::min(first_bad, badr);
        }
      }
      if (first_bad != INT64_MAX) {
        if (bad_record) *bad_record = base + (int64_t)at + first_bad;
        return fail(SCT_BAM_EFORMAT, "malformed BAM record in %s", in_paths[in]);
      }
      if (raise_missing && first_missing != INT64_MAX) {
        if (bad_record) *bad_record = base + (int64_t)at + first_missing;
        std::string names;
        for (int k = 0; k < n_tags; k++) names += std::string(k ? ", '" : "'") + std::string(tags + 2 * k, 2) + "'";
        return fail(SCT_BAM_MISSING_TAG, "Alignment encountered that is missing [%s] tag(s).", names.c_str());
      }
      w.advance();
    }
    if (rc < 0) return rc;
    if (in == 0) {
      header0 = w.header;
    } else {  // the chunks carry the first input's header: the references must agree
      const auto refs = [](const std::string& h) {
        const size_t off = 8 + (size_t)rd32((const uint8_t*)h.data() + 4);
        return h.substr(off);
      };
      if (refs(w.header) != refs(header0))
        return fail(SCT_BAM_VALUEERROR, "%s has another reference list than %s", in_paths[in], in_paths[0]);
    }
    base += (int64_t)ids.size();
  }

  // bins: barcodes in string order; rank, or rank % n_subfiles when there are more barcodes
  std::vector<std::pair<std::string, int32_t>> all;
  dict.collect(all);
  std::sort(all.begin(), all.end());
  const int32_t n_bc = (int32_t)all.size();
  const int32_t nb = n_bc < n_subfiles ? n_bc : n_subfiles;
  std::vector<int32_t> bin_of((size_t)dict.count() + 1, -1);
  for (int32_t r = 0; r < n_bc; r++) bin_of[all[r].second] = r % (nb > 0 ? nb : 1);
  if (nb == 0) return SCT_BAM_OK;  // no barcodes at all: no chunk (the reference writes none either)

  // outputs: header, then the records, then EOF
  std::vector<FILE*> files(nb, nullptr);
  struct Closer {
    std::vector<FILE*>& f;
    ~Closer() {
      for (FILE* x : f)
        if (x) fclose(x);
    }
  } closer{files};
  std::vector<z_stream> zs(n_threads);
  for (auto& z : zs) {
    memset(&z, 0, sizeof(z));
    deflateInit2(&z, level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY);
  }
  struct ZEnd {
    std::vector<z_stream>& zs;
    ~ZEnd() {
      for (auto& z : zs) deflateEnd(&z);
    }
  } zend{zs};
  std::vector<std::string> stage(nb);  // per chunk: uncompressed bytes not yet deflated
  // deflate every full 0xff00 piece of every chunk (or everything, at the end) in parallel
  auto flush = [&](bool final) -> int {
    struct Piece {
      int bin;
      size_t off, len;
    };
    std::vector<Piece> pieces;
    for (int b = 0; b < nb; b++) {
      const size_t full = final ? stage[b].size() : stage[b].size() / kBgzfMaxInput * kBgzfMaxInput;
      for (size_t o = 0; o < full; o += kBgzfMaxInput)
        pieces.push_back(Piece{b, o, std::min(kBgzfMaxInput, full - o)});
    }
    std::vector<std::vector<uint8_t>> out(pieces.size());
    int bad = 0;
#pragma omp parallel for num_threads(n_threads) schedule(dynamic, 1) reduction(| : bad)
    for (long k = 0; k < (long)pieces.size(); k++) {
      const Piece& p = pieces[k];
      if (!bgzf_block((const uint8_t*)stage[p.bin].data() + p.off, p.len, level, zs[omp_get_thread_num()], out[k]))
        bad = 1;
    }
    if (bad) return fail(SCT_BAM_EIO, "deflate failed");
    for (size_t k = 0; k < pieces.size(); k++)
      if (fwrite(out[k].data(), 1, out[k].size(), files[pieces[k].bin]) != out[k].size())
        return fail(SCT_BAM_EIO, "cannot write chunk %d", pieces[k].bin);
    for (int b = 0; b < nb; b++) {
      const size_t full = final ? stage[b].size() : stage[b].size() / kBgzfMaxInput * kBgzfMaxInput;
      stage[b].erase(0, full);
    }
    return SCT_BAM_OK;
  };
  for (int b = 0; b < nb; b++) {
    const std::string name = std::string(out_prefix) + "_" + std::to_string(b) + ".bam";
    files[b] = fopen(name.c_str(), "wb");
    if (!files[b]) return fail(SCT_BAM_EIO, "cannot create %s", name.c_str());
    stage[b] = header0;  // the header starts the chunk's uncompressed stream
  }
  int rc = flush(true);  // the header in its own members, as htslib writes it
  if (rc) return rc;

  // pass 2: records to their chunks, in file order
  for (int in = 0; in < n_in; in++) {
    Mapped m;
    rc = map_bam(in_paths[in], m);
    if (rc) return rc;
    Walker w(m, n_threads);
    const std::vector<int32_t>& ids = rec_bc[in];
    size_t at = 0;
    while ((rc = w.next(in_paths[in])) == 1) {
      const int64_t nw = (int64_t)w.starts.size();
      // stable parallel partition: per thread chunk, bytes per bin; prefix; copy
      const int T = n_threads;
      std::vector<std::vector<size_t>> bytes(T, std::vector<size_t>(nb, 0));
#pragma omp parallel num_threads(T)
      {
        const int t = omp_get_thread_num();
        const int64_t lo = nw * t / T, hi = nw * (t + 1) / T;
        for (int64_t i = lo; i < hi; i++) {
          const int32_t id = ids[at + i];
          if (!id) continue;
          bytes[t][bin_of[id]] += 4 + (size_t)rd32(w.buf.data() + w.starts[i]);
        }
      }
      std::vector<std::vector<size_t>> dst(T, std::vector<size_t>(nb, 0));
      for (int b = 0; b < nb; b++) {
        size_t o = stage[b].size();
        for (int t = 0; t < T; t++) {
          dst[t][b] = o;
          o += bytes[t][b];
        }
        stage[b].resize(o);
      }
#pragma omp parallel num_threads(T)
      {
        const int t = omp_get_thread_num();
        const int64_t lo = nw * t / T, hi = nw * (t + 1) / T;
        std::vector<size_t>& d = dst[t];
        for (int64_t i = lo; i < hi; i++) {
          const int32_t id = ids[at + i];
          if (!id) continue;
          const int b = bin_of[id];
          const size_t len = 4 + (size_t)rd32(w.buf.data() + w.starts[i]);
          memcpy(&stage[b][d[b]], w.buf.data() + w.starts[i], len);
          d[b] += len;
        }
      }
      at += (size_t)nw;
      w.advance();
      if ((rc = flush(false))) return rc;
    }
    if (rc < 0) return rc;
  }
  if ((rc = flush(true))) return rc;
  for (int b = 0; b < nb; b++)
    if (fwrite(kBgzfEof, 1, sizeof(kBgzfEof), files[b]) != sizeof(kBgzfEof))
      return fail(SCT_BAM_EIO, "cannot write chunk %d", b);
  for (int b = 0; b < nb; b++) {
    if (fclose(files[b]) != 0) {
      files[b] = nullptr;
      return fail(SCT_BAM_EIO, "cannot close chunk %d", b);
    }
    files[b] = nullptr;
  }
  *n_out = nb;
  return SCT_BAM_OK;
}

// TagSortBam's output (platform.py:60-97): the input's records in the order `perm` gives
// (perm[k] = input index of output record k), byte for byte, under the input's header.  The
// inflated records are held in memory (the reference holds every record in Python too); the
// output stream is assembled with parallel copies and deflated in parallel 0xff00-byte pieces.
int sct_bam_write_order(const char* in_path, const char* out_path, const int64_t* perm, int64_t n, int32_t level,
                        int32_t n_threads) {
  g_err.clear();
  if (!in_path || !out_path || n < 0 || (n > 0 && !perm)) return fail(SCT_BAM_EIO, "bad arguments");
  if (level < 0 || level > 9) return fail(SCT_BAM_EIO, "compression level %d outside 0..9", level);
  if (n_threads <= 0) n_threads = omp_get_max_threads();
  Mapped m;
  int rc = map_bam(in_path, m);
  if (rc) return rc;
  Walker w(m, n_threads);
  std::vector<uint8_t> recs;   // every record (block_size field included), in file order
  std::vector<uint64_t> at;    // record start in recs
  std::string header0;
  while ((rc = w.next(in_path)) == 1) {
    if (at.empty() && header0.empty()) header0 = w.header;
    if (!w.starts.empty()) {
      const uint64_t first = w.starts.front();
      const uint64_t last = w.starts.back() + 4 + rd32(w.buf.data() + w.starts.back());
      const uint64_t base = recs.size();
      recs.insert(recs.end(), w.buf.begin() + first, w.buf.begin() + last);
      for (uint64_t o : w.starts) at.push_back(base + (o - first));
    }
    w.advance();
  }
  if (rc < 0) return rc;
  if (header0.empty()) header0 = w.header;
  if ((int64_t)at.size() != n) return fail(SCT_BAM_EIO, "%s holds %zu records, the order %lld", in_path, at.size(), (long long)n);
  // output offsets: the permuted records' sizes, scanned per thread
  const int T = n_threads;
  std::vector<uint64_t> part(T + 1, 0);
  int bad = 0;
#pragma omp parallel num_threads(T) reduction(| : bad)
  {
    const int t = omp_get_thread_num();
    const int64_t lo = n * t / T, hi = n * (t + 1) / T;
    uint64_t sz = 0;
    for (int64_t k = lo; k < hi; k++) {
      const int64_t i = perm[k];
      if (i < 0 || i >= n) {
        bad = 1;
        break;
      }
      sz += 4 + (uint64_t)rd32(recs.data() + at[i]);
    }
    part[t + 1] = sz;
  }
  if (bad) return fail(SCT_BAM_EIO, "the order holds an index outside 0..%lld", (long long)(n - 1));
  for (int t = 0; t < T; t++) part[t + 1] += part[t];
  std::vector<uint8_t> out(part[T]);
#pragma omp parallel num_threads(T)
  {
    const int t = omp_get_thread_num();
    const int64_t lo = n * t / T, hi = n * (t + 1) / T;
    uint64_t o = part[t];
    for (int64_t k = lo; k < hi; k++) {
      const uint64_t len = 4 + (uint64_t)rd32(recs.data() + at[perm[k]]);
      memcpy(out.data() + o, recs.data() + at[perm[k]], len);
      o += len;
    }
  }
  std::vector<uint8_t>().swap(recs);
  std::vector<z_stream> zs(n_threads);
  for (auto& z : zs) {
    memset(&z, 0, sizeof(z));
    deflateInit2(&z, level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY);
  }
  struct ZEnd {
    std::vector<z_stream>& zs;
    ~ZEnd() {
      for (auto& z : zs) deflateEnd(&z);
    }
  } zend{zs};
  FILE* f = fopen(out_path, "wb");
  if (!f) return fail(SCT_BAM_EIO, "cannot create %s", out_path);
  struct Closer {
    FILE*& f;
    ~Closer() {
      if (f) fclose(f);
    }
  } closer{f};
  // the header in its own members, as htslib writes it, then the records, then EOF
  for (int pass = 0; pass < 2; pass++) {
    const uint8_t* src = pass == 0 ? (const uint8_t*)header0.data() : out.data();
    const size_t total = pass == 0 ? header0.size() : out.size();
    const size_t np = (total + kBgzfMaxInput - 1) / kBgzfMaxInput;
    std::vector<std::vector<uint8_t>> z(np);
#pragma omp parallel for num_threads(n_threads) schedule(dynamic, 1) reduction(| : bad)
    for (long k = 0; k < (long)np; k++) {
      const size_t o = (size_t)k * kBgzfMaxInput;
      if (!bgzf_block(src + o, std::min(kBgzfMaxInput, total - o), level, zs[omp_get_thread_num()], z[k])) bad = 1;
    }
    if (bad) return fail(SCT_BAM_EIO, "deflate failed");
    for (size_t k = 0; k < np; k++)
      if (fwrite(z[k].data(), 1, z[k].size(), f) != z[k].size()) return fail(SCT_BAM_EIO, "cannot write %s", out_path);
  }
  if (fwrite(kBgzfEof, 1, sizeof(kBgzfEof), f) != sizeof(kBgzfEof)) return fail(SCT_BAM_EIO, "cannot write %s", out_path);
  FILE* g = f;
  f = nullptr;
  if (fclose(g) != 0) return fail(SCT_BAM_EIO, "cannot close %s", out_path);
  return SCT_BAM_OK;
}

}  // extern "C"
