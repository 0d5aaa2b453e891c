// synthbam -- a cell-sorted, 10x-v2-shaped BAM with the config-2 record statistics of SURVEY.md
// §8(d), for the end-to-end drop-in bench (tools/e2e_bench.py --synth): the device decoder's
// interning tables and the metrics see tens of thousands of Zipf-skewed gene names, ~10^6 random
// 10-mer UMIs per run, soft clips, CR != CB and UR != UB.
//
//   synthbam OUT.bam N_RECORDS [SEED]
//
// Cells: N / 10000 of them (reads per cell ~ lognormal(0, 1) weights, mean 10k), 16-mer barcodes
// written in sorted order.  Per cell, molecules of Geometric(0.35) reads; GE ~ Zipf(1.1) over 30,000
// gene names whose string order is a random permutation of their frequency rank (real gene names
// are not sorted by expression); 6 % without GE, 1 % "A,B" multi-gene values; UB a uniform 10-mer.
// Mapped reads (95 %): ref U{0..24}, pos = the molecule's anchor + 50 U{0..3}, 70 % reverse, 16 %
// duplicates, XF CODING .85 / INTRONIC .05 / UTR .03 / INTERGENIC .07, NH 1 (90 %) else U{2..10},
// 5 % spliced (a 500-base N); unmapped reads have no XF and NH 0.  13 % soft-clipped 1-29 bases at
// one end.  Read length 98, CY 16, UY 10; Phred binned {2,8,12,22,27,32,37,41} with the weights of
// small-cell-sorted.bam; CR != CB 1 %, UR != UB 0.2 %.  BGZF members of 0xff00 payload bytes, zlib
// level 6, compressed on all cores (OpenMP), then the EOF member.
#include <omp.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#include <algorithm>
#include <cmath>
#include <string>
#include <vector>

namespace {

struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull) {}
  uint64_t next() {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return s * 0x2545F4914F6CDD1Dull;
  }
  double u() { return (next() >> 11) * 0x1.0p-53; }
  uint32_t below(uint32_t n) { return (uint32_t)(u() * n); }
};

const int kPhred[8] = {2, 8, 12, 22, 27, 32, 37, 41};
const double kWGenomic[8] = {3, 427, 5416, 3969, 4536, 7514, 12909, 29514};
const double kWCY[8] = {1, 0, 59, 33, 102, 1578, 2253, 6470};
const double kWUY[8] = {0, 0, 25, 35, 47, 105, 353, 5995};

struct Cdf {
  double c[8];
  explicit Cdf(const double* w) {
    double t = 0;
    for (int i = 0; i < 8; i++) t += w[i];
    double a = 0;
    for (int i = 0; i < 8; i++) c[i] = (a += w[i] / t);
  }
  int draw(Rng& r) const {
    const double x = r.u();
    for (int i = 0; i < 7; i++)
      if (x < c[i]) return kPhred[i];
    return kPhred[7];
  }
};

void put32(std::string& b, uint32_t v) { b.append((const char*)&v, 4); }
void put16(std::string& b, uint16_t v) { b.append((const char*)&v, 2); }
void ztag(std::string& b, const char* k, const std::string& v) {
  b.append(k, 2);
  b.push_back('Z');
  b.append(v);
  b.push_back('\0');
}
std::string qual_string(Rng& r, const Cdf& cdf, int n) {
  std::string s(n, '!');
  for (int i = 0; i < n; i++) s[i] = (char)(33 + cdf.draw(r));
  return s;
}
std::string kmer(Rng& r, int n) {
  static const char A[4] = {'A', 'C', 'G', 'T'};
  std::string s(n, 'A');
  for (int i = 0; i < n; i++) s[i] = A[r.next() >> 62];
  return s;
}

void bgzf(const std::string& raw, std::string& out) {
  const size_t kBlock = 0xff00;
  std::vector<unsigned char> comp(compressBound(kBlock) + 64);
  for (size_t i = 0; i < raw.size(); i += kBlock) {
    const size_t n = std::min(kBlock, raw.size() - i);
    z_stream z;
    memset(&z, 0, sizeof(z));
    deflateInit2(&z, 6, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY);
    z.next_in = (Bytef*)raw.data() + i;
    z.avail_in = (uInt)n;
    z.next_out = comp.data();
    z.avail_out = (uInt)comp.size();
    deflate(&z, Z_FINISH);
    const size_t clen = z.total_out;
    deflateEnd(&z);
    const unsigned char head[18] = {31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 66, 67, 2, 0,
                                    (unsigned char)((clen + 25) & 0xff), (unsigned char)((clen + 25) >> 8)};
    out.append((const char*)head, 18);
    out.append((const char*)comp.data(), clen);
    const uint32_t crc = (uint32_t)crc32(0, (const Bytef*)raw.data() + i, (uInt)n), isz = (uint32_t)n;
    out.append((const char*)&crc, 4);
    out.append((const char*)&isz, 4);
  }
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: synthbam OUT.bam N_RECORDS [SEED]\n");
    return 2;
  }
  const int64_t n = atoll(argv[2]);
  const uint64_t seed = argc > 3 ? strtoull(argv[3], nullptr, 10) : 0;
  const int n_cells = (int)std::max<int64_t>(1, n / 10000);
  const int n_genes = 30000, n_refs = 25;
  Rng g0(seed);
  // genes: Zipf(1.1) over ranks; names in a random order of the ranks
  std::vector<double> zcdf(n_genes);
  double zt = 0;
  for (int k = 0; k < n_genes; k++) zcdf[k] = (zt += std::pow(k + 1.0, -1.1));
  for (double& v : zcdf) v /= zt;
  std::vector<int> perm(n_genes);
  for (int k = 0; k < n_genes; k++) perm[k] = k;
  for (int k = n_genes - 1; k > 0; k--) std::swap(perm[k], perm[g0.below((uint32_t)k + 1)]);
  std::vector<std::string> gname(n_genes);
  for (int k = 0; k < n_genes; k++) {
    char b[32];
    snprintf(b, sizeof(b), "ENSG%011d", perm[k] * 7 + 3);
    gname[k] = b;
  }
  // cells: lognormal(0, 1) weights -> record counts summing to n; barcodes sorted
  std::vector<double> w(n_cells);
  double wt = 0;
  for (int c = 0; c < n_cells; c++) {
    const double u1 = std::max(g0.u(), 1e-300), u2 = g0.u();
    w[c] = std::exp(std::sqrt(-2 * std::log(u1)) * std::cos(2 * M_PI * u2));
    wt += w[c];
  }
  std::vector<int64_t> cnt(n_cells);
  int64_t got = 0;
  for (int c = 0; c < n_cells; c++) got += (cnt[c] = (int64_t)std::floor(w[c] / wt * (double)n));
  for (int64_t k = 0; got < n; k++, got++) cnt[k % n_cells]++;
  std::vector<std::string> cb(n_cells);
  for (int c = 0; c < n_cells; c++) cb[c] = kmer(g0, 16);
  std::sort(cb.begin(), cb.end());
  cb.erase(std::unique(cb.begin(), cb.end()), cb.end());
  if ((int)cb.size() != n_cells) {
    fprintf(stderr, "barcode collision; use another seed\n");
    return 1;
  }
  std::vector<int64_t> first(n_cells + 1, 0);
  for (int c = 0; c < n_cells; c++) first[c + 1] = first[c] + cnt[c];
  const Cdf cg(kWGenomic), cc(kWCY), cu(kWUY);

  // header
  std::string hdr("BAM\1", 4);
  const std::string text = "@HD\tVN:1.4\tSO:unsorted\n";
  put32(hdr, (uint32_t)text.size());
  hdr += text;
  put32(hdr, (uint32_t)n_refs);
  for (int r = 0; r < n_refs; r++) {
    char b[16];
    snprintf(b, sizeof(b), "chr%d", r + 1);
    put32(hdr, (uint32_t)strlen(b) + 1);
    hdr.append(b, strlen(b) + 1);
    put32(hdr, 1u << 28);
  }
  // cells in chunks, each chunk's records then its BGZF members built by one thread
  const int n_chunks = std::max(1, std::min(n_cells, omp_get_max_threads() * 8));
  std::vector<std::string> members(n_chunks);
#pragma omp parallel for schedule(dynamic, 1)
  for (int ch = 0; ch < n_chunks; ch++) {
    const int c0 = (int)((int64_t)n_cells * ch / n_chunks), c1 = (int)((int64_t)n_cells * (ch + 1) / n_chunks);
    std::string raw;
    if (ch == 0) raw = hdr;
    for (int c = c0; c < c1; c++) {
      Rng r(seed * 1000003 + (uint64_t)c + 1);
      int64_t left = cnt[c], qn = first[c];
      while (left > 0) {
        // one molecule: Geometric(0.35) reads sharing UB, GE, ref, anchor
        int reads = 1;
        while (r.u() > 0.35) reads++;
        if (reads > left) reads = (int)left;
        left -= reads;
        const std::string ub = kmer(r, 10);
        const double gx = r.u();
        std::string ge;
        if (gx >= 0.06) {
          const int k = (int)(std::lower_bound(zcdf.begin(), zcdf.end(), r.u()) - zcdf.begin());
          ge = gname[std::min(k, n_genes - 1)];
          if (gx < 0.07) ge += "," + gname[0];
        }
        const int ref = (int)r.below(n_refs);
        const int32_t anchor = (int32_t)r.below(1u << 27);
        for (int rd = 0; rd < reads; rd++, qn++) {
          const bool unmapped = r.u() < 0.05;
          std::string b;
          b.reserve(420);
          char qname[24];
          const int lrn = snprintf(qname, sizeof(qname), "R%011lld", (long long)qn) + 1;
          const int lseq = 98;
          int clip = r.u() < 0.13 ? 1 + (int)r.below(29) : 0;
          const bool clip_front = r.u() < 0.5;
          const bool spliced = !unmapped && r.u() < 0.05;
          std::vector<uint32_t> cig;
          if (clip && clip_front) cig.push_back((uint32_t)clip << 4 | 4);
          const int m = lseq - clip;
          if (spliced && m > 41) {
            cig.push_back(40u << 4 | 0);
            cig.push_back(500u << 4 | 3);
            cig.push_back((uint32_t)(m - 40) << 4 | 0);
          } else {
            cig.push_back((uint32_t)m << 4 | 0);
          }
          if (clip && !clip_front) cig.push_back((uint32_t)clip << 4 | 4);
          uint16_t flag = 0;
          if (unmapped) flag |= 0x4;
          else {
            if (r.u() < 0.70) flag |= 0x10;
            if (r.u() < 0.16) flag |= 0x400;
          }
          const int32_t pos = unmapped ? -1 : anchor + 50 * (int32_t)r.below(4);
          put32(b, 0);  // block_size, patched below
          put32(b, (uint32_t)(unmapped ? -1 : ref));
          put32(b, (uint32_t)pos);
          b.push_back((char)lrn);
          b.push_back((char)(unmapped ? 0 : 255));
          put16(b, 4680);  // bin (unused by the decoders)
          put16(b, (uint16_t)cig.size());
          put16(b, flag);
          put32(b, (uint32_t)lseq);
          put32(b, 0xffffffffu);
          put32(b, 0xffffffffu);
          put32(b, 0);
          b.append(qname, lrn);
          for (uint32_t x : cig) put32(b, x);
          for (int i = 0; i < (lseq + 1) / 2; i++) b.push_back((char)(0x12 + (r.next() >> 61)));
          for (int i = 0; i < lseq; i++) b.push_back((char)cg.draw(r));
          // tags: CB / CR / CY / UB / UR / UY / GE / XF / NH
          ztag(b, "CB", cb[c]);
          std::string cr = cb[c];
          if (r.u() < 0.01) cr[r.below(16)] = 'N';
          ztag(b, "CR", cr);
          ztag(b, "CY", qual_string(r, cc, 16));
          ztag(b, "UB", ub);
          std::string ur = ub;
          if (r.u() < 0.002) ur[r.below(10)] = 'N';
          ztag(b, "UR", ur);
          ztag(b, "UY", qual_string(r, cu, 10));
          if (!ge.empty()) ztag(b, "GE", ge);
          if (!unmapped) {
            const double x = r.u();
            ztag(b, "XF", x < 0.85 ? "CODING" : x < 0.90 ? "INTRONIC" : x < 0.93 ? "UTR" : "INTERGENIC");
          }
          b.append("NHC", 3);
          b.push_back((char)(unmapped ? 0 : (r.u() < 0.9 ? 1 : 2 + (int)r.below(9))));
          const uint32_t bs = (uint32_t)b.size() - 4;
          memcpy(&b[0], &bs, 4);
          raw += b;
        }
      }
    }
    bgzf(raw, members[ch]);
  }
  FILE* fo = fopen(argv[1], "wb");
  if (!fo) {
    perror(argv[1]);
    return 1;
  }
  size_t total = 0;
  for (auto& m : members) {
    fwrite(m.data(), 1, m.size(), fo);
    total += m.size();
  }
  static const unsigned char eof[28] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 0x42, 0x43,
                                        2,    0,    0x1b, 0, 3, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  fwrite(eof, 1, 28, fo);
  fclose(fo);
  fprintf(stderr, "synthbam: %lld records, %d cells, %zu bytes\n", (long long)n, n_cells, total + 28);
  return 0;
}
