// csvfmt.cpp -- metric CSV text (Python str / float.__repr__) and parallel gzip (include/sct_csv.h).
//
// float.__repr__ is the shortest decimal string that round-trips (Python's 'r' format,
// Py_DTSF_ADD_DOT_0): digits and exponent from std::to_chars' shortest scientific form, then
// Python's layout rule (pystrtod.c format_float_short): positional when -4 < decpt <= 16, with
// ".0" added to integral values; otherwise d[.ddd]e+XX with at least two exponent digits.
#include <math.h>
#include <omp.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#include <charconv>
#include <string>
#include <vector>

#include "../../include/sct_csv.h"

namespace {

int repr_double(double x, char* out) {
  char* p = out;
  if (isnan(x)) {
    memcpy(out, "nan", 4);
    return 3;
  }
  if (isinf(x)) {
    if (x < 0) *p++ = '-';
    memcpy(p, "inf", 4);
    return (int)(p - out) + 3;
  }
  if (x == 0.0) {
    if (signbit(x)) *p++ = '-';
    memcpy(p, "0.0", 4);
    return (int)(p - out) + 3;
  }
  char sci[40];
  const auto r = std::to_chars(sci, sci + sizeof(sci), x, std::chars_format::scientific);
  *r.ptr = 0;
  const char* s = sci;
  if (*s == '-') *p++ = '-', s++;
  char digits[24] = {0};
  int nd = 0;
  while (*s && *s != 'e') {
    if (*s != '.') digits[nd++] = *s;
    s++;
  }
  const int e = atoi(s + 1);  // exponent of the first digit
  const int decpt = e + 1;
  if (decpt > -4 && decpt <= 16) {
    if (decpt <= 0) {
      *p++ = '0', *p++ = '.';
      for (int i = 0; i < -decpt; i++) *p++ = '0';
      for (int i = 0; i < nd; i++) *p++ = digits[i];
    } else if (decpt >= nd) {
      for (int i = 0; i < nd; i++) *p++ = digits[i];
      for (int i = nd; i < decpt; i++) *p++ = '0';
      *p++ = '.', *p++ = '0';
    } else {
      for (int i = 0; i < decpt; i++) *p++ = digits[i];
      *p++ = '.';
      for (int i = decpt; i < nd; i++) *p++ = digits[i];
    }
  } else {
    *p++ = digits[0];
    if (nd > 1) {
      *p++ = '.';
      for (int i = 1; i < nd; i++) *p++ = digits[i];
    }
    const int ex = decpt - 1;
    *p++ = 'e';
    *p++ = ex < 0 ? '-' : '+';
    const int a = ex < 0 ? -ex : ex;
    if (a < 10) *p++ = '0';
    const auto q = std::to_chars(p, p + 8, a);
    p = q.ptr;
  }
  *p = 0;
  return (int)(p - out);
}

}  // namespace

extern "C" {

int32_t sct_csv_repr_double(double x, char* buf, int32_t cap) {
  char tmp[40];
  const int n = repr_double(x, tmp);
  if (!buf || cap < n + 1) return -1;
  memcpy(buf, tmp, (size_t)n + 1);
  return n;
}

int sct_csv_format_rows(int64_t rows, const char* names, const int64_t* name_off, int32_t ncols,
                        const int32_t* kind, const int32_t* slot, const int64_t* ints, int32_t ints_stride,
                        const double* floats, int32_t floats_stride, int32_t threads, char** out,
                        int64_t* out_len) {
  if (!out || !out_len || rows < 0 || ncols < 0) return -1;
  if (threads <= 0) threads = omp_get_max_threads();
  const int64_t per = rows / threads + 1;
  std::vector<std::string> parts((size_t)threads);
#pragma omp parallel num_threads(threads)
  {
    const int t = omp_get_thread_num();
    const int64_t r0 = (int64_t)t * per, r1 = r0 + per < rows ? r0 + per : rows;
    std::string& s = parts[(size_t)t];
    s.reserve(r1 > r0 ? (size_t)(r1 - r0) * (32 + 12 * (size_t)ncols) : 0);
    char buf[48];
    for (int64_t r = r0; r < r1; r++) {
      s.append(names + name_off[r], (size_t)(name_off[r + 1] - name_off[r]));
      for (int c = 0; c < ncols; c++) {
        s.push_back(',');
        if (kind[c] == SCT_CSV_INT) {
          const auto q = std::to_chars(buf, buf + sizeof(buf), ints[r * ints_stride + slot[c]]);
          s.append(buf, (size_t)(q.ptr - buf));
        } else {
          s.append(buf, (size_t)repr_double(floats[r * floats_stride + slot[c]], buf));
        }
      }
      s.push_back('\n');
    }
  }
  size_t total = 0;
  for (auto& s : parts) total += s.size();
  char* o = (char*)malloc(total ? total : 1);
  if (!o) return -1;
  size_t off = 0;
  for (auto& s : parts) {
    memcpy(o + off, s.data(), s.size());
    off += s.size();
  }
  *out = o;
  *out_len = (int64_t)total;
  return 0;
}

int sct_csv_gzip(const char* data, int64_t len, int32_t level, int64_t chunk, int32_t threads, char** out,
                 int64_t* out_len) {
  if (!out || !out_len || len < 0) return -1;
  if (threads <= 0) threads = omp_get_max_threads();
  if (chunk <= 0) chunk = 1 << 22;
  const int64_t nchunks = len ? (len + chunk - 1) / chunk : 1;
  std::vector<std::string> parts((size_t)nchunks);
  int bad = 0;
#pragma omp parallel for num_threads(threads) schedule(dynamic, 1) reduction(| : bad)
  for (int64_t k = 0; k < nchunks; k++) {
    const int64_t b = k * chunk, n = (b + chunk < len ? chunk : len - b);
    z_stream z;
    memset(&z, 0, sizeof(z));
    if (deflateInit2(&z, level, Z_DEFLATED, 15 + 16, 8, Z_DEFAULT_STRATEGY) != Z_OK) {
      bad |= 1;
      continue;
    }
    std::string& s = parts[(size_t)k];
    s.resize(deflateBound(&z, (uLong)n) + 32);
    z.next_in = (Bytef*)(data + b);
    z.avail_in = (uInt)n;
    z.next_out = (Bytef*)&s[0];
    z.avail_out = (uInt)s.size();
    if (deflate(&z, Z_FINISH) != Z_STREAM_END) bad |= 1;
    s.resize(z.total_out);
    deflateEnd(&z);
  }
  if (bad) return -1;
  size_t total = 0;
  for (auto& s : parts) total += s.size();
  char* o = (char*)malloc(total ? total : 1);
  if (!o) return -1;
  size_t off = 0;
  for (auto& s : parts) {
    memcpy(o + off, s.data(), s.size());
    off += s.size();
  }
  *out = o;
  *out_len = (int64_t)total;
  return 0;
}

void sct_csv_free(char* p) { free(p); }

}  // extern "C"
