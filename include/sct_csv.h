/* sct_csv.h -- native metric CSV text and parallel gzip (host C++, zlib, OpenMP).
 *
 * Replaces the per-value str() formatting of the reference's MetricCSVWriter.write
 * (src/sctools/metrics/writer.py:84-103: str(int), float.__repr__ for floats) and its
 * single-threaded gzip.open(..., "wt") (writer.py:55-61) for the bulk rows the gatherers
 * write.  The text is byte-identical to Python's; the .csv.gz is a sequence of gzip members
 * (RFC 1952 allows it; gzip, zcat, Python and pandas read it as one stream).
 */
#ifndef SCT_CSV_H
#define SCT_CSV_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SCT_CSV_INT 0
#define SCT_CSV_FLOAT 1

/* Python repr() of x (float.__repr__) into buf (NUL-terminated); returns the length, or -1
 * if cap is too small (32 bytes always suffice). */
int32_t sct_csv_repr_double(double x, char* buf, int32_t cap);

/* CSV lines "name,v1,...,vk\n" for `rows` rows.  Row r's name is the UTF-8 bytes
 * names[name_off[r] .. name_off[r + 1]); column c is ints[r * ints_stride + slot[c]]
 * (kind[c] == SCT_CSV_INT) or floats[r * floats_stride + slot[c]] (SCT_CSV_FLOAT).
 * threads <= 0: all cores.  *out is malloc'd (free with sct_csv_free). */
int sct_csv_format_rows(int64_t rows, const char* names, const int64_t* name_off, int32_t ncols,
                        const int32_t* kind, const int32_t* slot, const int64_t* ints, int32_t ints_stride,
                        const double* floats, int32_t floats_stride, int32_t threads, char** out,
                        int64_t* out_len);

/* gzip of data[0 .. len) as independent members of `chunk` input bytes each, compressed in
 * parallel at `level` (the reference's gzip.open uses 9).  *out is malloc'd. */
int sct_csv_gzip(const char* data, int64_t len, int32_t level, int64_t chunk, int32_t threads, char** out,
                 int64_t* out_len);

void sct_csv_free(char* p);

#ifdef __cplusplus
}
#endif

#endif /* SCT_CSV_H */
