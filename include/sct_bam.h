/* sct_bam.h -- native BAM -> columnar decoder for the metric path (host C++, zlib, OpenMP).
 *
 * Replaces the per-record pysam reads of the reference's aggregation loop
 * (MetricAggregator.parse_molecule, aggregator.py:251-334; CellMetrics.parse_extra_fields,
 * aggregator.py:507-530; pysam 0.16 AlignedSegment.query_alignment_qualities /
 * get_cigar_stats) with one parallel pass: BGZF blocks are inflated concurrently,
 * records are parsed concurrently, and the CB / UB / GE tag strings are dictionary-encoded
 * to ids that are ranks of the sorted strings with a missing tag first (ids compare as the
 * strings compare).  Output: the 32-byte-per-record SoA columns of include/sctools_gpu.h.
 *
 * The decode validates exactly as sctools_amd.columnar.columnarize (and so the reference):
 * the FIRST offending record in file order decides the error, reported as a code below
 * and a message (the Python layer raises the reference's exception types).
 */
#ifndef SCT_BAM_H
#define SCT_BAM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SCT_BAM_OK 0
#define SCT_BAM_EIO -1          /* cannot open / read / inflate the file            */
#define SCT_BAM_EFORMAT -2      /* not a BAM file or a truncated record             */
#define SCT_BAM_KEYERROR -10    /* a required tag is missing (KeyError)             */
#define SCT_BAM_TYPEERROR -11   /* missing base qualities (TypeError)               */
#define SCT_BAM_ZERODIV -12     /* empty quality string (ZeroDivisionError)         */
#define SCT_BAM_VALUEERROR -13  /* invalid clipping, or a record beyond the 32-byte columnar limits */
#define SCT_BAM_EMPTY -14       /* no records (RuntimeError: StopIteration in iter_tag_groups) */
#define SCT_BAM_MISSING_TAG -15 /* sct_bam_split: a record carries none of the tags (RuntimeError, bam.py:286-289) */
#define SCT_BAM_ETYPED -16      /* sct_bam_decode*: a dictionary tag holds a float or array value (or, for
                                 * SCT_BAM_SORT_KEYS, an integer): decode with the Python reader instead */

#define SCT_BAM_CELL_METRICS 0 /* require CY (and CR where CB is present), as CellMetrics does   */
#define SCT_BAM_GENE_METRICS 1 /* records of multi-gene GE values are not validated (gatherer.py:210-212) */
#define SCT_BAM_COUNT_MATRIX 2 /* CountMatrix.from_sorted_tagged_bam (count.py:134-328): only the cell /
                                * molecule / gene tags, XF and the query name are read, nothing is
                                * validated, an empty file is 0 records, and the "qhead" column is set */

#define SCT_BAM_SORT_KEYS 3   /* TagSortBam / VerifyBamSort keys (bam.py:638-724): the three dictionary tags
                                * (a missing tag and an empty value are both id 0: get_tag_or_default's "")
                                * and the query name, ranked into a fourth dictionary (column "qname",
                                * int32); nothing is validated, an empty file is 0 records */

#define SCT_BAM_TAG_CB 0
#define SCT_BAM_TAG_UB 1
#define SCT_BAM_TAG_GE 2
#define SCT_BAM_QNAME 3 /* SCT_BAM_SORT_KEYS: the query-name dictionary */

typedef struct sct_bam sct_bam_t;

/* Decode `path` (BAM).  n_threads <= 0: all cores.  On success *out owns the columns and
 * dictionaries until sct_bam_close.  On a validation error *out is NULL, *bad_record (if
 * set) is the offending record's index, and sct_bam_last_error() holds the message. */
int sct_bam_decode(const char* path, int32_t metric_mode, int32_t n_threads, sct_bam_t** out,
                   int64_t* bad_record);

/* As sct_bam_decode, with the three dictionary tags named by `tags` (6 characters: cell,
 * molecule, gene tag, e.g. "CBUBGE" -- the CreateCountMatrix -c / -m / -g options,
 * platform.py:402-429).  The metric modes require "CBUBGE". */
int sct_bam_decode_tags(const char* path, int32_t metric_mode, const char* tags, int32_t n_threads,
                        sct_bam_t** out, int64_t* bad_record);

/* Message of the calling thread's last error ("" if none). */
const char* sct_bam_last_error(void);

/* Number of records. */
int64_t sct_bam_n(const sct_bam_t* b);

/* Host pointer to a column by name (the sct_records_t field names: "cell", "umi", "gene",
 * "ref", "pos", "gq_sum", "gq_len", "gq_gt30", "bits", "xf", "cy_gt30", "cy_len",
 * "uy_gt30", "uy_len"), or "qhead" (uint8: 1 where the record's query name differs from the
 * previous record's -- the itertools.groupby of count.py:83-86 -- SCT_BAM_COUNT_MATRIX only),
 * or "qname" (int32 rank of the query name, SCT_BAM_SORT_KEYS only);
 * NULL for an unknown name.  Valid until sct_bam_close. */
const void* sct_bam_column(const sct_bam_t* b, const char* name);

/* Dictionary of tag `which` (SCT_BAM_TAG_*, or SCT_BAM_QNAME): *n entries in id order; entry i is the UTF-8
 * string bytes[offsets[i] .. offsets[i + 1]); *has_none = 1 when id 0 is the missing value
 * (its bytes are empty). */
int sct_bam_dictionary(const sct_bam_t* b, int32_t which, int64_t* n, const char** bytes,
                       const int64_t** offsets, int32_t* has_none);

void sct_bam_close(sct_bam_t* b);

/* SplitBam (bam.split, bam.py:361-488; platform.py:153-223): the records of the input BAMs
 * into chunk files `<out_prefix>_<k>.bam`, k = 0 .. *n_out - 1, every barcode in exactly one
 * chunk.  A record's barcode is the value of the first of the `n_tags` two-character tags in
 * `tags` (priority order, e.g. "CBCR") it carries; records with none raise
 * SCT_BAM_MISSING_TAG when raise_missing, else they are dropped.  Barcodes are ranked in
 * string order and chunk k gets the barcodes of rank k (mod n_subfiles when there are more
 * barcodes than chunks), so *n_out = min(#barcodes, n_subfiles).  Records keep their file
 * order; several inputs (same reference list) are concatenated in input order.  Each chunk is
 * a BGZF file: the first input's header, the records (deflate `level` 0-9, 6 as htslib's
 * default), the EOF member.  n_threads <= 0: all cores.  On an error *bad_record (if set) is
 * the offending record's index over all inputs. */
int sct_bam_split(const char* const* in_paths, int32_t n_in, const char* out_prefix, const char* tags,
                  int32_t n_tags, int32_t n_subfiles, int32_t raise_missing, int32_t level, int32_t n_threads,
                  int32_t* n_out, int64_t* bad_record);

/* TagSortBam's output (platform.py:60-97, pysam writes the sorted records under the input's
 * header): the records of `in_path` written to `out_path` in the order `perm` gives
 * (perm[k] = the input index of output record k, a permutation of 0..n-1), byte for byte,
 * as BGZF (header members, 0xff00-byte record members, EOF) at zlib `level`. */
int sct_bam_write_order(const char* in_path, const char* out_path, const int64_t* perm, int64_t n, int32_t level,
                        int32_t n_threads);

#ifdef __cplusplus
}
#endif

#endif /* SCT_BAM_H */
