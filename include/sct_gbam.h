/* sct_gbam.h -- BAM -> columnar decode on the device (libsct_gbam.so, HIP for gfx950).
 *
 * The same 32-byte SoA columns and dictionaries as include/sct_bam.h's SCT_BAM_CELL_METRICS /
 * SCT_BAM_GENE_METRICS decode, produced on the GPU: the compressed file is copied to HBM once,
 * every BGZF member is inflated by one wavefront (Huffman tables and the 32 KB window in LDS),
 * record starts are found per member and verified against the previous member's walk, each
 * record is parsed by one lane (the validation of sct_bam.h, the aligned-quality sums, the tag
 * walk) and the CB / UB / GE strings are interned in device hash tables; only the distinct
 * strings come back to the host, to be ranked in Python's sorted() order.
 *
 * It replaces the same reference reads as sct_bam.h (the per-record pysam loop of
 * MetricAggregator.parse_molecule, aggregator.py:251-334, and CellMetrics.parse_extra_fields,
 * aggregator.py:507-530; the native analogue is fastqpreprocessing/src/htslib_tagsort.cpp:106-218).
 *
 * The device path handles the common file; anything else -- a record that fails validation, a
 * typed (non-string) dictionary tag, non-ASCII dictionary bytes, a malformed deflate stream --
 * makes the call return SCT_GBAM_HOST without raising, and the caller decodes the file with
 * sct_bam_decode, which reports the reference's exception for the first offending record.
 */
#ifndef SCT_GBAM_H
#define SCT_GBAM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SCT_GBAM_HOST 1 /* not decodable on the device as the reference would read it: use sct_bam_decode */

typedef struct sct_gbam sct_gbam_t;

/* Phase 1: map `path`, copy it to device `device`, inflate every BGZF member and locate the
 * alignment records, on `stream` (a hipStream_t, NULL: the default stream).  On SCT_BAM_OK
 * *out owns the device buffers and *n_records is the record count.  Returns SCT_GBAM_HOST or an
 * SCT_BAM_E* code (sct_bam.h) otherwise, with *out NULL. */
int sct_gbam_open(const char* path, int32_t device, void* stream, sct_gbam_t** out, int64_t* n_records);

/* Phase 1 for one of `n_parts` devices decoding one file together (GatherCellMetrics(devices=N)):
 * part `part` takes the BGZF members from the first one starting at or after part/n_parts of the
 * file's bytes to the next part's first (byte-balanced; part 0 keeps the header's) and the records
 * starting in their payload; a record cut by the part's end is read on from the next part's
 * members.  first_start: the payload offset of the part's first record, or -1 to find it inside the
 * part (then check it: sct_gbam_part_bounds).  A part may hold no records (*n_records 0: skip its
 * parse).  Same returns as sct_gbam_open. */
int sct_gbam_open_part(const char* path, int32_t part, int32_t n_parts, int64_t first_start, int32_t device,
                       void* stream, sct_gbam_t** out, int64_t* n_records);

/* Payload offsets of a part's first record and of the first record after the part (its walk's
 * landing).  Part p's first_start must equal part p-1's end_landing; if not, reopen part p with
 * first_start = part p-1's end_landing (the walk from inside part p guessed wrong). */
int sct_gbam_part_bounds(const sct_gbam_t* h, int64_t* first_start, int64_t* end_landing);

/* After every part's parse: the parts' dictionaries `which` merged into one ranked dictionary (the
 * sorted union, the missing tag first if any part has it; sct_gbam_dictionary(parts[0], which)
 * returns it) and remap[p][i] = the merged id of part p's id i (caller-sized host arrays, one entry
 * per id of part p's dictionary).  Then sct_gbam_remap renumbers each part's column. */
int sct_gbam_merge_dictionaries(sct_gbam_t* const* parts, int32_t n_parts, int32_t which, int32_t* const* remap);

/* column[i] = remap[column[i]] for the n int32 ids of a device column, on the part's device and
 * stream (remap: n_ids host entries). */
int sct_gbam_remap(sct_gbam_t* h, const int32_t* remap, int64_t n_ids, void* column, int64_t n);

/* Phase 2: parse the records into the caller's device columns, in the order of
 * sct_records_t (include/sctools_gpu.h): cell, umi, gene, ref, pos (int32), gq_sum, gq_len,
 * gq_gt30 (uint16), bits, xf, cy_gt30, cy_len, uy_gt30, uy_len (uint8); each holds
 * n_records elements.  metric_mode: SCT_BAM_CELL_METRICS or SCT_BAM_GENE_METRICS.
 * Returns SCT_BAM_OK, SCT_GBAM_HOST, or SCT_BAM_EIO on a device error. */
int sct_gbam_parse(sct_gbam_t* h, int32_t metric_mode, void* const* columns);

/* Phase 2, count-matrix mode (sct_bam.h SCT_BAM_COUNT_MATRIX; CountMatrix.from_sorted_tagged_bam,
 * count.py:134-328): `tags` holds the cell, molecule and gene tag names (6 characters, as
 * sct_bam_decode_tags); columns: cell, umi, gene (int32), xf (uint8: 0 no XF tag, 4 INTERGENIC,
 * 5 any other value), qhead (uint8: 1 where the record's query name differs from the previous
 * record's -- the itertools.groupby of count.py:83-86), each n_records elements.  No validation,
 * as the reference reads only these tags.  A non-string value of a named tag returns
 * SCT_GBAM_HOST (the host decoder applies the reference's str() or raises its error).
 * Returns SCT_BAM_OK, SCT_GBAM_HOST, or SCT_BAM_EIO on a device error. */
int sct_gbam_parse_count(sct_gbam_t* h, const char* tags, void* const* columns);

/* The ranked dictionary `which` (SCT_BAM_TAG_CB / _UB / _GE) after sct_gbam_parse(_count), as
 * sct_bam_dictionary: *n names, names[i] = bytes[offsets[i] .. offsets[i+1]), entry 0 the
 * missing tag when *has_none.  Valid until sct_gbam_close. */
int sct_gbam_dictionary(const sct_gbam_t* h, int32_t which, int64_t* n, const char** bytes,
                        const int64_t** offsets, int32_t* has_none);

/* Copy `n` inflated bytes from offset `off` of the concatenated BGZF payload to host `dst`
 * (tests compare it with zlib).  *total (if set) receives the payload length. */
int sct_gbam_read_inflated(const sct_gbam_t* h, uint64_t off, uint64_t n, void* dst, uint64_t* total);

/* Seconds spent per stage: [0] map + scan, [1] copy to the device (in pieces, each piece's members
 * inflating while the next piece copies), [2] the inflate left after the last piece, [3] record
 * starts, [4] parse + intern, [5] dictionaries, [6] members, [7] record-start repair rounds. */
int sct_gbam_timing(const sct_gbam_t* h, double* t8);

/* Decode windows of the file (1: the whole payload was resident at once).  A BAM whose payload
 * exceeds SCT_GBAM_WINDOW_BYTES (default: a quarter of the device's free memory) is decoded in
 * windows of whole BGZF members, twice inflated: sct_gbam_open proves record starts and counts
 * records window by window, sct_gbam_parse re-inflates and parses them, so device memory holds one
 * window's payload, the columns and the dictionaries (the reference reads in bounded memory too:
 * bam.py:361-488 splits, htslib_tagsort.cpp:308-393 streams). */
int64_t sct_gbam_windows(const sct_gbam_t* h);

/* Free the device buffers. */
void sct_gbam_close(sct_gbam_t* h);

/* Message of the calling thread's last error ("" if none). */
const char* sct_gbam_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
