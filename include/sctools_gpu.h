/*
 * sctools_gpu.h -- C-ABI of libsctools_gpu.so, the MI355X (gfx950) metric engine.
 *
 * This is the drop-in boundary for the reference's per-record Python hot loop.
 * Every entry point below names the reference interface it replaces
 * (file:line into fredlas/sctools, src/sctools/...).  The reference has no
 * native FFI for this path; the binding a maintainer would
 * add on the reference side is a ctypes stub, shown in INTEGRATION.md.
 *
 * Conventions
 *   - Plain pointers and sizes only.  Record columns, workspace, partials and
 *     outputs are DEVICE pointers (hipMalloc / torch CUDA tensors) unless a
 *     parameter says "host".  `stream` is a hipStream_t passed as void*
 *     (NULL = the legacy default stream).
 *   - The library never allocates or frees caller memory.  Workspace is
 *     caller-provided and sized by sct_workspace_size().
 *   - Return 0 on success, a negative SCT_E* code on failure; the message is
 *     available from sct_last_error() (thread-local).
 *   - Reentrant: one call per (device, stream) at a time; no global mutable
 *     state besides the thread-local error string.
 */
#ifndef SCTOOLS_GPU_H
#define SCTOOLS_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SCT_ABI_VERSION 2

/* ---- error codes ---- */
#define SCT_OK 0
#define SCT_EINVAL (-1)  /* bad argument / shape */
#define SCT_EHIP (-2)    /* HIP runtime error */
#define SCT_ENOMEM (-3)  /* workspace too small */
#define SCT_ENCCL (-4)   /* RCCL error */

/* ---- per-record columns: the 32-byte SoA record ----
 * Read by the reference per record in MetricAggregator.parse_molecule
 * (metrics/aggregator.py:251-334) and CellMetrics.parse_extra_fields
 * (metrics/aggregator.py:507-530). */
#define SCT_B_UNMAPPED 0x01u     /* flag & 0x4                       */
#define SCT_B_REVERSE 0x02u      /* flag & 0x10                      */
#define SCT_B_DUPLICATE 0x04u    /* flag & 0x400                     */
#define SCT_B_SPLICED 0x08u      /* CIGAR N length > 0               */
#define SCT_B_NH1 0x10u          /* NH == 1                          */
#define SCT_B_PERFECT_UMI 0x20u  /* UR and UB present, UR == UB      */
#define SCT_B_HAS_CB 0x40u       /* CB present                       */
#define SCT_B_PERFECT_CB 0x80u   /* CB present, CR == CB             */

#define SCT_XF_ABSENT 0
#define SCT_XF_CODING 1
#define SCT_XF_INTRONIC 2
#define SCT_XF_UTR 3
#define SCT_XF_INTERGENIC 4
#define SCT_XF_OTHER 5

typedef struct sct_records {
  int64_t n;                /* number of records                              */
  const int32_t* cell;      /* CB dictionary id (missing CB is an id)         */
  const int32_t* umi;       /* UB dictionary id                               */
  const int32_t* gene;      /* GE dictionary id                               */
  const int32_t* ref;       /* reference_id                                   */
  const int32_t* pos;       /* 0-based leftmost position                      */
  const uint16_t* gq_sum;   /* sum(query_alignment_qualities)                 */
  const uint16_t* gq_len;   /* len(query_alignment_qualities)                 */
  const uint16_t* gq_gt30;  /* #query_alignment_qualities > 30                */
  const uint8_t* bits;      /* SCT_B_*                                        */
  const uint8_t* xf;        /* SCT_XF_*                                       */
  const uint8_t* cy_gt30;   /* #CY phred > 30                                 */
  const uint8_t* cy_len;    /* len(CY)                                        */
  const uint8_t* uy_gt30;   /* #UY phred > 30                                 */
  const uint8_t* uy_len;    /* len(UY)                                        */
} sct_records_t;

/* ---- what an entity is ---- */
#define SCT_MODE_CELL 0         /* maximal run of equal `cell` (GatherCellMetrics, gatherer.py:116-159) */
#define SCT_MODE_GENE 1         /* maximal run of equal `gene` (GatherGeneMetrics, gatherer.py:189-232) */
#define SCT_MODE_GENE_GROUPED 2 /* every record of a gene id: per-gene partials, additive across
                                   cell shards; replaces MergeGeneMetrics (merge.py:74-191)          */

/* ---- how mean / variance are computed ---- */
#define SCT_FLOAT_EXACT_SUM 0 /* order-free exact fixed-point sums (x * 2^68 is an integer),
                                 correctly rounded mean and variance; independent of order,
                                 tiling and GPU count; within 1e-12 relative of Welford           */
#define SCT_FLOAT_WELFORD 1   /* sequential Welford in record order (stats.py:82-99): bit-identical
                                 to the reference; RUN modes only                                 */

typedef struct sct_plan {
  int64_t n_records;
  int64_t max_entities; /* upper bound on RUN-mode rows (from sct_count_entities);
                           0 = n_records.  Sizes the workspace.           */
  int32_t mode;         /* SCT_MODE_*                                     */
  int32_t float_mode;   /* SCT_FLOAT_*                                    */
  int32_t n_cell_ids;   /* dictionary sizes: ids are in [0, n_*_ids)      */
  int32_t n_gene_ids;
  int32_t n_umi_ids;
  int32_t flags;        /* SCT_PLAN_* bits                                */
} sct_plan_t;

/* plan.flags: size the workspace for grouped gene partials next to cell rows
 * (sct_cell_metrics_gene_partials).  Implied by SCT_MODE_GENE_GROUPED. */
#define SCT_PLAN_GENE_PARTIALS 0x1

/* ---- output rows ----
 * ints [rows][SCT_NI] (int64) and floats [rows][SCT_NF] (double).  Column
 * names follow the reference header (MetricAggregator.__init__,
 * aggregator.py:132-189; CellMetrics 437-461; GeneMetrics 561-569). */
#define SCT_NI 24
#define SCT_I_N_READS 0
#define SCT_I_NOISE_READS 1 /* always 0 (not implemented by the reference either) */
#define SCT_I_PERFECT_MOLECULE_BARCODES 2
#define SCT_I_READS_MAPPED_EXONIC 3
#define SCT_I_READS_MAPPED_INTRONIC 4
#define SCT_I_READS_MAPPED_UTR 5
#define SCT_I_READS_MAPPED_UNIQUELY 6
#define SCT_I_READS_MAPPED_MULTIPLE 7
#define SCT_I_DUPLICATE_READS 8
#define SCT_I_SPLICED_READS 9
#define SCT_I_ANTISENSE_READS 10 /* always 0 */
#define SCT_I_N_MOLECULES 11
#define SCT_I_N_FRAGMENTS 12
#define SCT_I_FRAGMENTS_SINGLE 13
#define SCT_I_MOLECULES_SINGLE 14
#define SCT_I_PERFECT_CELL_BARCODES 15 /* cell */
#define SCT_I_READS_MAPPED_INTERGENIC 16 /* cell */
#define SCT_I_READS_UNMAPPED 17 /* cell */
#define SCT_I_READS_TOO_MANY_LOCI 18 /* always 0 */
#define SCT_I_N_K1 19        /* cell: n_genes; gene: number_cells_expressing */
#define SCT_I_K1_MULTIPLE 20 /* cell: genes_detected_multiple_observations; gene: number_cells_detected_multiple */
#define SCT_I_N_MITO_GENES 21 /* cell */
#define SCT_I_N_MITO_MOLECULES 22 /* cell (counts reads, as the reference does) */
#define SCT_I_ENTITY 23       /* RUN modes: index of the entity's first record; GROUPED: gene id */

#define SCT_NF 12
#define SCT_F_UY_MEAN 0 /* molecule_barcode_fraction_bases_above_30_mean */
#define SCT_F_UY_VAR 1
#define SCT_F_GQF_MEAN 2 /* genomic_reads_fraction_bases_quality_above_30_mean */
#define SCT_F_GQF_VAR 3
#define SCT_F_GQ_MEAN 4 /* genomic_read_quality_mean */
#define SCT_F_GQ_VAR 5
#define SCT_F_READS_PER_MOLECULE 6
#define SCT_F_READS_PER_FRAGMENT 7
#define SCT_F_FRAGMENTS_PER_MOLECULE 8
#define SCT_F_CY_VAR 9 /* cell_barcode_fraction_bases_above_30_variance */
#define SCT_F_CY_MEAN 10
#define SCT_F_PCT_MITO 11

/* ---- additive partials (GROUPED mode; also the internal RUN-mode row state) ----
 * int64 [rows][SCT_NP]: 24 counter slots, then per float stream (UY frac,
 * genomic frac, genomic mean quality, CY frac) 3 lanes of sum(x*2^68) and 5
 * lanes of sum((x*2^68)^2); a lane holds a sum of 32-bit limb values, so
 * lanes are plain int64 sums and partials of disjoint record sets add
 * lane-wise (this is what the RCCL all-reduce sums).  Slot 20 of a RUN-mode
 * row holds the entity's first record index and is not additive. */
#define SCT_NP 64
#define SCT_P_FLOAT_BASE 24
#define SCT_P_STREAM_LANES 8

/* ABI version of the loaded library (== SCT_ABI_VERSION). */
int sct_abi_version(void);

/* Last error message of the calling thread ("" if none). */
const char* sct_last_error(void);

/* Device workspace bytes needed for `plan`. */
int sct_workspace_size(const sct_plan_t* plan, size_t* bytes);

/* Number of output rows for `plan` (RUN modes: entity runs; GROUPED:
 * n_gene_ids).  Replaces the entity enumeration of bam.iter_tag_groups
 * (bam.py:492-540).  Synchronizes `stream`. */
int sct_count_entities(const sct_plan_t* plan, const sct_records_t* rec, void* workspace,
                       size_t workspace_bytes, int64_t* n_entities /* host */, void* stream);

/* Full metric rows for RUN modes (cell or gene entities, file order).
 * Replaces GatherCellMetrics.extract_metrics / GatherGeneMetrics.extract_metrics'
 * aggregation (gatherer.py:134-159 / 207-232): MetricAggregator.parse_molecule
 * (aggregator.py:236-334), parse_extra_fields (492-530, 580-595) and finalize
 * (342-387, 463-490, 571-578).  `gene_is_mito`/`gene_is_multi` are device
 * uint8[n_gene_ids].  `out_ints`/`out_floats` hold `capacity` rows; the row
 * count is returned in *n_rows (host).  Gene rows of multi-gene runs are
 * computed like any other; the caller drops them (gatherer.py:210-212). */
int sct_compute_metrics(const sct_plan_t* plan, const sct_records_t* rec,
                        const uint8_t* gene_is_mito, const uint8_t* gene_is_multi,
                        void* workspace, size_t workspace_bytes, int64_t* out_ints,
                        double* out_floats, int64_t capacity, int64_t* n_rows /* host */,
                        void* stream);

/* Per-gene additive partials (GROUPED mode) of this rank's records, written
 * to `partials` [n_gene_ids][SCT_NP] (overwritten).  Records must be
 * cell-sorted with every cell id in one run (SCT_EINVAL otherwise) and
 * cell-sharded across calls: the SplitBam invariant (bam.py:439-448).  The
 * (gene, cell, umi) Counters of the gene view are resolved in the cell-sorted
 * order, so this runs the cell pipeline internally.  Synchronizes `stream`. */
int sct_gene_partials(const sct_plan_t* plan, const sct_records_t* rec, void* workspace,
                      size_t workspace_bytes, int64_t* partials, void* stream);

/* Cell rows (as sct_compute_metrics with SCT_MODE_CELL) AND grouped gene
 * partials (as sct_gene_partials) from one pass over cell-sorted records:
 * GatherCellMetrics + GatherGeneMetrics of the same shard sharing one sort.
 * `plan->mode` must be SCT_MODE_CELL with SCT_PLAN_GENE_PARTIALS in flags. */
int sct_cell_metrics_gene_partials(const sct_plan_t* plan, const sct_records_t* rec,
                                   const uint8_t* gene_is_mito, void* workspace,
                                   size_t workspace_bytes, int64_t* out_ints, double* out_floats,
                                   int64_t capacity, int64_t* n_rows /* host */,
                                   int64_t* gene_partials, void* stream);

/* Finalize `rows` partial rows into output rows (floats and ratios; the
 * reference's finalize(), aggregator.py:342-387, 463-490, 571-578).  `mode`
 * selects cell or gene columns; entity ids are written as the row index. */
int sct_finalize_partials(int32_t mode, const int64_t* partials, int64_t rows, int64_t* out_ints,
                          double* out_floats, void* stream);

/* ---- multi-GPU: the gene-partial all-reduce ----
 * Replaces MergeGeneMetrics' CSV merge of cell-disjoint chunks (merge.py:74-191; the
 * chunks come from SplitBam, bam.py:361-488).  Each rank holds [rows][SCT_NP] int64
 * partial rows of its cell shard (sct_gene_partials / sct_cell_metrics_gene_partials);
 * their lanes are plain integer sums, so one in-place sum all-reduce over RCCL (xGMI)
 * gives every rank the rows of the union of the shards, bit for bit, in any rank order;
 * sct_finalize_partials then yields the unsharded gene rows.
 * `comm` is an ncclComm_t (RCCL) passed as void*: from the helpers below or from the
 * caller's own RCCL setup.  Does not synchronize `stream`. */
int sct_allreduce_gene_partials(int64_t* partials, int64_t rows, void* comm, void* stream);

/* Communicator helpers for callers without their own RCCL setup.
 * One process, several devices: sct_comm_init_all fills comms[0..ndev) (ncclCommInitAll);
 * drive each from its own host thread (or one thread with group calls).
 * One process per device: rank 0 calls sct_comm_unique_id (id: >= 128 bytes, host), the id
 * travels out of band, then every rank calls sct_comm_init_rank on its device. */
int sct_comm_unique_id(uint8_t* id, size_t bytes);
int sct_comm_init_rank(void** comm, int nranks, const uint8_t* id, size_t bytes, int rank, int device);
int sct_comm_init_all(void** comms, int ndev, const int* devices);
int sct_comm_destroy(void* comm);
/* Abort a communicator whose peers may never arrive (ncclCommAbort): a rank failed before
 * or during the all-reduce.  Pending RCCL work on it is cancelled and the communicator is
 * freed; it must not be used or destroyed afterwards.  (New plumbing: the reference merges
 * CSV files and has no collective to abort.) */
int sct_comm_abort(void* comm);

/* ---- tag sort (TagSortBam / bam.sort_by_tags_and_queryname, bam.py:638-709;
 *      platform.py:55-104) ---- */
#define SCT_ORDER_CELL 0          /* CB only: what cell metrics need (input order kept within a cell) */
#define SCT_ORDER_CELL_UMI_GENE 1 /* CB, UB, GE: TagSortBam's order for GatherCellMetrics          */
#define SCT_ORDER_GENE_CELL_UMI 2 /* GE, CB, UB: TagSortBam's order for GatherGeneMetrics          */

/* Device workspace bytes for sct_tag_sort / sct_verify_sort of plan->n_records
 * records (plan: n_records and the three dictionary sizes; mode, float_mode
 * and flags are ignored). */
int sct_tag_sort_workspace_size(const sct_plan_t* plan, size_t* bytes);

/* Stable sort of `in` into `out` (caller-allocated device columns of n records,
 * written; must not alias `in`) by the `order` fields (dictionary ids: ranks of
 * the sorted tag strings, a missing tag first, as bam.get_tag_or_default(..., "")
 * sorts), then by `tiebreak` (nullable device int32 ids in [0, n_tiebreak_ids):
 * the query-name rank).  Without a tiebreak, ties keep input order (Python's
 * sorted() is stable).  Does not synchronize without a tiebreak; with one it synchronizes
 * `stream` once (to size the tiebreak pass over runs of equal tag fields). */
int sct_tag_sort(const sct_plan_t* plan, const sct_records_t* in, const int32_t* tiebreak,
                 int32_t n_tiebreak_ids, int32_t order, const sct_records_t* out, void* workspace,
                 size_t workspace_bytes, void* stream);

/* verify_sort (bam.py:712-724; VerifyBamSort, platform.py:107-143): *first_violation
 * (host) = the first index j with record j ordered before record j-1, or -1 if
 * `rec` is sorted by `order` (then `tiebreak`, if given).  Synchronizes `stream`. */
int sct_verify_sort(const sct_plan_t* plan, const sct_records_t* rec, const int32_t* tiebreak,
                    int32_t order, void* workspace, size_t workspace_bytes,
                    int64_t* first_violation /* host */, void* stream);

/* ---- multi-GPU for unsorted input: cell bins exchanged between devices ----
 * The reference's route for an unsorted BAM: SplitBam gives every cell barcode a bin
 * (bam.py:439-448), writes each input's records to their bins (write_barcodes_to_bins,
 * bam.py:454-463) and merges each bin's pieces (bam.py:465-480); every chunk is then sorted
 * (TagSortBam, platform.py:55-97) and measured.  Here each device bins its part of the records
 * (sct_bin_records), the devices swap bins over RCCL (sct_exchange_counts, then
 * sct_exchange_records: bin r of every rank to rank r, in rank order), and each device sorts
 * and measures its cells (sct_tag_sort, sct_cell_metrics_gene_partials), the gene partials
 * summed by sct_allreduce_gene_partials.  Bins keep input order, so a rank whose parts are
 * consecutive file ranges receives its cells' records in file order. */
#define SCT_MAX_BINS 256

/* Device workspace bytes for sct_bin_records of plan->n_records records into n_bins bins. */
int sct_bin_workspace_size(const sct_plan_t* plan, int32_t n_bins, size_t* bytes);

/* Stable partition of `in` into `out` (caller-allocated device columns of n records; must not
 * alias `in`) by the bin of each record's cell: bin_of_cell[cell] (device uint8 per cell id,
 * values >= n_bins go to the last bin), or, when bin_of_cell is NULL, contiguous id ranges
 * cell * n_bins / n_cell_ids (ids are ranks of the sorted barcodes, so bins follow barcode
 * order).  Bin 0's records first; input order kept inside a bin.  `tiebreak` (nullable device
 * int32) is carried along into `tiebreak_out`.  bin_counts: device int64[n_bins], written.
 * 1 <= n_bins <= SCT_MAX_BINS.  Does not synchronize `stream`. */
int sct_bin_records(const sct_plan_t* plan, const sct_records_t* in, const int32_t* tiebreak,
                    const uint8_t* bin_of_cell, int32_t n_bins, const sct_records_t* out,
                    int32_t* tiebreak_out, int64_t* bin_counts, void* workspace, size_t workspace_bytes,
                    void* stream);

/* Every rank's bin counts swapped: recv_counts[p] (device int64[n_ranks]) = send_counts[me] of
 * rank p (device int64[n_ranks], this rank's bin sizes).  n_ranks = the communicator's size. */
int sct_exchange_counts(const int64_t* send_counts, int64_t* recv_counts, int32_t n_ranks, void* comm,
                        void* stream);

/* The binned records swapped: bin p of this rank (send_counts[p] records from the start of
 * bin p in `binned`) goes to rank p; `out` (out->n = sum(recv_counts)) receives rank 0's
 * piece first, then rank 1's, ... .  send_counts / recv_counts are HOST int64[n_ranks]
 * (sct_exchange_counts' result, copied back).  `tiebreak` / `tiebreak_out`: an optional int32
 * column exchanged alongside (both or neither).  One RCCL group of send/recv pairs per peer
 * and column; this rank's own bin is a device copy.  Does not synchronize `stream`. */
int sct_exchange_records(const sct_records_t* binned, const int32_t* tiebreak, const int64_t* send_counts,
                         const int64_t* recv_counts, int32_t n_ranks, const sct_records_t* out,
                         int32_t* tiebreak_out, void* comm, void* stream);

/* ---- count matrix (CountMatrix.from_sorted_tagged_bam, count.py:134-328) ---- */

#define SCT_COUNT_SKIP (-1)    /* gene_col: never counted (missing tag, or a multi-gene "a,b" value) */
#define SCT_COUNT_UNKNOWN (-2) /* gene_col: a single gene name outside the annotation (KeyError) */

typedef struct sct_count_input {
  int64_t n;            /* records, in file order */
  const int32_t* cell;  /* device, dictionary ids of the cell / molecule / gene tags */
  const int32_t* umi;
  const int32_t* gene;
  const uint8_t* xf;    /* device, SCT_XF_* */
  const uint8_t* qhead; /* device, 1 where the query name differs from the previous record's */
  int32_t n_cell_ids, n_umi_ids, n_gene_ids;
  int32_t cell_none, umi_none; /* id of a missing cell / molecule tag, or -1 */
  const int32_t* gene_col;     /* device [n_gene_ids]: matrix column, SCT_COUNT_SKIP or SCT_COUNT_UNKNOWN */
  int32_t n_cols;              /* annotation genes (matrix columns) */
} sct_count_input_t;

typedef struct sct_count_output {
  int32_t* row_cell;  /* device [n_cell_ids]: cell id of each row, rows in order of each cell's first counted molecule */
  int32_t* indptr;    /* device [n_cell_ids + 1]: CSR row pointers (n_rows + 1 written) */
  int32_t* indices;   /* device [n]: CSR column indices, ascending within a row */
  uint32_t* data;     /* device [n]: molecules (distinct molecule barcodes) per (cell, gene) */
  int64_t n_rows;     /* host, set on return */
  int64_t nnz;        /* host, set on return */
  int64_t unknown_record; /* host: first record (file order) of a counted molecule whose gene is
                           * SCT_COUNT_UNKNOWN -- the reference's KeyError -- or -1 */
  int64_t n_sorted;       /* host: molecule keys sorted (the counted query-name groups) */
} sct_count_output_t;

/* Device workspace bytes for sct_count_matrix. */
int sct_count_matrix_workspace_size(const sct_count_input_t* in, size_t* bytes);

/* The cells x genes molecule-count matrix in CSR form, as the reference builds it: records
 * are grouped by runs of equal query name; a group counts when its first record has both
 * barcodes and exactly one distinct single gene name is carried by its alignments with an
 * XF tag other than INTERGENIC; a (cell, molecule, gene) triple counts once.  On
 * unknown_record >= 0 the matrix outputs are not written.  Synchronizes `stream`. */
int sct_count_matrix(const sct_count_input_t* in, sct_count_output_t* out, void* workspace, size_t workspace_bytes,
                     void* stream);

/* Optional kernel timing: while enabled, every kernel launch is bracketed by
 * HIP events on its launch stream.  sct_profile_read waits for the events,
 * fills up to `max_kernels` (name, total ms, launches) triples (host arrays;
 * names stay valid until the next read), resets, and returns the number of
 * distinct kernels seen.  sct_profile_only restricts the timing to the kernels
 * of one name (NULL or "": all kernels), so a caller can time one kernel
 * without bracketing every launch.  Thread-local. */
int sct_profile_enable(int on);
int sct_profile_only(const char* kernel_name);
int sct_profile_read(const char** names, double* ms, int64_t* launches, int max_kernels);
/* sct_profile_read plus, per kernel, the items its timed launches processed in all (records,
 * payloads or sort items: what the algorithmic bytes per item of the roofline multiply), or -1
 * when a launch of that kernel does not report them. */
int sct_profile_read_items(const char** names, double* ms, int64_t* launches, int64_t* items, int max_kernels);

#ifdef __cplusplus
}
#endif

#endif /* SCTOOLS_GPU_H */
