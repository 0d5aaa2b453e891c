"""
Metric aggregators -- same classes, attribute names and attribute order as the
reference (``/root/reference/src/sctools/metrics/aggregator.py``:
``MetricAggregator`` 46-387, ``CellMetrics`` 390-530, ``GeneMetrics``
533-595), so ``vars(CellMetrics())`` yields the reference CSV header and
existing callers of the aggregator protocol keep working.

``parse_molecule`` keeps the reference's per-record protocol: the plain
counters (``n_reads``, ``perfect_molecule_barcodes``, ``reads_mapped_*``,
``duplicate_reads``, ``spliced_reads``, ``perfect_cell_barcodes``,
``reads_unmapped`` ...) are host integers updated record by record in the
reference's order, and a missing tag raises its ``KeyError`` (or the empty
quality string its ``ZeroDivisionError``) inside the ``parse_molecule`` call
that reads it, after the counters the reference has already updated for that
record.  Each record's numeric fields are buffered with its tags; ``finalize``
runs the entity through the HIP engine (one launch sequence per entity -- the
gatherers batch every entity of a file into one launch sequence instead) for
the distinct counts and the Welford mean / variance, and fills every public
attribute from the engine's row.  ``finalize`` of an aggregator that parsed
nothing gives the reference's values (zero counts, 0.0 means, NaN variances
and ratios) without a launch.

A record that raises part-way (round 5): the reference has by then fed it to some
of its state.  A mapped read without an XF or NH tag (``KeyError``, aggregator.py:305 / 317) has
reached its molecule and fragment histograms and its UY / genomic Welford streams (264-303), so it
is buffered with the fields read so far before the error propagates; ``finalize()`` then takes the
distinct counts and the streams from the engine (that record included) and keeps the host's
integer counters, which stopped exactly where the reference's stopped.  A caller that catches the
error and calls ``finalize()`` -- at once, or after parsing more records -- gets the reference's
values (tests/golden/protocol: ``final_after_error``, ``final_continued``).  Remaining gap: a
record that raises earlier -- ``KeyError`` on CR (after its CY sample, 507-520) or UY, or
``TypeError`` / ``ZeroDivisionError`` on its qualities (after its UY sample) -- has fed only part of
a record's streams, which the engine's record format cannot express; it is not buffered, so
``finalize()`` after catching such an error leaves it out of the streams and distinct counts.
"""

from typing import Sequence

import numpy as np

from sctools_amd import _native as N
from sctools_amd import columnar as C
from sctools_amd import consts
from sctools_amd.metrics import rows as R

_NAN = float("nan")


class MetricAggregator:
    _MODE = None

    def __init__(self):
        # attribute order == reference header order (aggregator.py:141-189)
        self.n_reads: int = 0
        self.noise_reads: int = 0
        self._fragment_histogram = None
        self._molecule_histogram = None
        self._molecule_barcode_fraction_bases_above_30 = None
        self.perfect_molecule_barcodes = 0
        self._genomic_reads_fraction_bases_quality_above_30 = None
        self._genomic_read_quality = None
        self.reads_mapped_exonic = 0
        self.reads_mapped_intronic = 0
        self.reads_mapped_utr = 0
        self.reads_mapped_uniquely = 0
        self.reads_mapped_multiple = 0
        self.duplicate_reads = 0
        self.spliced_reads = 0
        self.antisense_reads = 0
        self._plus_strand_reads = 0
        self.molecule_barcode_fraction_bases_above_30_mean: float = None
        self.molecule_barcode_fraction_bases_above_30_variance: float = None
        self.genomic_reads_fraction_bases_quality_above_30_mean: float = None
        self.genomic_reads_fraction_bases_quality_above_30_variance: float = None
        self.genomic_read_quality_mean: float = None
        self.genomic_read_quality_variance: float = None
        self.n_molecules: float = None
        self.n_fragments: float = None
        self.reads_per_molecule: float = None
        self.reads_per_fragment: float = None
        self.fragments_per_molecule: float = None
        self.fragments_with_single_read_evidence: int = None
        self.molecules_with_single_read_evidence: int = None
        self._buffered = []  # (tags, numeric fields) per parsed record
        self._extra = (0, 0)  # the subclass's CY counts of the record being parsed

    # ---- aggregator protocol (aggregator.py:236-340) ----
    def parse_molecule(self, tags: Sequence[str], records) -> None:
        """aggregator.py:251-334, record by record: the subclass fields first, then the counters,
        raising where the reference raises.

        A mapped read without an XF or NH tag is buffered before its KeyError propagates (the
        reference has counted it in its histograms and streams by then; see the module docstring)."""
        for record in records:
            self._extra = (0, 0)
            self.parse_extra_fields(tags=tags, record=record)
            cg, cl = self._extra
            self.n_reads += 1
            ug, ul = C._frac_counts(record.get_tag(consts.QUALITY_MOLECULE_BARCODE_TAG_KEY))
            try:
                self.perfect_molecule_barcodes += record.get_tag(
                    consts.RAW_MOLECULE_BARCODE_TAG_KEY) == record.get_tag(consts.MOLECULE_BARCODE_TAG_KEY)
            except KeyError:
                pass
            aq = record.query_alignment_qualities
            if aq is None:
                raise TypeError("'NoneType' object is not iterable")
            if len(aq) == 0:
                raise ZeroDivisionError("division by zero")
            flag = record.flag
            b = C.B_PERFECT_UMI if _perfect_umi(record) else 0
            cb = record.get_tag(consts.CELL_BARCODE_TAG_KEY) if record.has_tag(consts.CELL_BARCODE_TAG_KEY) else None
            if cb is not None:
                b |= C.B_HAS_CB
                if self._MODE == "cell" and record.get_tag(consts.RAW_CELL_BARCODE_TAG_KEY) == cb:
                    b |= C.B_PERFECT_CB
            xfv = record.get_tag(consts.ALIGNMENT_LOCATION_TAG_KEY) if record.has_tag(
                consts.ALIGNMENT_LOCATION_TAG_KEY) else None
            x = C.XF_ABSENT if xfv is None else C._XF_CODE.get(xfv, C.XF_OTHER)
            if flag & 0x10:
                b |= C.B_REVERSE
            if flag & 0x400:
                b |= C.B_DUPLICATE
            s = sum(aq)
            gq = (s, len(aq), sum(1 for q in aq if q > 30))
            if flag & 0x4:
                b |= C.B_UNMAPPED
            else:
                try:
                    alignment_location = record.get_tag(consts.ALIGNMENT_LOCATION_TAG_KEY)
                except KeyError:
                    self._buffer_partial(tags, record, gq, b, x, cg, cl, ug, ul)
                    raise
                if alignment_location == consts.CODING_ALIGNMENT_LOCATION_TAG_VALUE:
                    self.reads_mapped_exonic += 1
                elif alignment_location == consts.INTRONIC_ALIGNMENT_LOCATION_TAG_VALUE:
                    self.reads_mapped_intronic += 1
                elif alignment_location == consts.UTR_ALIGNMENT_LOCATION_TAG_VALUE:
                    self.reads_mapped_utr += 1
                try:
                    nh = record.get_tag(consts.NUMBER_OF_HITS_TAG_KEY)
                except KeyError:
                    self._buffer_partial(tags, record, gq, b, x, cg, cl, ug, ul)
                    raise
                if nh == 1:
                    self.reads_mapped_uniquely += 1
                    b |= C.B_NH1
                else:
                    self.reads_mapped_multiple += 1
                if flag & 0x400:
                    self.duplicate_reads += 1
                n_len = record.n_skip_length() if hasattr(record, "n_skip_length") else \
                    record.get_cigar_stats()[0][3]
                if n_len:
                    self.spliced_reads += 1
                    b |= C.B_SPLICED
                self._plus_strand_reads += not (flag & 0x10)
            if not _fits(gq, cl, ul):
                raise ValueError("record %s exceeds the 32-byte columnar limits" % getattr(record, "query_name", "?"))
            num = (record.reference_id, record.pos) + gq + (b, x, cg, cl, ug, ul)
            self._buffered.append((tuple(tags), num))

    def _buffer_partial(self, tags, record, gq, b, x, cg, cl, ug, ul) -> None:
        """A mapped read about to raise KeyError on XF or NH (aggregator.py:305 / 317): buffered as
        the reference has consumed it -- its molecule and fragment keys and its stream samples -- so
        the engine's distinct counts and streams include it; the XF / NH counters it never reached are
        the host's (_fill keeps them).  A record past the columnar limits stays out (the KeyError
        still propagates)."""
        if _fits(gq, cl, ul):
            self._buffered.append((tuple(tags), (record.reference_id, record.pos) + gq + (b, x, cg, cl, ug, ul)))

    def parse_extra_fields(self, tags: Sequence[str], record) -> None:
        """Per-record hook of the subclasses (aggregator.py:336-340)."""
        raise NotImplementedError

    def _run_engine(self, mitochondrial_genes=frozenset(), float_mode="welford"):
        from sctools_amd.metrics.single import aggregate_buffered

        if not self._buffered:
            self._fill_empty()
            return
        ints, floats = aggregate_buffered(self._MODE, self._buffered, mitochondrial_genes, float_mode)
        self._fill(ints, floats)

    def _fill_empty(self) -> None:
        """finalize() with nothing parsed (aggregator.py:350-387): Welford means 0.0 and variances NaN
        (stats.py:77-100), zero distinct counts, NaN ratios; the counters stay as they are."""
        for name, kind, _ in R.columns_for(self._MODE):
            if kind == R.I:
                if getattr(self, name) is None:
                    setattr(self, name, 0)
            elif name.endswith("_mean") or name == "pct_mitochondrial_molecules":
                setattr(self, name, 0.0)
            else:
                setattr(self, name, _NAN)

    def _fill(self, ints: np.ndarray, floats: np.ndarray) -> None:
        """Every public attribute from the engine's row, except the per-record counters the host keeps
        in the reference's order (they differ from the engine's only after a caught error)."""
        for name, kind, slot in R.columns_for(self._MODE):
            if name in _HOST_COUNTERS:
                continue
            v = ints[slot] if kind == R.I else floats[slot]
            setattr(self, name, int(v) if kind == R.I else float(v))

    def finalize(self) -> None:
        self._run_engine()


# counters parse_molecule / parse_extra_fields keep record by record (aggregator.py:259-334, 507-527)
_HOST_COUNTERS = frozenset((
    "n_reads", "noise_reads", "perfect_molecule_barcodes", "reads_mapped_exonic", "reads_mapped_intronic",
    "reads_mapped_utr", "reads_mapped_uniquely", "reads_mapped_multiple", "duplicate_reads", "spliced_reads",
    "antisense_reads", "perfect_cell_barcodes", "reads_mapped_intergenic", "reads_unmapped",
    "reads_mapped_too_many_loci"))


def _fits(gq, cl, ul) -> bool:
    """The 32-byte record's field widths (uint16 genomic quality sums, uint8 barcode lengths)."""
    return gq[1] <= 0xFFFF and gq[0] <= 0xFFFF and cl <= 0xFF and ul <= 0xFF


def _perfect_umi(record) -> bool:
    try:
        return record.get_tag(consts.RAW_MOLECULE_BARCODE_TAG_KEY) == record.get_tag(consts.MOLECULE_BARCODE_TAG_KEY)
    except KeyError:
        return False


class CellMetrics(MetricAggregator):
    _MODE = "cell"

    def __init__(self):
        super().__init__()
        # aggregator.py:441-461
        self._cell_barcode_fraction_bases_above_30 = None
        self.perfect_cell_barcodes = 0
        self.reads_mapped_intergenic = 0
        self.reads_unmapped = 0
        self.reads_mapped_too_many_loci = 0
        self._genes_histogram = None
        self.cell_barcode_fraction_bases_above_30_variance: float = None
        self.cell_barcode_fraction_bases_above_30_mean: float = None
        self.n_genes: int = None
        self.genes_detected_multiple_observations: int = None
        self.n_mitochondrial_genes: int = None
        self.n_mitochondrial_molecules: int = None
        self.pct_mitochondrial_molecules: float = None

    def parse_extra_fields(self, tags: Sequence[str], record) -> None:
        """aggregator.py:507-530: CY first, then CB / CR, then XF."""
        self._extra = C._frac_counts(record.get_tag(consts.QUALITY_CELL_BARCODE_TAG_KEY))
        if record.has_tag(consts.CELL_BARCODE_TAG_KEY):
            raw_cell_barcode_tag = record.get_tag(consts.RAW_CELL_BARCODE_TAG_KEY)
            self.perfect_cell_barcodes += raw_cell_barcode_tag == record.get_tag(consts.CELL_BARCODE_TAG_KEY)
        try:
            if record.get_tag(consts.ALIGNMENT_LOCATION_TAG_KEY) == consts.INTERGENIC_ALIGNMENT_LOCATION_TAG_VALUE:
                self.reads_mapped_intergenic += 1
        except KeyError:
            self.reads_unmapped += 1

    def finalize(self, mitochondrial_genes=set()):
        self._run_engine(mitochondrial_genes=mitochondrial_genes)


class GeneMetrics(MetricAggregator):
    _MODE = "gene"

    def __init__(self):
        super().__init__()
        # aggregator.py:564-569
        self._cells_histogram = None
        self.number_cells_detected_multiple: int = None
        self.number_cells_expressing: int = None

    def parse_extra_fields(self, tags: Sequence[str], record) -> None:
        """aggregator.py:595: the cell tag feeds the distinct cell count at finalize()."""
        return None

    def finalize(self):
        self._run_engine()


# sanity: the public attribute order must be the writer's column order
assert [k for k in vars(CellMetrics()) if not k.startswith("_")] == [c for c, _, _ in R.CELL_COLUMNS]
assert [k for k in vars(GeneMetrics()) if not k.startswith("_")] == [c for c, _, _ in R.GENE_COLUMNS]
_ = N  # layout constants live in _native
