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

A record that raises part-way (rounds 5-6): the reference has by then fed
it to some of its state, in its own order (aggregator.py:257-334, 507-530):

* CR missing under a CB (cell, 518): its CY sample only (507-514);
* UY missing or empty (270): the subclass fields (CY sample, the gene / cell histogram), n_reads and
  the molecule histogram (259-264);
* no or empty base qualities (288): those and the UY sample (266-273);
* a mapped read without XF or NH (305 / 317): all of it up to and including the fragment
  histogram (303) and both genomic streams (287-292).

Each buffered record carries the set of the reference's states it fed ("fed" bits).  ``finalize()``
takes the distinct counts and ratios from an engine run over the records that reached n_reads (a
record that stopped before its fragment histogram marked unmapped there, so it adds a molecule but
no fragment), and each Welford stream from an engine run over exactly the records that fed that
stream, in file order; the host's integer counters stopped exactly where the reference's stopped.
A caller that catches the error and calls ``finalize()`` -- at once, or after parsing more records
-- gets the reference's values (tests/golden/protocol: ``final_after_error``, ``final_continued``).
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
        self._buffered = []  # (tags, numeric fields, fed bits) per parsed record
        self._extra = (0, 0)  # the subclass's CY counts of the record being parsed

    # ---- aggregator protocol (aggregator.py:236-340) ----
    def parse_molecule(self, tags: Sequence[str], records) -> None:
        """aggregator.py:251-334, record by record: the subclass fields first, then the counters,
        raising where the reference raises.

        A record that raises part-way is buffered with the states the reference fed before the
        exception propagates (see the module docstring)."""
        for record in records:
            self._extra = None
            try:
                self.parse_extra_fields(tags=tags, record=record)
            except Exception:
                if self._extra is not None:  # cell: the CY sample was taken, CR raised (518)
                    self._buffer(tags, record, FED_CY, cy=self._extra)
                raise
            cy = self._extra if self._extra is not None else (0, 0)
            fed = FED_CORE | FED_CY
            self.n_reads += 1
            try:
                uy = C._frac_counts(record.get_tag(consts.QUALITY_MOLECULE_BARCODE_TAG_KEY))
            except (KeyError, ZeroDivisionError):  # after the molecule histogram (264-270)
                self._buffer(tags, record, fed, cy=cy)
                raise
            fed |= FED_UY
            try:
                self.perfect_molecule_barcodes += record.get_tag(
                    consts.RAW_MOLECULE_BARCODE_TAG_KEY) == record.get_tag(consts.MOLECULE_BARCODE_TAG_KEY)
            except KeyError:
                pass
            aq = record.query_alignment_qualities
            if aq is None or len(aq) == 0:  # _quality_above_threshold (288): after the UY sample
                self._buffer(tags, record, fed, cy=cy, uy=uy)
                if aq is None:
                    raise TypeError("'NoneType' object is not iterable")
                raise ZeroDivisionError("division by zero")
            fed |= FED_GQ
            flag = record.flag
            s = sum(aq)
            gq = (s, len(aq), sum(1 for q in aq if q > 30))
            if not flag & 0x4:
                fed |= FED_FRAG  # the fragment histogram (303) precedes the XF / NH reads
                try:
                    alignment_location = record.get_tag(consts.ALIGNMENT_LOCATION_TAG_KEY)
                except KeyError:
                    self._buffer(tags, record, fed, cy=cy, uy=uy, gq=gq)
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
                    self._buffer(tags, record, fed, cy=cy, uy=uy, gq=gq)
                    raise
                if nh == 1:
                    self.reads_mapped_uniquely += 1
                else:
                    self.reads_mapped_multiple += 1
                if flag & 0x400:
                    self.duplicate_reads += 1
                n_len = record.n_skip_length() if hasattr(record, "n_skip_length") else \
                    record.get_cigar_stats()[0][3]
                if n_len:
                    self.spliced_reads += 1
                self._plus_strand_reads += not (flag & 0x10)
            else:
                nh = n_len = None
            num = self._fields(record, cy, uy, gq, nh, n_len)
            if num is None:
                raise ValueError("record %s exceeds the 32-byte columnar limits" % getattr(record, "query_name", "?"))
            self._buffered.append((tuple(tags), num, FED_ALL))

    def _fields(self, record, cy, uy, gq, nh=None, n_len=None):
        """The record's 32-byte numeric fields (columnar.record_fields' layout); a stream the record
        never reached gets a neutral stand-in sample (a = 0, b = 1: its run never reports that stream).
        None if a field exceeds its column width."""
        cy = cy if cy is not None else (0, 1)
        uy = uy if uy is not None else (0, 1)
        gq = gq if gq is not None else (0, 1, 0)
        if not _fits(gq, cy[1], uy[1]):
            return None
        flag = record.flag
        b = C.B_PERFECT_UMI if _perfect_umi(record) else 0
        cb = record.get_tag(consts.CELL_BARCODE_TAG_KEY) if record.has_tag(consts.CELL_BARCODE_TAG_KEY) else None
        if cb is not None:
            b |= C.B_HAS_CB
            if self._MODE == "cell" and record.has_tag(consts.RAW_CELL_BARCODE_TAG_KEY) and \
                    record.get_tag(consts.RAW_CELL_BARCODE_TAG_KEY) == cb:
                b |= C.B_PERFECT_CB
        xfv = record.get_tag(consts.ALIGNMENT_LOCATION_TAG_KEY) if record.has_tag(
            consts.ALIGNMENT_LOCATION_TAG_KEY) else None
        x = C.XF_ABSENT if xfv is None else C._XF_CODE.get(xfv, C.XF_OTHER)
        if flag & 0x10:
            b |= C.B_REVERSE
        if flag & 0x400:
            b |= C.B_DUPLICATE
        if flag & 0x4:
            b |= C.B_UNMAPPED
        if nh == 1:
            b |= C.B_NH1
        if n_len:
            b |= C.B_SPLICED
        return (record.reference_id, record.pos) + tuple(gq) + (b, x, cy[0], cy[1], uy[0], uy[1])

    def _buffer(self, tags, record, fed, cy=None, uy=None, gq=None) -> None:
        """A record about to raise, buffered with the states it fed (``fed`` bits).  A record past
        the columnar limits stays out (the exception still propagates)."""
        num = self._fields(record, cy, uy, gq)
        if num is not None:
            self._buffered.append((tuple(tags), num, fed))

    def parse_extra_fields(self, tags: Sequence[str], record) -> None:
        """Per-record hook of the subclasses (aggregator.py:336-340)."""
        raise NotImplementedError

    def _run_engine(self, mitochondrial_genes=frozenset(), float_mode="welford"):
        from sctools_amd.metrics.single import aggregate_buffered

        buf = self._buffered
        core = [i for i, (_, _, f) in enumerate(buf) if f & FED_CORE]

        def run(idx, core_run):
            items = []
            for i in idx:
                tags, num, f = buf[i]
                if core_run and not f & FED_FRAG and not num[5] & C.B_UNMAPPED:
                    # stopped before its fragment histogram (303): a molecule, but no fragment
                    num = num[:5] + (num[5] | C.B_UNMAPPED,) + num[6:]
                items.append((tags, num))
            return aggregate_buffered(self._MODE, items, mitochondrial_genes, float_mode)

        if core:
            self._fill(*run(core, True))
        else:
            self._fill_empty()
        # every Welford stream over exactly the records that fed it (file order)
        for bit, names in _STREAMS[self._MODE]:
            idx = [i for i, (_, _, f) in enumerate(buf) if f & bit]
            if idx == core and core:
                continue
            if not idx:
                vals = {n: (0.0 if n.endswith("_mean") else _NAN) for n in names}
            else:
                _, floats = run(idx, False)
                vals = {n: float(floats[slot]) for n, kind, slot in R.columns_for(self._MODE) if n in names}
            for n in names:
                setattr(self, n, vals[n])

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


# the reference states a buffered record may have fed before raising (parse_molecule)
FED_CORE = 1   # n_reads, the molecule histogram, the subclass histogram (aggregator.py:259-264, 530, 595)
FED_UY = 2     # the UY Welford sample (266-273)
FED_GQ = 4     # both genomic Welford samples (287-292)
FED_CY = 8     # the CY Welford sample (cell, 507-514)
FED_FRAG = 16  # the fragment histogram (303)
FED_ALL = 31

# the Welford streams of each mode: (fed bit, mean / variance attribute names)
_STREAMS = {
    "cell": ((FED_UY, ("molecule_barcode_fraction_bases_above_30_mean",
                       "molecule_barcode_fraction_bases_above_30_variance")),
             (FED_GQ, ("genomic_reads_fraction_bases_quality_above_30_mean",
                       "genomic_reads_fraction_bases_quality_above_30_variance",
                       "genomic_read_quality_mean", "genomic_read_quality_variance")),
             (FED_CY, ("cell_barcode_fraction_bases_above_30_variance",
                       "cell_barcode_fraction_bases_above_30_mean"))),
    "gene": ((FED_UY, ("molecule_barcode_fraction_bases_above_30_mean",
                       "molecule_barcode_fraction_bases_above_30_variance")),
             (FED_GQ, ("genomic_reads_fraction_bases_quality_above_30_mean",
                       "genomic_reads_fraction_bases_quality_above_30_variance",
                       "genomic_read_quality_mean", "genomic_read_quality_variance"))),
}

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
