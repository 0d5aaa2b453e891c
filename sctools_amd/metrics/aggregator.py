"""
Metric aggregators -- same classes, attribute names and attribute order as the
reference (``/root/reference/src/sctools/metrics/aggregator.py``:
``MetricAggregator`` 46-387, ``CellMetrics`` 390-530, ``GeneMetrics``
533-595), so ``vars(CellMetrics())`` yields the reference CSV header and
existing callers of the aggregator protocol keep working.

The arithmetic does not live here.  ``parse_molecule`` buffers the records of
the entity; ``finalize`` columnarizes them and runs the single entity through
the HIP engine (one launch sequence per entity -- the gatherers batch every
entity of a file into one launch sequence instead).  The public attributes
are then filled from the engine's output row.
"""

from typing import Sequence

import numpy as np

from sctools_amd import _native as N
from sctools_amd.metrics import rows as R


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
        self._buffered = []

    # ---- aggregator protocol (aggregator.py:236-340) ----
    def parse_molecule(self, tags: Sequence[str], records) -> None:
        for record in records:
            self.parse_extra_fields(tags=tags, record=record)
            self._buffered.append((tuple(tags), record))

    def parse_extra_fields(self, tags: Sequence[str], record) -> None:
        """Per-record hook; the engine computes the subclass fields at finalize()."""
        return None

    def _run_engine(self, mitochondrial_genes=frozenset(), float_mode="welford"):
        from sctools_amd.metrics.single import aggregate_buffered

        ints, floats = aggregate_buffered(self._MODE, self._buffered, mitochondrial_genes, float_mode)
        self._fill(ints, floats)

    def _fill(self, ints: np.ndarray, floats: np.ndarray) -> None:
        for name, kind, slot in R.columns_for(self._MODE):
            v = ints[slot] if kind == R.I else floats[slot]
            setattr(self, name, int(v) if kind == R.I else float(v))

    def finalize(self) -> None:
        self._run_engine()


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

    def finalize(self):
        self._run_engine()


# sanity: the public attribute order must be the writer's column order
assert [k for k in vars(CellMetrics()) if not k.startswith("_")] == [c for c, _, _ in R.CELL_COLUMNS]
assert [k for k in vars(GeneMetrics()) if not k.startswith("_")] == [c for c, _, _ in R.GENE_COLUMNS]
_ = N  # layout constants live in _native
