"""
Metric gatherers -- drop-in for the reference's ``sctools.metrics.gatherer``
(``/root/reference/src/sctools/metrics/gatherer.py:38-232``).

Same classes, constructor signature and ``extract_metrics(mode)`` behaviour:
read a BAM ('rb') or SAM ('r'), aggregate per cell-barcode run
(``GatherCellMetrics``) or per gene run (``GatherGeneMetrics``, multi-gene
runs skipped), write ``output_stem.csv.gz`` (or ``.csv``) with the reference's
header and row format.

The per-record aggregation runs on the GPU (``sctools_amd.engine``): the host
decodes the file into columns (``sctools_amd.columnar``), raising the same
exception types the reference raises, and the HIP engine computes every row
in one launch sequence.  ``float_mode='welford'`` (default) reproduces the
reference's sequential Welford floats bit for bit; ``'exact'`` computes
correctly rounded mean / variance from exact sums (order independent,
within 1e-12 of Welford).
"""

from typing import Optional, Set

import numpy as np

from sctools_amd import columnar
from sctools_amd import _native as N
from sctools_amd.metrics import rows as R
from sctools_amd.metrics.aggregator import CellMetrics, GeneMetrics
from sctools_amd.metrics.writer import MetricCSVWriter


def compute_rows(cols: columnar.Columns, mode: str, mitochondrial_gene_ids=frozenset(),
                 float_mode: str = "welford", device=None):
    """Run the engine on host columns; returns (ints, floats) numpy rows of every entity run."""
    import torch

    from sctools_amd import engine as E

    eng = E.get_engine(device)
    dev_cols = E.to_device(cols.arrays, eng.device)
    mito, multi = cols.gene_flags(mitochondrial_gene_ids)
    dims = E.Dims(len(cols.cells), len(cols.genes), len(cols.umis))
    gm = torch.from_numpy(mito).to(eng.device)
    gx = torch.from_numpy(multi).to(eng.device)
    ints, floats = eng.compute(dev_cols, mode, dims, gm, gx, float_mode=float_mode)
    return ints.cpu().numpy(), floats.cpu().numpy()


def write_rows(writer: MetricCSVWriter, mode: str, cols: columnar.Columns, ints: np.ndarray,
               floats: np.ndarray) -> None:
    key = cols.arrays["cell" if mode == "cell" else "gene"]
    names_of = cols.cells.names if mode == "cell" else cols.genes.names
    names = [names_of[key[i]] for i in ints[:, N.I_ENTITY]]
    keep, kept = R.select_rows(mode, ints, names)
    writer.write_bytes(R.format_rows_bytes(mode, kept, ints[keep], floats[keep]))


class MetricGatherer:
    """Gathers metrics from an experiment (``gatherer.py:38-86``)."""

    def __init__(self, bam_file: str, output_stem: str, mitochondrial_gene_ids: Set[str] = set(),
                 compress: bool = True, float_mode: str = "welford", device: Optional[str] = None):
        self._bam_file = bam_file
        self._output_stem = output_stem
        self._compress = compress
        self._mitochondrial_gene_ids = mitochondrial_gene_ids
        self._float_mode = float_mode
        self._device = device

    @property
    def bam_file(self) -> str:
        """the bam file that metrics are generated from"""
        return self._bam_file

    def extract_metrics(self, mode: str = "rb") -> None:
        raise NotImplementedError


class GatherCellMetrics(MetricGatherer):
    """Per-cell metrics of a cell-sorted BAM (``gatherer.py:89-159``)."""

    def extract_metrics(self, mode: str = "rb") -> None:
        with MetricCSVWriter(self._output_stem, self._compress) as out:
            out.write_header(vars(CellMetrics()))
            cols = columnar.columnarize(self.bam_file, mode, columnar.MODE_CELL)
            ints, floats = compute_rows(cols, "cell", self._mitochondrial_gene_ids, self._float_mode,
                                        self._device)
            write_rows(out, "cell", cols, ints, floats)


class GatherGeneMetrics(MetricGatherer):
    """Per-gene metrics of a gene-sorted BAM (``gatherer.py:162-232``); multi-gene runs skipped."""

    def extract_metrics(self, mode: str = "rb") -> None:
        with MetricCSVWriter(self._output_stem, self._compress) as out:
            out.write_header(vars(GeneMetrics()))
            cols = columnar.columnarize(self.bam_file, mode, columnar.MODE_GENE)
            ints, floats = compute_rows(cols, "gene", frozenset(), self._float_mode, self._device)
            write_rows(out, "gene", cols, ints, floats)
