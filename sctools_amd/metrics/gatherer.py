"""
Metric gatherers -- drop-in for the reference's ``sctools.metrics.gatherer``
(``/root/reference/src/sctools/metrics/gatherer.py:38-232``).

Same classes, constructor signature and ``extract_metrics(mode)`` behaviour:
read a BAM ('rb') or SAM ('r'), aggregate per cell-barcode run
(``GatherCellMetrics``) or per gene run (``GatherGeneMetrics``, multi-gene
runs skipped), write ``output_stem.csv.gz`` (or ``.csv``) with the reference's
header and row format.

The per-record aggregation runs on the GPU (``sctools_amd.engine``): a BAM is
inflated and parsed into columns on the same GPU (``sctools_amd.gbam``; a file
it declines -- one the reference rejects -- is decoded on the host by
``sctools_amd.columnar``, raising the same exception types the reference
raises), and the HIP engine computes every row in one launch sequence.
``float_mode='welford'`` (default) reproduces the reference's sequential Welford floats bit for bit; ``'exact'`` computes
correctly rounded mean / variance from exact sums (order independent,
within 1e-12 of Welford).

``devices=N`` (optional) spreads the entity runs over N GPUs, one host thread each
(``sctools_amd.multigpu``): same rows, same order.  ``GatherCellAndGeneMetrics`` (new) writes
the cell rows of a cell-sorted file and, from the same pass, its gene rows as TagSortBam by
(GE, CB, UB) + ``GatherGeneMetrics`` would give them -- the SplitBam + per-chunk metrics +
``MergeGeneMetrics`` workflow in one call, the gene partials of the devices' cell ranges summed
by an RCCL all-reduce.
"""

from typing import Optional, Set

import numpy as np

from sctools_amd import columnar
from sctools_amd import _native as N
from sctools_amd.metrics import rows as R
from sctools_amd.metrics.aggregator import CellMetrics, GeneMetrics
from sctools_amd.metrics.writer import MetricCSVWriter


def compute_rows(cols: columnar.Columns, mode: str, mitochondrial_gene_ids=frozenset(),
                 float_mode: str = "welford", device=None, devices=None):
    """Run the engine on host columns; returns (ints, floats) numpy rows of every entity run."""
    import torch

    from sctools_amd import engine as E

    if devices is not None:
        from sctools_amd import multigpu

        return multigpu.compute_rows(cols, mode, mitochondrial_gene_ids, float_mode, devices)

    eng = E.get_engine(device)
    if cols.on_device:
        dev_cols = cols.arrays
    else:
        dev_cols = E.to_device(cols.arrays, eng.device)
    mito, multi = cols.gene_flags(mitochondrial_gene_ids)
    dims = E.Dims(len(cols.cells), len(cols.genes), len(cols.umis))
    gm = torch.from_numpy(mito).to(eng.device)
    gx = torch.from_numpy(multi).to(eng.device)
    ints, floats = eng.compute(dev_cols, mode, dims, gm, gx, float_mode=float_mode)
    return ints.cpu().numpy(), floats.cpu().numpy()


def write_rows(writer: MetricCSVWriter, mode: str, cols: columnar.Columns, ints: np.ndarray,
               floats: np.ndarray) -> None:
    ids = cols.column_at("cell" if mode == "cell" else "gene", ints[:, N.I_ENTITY])
    names_of = cols.cells.names if mode == "cell" else cols.genes.names
    names = [names_of[i] for i in ids.tolist()]
    keep, kept = R.select_rows(mode, ints, names)
    writer.write_bytes(R.format_rows_bytes(mode, kept, ints[keep], floats[keep]))


class MetricGatherer:
    """Gathers metrics from an experiment (``gatherer.py:38-86``)."""

    def __init__(self, bam_file: str, output_stem: str, mitochondrial_gene_ids: Set[str] = set(),
                 compress: bool = True, float_mode: str = "welford", device: Optional[str] = None,
                 devices=None, gpu_decode: bool = True):
        self._bam_file = bam_file
        self._output_stem = output_stem
        self._compress = compress
        self._mitochondrial_gene_ids = mitochondrial_gene_ids
        self._float_mode = float_mode
        self._device = device
        self._devices = devices  # None: one device (`device`); int N or device list: multigpu
        self._gpu_decode = gpu_decode  # inflate and parse a BAM on the (first) device (gbam)

    def _columns(self, mode: str, metric_mode: str) -> columnar.Columns:
        """The file's columns: a BAM is decoded on the GPU that computes the metrics (the first of
        several devices); a file the device decoder declines, and SAM text, go through the host
        decoder, which raises the reference's exception."""
        if self._gpu_decode and mode == "rb":
            from sctools_amd import engine as E
            from sctools_amd import gbam

            if gbam.available():
                if self._devices is None:
                    dev = E.get_engine(self._device).device
                    return columnar.columnarize(self.bam_file, mode, metric_mode, device=dev)
                # several devices: each decodes its part of the file (no device holds it all), the
                # parts re-cut at entity runs; a file the device path declines: the host decoder
                import torch

                from sctools_amd import multigpu

                devs = [torch.device("cuda", d) for d in multigpu.parse_devices(self._devices)]
                key = "cell" if metric_mode == columnar.MODE_CELL else "gene"
                got = columnar.columnarize_parts(self.bam_file, metric_mode, devs, key)
                if got is not None:
                    return got
        return columnar.columnarize(self.bam_file, mode, metric_mode)

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
            cols = self._columns(mode, columnar.MODE_CELL)
            ints, floats = compute_rows(cols, "cell", self._mitochondrial_gene_ids, self._float_mode,
                                        self._device, self._devices)
            write_rows(out, "cell", cols, ints, floats)


class GatherGeneMetrics(MetricGatherer):
    """Per-gene metrics of a gene-sorted BAM (``gatherer.py:162-232``); multi-gene runs skipped."""

    def extract_metrics(self, mode: str = "rb") -> None:
        with MetricCSVWriter(self._output_stem, self._compress) as out:
            out.write_header(vars(GeneMetrics()))
            cols = self._columns(mode, columnar.MODE_GENE)
            ints, floats = compute_rows(cols, "gene", frozenset(), self._float_mode, self._device,
                                        self._devices)
            write_rows(out, "gene", cols, ints, floats)


def write_rows_of_ids(writer: MetricCSVWriter, mode: str, cols: columnar.Columns, ints: np.ndarray,
                      floats: np.ndarray, ids: np.ndarray) -> None:
    """Rows whose entity ids are given (records re-sorted on the device: no file position to look up)."""
    names_of = cols.cells.names if mode == "cell" else cols.genes.names
    names = [names_of[i] for i in ids.tolist()]
    keep, kept = R.select_rows(mode, ints, names)
    writer.write_bytes(R.format_rows_bytes(mode, kept, ints[keep], floats[keep]))


def query_name_ranks(bam_file: str, mode: str):
    """(rank of each record's query name among the file's sorted names, number of names): the last
    field of TagSortBam's order (bam.py:638-709), decoded on the host (bamdec.cpp sort-key mode).
    SAM input: (None, 0) -- ties then keep input order."""
    if mode != "rb":
        return None, 0
    from sctools_amd import bamnative

    arrays, names = bamnative.decode(bam_file, "sortkeys")
    return arrays["qname"], max(1, len(names[3]))


def write_grouped_gene_rows(writer: MetricCSVWriter, cols: columnar.Columns, ints: np.ndarray,
                            floats: np.ndarray) -> None:
    """Gene rows indexed by gene id: ids with reads, multi-gene values skipped, in id order (the
    sorted order of the gene strings, None first -- TagSortBam's order, bam.py:698-709)."""
    names = [cols.genes.names[g] for g in ints[:, N.I_ENTITY]]
    keep, kept = R.select_rows("gene_grouped", ints, names)
    writer.write_bytes(R.format_rows_bytes("gene", kept, ints[keep], floats[keep]))


class GatherCellAndGeneMetrics(MetricGatherer):
    """Cell rows AND gene rows of one cell-sorted BAM, from one decode and one device pass.

    Cell rows: as ``GatherCellMetrics``.  Gene rows: every record of a gene id aggregated
    together, as ``GatherGeneMetrics`` reports them for the same records re-sorted by
    (GE, CB, UB) (TagSortBam), with exact-sum floats (within 1e-12 of Welford); it replaces
    SplitBam + per-chunk ``CalculateGeneMetrics`` + ``MergeGeneMetrics`` (merge.py:74-191) with
    an exact RCCL all-reduce of per-gene partials when ``devices`` > 1.
    """

    def __init__(self, bam_file: str, output_stem: str, gene_output_stem: str,
                 mitochondrial_gene_ids: Set[str] = set(), compress: bool = True, float_mode: str = "welford",
                 devices=1):
        super().__init__(bam_file, output_stem, mitochondrial_gene_ids, compress, float_mode, None, devices)
        self._gene_output_stem = gene_output_stem

    def extract_metrics(self, mode: str = "rb") -> None:
        from sctools_amd import multigpu

        cols = self._columns(mode, columnar.MODE_CELL)
        if multigpu.cells_twice(cols):
            # not cell-sorted: the rows of TagSortBam by (CB, UB, GE, query name) + GatherCellMetrics
            # (and by (GE, CB, UB) + GatherGeneMetrics), the cell bins swapped between the devices
            tie, n_tie = (None, 0) if self._float_mode == "exact" else query_name_ranks(self.bam_file, mode)
            (ci, cf, ids), (gi, gf) = multigpu.sorted_cell_and_gene_rows(
                cols, self._mitochondrial_gene_ids, self._float_mode, self._devices, tie, n_tie)
            with MetricCSVWriter(self._output_stem, self._compress) as out:
                out.write_header(vars(CellMetrics()))
                write_rows_of_ids(out, "cell", cols, ci, cf, ids)
        else:
            (ci, cf), (gi, gf) = multigpu.compute_cell_and_gene_rows(cols, self._mitochondrial_gene_ids,
                                                                     self._float_mode, self._devices)
            with MetricCSVWriter(self._output_stem, self._compress) as out:
                out.write_header(vars(CellMetrics()))
                write_rows(out, "cell", cols, ci, cf)
        with MetricCSVWriter(self._gene_output_stem, self._compress) as out:
            out.write_header(vars(GeneMetrics()))
            write_grouped_gene_rows(out, cols, gi, gf)
