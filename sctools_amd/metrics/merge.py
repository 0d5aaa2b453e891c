"""
Host-side merges of per-chunk metric CSVs -- same interface and semantics as
the reference's ``sctools.metrics.merge`` (``/root/reference/src/sctools/metrics/merge.py:31-191``):

* ``MergeCellMetrics``: chunks hold disjoint cells, so rows are concatenated.
* ``MergeGeneMetrics``: rows of the same gene are combined: 17 count columns
  summed, the 6 mean / variance columns averaged weighted by ``n_reads``, and
  ``reads_per_molecule``, ``fragments_per_molecule``, ``reads_per_fragment``
  recomputed; files are folded in pairwise order like the reference.

Output is always ``<stem>.csv.gz`` written by pandas.  These keep CLI
compatibility for scattered workflows; the multi-GPU path replaces the gene
merge with an exact RCCL all-reduce of per-gene partials (sctools_amd.distributed).
"""

from typing import List, Sequence

import numpy as np
import pandas as pd

_SUM_COLUMNS = [
    "n_reads", "noise_reads", "perfect_molecule_barcodes", "reads_mapped_exonic", "reads_mapped_intronic",
    "reads_mapped_utr", "reads_mapped_uniquely", "reads_mapped_multiple", "duplicate_reads", "spliced_reads",
    "antisense_reads", "n_molecules", "n_fragments", "fragments_with_single_read_evidence",
    "molecules_with_single_read_evidence", "number_cells_detected_multiple", "number_cells_expressing",
]
_AVERAGE_COLUMNS = [
    "molecule_barcode_fraction_bases_above_30_mean", "molecule_barcode_fraction_bases_above_30_variance",
    "genomic_reads_fraction_bases_quality_above_30_mean", "genomic_reads_fraction_bases_quality_above_30_variance",
    "genomic_read_quality_mean", "genomic_read_quality_variance",
]


class MergeMetrics:
    def __init__(self, metric_files: Sequence[str], output_file: str):
        self._metric_files = metric_files
        if not output_file.endswith(".csv.gz"):
            output_file += ".csv.gz"
        self._output_file = output_file

    def execute(self) -> None:
        raise NotImplementedError


class MergeCellMetrics(MergeMetrics):
    def execute(self) -> None:
        frames: List[pd.DataFrame] = [pd.read_csv(f, index_col=0) for f in self._metric_files]
        pd.concat(frames, axis=0).to_csv(self._output_file, compression="gzip")


class MergeGeneMetrics(MergeMetrics):
    @staticmethod
    def _merge_pair(nucleus: pd.DataFrame, leaf: pd.DataFrame) -> pd.DataFrame:
        both = pd.concat([nucleus, leaf], axis=0)
        # the gatherer writes a ``None`` row for reads without GE; read_csv makes its index NaN
        # and the reference's groupby(level=0) drops such rows (merge.py:176, dropna default)
        both = both[both.index.notna()]
        if both.shape[0] == 0:
            raise ValueError("no gene rows left to merge: every row has a missing (None) gene index")
        grouped = both.groupby(level=0)
        summed = grouped.agg({c: "sum" for c in _SUM_COLUMNS})
        weights = both["n_reads"].to_numpy(dtype=np.float64)
        averaged = {}
        codes = grouped.ngroup().to_numpy()
        n_groups = summed.shape[0]
        wsum = np.bincount(codes, weights=weights, minlength=n_groups)
        if (wsum == 0).any():  # np.average raises on zero weights (merge.py:108-138)
            raise ZeroDivisionError("Weights sum to zero, can't be normalized")
        for c in _AVERAGE_COLUMNS:
            vals = both[c].to_numpy(dtype=np.float64)
            # np.average(x, weights=n_reads) per group; NaN propagates like the reference
            averaged[c] = np.bincount(codes, weights=vals * weights, minlength=n_groups) / wsum
        averaged = pd.DataFrame(averaged, index=summed.index)
        merged = pd.concat([summed, averaged], axis=1)
        recalculated = pd.DataFrame({
            "reads_per_molecule": merged["n_reads"] / merged["n_molecules"],
            "fragments_per_molecule": merged["n_fragments"] / merged["n_molecules"],
            "reads_per_fragment": merged["n_reads"] / merged["n_fragments"],
        })
        return pd.concat([merged, recalculated], axis=1)

    def execute(self) -> None:
        nucleus = pd.read_csv(self._metric_files[0], index_col=0)
        for filename in self._metric_files[1:]:
            nucleus = self._merge_pair(nucleus, pd.read_csv(filename, index_col=0))
        nucleus.to_csv(self._output_file, compression="gzip")
