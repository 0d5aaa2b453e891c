"""
Output column layout and CSV row text.

The header of a metric CSV is ``vars(aggregator)`` minus private keys, in
attribute-assignment order (``MetricCSVWriter.write_header``,
``/root/reference/src/sctools/metrics/writer.py:71-82``; attribute order from
``MetricAggregator.__init__`` aggregator.py:132-189, ``CellMetrics.__init__``
437-461, ``GeneMetrics.__init__`` 561-569).  Values are written with ``str``
(``writer.py:96``), i.e. Python ``repr`` for floats, and a ``None`` entity is
written as ``None`` (``writer.py:99-103``).

Each column maps to one slot of the engine's output rows (int64 ``ints`` or
float64 ``floats``, see ``include/sctools_gpu.h``).
"""

from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np

from sctools_amd import _native as N

I, F = "i", "f"

COMMON_COLUMNS: List[Tuple[str, str, int]] = [
    ("n_reads", I, N.I_N_READS),
    ("noise_reads", I, N.I_NOISE_READS),
    ("perfect_molecule_barcodes", I, N.I_PERFECT_UMI),
    ("reads_mapped_exonic", I, N.I_EXONIC),
    ("reads_mapped_intronic", I, N.I_INTRONIC),
    ("reads_mapped_utr", I, N.I_UTR),
    ("reads_mapped_uniquely", I, N.I_UNIQUE),
    ("reads_mapped_multiple", I, N.I_MULTIPLE),
    ("duplicate_reads", I, N.I_DUP),
    ("spliced_reads", I, N.I_SPLICED),
    ("antisense_reads", I, N.I_ANTISENSE),
    ("molecule_barcode_fraction_bases_above_30_mean", F, N.F_UY_MEAN),
    ("molecule_barcode_fraction_bases_above_30_variance", F, N.F_UY_VAR),
    ("genomic_reads_fraction_bases_quality_above_30_mean", F, N.F_GQF_MEAN),
    ("genomic_reads_fraction_bases_quality_above_30_variance", F, N.F_GQF_VAR),
    ("genomic_read_quality_mean", F, N.F_GQ_MEAN),
    ("genomic_read_quality_variance", F, N.F_GQ_VAR),
    ("n_molecules", I, N.I_N_MOL),
    ("n_fragments", I, N.I_N_FRAG),
    ("reads_per_molecule", F, N.F_RPM),
    ("reads_per_fragment", F, N.F_RPF),
    ("fragments_per_molecule", F, N.F_FPM),
    ("fragments_with_single_read_evidence", I, N.I_FRAG_SINGLE),
    ("molecules_with_single_read_evidence", I, N.I_MOL_SINGLE),
]

CELL_COLUMNS = COMMON_COLUMNS + [
    ("perfect_cell_barcodes", I, N.I_PERFECT_CB),
    ("reads_mapped_intergenic", I, N.I_INTERGENIC),
    ("reads_unmapped", I, N.I_UNMAPPED),
    ("reads_mapped_too_many_loci", I, N.I_TOO_MANY_LOCI),
    ("cell_barcode_fraction_bases_above_30_variance", F, N.F_CY_VAR),
    ("cell_barcode_fraction_bases_above_30_mean", F, N.F_CY_MEAN),
    ("n_genes", I, N.I_N_K1),
    ("genes_detected_multiple_observations", I, N.I_K1_MULTI),
    ("n_mitochondrial_genes", I, N.I_MITO_GENES),
    ("n_mitochondrial_molecules", I, N.I_MITO_READS),
    ("pct_mitochondrial_molecules", F, N.F_PCT_MITO),
]

GENE_COLUMNS = COMMON_COLUMNS + [
    ("number_cells_detected_multiple", I, N.I_K1_MULTI),
    ("number_cells_expressing", I, N.I_N_K1),
]


def columns_for(mode: str):
    return CELL_COLUMNS if mode == "cell" else GENE_COLUMNS


def header_line(mode: str) -> str:
    return "," + ",".join(name for name, _, _ in columns_for(mode)) + "\n"


def entity_name(value) -> str:
    # MetricCSVWriter.write: str index, or repr(None) -> 'None' (writer.py:99-103)
    return "None" if value is None else str(value)


def format_rows(mode: str, names: Sequence, ints: np.ndarray, floats: np.ndarray) -> Iterable[str]:
    """CSV lines (with trailing newline) for rows ``ints``/``floats`` named ``names``."""
    cols = columns_for(mode)
    per_col = []
    for _, kind, slot in cols:
        src = ints[:, slot] if kind == I else floats[:, slot]
        per_col.append(src.tolist())  # Python int / float: str() == reference text
    for r, name in enumerate(names):
        yield entity_name(name) + "," + ",".join([str(c[r]) for c in per_col]) + "\n"


def format_rows_bytes(mode: str, names: Sequence, ints: np.ndarray, floats: np.ndarray) -> bytes:
    """All CSV lines as UTF-8 bytes: the native formatter (libsct_csv.so, all cores, the same text
    as format_rows) when it is built, else format_rows."""
    from sctools_amd import csvnative

    if not csvnative.available():
        return "".join(format_rows(mode, names, ints, floats)).encode("utf-8")
    cols = columns_for(mode)
    kinds = [csvnative.INT if kind == I else csvnative.FLOAT for _, kind, _ in cols]
    slots = [slot for _, _, slot in cols]
    return csvnative.format_rows([entity_name(n) for n in names], kinds, slots, ints, floats)


def select_rows(mode: str, ints: np.ndarray, entity_names: Sequence[Optional[str]],
                gene_is_multi: Optional[np.ndarray] = None):
    """Row indices to emit and their entity names.

    RUN modes: every entity, except gene runs whose GE is multi-gene
    (``gatherer.py:210-212``).  GROUPED: gene ids that have reads and are not
    multi-gene, in id order.
    """
    keep = []
    names = []
    for r in range(ints.shape[0]):
        name = entity_names[r]
        if mode != "cell":
            if ints[r, N.I_N_READS] == 0:
                continue
            if name is not None and len(str(name).split(",")) > 1:
                continue
        keep.append(r)
        names.append(name)
    return np.asarray(keep, dtype=np.int64), names
