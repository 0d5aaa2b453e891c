"""
sctools_amd: MI355X-native per-cell / per-gene metric aggregation.

Drop-in for ``sctools.metrics`` (GatherCellMetrics / GatherGeneMetrics,
MetricCSVWriter, MergeCellMetrics / MergeGeneMetrics) whose hot path runs as
hand-written HIP kernels for gfx950 behind the C-ABI in
``include/sctools_gpu.h``.  See DESIGN.md.
"""

__version__ = "0.1.0"
