"""Drop-in for ``sctools.metrics``: gatherers, aggregators, writer and merges."""

from sctools_amd.metrics.aggregator import CellMetrics, GeneMetrics, MetricAggregator  # noqa: F401
from sctools_amd.metrics.gatherer import (  # noqa: F401
    GatherCellAndGeneMetrics, GatherCellMetrics, GatherGeneMetrics, MetricGatherer)
from sctools_amd.metrics.merge import MergeCellMetrics, MergeGeneMetrics, MergeMetrics  # noqa: F401
from sctools_amd.metrics.writer import MetricCSVWriter  # noqa: F401
