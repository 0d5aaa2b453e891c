"""
The aggregator protocol on the engine: ``MetricAggregator.parse_molecule``
buffers (tags, numeric fields) pairs -- the fields ``columnar.record_fields``
would give, read while the counters are updated; ``finalize`` turns the
buffered entity into columns and runs it through the HIP engine as a
single-entity batch.

Record semantics follow ``parse_molecule`` / ``parse_extra_fields``
(``/root/reference/src/sctools/metrics/aggregator.py:236-334, 492-530, 580-595``):
the molecule / gene / cell keys come from the ``tags`` tuple passed by the
caller, every other field from the record itself.
"""

import numpy as np

from sctools_amd import columnar


def aggregate_buffered(mode: str, buffered, mitochondrial_genes=frozenset(), float_mode="welford"):
    if not buffered:
        raise ValueError("no buffered records (an empty aggregator finalizes without the engine)")
    is_cell = mode == "cell"
    cell_v, umi_v, gene_v, numeric = [], [], [], []
    for tags, num in buffered:
        numeric.append(num)
        if is_cell:  # tags = (CB, UB, GE)
            cell_v.append(tags[0])
            umi_v.append(tags[1])
            gene_v.append(tags[2])
        else:  # tags = (GE, CB, UB)
            gene_v.append(tags[0])
            cell_v.append(tags[1])
            umi_v.append(tags[2])
    cols = columnar.build_columns(cell_v, umi_v, gene_v, numeric)
    from sctools_amd.metrics.gatherer import compute_rows

    ints, floats = compute_rows(cols, mode, mitochondrial_genes, float_mode)
    assert ints.shape[0] == 1, "a buffered entity is one run"
    return ints[0], floats[0]
