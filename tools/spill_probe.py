"""Experiment helper: records missing from the gene partials (n - sum n_reads) on the bench data."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from sctools_amd import engine as E  # noqa: E402
from sctools_amd import synth  # noqa: E402

dev = torch.device("cuda", 0)
eng = E.get_engine(dev)
d = synth.generate(synth.SynthConfig(n_reads=int(sys.argv[1]) if len(sys.argv) > 1 else 20_000_000), device=dev,
                   chunk=16_000_000)
dims = E.Dims(d.n_cell_ids, d.n_gene_ids, d.n_umi_ids)
part = eng.gene_partials(d.cols, dims)
n = d.cols["cell"].numel()
print("records", n, "missing", n - int(part[:, 0].sum().item()))
