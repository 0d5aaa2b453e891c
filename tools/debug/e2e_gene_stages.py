import sys, time, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch
from sctools_amd import columnar
from sctools_amd.metrics import gatherer as G
from sctools_amd.metrics.aggregator import GeneMetrics
from sctools_amd.metrics.writer import MetricCSVWriter
bam = "/tmp/sct_e2e_gene_24000000.bam"
dev = torch.device("cuda", 0)
for rep in range(2):
    t0 = time.perf_counter()
    cols = columnar.columnarize(bam, "rb", "gene", device=dev)
    torch.cuda.synchronize(); t1 = time.perf_counter()
    ints, floats = G.compute_rows(cols, "gene", float_mode="welford", device=dev)
    t2 = time.perf_counter()
    with MetricCSVWriter("/tmp/eg2", compress=True) as w:
        w.write_header(vars(GeneMetrics()))
        G.write_rows(w, "gene", cols, ints, floats)
    t3 = time.perf_counter()
    print("decode %.3f compute %.3f csv %.3f rows %d on_device %s" % (t1 - t0, t2 - t1, t3 - t2, ints.shape[0], cols.on_device))
