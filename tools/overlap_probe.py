"""Experiments only: do two batches in flight on one GPU (two host threads, two streams, two engine
workspaces) raise the config-2 step throughput?  Times K steps one after another, then the same K
steps as K/2 per thread on two threads at once (each thread its own stream, Engine and partials)."""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def main():
    from sctools_amd import engine as E
    from sctools_amd import synth

    dev = torch.device("cuda", 0)
    cells = 10_000
    cfg = synth.SynthConfig(n_reads=100_000_000, n_cells=cells, n_genes=30_000, seed=0)
    data = synth.generate(cfg, device=dev, chunk=16_000_000)
    dims = E.Dims(data.n_cell_ids, data.n_gene_ids, data.n_umi_ids)
    mito = torch.from_numpy(data.gene_is_mito).to(dev)
    engs = [E.Engine(dev), E.Engine(dev)]
    n_ent = engs[0].count_entities(data.cols, "cell", dims)
    parts = [torch.empty((data.n_gene_ids, 64), dtype=torch.int64, device=dev) for _ in range(2)]
    streams = [torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)]

    def step(i):
        ci, cf, _ = engs[i].cell_and_gene(data.cols, dims, mito, n_entities=n_ent, partials=parts[i])
        engs[i].finalize_partials(parts[i])

    def run(i, k):
        with torch.cuda.stream(streams[i]):
            for _ in range(k):
                step(i)
        streams[i].synchronize()

    K = 10
    run(0, 2)
    run(1, 2)
    for rep in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(0, K)
        t1 = time.perf_counter()
        th = [threading.Thread(target=run, args=(i, K // 2)) for i in range(2)]
        t2 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        t3 = time.perf_counter()
        print("rep %d: one stream %.3f ms/step, two in flight %.3f ms/step" % (rep, (t1 - t0) / K * 1e3,
                                                                          (t3 - t2) / K * 1e3), flush=True)


if __name__ == "__main__":
    main()
