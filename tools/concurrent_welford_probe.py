"""Experiments only: three Welford drop-in cell passes at once on one device (three host threads,
each its own stream and Engine, as multigpu's devices=[0, 0, 0] runs them), wall time per round."""
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
    data = synth.generate(synth.SynthConfig(n_reads=30_000_000, n_cells=3_000, n_genes=30_000, seed=0), device=dev)
    dims = E.Dims(data.n_cell_ids, data.n_gene_ids, data.n_umi_ids)
    mito = torch.from_numpy(data.gene_is_mito).to(dev)
    multi = torch.from_numpy(data.gene_is_multi).to(dev)
    engs = [E.Engine(dev) for _ in range(3)]
    streams = [torch.cuda.Stream(device=dev) for _ in range(3)]

    def run(i):
        with torch.cuda.stream(streams[i]):
            engs[i].compute(data.cols, "cell", dims, mito, multi, float_mode="welford")
        streams[i].synchronize()

    for i in range(3):
        run(i)
    for rep in range(4):
        t0 = time.perf_counter()
        run(0)
        t1 = time.perf_counter()
        th = [threading.Thread(target=run, args=(i,)) for i in range(3)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        t2 = time.perf_counter()
        print("rep %d: one pass %.2f ms, three at once %.2f ms" % (rep, (t1 - t0) * 1e3, (t2 - t1) * 1e3), flush=True)


if __name__ == "__main__":
    main()
