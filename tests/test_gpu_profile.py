"""Kernel timing through the C-ABI (sct_profile_enable / sct_profile_only / sct_profile_read).

bench.py's roofline depends on it: an untimed pass times every kernel (the per-kernel table and
the dominant kernel), then the timed steps bracket only the dominant kernel's launches.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def setup():
    from sctools_amd import engine as E
    from sctools_amd import synth

    dev = torch.device("cuda", 0)
    eng = E.get_engine(dev)
    d = synth.generate(synth.SynthConfig(n_reads=300_000, n_cells=60, n_genes=2_000), device=dev)
    dims = E.Dims(d.n_cell_ids, d.n_gene_ids, d.n_umi_ids)
    mito = torch.from_numpy(d.gene_is_mito).to(dev)
    yield eng, d.cols, dims, mito
    eng.profile_enable(False)
    eng.profile_only("")


def test_every_kernel_is_timed_by_default(setup):
    eng, cols, dims, mito = setup
    eng.profile_only("")
    eng.profile_enable(True)
    eng.cell_and_gene(cols, dims, mito)
    torch.cuda.synchronize()
    eng.profile_enable(False)
    table = eng.profile_read()
    for k in ("heads", "build_keys", "hash_tile", "gene_emit", "gene_reduce"):
        assert k in table, sorted(table)
        ms, launches = table[k]
        assert ms > 0 and launches >= 1
    assert eng.profile_read() == {}  # a read resets


def test_profile_only_brackets_one_kernel(setup):
    eng, cols, dims, mito = setup
    eng.profile_only("build_keys")
    eng.profile_enable(True)
    for _ in range(3):
        eng.cell_and_gene(cols, dims, mito)
    torch.cuda.synchronize()
    eng.profile_enable(False)
    eng.profile_only("")
    prof = eng.profile_read()
    assert set(prof) == {"build_keys"}
    assert prof["build_keys"][1] == 3 and prof["build_keys"][0] > 0
