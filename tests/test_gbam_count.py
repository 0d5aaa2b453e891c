"""Device BAM decode in count-matrix mode (sct_gbam_parse_count, include/sct_gbam.h) against the
host decoder's count mode (libsct_bam.so, itself checked against the pure-Python reader and the
reference's golden matrices in test_count_cpu.py), and CountMatrix.from_sorted_tagged_bam with
the device decoder against the same call decoding on the host."""
import os
import re

import numpy as np
import pytest

import helpers as H
import test_gbam as G
from sctools_amd import bamnative, gbam
from sctools_amd import count as C

pytestmark = pytest.mark.gpu

BAMS = sorted(os.path.join(d, f) for d in (os.path.join(H.GOLDEN, "bam"), os.path.join(H.GOLDEN, "count"))
              for f in os.listdir(d) if f.endswith(".bam"))
TAGS = [("CB", "UB", "GE"), ("UB", "CB", "GE"), ("CR", "UR", "GE"), ("CB", "CB", "XX")]


def same_as_host(path, tags):
    want = bamnative.decode(path, "count", tags=tags)
    got = gbam.decode(path, "count", tags=tags)
    if want[0]["cell"].shape[0] == 0:
        assert got is None  # an empty file: the host path
        return None
    assert got is not None, (path, tags, gbam.last_error())
    cols, names = got
    arrays, want_names = want
    assert names == [list(n) for n in want_names]
    for c in gbam.COUNT_COLUMNS:
        assert np.array_equal(cols[c].cpu().numpy(), arrays[c]), (path, tags, c)
    return cols


@pytest.mark.parametrize("bam", BAMS, ids=os.path.basename)
@pytest.mark.parametrize("tags", TAGS, ids="-".join)
def test_count_columns_match_host_decoder(bam, tags):
    same_as_host(bam, tags)


def test_count_columns_across_members(tmp_path):
    """Members cutting records anywhere: a query-name group head compares names across members."""
    raw = G.payload(os.path.join(H.GOLDEN, "count", "synth_b_qname.bam"))
    path = str(tmp_path / "re.bam")
    G.rebgzf(raw, path, level=6, block=997)
    cols = same_as_host(path, ("CB", "UB", "GE"))
    assert cols is not None and int(cols["qhead"].sum()) < cols["qhead"].numel()  # some multi-record groups


def test_typed_tag_declines():
    """NH holds integers: the device path declines; the host decoder keys their str()."""
    path = os.path.join(H.GOLDEN, "bam", "small-cell-sorted.bam")
    assert gbam.decode(path, "count", tags=("NH", "UB", "GE")) is None
    bamnative.decode(path, "count", tags=("NH", "UB", "GE"))


def _rb_cases():
    import test_count_cpu as T

    return [c for c in T.CASES if T.case_input(c)[1] == "rb"]


@pytest.mark.parametrize("case", _rb_cases())
@pytest.mark.parametrize("gpu_decode", [True, False])
def test_count_matrix_both_decoders_match_reference(case, gpu_decode):
    """The reference's golden matrix (or its KeyError) whichever decoder reads the BAM."""
    import test_count_cpu as T

    path, mode = T.case_input(case)

    def run():
        m = C.CountMatrix.from_sorted_tagged_bam(path, T.case_genes(case), open_mode=mode, device="cuda:0",
                                                 gpu_decode=gpu_decode)
        return m.matrix, m.row_index, m.col_index

    T.check_case(case, run)


def test_count_matrix_many_members(tmp_path):
    """26 replicas of a query-name-grouped file (new cell barcodes per replica) over hundreds of
    members: device and host decodes give the same matrix."""
    import test_count_cpu as T

    raw = G.payload(os.path.join(H.GOLDEN, "count", "synth_b_qname.bam"))
    hdr_end = G._header_end(raw)
    body = raw[hdr_end:]
    reps = [re.sub(rb"CBZ.", b"CBZ" + bytes([65 + r % 26]), body) for r in range(26)]
    path = str(tmp_path / "big.bam")
    G.rebgzf(raw[:hdr_end] + b"".join(reps), path, level=6, block=65280)
    same_as_host(path, ("CB", "UB", "GE"))
    genes = T.case_genes("synth_b_qname")
    a = C.CountMatrix.from_sorted_tagged_bam(path, genes, device="cuda:0")
    b = C.CountMatrix.from_sorted_tagged_bam(path, genes, device="cuda:0", gpu_decode=False)
    assert a.matrix.shape == b.matrix.shape and (a.matrix != b.matrix).nnz == 0
    assert np.array_equal(a.row_index, b.row_index)
