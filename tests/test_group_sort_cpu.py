"""The group tag sort's key layout (sctools_amd/csrc/tagsort.h, round 6), restated in numpy: an LSD
sort on the group key K1 = (cell, top `ub` umi bits) followed by a stable sort of every group by
W = (low umi bits, gene, tiebreak) is numpy's stable lexsort by (CB, UB, GE, tiebreak) -- the order of
bam.sort_by_tags_and_queryname (bam.py:698-709).  The `ub` rule is sct_tag_sort's: W must fit 52 bits
(12 bits of the 64-bit wave key hold the group's start lane and the lane), and ub fills K1 to the width
its passes sort anyway: the 9-bit top digit of the MSD pass plus whole 8-bit segmented passes (the
default when K1 needs more than 8 bits), else whole 8-bit LSD digits.  The GPU tests check the kernels
themselves (tests/test_gpu_tagsort.py)."""
import numpy as np
import pytest


def bitlen(v):  # bits for ids 0..v-1 (util.h bitlen)
    return 0 if v <= 1 else int(v - 1).bit_length()


MSD_BITS = 9  # tagsort.h kMsdBits


def group_bits(n_cell, n_umi, n_gene, n_tie):
    """(c, u, g, t, ub, ul, kw, seg): kw = the sorted key width, seg = its 8-bit segmented (MSD path) or
    LSD passes."""
    c, u, g, t = bitlen(n_cell), bitlen(n_umi), bitlen(n_gene), (bitlen(n_tie) if n_tie else 0)
    ub_min = max(0, u + g + t - 52)
    passes = (c + ub_min + 7) // 8
    if ub_min > u or passes > 4:
        return None  # the general path
    if c + ub_min > 8:  # MSD pass + segmented passes
        seg = max(0, -(-(c + ub_min - MSD_BITS) // 8))
        kw = min(32, MSD_BITS + 8 * seg)
    else:
        seg = passes
        kw = 8 * passes
    ub = min(u, kw - c)
    return c, u, g, t, ub, u - ub, kw, seg


@pytest.mark.parametrize("dims", [(10_000, 1 << 20, 30_000, 90_000_000), (300, 1 << 20, 2000, 1000),
                                  (300, 1 << 20, 2000, 0), (1, 1, 1, 0), (62_500, 1 << 24, 120_000, 0),
                                  (500_000, 1 << 20, 30_000, 1 << 28)])
def test_group_key_order_is_lexsort(dims):
    n_cell, n_umi, n_gene, n_tie = dims
    gb = group_bits(n_cell, n_umi, n_gene, n_tie)
    rng = np.random.default_rng(sum(dims) % 1000)
    n = 50_000
    cell = rng.integers(0, n_cell, n).astype(np.uint64)
    umi = rng.integers(0, min(n_umi, 64), n).astype(np.uint64) * (n_umi // min(n_umi, 64))  # collide on purpose
    gene = rng.integers(0, min(n_gene, 50), n).astype(np.uint64)
    tie = rng.integers(0, max(1, min(n_tie, 20)), n).astype(np.uint64)
    want = np.lexsort((tie, gene, umi, cell)) if n_tie else np.lexsort((gene, umi, cell))
    if gb is None:
        assert n_cell == 500_000  # (this case needs more than 4 radix passes: the general path)
        return
    c, u, g, t, ub, ul, kw, seg = gb
    assert ul + g + t <= 52 and c + ub <= kw <= 32
    k1 = (cell << np.uint64(ub)) | (umi >> np.uint64(ul))
    w = ((umi & np.uint64((1 << ul) - 1)) << np.uint64(g + t)) | (gene << np.uint64(t)) | (tie if t else 0)
    got = np.lexsort((w, k1))  # stable: ties keep input order, as the LSD passes and the lane key do
    assert np.array_equal(got, want)


@pytest.mark.parametrize("n_gene", [30_000, 60_001])
def test_config5_widths(n_gene):
    """Config 5 (10k cells, 10-mer UMIs, 30k genes -- 60,001 gene ids with the missing-GE id and the
    multi-gene strings, as synth generates them --, ~94M query names): a 24- or 25-bit group key, the
    MSD pass's 9-bit digit and two segmented passes (an 8-bit top digit needed three for 25 bits)."""
    c, u, g, t, ub, ul, kw, seg = group_bits(10_000, 1 << 20, n_gene, 93_500_000)
    assert (c, ub, kw, seg) == (14, 11, 25, 2) and ul + g + t <= 52
