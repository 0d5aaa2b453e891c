"""Native BAM decoder (libsct_bam.so, include/sct_bam.h) against the pure-Python decoder.

The Python decoder (sctools_amd.columnar + sctools_amd.bam) is checked against the
reference's outputs elsewhere (test_api_cpu, the GPU golden tests); here the native one
must give identical columns and dictionaries on every fixture, raise the same exception
class at the same first record on every error path the reference has (missing CY / CR /
UY / XF / NH, missing or empty qualities, empty quality strings, an empty file), and
handle records cut across BGZF blocks and decode windows.
"""
import copy
import os

import numpy as np
import pytest

import bamwriter
import helpers as H
from sctools_amd import bamnative, columnar
from sctools_amd.bam import open_alignments


def both(path, mode):
    a = columnar.columnarize(path, "rb", mode, native=True)
    b = columnar.columnarize(path, "rb", mode, native=False)
    return a, b


def same(a, b):
    assert a.cells.names == b.cells.names
    assert a.umis.names == b.umis.names
    assert a.genes.names == b.genes.names
    for k in b.arrays:
        assert a.arrays[k].dtype == b.arrays[k].dtype, k
        assert np.array_equal(a.arrays[k], b.arrays[k]), k


def test_library_exports():
    lib = bamnative.load()
    for name in bamnative.EXPORTED:
        assert hasattr(lib, name), name


@pytest.mark.parametrize("bam", H.BAMS)
@pytest.mark.parametrize("mode", ["cell", "gene"])
def test_fixtures_identical_to_python_decoder(bam, mode):
    same(*both(os.path.join(H.GOLDEN, "bam", bam + ".bam"), mode))


def records(name="small-cell-sorted"):
    return list(open_alignments(os.path.join(H.GOLDEN, "bam", name + ".bam"), "rb"))


def test_many_blocks_and_windows(tmp_path, monkeypatch):
    """~40k records in ~60 KB BGZF blocks, decoded in 100 KB windows: records cut across blocks
    and across windows (the carry path) decode exactly."""
    recs = records("cell-sorted-missing-cb") * 3
    p = str(tmp_path / "big.bam")
    bamwriter.write_bam(p, recs)
    b = columnar.columnarize(p, "rb", "gene", native=False)
    monkeypatch.setenv("SCT_BAM_WINDOW", str(100_000))
    a = columnar.columnarize(p, "rb", "gene", native=True)
    same(a, b)
    assert a.n == 3 * 13236


def mutate(recs, k, fn):
    out = [copy.copy(r) for r in recs]
    r = out[k]
    r._tags = dict(r._tags)
    fn(r)
    return out


def drop(tag):
    return lambda r: r._tags.pop(tag, None)


def setter(tag, v):
    def f(r):
        r._tags[tag] = v
    return f


def no_quals(r):
    r._qual = None


CASES = [
    ("cell", drop("CY"), KeyError),
    ("cell", drop("CR"), KeyError),
    ("cell", drop("UY"), KeyError),
    ("gene", drop("UY"), KeyError),
    ("cell", drop("XF"), KeyError),
    ("gene", drop("NH"), KeyError),
    ("cell", setter("CY", ""), ZeroDivisionError),
    ("gene", setter("UY", ""), ZeroDivisionError),
    ("cell", no_quals, TypeError),
    ("gene", no_quals, TypeError),
]


@pytest.mark.parametrize("mode,fn,exc", CASES)
def test_errors_match_python_decoder(tmp_path, mode, fn, exc):
    recs = records()
    k = next(i for i, r in enumerate(recs) if not r.flag & 4 and "CB" in r._tags and i > 100)
    p = str(tmp_path / "bad.bam")
    bamwriter.write_bam(p, mutate(recs, k, fn))
    with pytest.raises(exc):
        columnar.columnarize(p, "rb", mode, native=False)
    with pytest.raises(exc):
        columnar.columnarize(p, "rb", mode, native=True)


def test_first_error_in_file_order_wins(tmp_path):
    """Two bad records: the earlier one's class is raised (KeyError), not the later one's."""
    recs = records()
    ks = [i for i, r in enumerate(recs) if not r.flag & 4 and "CB" in r._tags]
    bad = mutate(recs, ks[10], drop("NH"))
    bad = mutate(bad, ks[5], no_quals)  # earlier: TypeError
    p = str(tmp_path / "two.bam")
    bamwriter.write_bam(p, bad)
    with pytest.raises(TypeError):
        columnar.columnarize(p, "rb", "cell", native=False)
    with pytest.raises(TypeError):
        columnar.columnarize(p, "rb", "cell", native=True)


def test_multi_gene_runs_skip_validation_in_gene_mode(tmp_path):
    """gatherer.py:210-212: a multi-gene GE run is skipped, so its records are not validated."""
    recs = records("small-gene-sorted")
    k = 50
    bad = mutate(recs, k, lambda r: (r._tags.__setitem__("GE", "A,B"), r._tags.pop("UY", None)))
    p = str(tmp_path / "multi.bam")
    bamwriter.write_bam(p, bad)
    same(*both(p, "gene"))
    with pytest.raises(KeyError):
        columnar.columnarize(p, "rb", "cell", native=True)


def test_empty_bam_raises_runtime_error(tmp_path):
    p = str(tmp_path / "empty.bam")
    bamwriter.write_bam(p, [])
    with pytest.raises(RuntimeError):
        columnar.columnarize(p, "rb", "cell", native=True)
