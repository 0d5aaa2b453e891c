"""Native CSV text (libsct_csv.so) against Python's str / float.__repr__, and its gzip members.

The reference writes every value with str() (writer.py:84-103); the native formatter must give
the same bytes for every double (checked on random bit patterns, the ratios the metrics
produce, and the edge cases of Python's repr layout), and its parallel gzip must decompress to
the text with the standard readers.
"""
import gzip
import math

import numpy as np
import pytest

from sctools_amd import csvnative
from sctools_amd.metrics import rows as R
from sctools_amd.metrics.writer import MetricCSVWriter

EDGES = [0.0, -0.0, 1.0, -1.0, 0.1, 1e-5, 1e-4, 1.5e-4, 0.0001, 0.00012, 1e15, 1e16, 1.5e16, 9999999999999998.0,
         1e100, 1e-100, 5e-324, 2.2250738585072014e-308, 1.7976931348623157e308, 123456789.125, 2.5, 1 / 3, 2 / 3,
         100.0, 1e21, 1e22, 12345678901234567890.0, float("nan"), float("inf"), float("-inf")]


def test_exports():
    lib = csvnative.load()
    for name in csvnative.EXPORTED:
        assert hasattr(lib, name)


def test_repr_edges():
    for v in EDGES:
        assert csvnative.repr_double(v) == repr(v), v


def test_repr_random_bit_patterns_and_ratios():
    rng = np.random.default_rng(0)
    bits = rng.integers(0, 2 ** 63, 200_000, dtype=np.int64).view(np.float64)
    bits = bits[np.isfinite(bits)]
    ratios = rng.integers(0, 100_000, 100_000) / rng.integers(1, 1000, 100_000)
    for v in np.concatenate([bits, -bits[:1000], ratios]):
        v = float(v)
        assert csvnative.repr_double(v) == repr(v), v


def random_rows(n, seed=1):
    rng = np.random.default_rng(seed)
    ints = rng.integers(-5, 10 ** 9, (n, 24)).astype(np.int64)
    floats = rng.random((n, 12)) * 10.0 ** rng.integers(-8, 20, (n, 12))
    floats[rng.random((n, 12)) < 0.05] = np.nan
    floats[:, 3] = np.round(floats[:, 3])
    names = [None if i % 97 == 0 else "AAAC%06dé" % i for i in range(n)]
    return names, ints, floats


@pytest.mark.parametrize("mode", ["cell", "gene"])
def test_rows_bytes_identical_to_python(mode):
    names, ints, floats = random_rows(20_000)
    py = "".join(R.format_rows(mode, names, ints, floats)).encode("utf-8")
    assert R.format_rows_bytes(mode, names, ints, floats) == py


def test_gzip_members_decompress(tmp_path):
    data = b"".join(b"line %d,%r\n" % (i, math.sqrt(i)) for i in range(300_000))
    z = csvnative.gzip(data, level=9, chunk=1 << 20)
    assert gzip.decompress(z) == data
    p = tmp_path / "x.gz"
    p.write_bytes(z)
    with gzip.open(p, "rt") as f:
        assert f.read().encode() == data


def test_writer_file_matches_python_text(tmp_path):
    names, ints, floats = random_rows(5_000, seed=2)
    w = MetricCSVWriter(str(tmp_path / "native"), compress=True)
    w.write_header({"a": 1, "_x": 2, "b": 3})
    w.write("idx", {"a": 1.5, "b": None})
    w.write_bytes(R.format_rows_bytes("cell", names, ints, floats))
    w.close()
    expected = ",a,b\nidx,1.5,None\n" + "".join(R.format_rows("cell", names, ints, floats))
    with gzip.open(w.filename, "rt") as f:
        assert f.read() == expected
    w2 = MetricCSVWriter(str(tmp_path / "plain"), compress=False)
    w2.write_header({"a": 1, "b": 3})
    w2.write_bytes(R.format_rows_bytes("gene", names, ints, floats))
    w2.close()
    assert open(w2.filename).read() == ",a,b\n" + "".join(R.format_rows("gene", names, ints, floats))
