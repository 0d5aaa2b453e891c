"""Host-side pieces of the device decode path (no GPU): the lazily decoded dictionaries the device
decoder hands over (columnar.PackedDictionary) and the Columns helpers the gatherers use for host
and device columns alike."""
import numpy as np

from sctools_amd import columnar


def packed(names, has_none):
    raw = b"".join(b"" if n is None else n.encode() for n in names)
    off = np.zeros(len(names) + 1, dtype=np.int64)
    off[1:] = np.cumsum([0 if n is None else len(n.encode()) for n in names])
    return columnar.PackedDictionary(raw, off, has_none)


def test_packed_dictionary_matches_the_eager_one():
    values = [None, "AAAC", "AAAG", "TTTT"]
    d = packed(values, True)
    e = columnar.Dictionary(values, presorted=True)
    assert len(d) == len(e) == 4
    assert d.names == e.names
    assert d.index == e.index
    assert d.names[0] is None


def test_packed_dictionary_without_missing_value_and_empty():
    d = packed(["G1", "G2"], False)
    assert d.names == ["G1", "G2"] and d.index["G2"] == 1
    empty = columnar.PackedDictionary(b"", np.zeros(1, dtype=np.int64), False)
    assert len(empty) == 0 and empty.names == []


def test_packed_dictionary_decodes_lazily():
    d = packed(["x%d" % i for i in range(1000)], False)
    assert d._names is None and len(d) == 1000  # counting needs no strings
    assert d.names[999] == "x999"


def test_host_columns_helpers():
    arrays = {"cell": np.array([3, 3, 5, 7], dtype=np.int32), "gene": np.array([1, 2, 1, 0], dtype=np.int32)}
    cols = columnar.Columns(arrays, packed(["a"], False), packed([], False), packed(["g"], False))
    assert not cols.on_device
    assert cols.host() is cols
    assert cols.n == 4
    assert cols.column_at("cell", np.array([0, 2, 3])).tolist() == [3, 5, 7]
