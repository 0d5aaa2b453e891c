"""Exact fixed-point mean / variance (sctools_amd/csrc/fixedpt.h), host build.

The same header runs on the device in the SCT_FLOAT_EXACT_SUM path.  Here it
is checked against exact rational arithmetic: mean and variance must be the
correctly rounded values of the exact rationals, for the value shapes the
metric streams produce (k/len fractions and sum/len mean qualities).
"""
import ctypes
import os
import subprocess
from fractions import Fraction

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "native", "libfxcheck.so")


@pytest.fixture(scope="module")
def fx():
    if not os.path.exists(LIB):
        subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared", "-o", LIB,
                        os.path.join(HERE, "native", "fxcheck.cpp")], check=True)
    lib = ctypes.CDLL(LIB)
    lib.fx_stats.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_double),
                             ctypes.POINTER(ctypes.c_double), ctypes.c_void_p]
    return lib


def run(fx, xs):
    x = np.ascontiguousarray(np.asarray(xs, dtype=np.float64))
    m, v = ctypes.c_double(), ctypes.c_double()
    fx.fx_stats(x.ctypes.data, x.shape[0], ctypes.byref(m), ctypes.byref(v), None)
    return m.value, v.value


def exact(xs):
    fs = [Fraction(float(x)) for x in xs]
    n = len(fs)
    mean = sum(fs) / n
    var = sum((f - mean) ** 2 for f in fs) / (n - 1) if n > 1 else None
    return float(mean), (float(var) if var is not None else float("nan"))


@pytest.mark.parametrize("seed", range(12))
def test_correctly_rounded_against_fractions(fx, seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 400))
    kind = seed % 3
    if kind == 0:
        L = rng.integers(1, 99, n)
        xs = rng.integers(0, L + 1) / L
    elif kind == 1:
        L = rng.integers(1, 99, n)
        xs = rng.integers(0, 42 * L + 1) / L
    else:
        xs = rng.integers(0, 11, n) / 10.0
    m, v = run(fx, xs)
    em, ev = exact(xs)
    assert m == em
    if n > 1:
        assert v == ev
    else:
        assert np.isnan(v)


def test_constant_stream_has_zero_variance(fx):
    m, v = run(fx, [0.9] * 1000)
    assert m == 0.9 and v == 0.0


def test_extreme_values(fx):
    xs = [1 / 65535, 93.0, 0.0, 1.0, 1 / 3, 2 / 3]
    m, v = run(fx, xs)
    em, ev = exact(xs)
    assert m == em and v == ev


def test_partials_add(fx):
    """Lanes of disjoint record sets add: the multi-GPU merge is a plain int64 sum."""
    rng = np.random.default_rng(5)
    L = rng.integers(1, 99, 3000)
    xs = rng.integers(0, L + 1) / L
    lanes = []
    for part in (xs[:1000], xs[1000:2500], xs[2500:]):
        arr = np.zeros(8, dtype=np.int64)
        x = np.ascontiguousarray(part)
        m, v = ctypes.c_double(), ctypes.c_double()
        fx.fx_stats(x.ctypes.data, x.shape[0], ctypes.byref(m), ctypes.byref(v), arr.ctypes.data)
        lanes.append(arr)
    tot = np.sum(lanes, axis=0)
    fx.fx_finalize_lanes.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_double),
                                     ctypes.POINTER(ctypes.c_double)]
    m, v = ctypes.c_double(), ctypes.c_double()
    fx.fx_finalize_lanes(tot.ctypes.data, 3000, ctypes.byref(m), ctypes.byref(v))
    em, ev = exact(xs)
    assert m.value == em and v.value == ev


def test_division_free_quotient_is_exact():
    """ratio_rcp (csrc/util.h) == IEEE a / b for every a, b < 2^16 (exhaustive, ~4.3e9 pairs)."""
    exe = os.path.join(HERE, "native", "divcheck")
    subprocess.run(["gcc", "-O2", "-fopenmp", "-ffp-contract=off", "-o", exe,
                    os.path.join(HERE, "native", "divcheck.c"), "-lm"], check=True)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    tot, bad = (int(v) for v in out.stdout.split())
    assert tot == 65535 * 65536
    assert bad == 0 and out.returncode == 0


def test_welford_chain_division_is_ieee(tmp_path):
    """The Welford chains divide by the record count without a division instruction (finalize.h):
    both the Markstein form RN(q0 + r y) and the double-double form fma(delta, y_hi, RN(delta y_lo))
    must be the IEEE quotient for every delta / k the chain can meet (20M random cases here)."""
    exe = str(tmp_path / "welfdiv")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", exe, os.path.join(HERE, "native", "welfdiv.c"), "-lm"],
                   check=True)
    out = subprocess.run([exe, "20000000", "7"], check=True, capture_output=True, text=True).stdout
    assert out.strip().splitlines()[-1] == "0 0", out
