"""GPU checks of the device helpers the SIM1 scan kernel is built from (csrc/fastmath.hpp,
csrc/blockscan.hpp), through the test-only probe library tests/native/bin/libblockscan_probe.so
(tests/native/Makefile; built by __graft_entry__.build()):

  * fm_log / fm_exp / fm_div / fm_rcp within 1 ulp of numpy (glibc) over the ranges the
    Riemann solver feeds them (pressures, the exponents of pk3 / pl / dz2);
  * the DPP block hand-overs and Kogge-Stone block sums against their definitions;
  * tri_solve (partitioned Thomas, NB = 8 blocks of 9 rows) against a sequential Thomas sweep
    in numpy: the pp-type system (strongly diagonally dominant) with the Möbius-scan pivots, and
    the w-type system (nearly singular: acoustic coupling ~1e8 against masses ~1e2, also 1e3
    times lighter layers) with the serial pivots, both at 1e-12 of the mean |x| (the column
    sweep itself is ~1e-14 from an extended-precision solve on these systems).
"""
import ctypes
import os

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

LIB = os.path.join(ROOT, "tests", "native", "bin", "libblockscan_probe.so")


@pytest.fixture(scope="module")
def probe(require_gpu):
    assert os.path.exists(LIB), "tests/native/bin/libblockscan_probe.so not built (make -C tests/native)"
    lib = ctypes.CDLL(LIB)
    P = ctypes.POINTER(ctypes.c_double)
    lib.probe_math.argtypes = [ctypes.c_int, P, P, P, ctypes.c_int]
    lib.probe_shift.argtypes = [P, P]
    lib.probe_tri.argtypes = [ctypes.c_int, P, P, P, P, P, ctypes.c_int]
    return lib


def _p(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _ulps(got, want):
    return np.abs(got - want) / np.spacing(np.abs(want))


@pytest.mark.parametrize("kind,lo,hi", [(0, 1e-3, 2e5), (0, 0.05, 20.0), (1, -30.0, 30.0), (1, -8.0, 17.0),
                                        (2, 0.1, 1e9), (3, 1e-6, 1e12)])
def test_fastmath_ulps(probe, kind, lo, hi):
    r = np.random.default_rng(7 + kind)
    n = 1 << 20
    if kind == 1:
        x = r.uniform(lo, hi, n)
    else:
        x = np.exp(r.uniform(np.log(lo), np.log(hi), n))
    y = np.exp(r.uniform(np.log(0.1), np.log(1e9), n))
    out = np.zeros(n)
    assert probe.probe_math(kind, _p(x), _p(y), _p(out), n) == 0
    want = [np.log(x), np.exp(x), x / y, 1.0 / x][kind]
    worst = _ulps(out, want).max()
    assert worst <= 1.0, f"kind {kind}: {worst:.2f} ulp"


def test_block_shifts_and_sums(probe):
    v = np.arange(64, dtype=np.float64) * 1.5 + 1.0
    out = np.zeros(384)
    assert probe.probe_shift(_p(v), _p(out)) == 0
    lane = np.arange(64)
    prev = np.where(lane % 16 == 0, 0.0, np.roll(v, 1))
    nxt = np.where(lane % 16 == 15, 0.0, np.roll(v, -1))
    assert np.array_equal(out[0:64][lane % 8 != 0], prev[lane % 8 != 0])
    assert np.array_equal(out[64:128][lane % 8 != 7], nxt[lane % 8 != 7])
    g8 = v.reshape(8, 8)
    assert np.allclose(out[128:192], np.cumsum(g8, axis=1).ravel(), rtol=1e-15)
    assert np.allclose(out[192:256], np.cumsum(g8[:, ::-1], axis=1)[:, ::-1].ravel(), rtol=1e-15)
    assert np.array_equal(out[256:320][lane % 16 >= 4], np.roll(v, 4)[lane % 16 >= 4])
    assert np.allclose(out[320:384], np.cumsum(v.reshape(4, 16), axis=1).ravel(), rtol=1e-15)


def _thomas(a, d, c, r):
    n = d.shape[-1]
    gam = np.zeros_like(d)
    y = np.zeros_like(d)
    bet = d[:, 0].copy()
    y[:, 0] = r[:, 0] / bet
    for k in range(1, n):
        gam[:, k] = c[:, k - 1] / bet
        bet = d[:, k] - a[:, k] * gam[:, k]
        y[:, k] = (r[:, k] - a[:, k] * y[:, k - 1]) / bet
    x = y.copy()
    for k in range(n - 2, -1, -1):
        x[:, k] = y[:, k] - gam[:, k + 1] * x[:, k + 1]
    return x


def _system(kind, ncol, r):
    n = 72
    dm = (100.0 + 900.0 * r.random((ncol, n))) * (1e-3 if kind == "wlight" else 1.0)
    if kind == "pp":
        g = np.concatenate([dm[:, :-1] / dm[:, 1:], np.zeros((ncol, 1))], axis=1)
        a = np.ones((ncol, n))
        d = 2.0 * (1.0 + g)
        d[:, -1] = 2.0
        c = g
        rhs = 3e3 * r.standard_normal((ncol, n))
    else:
        dz = -(50.0 + 500.0 * r.random((ncol, n)))
        pem = 1e5 * np.linspace(0.01, 1.0, n + 1)
        t1g = 5.7e5
        aa = np.zeros((ncol, n + 1))
        aa[:, 1:n] = t1g / (dz[:, :-1] + dz[:, 1:]) * pem[1:n]
        p1 = t1g / dz[:, -1] * pem[n]
        a = aa[:, :n].copy()
        c = np.concatenate([aa[:, 1:n], np.zeros((ncol, 1))], axis=1)
        d = dm - aa[:, :n] - np.concatenate([aa[:, 1:n], p1[:, None]], axis=1)
        rhs = dm * r.standard_normal((ncol, n)) + 1e3 * r.standard_normal((ncol, n))
    a[:, 0] = 0.0
    return a, d, c, rhs


@pytest.mark.parametrize("kind,mobius", [("pp", 1), ("w", 0), ("wlight", 0)])
def test_tri_solve_vs_thomas(probe, kind, mobius):
    r = np.random.default_rng(11)
    ncol = 1000
    a, d, c, rhs = _system(kind, ncol, r)
    x = np.zeros_like(d)
    assert probe.probe_tri(ncol, _p(a), _p(d), _p(c), _p(rhs), _p(x), mobius) == 0
    want = _thomas(a, d, c, rhs)
    err = np.abs(x - want).max(axis=1) / np.abs(want).mean(axis=1)
    assert err.max() <= 1e-12, f"{kind}: worst column {err.max():.2e}"
    # the pivots and the substitution run from the same factors in every block: a column's
    # blocks agree with the sequential sweep on their first rows as on their last
    assert np.isfinite(x).all()
