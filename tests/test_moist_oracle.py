"""CPU known-answer and property tests of the moist column oracle (oracle/moist.py),
SURVEY.md §8a row A13.  The GEOS moist schemes are external to the reference, so the
oracle is parity unpinned; these pin its physics: the saturation tables' anchor point
and ordering, column mass conservation of fillq2zero and of the GFDL-style step
(total water + surface precipitation, to round-off), positivity, the saturation
adjustment's target, and the buoyancy / LCL diagnostics on constructed columns."""
import numpy as np

from moist_inputs import moist_state
from oracle import moist as om

SHAPE = (2, 30, 9, 12)


def test_saturation_tables():
    tw, ti, dw, di = om.tables()
    n0 = int(round((om.T_ICE - om.TABLE_T0) / om.TABLE_DT))
    assert tw[n0] == om.E00 and ti[n0] == om.E00          # es(T0) = e00 exactly
    assert np.all(np.diff(tw) > 0) and np.all(np.diff(ti) > 0)
    assert np.all(ti[:n0] <= tw[:n0])                      # ice below water under T0
    assert abs(om.es_water(373.15) / 101325.0 - 1.0) < 0.025  # boiling point within the form's 2 %
    t = np.linspace(200.0, 310.0, 57)
    qs, dqs = om.qsat(t, np.full_like(t, 8.0e4))
    fd = (om.qsat(t + 0.01, np.full_like(t, 8.0e4))[0] - om.qsat(t - 0.01, np.full_like(t, 8.0e4))[0]) / 0.02
    assert np.allclose(dqs, fd, rtol=2e-2)


def test_fillq2zero_conserves_and_fills():
    st = moist_state(SHAPE)
    q = st["ql"][0]
    dp = st["delp"][0]
    out, fill = om.fillq2zero(q, dp)
    assert np.all(out >= 0.0)
    tot0 = np.maximum(np.einsum("k...,k...->...", q, dp), 0.0)
    tot1 = np.einsum("k...,k...->...", out, dp)
    assert np.allclose(tot1, tot0, rtol=1e-13, atol=1e-18)
    assert np.all(fill >= 0.0) and fill.max() > 0.0


def water(T, qv, ql, qr, qi, qs, qg, dp):
    return np.einsum("k...,k...->...", qv + ql + qr + qi + qs + qg, dp) / om.GRAV


def test_gfdl_1m_water_conservation_and_positivity():
    st = moist_state(SHAPE)
    dt = 450.0
    args = [st[k][0] for k in ("T", "delp", "delz", "pm", "qv", "ql", "qr", "qi", "qs", "qg")]
    (T, qv, ql, qr, qi, qs, qg), prec = om.gfdl_1m(*args, dt)
    w0 = water(None, *(st[k][0] for k in ("qv", "ql", "qr", "qi", "qs", "qg")), st["delp"][0])
    w1 = water(None, qv, ql, qr, qi, qs, qg, st["delp"][0]) + sum(prec)
    assert np.allclose(w1, w0, rtol=1e-12)
    for q in (ql, qr, qi, qs, qg):
        assert q.min() >= -1e-18
    assert sum(p.sum() for p in prec) > 0.0
    assert np.all(np.abs(T - st["T"][0]) < 30.0)


def test_gfdl_1m_saturation_adjustment_target():
    """a warm supersaturated cloud-free column with nothing to precipitate ends at
    saturation after the one-step adjustment (to the Newton step's accuracy)"""
    nk = 10
    pm = np.linspace(7.0e4, 9.5e4, nk)[:, None]
    T = np.linspace(285.0, 298.0, nk)[:, None]
    dp = np.full_like(pm, 2.5e3)
    dz = -om.RDGAS / om.GRAV * T * dp / pm
    qsw, _ = om.qsat(T, pm)
    qv = 1.05 * qsw
    z = np.zeros_like(pm)
    (T1, qv1, ql1, qr1, qi1, qs1, qg1), prec = om.gfdl_1m(T, dp, dz, pm, qv, z, z, z, z, z, 60.0)
    q1, _ = om.qsat(T1, pm)
    assert np.all(ql1 > 0.0) and np.all(T1 > T)
    assert np.allclose(qv1, q1, rtol=2e-3)
    assert np.all(qr1 == 0.0) and sum(p.sum() for p in prec) == 0.0


def test_buoyancy_lcl_and_cape():
    nk = 40
    pm = np.linspace(1.0e4, 1.0e5, nk)[:, None] * np.ones((1, 3))
    T = 300.0 * (pm / 1e5) ** om.KAPPA                  # dry adiabat
    zm = -om.RDGAS * 270.0 / om.GRAV * np.log(pm / 1e5)
    qv = np.zeros_like(pm)
    qv[:, 1] = om.qsat(T[-1:, 1], pm[-1:, 1])[0]        # column 1: saturated lowest layer
    qv[:, 2] = 0.5 * om.qsat(T[-1:, 2], pm[-1:, 2])[0]  # column 2: 50 % RH at the surface
    by, cape, cin, klcl = om.buoyancy(T, qv, pm, zm)
    assert klcl[0] == -1.0 and klcl[1] == nk - 1.0
    assert 0.0 <= klcl[2] < nk - 1.0
    assert np.all(cape >= 0.0) and np.all(cin <= 0.0)
    assert cape[1] > cape[0]
