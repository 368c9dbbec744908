"""CPU known-answer and property tests of the moist column oracles (oracle/moist.py,
oracle/gfdl_mp.py, oracle/geos_moist.py), SURVEY.md §8a row A13 / §8f row 2.  The GEOS
moist schemes are external to the reference, so the oracles are parity unpinned; these
pin their physics: the saturation tables' anchor point and ordering, column mass
conservation of fillq2zero, of the Lagrangian sedimentation and of the whole GFDL
microphysics step (total water + surface precipitation, to round-off), positivity, the
PPM profile's exactness and monotonicity, the PDF condensation's water and enthalpy
budget, RADCOUPLE's caps and the activation's monotonicity in the updraft, and the
buoyancy / LCL diagnostics on constructed columns."""
import numpy as np

from moist_inputs import moist_state
from oracle import geos_moist as gm
from oracle import gfdl_mp as mp
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


def water(qv, ql, qr, qi, qs, qg, dp):
    return np.einsum("k...,k...->...", qv + ql + qr + qi + qs + qg, dp) / om.GRAV


def cols(st, names, s=0, n=24):
    """the first n columns of sub-domain s as [k, n] arrays"""
    return [st[k][s].reshape(st[k].shape[1], -1)[:, :n] for k in names]


def test_cs_profile_exact_for_constant_and_monotone():
    dz = np.linspace(100.0, 400.0, 20)
    aL, aR, a6 = mp.cs_profile_mono(np.full(20, 3.0), dz)
    assert np.all(aL == 3.0) and np.all(aR == 3.0) and np.all(a6 == 0.0)
    r = np.random.default_rng(3)
    a = np.abs(r.standard_normal(20))
    aL, aR, a6 = mp.cs_profile_mono(a, dz)
    # every parabola stays within [min, max] of its edge values and the mean (monotone)
    for k in range(20):
        x = np.linspace(0.0, 1.0, 41)
        p = aL[k] + x * (aR[k] - aL[k] + a6[k] * (1.0 - x))
        lo, hi = min(aL[k], aR[k], a[k]), max(aL[k], aR[k], a[k])
        assert p.min() >= lo - 1e-12 and p.max() <= hi + 1e-12
        assert abs(aL[k] + 0.5 * (aR[k] - aL[k]) + a6[k] / 6.0 - a[k]) <= 1e-12 * max(1.0, a[k])


def test_lagrangian_fall_conserves_and_is_identity_at_rest():
    r = np.random.default_rng(4)
    n = 30
    dz = -(200.0 + 300.0 * r.random(n))
    ze = np.concatenate([np.cumsum(-dz[::-1])[::-1], [0.0]])
    dp = 800.0 + 400.0 * r.random(n)
    q = 1e-4 * r.random(n)
    qn, m1 = mp.lagrangian_fall_ppm(ze, ze.copy(), dp, q)
    assert np.allclose(qn, q, rtol=1e-13) and abs(m1[-1]) < 1e-16
    vt = 2.0 + 3.0 * r.random(n)
    zt = mp.fallen_edges(ze, vt, 150.0)
    qn, m1 = mp.lagrangian_fall_ppm(ze, zt, dp, q)
    assert np.all(qn >= -1e-20)
    assert abs((qn * dp).sum() + m1[-1] - (q * dp).sum()) <= 1e-14 * (q * dp).sum()
    assert m1[-1] > 0.0


def test_gfdl_mp_water_conservation_and_positivity():
    st = moist_state(SHAPE)
    dt = 450.0
    T, dp, dz, *qs = cols(st, ("T", "delp", "delz", "qv", "ql", "qr", "qi", "qs", "qg"))
    (T1, *q1), prec = mp.mpdrv(T, dp, dz, *qs, dt)
    w0 = water(*qs, dp)
    w1 = water(*q1, dp) + sum(prec)
    assert np.allclose(w1, w0, rtol=1e-13)
    for q in q1[1:]:
        assert q.min() >= -1e-18
    assert q1[0].min() >= 0.0
    assert sum(p.sum() for p in prec) > 0.0
    assert np.all(np.abs(T1 - T) < 30.0)
    assert np.all(np.isfinite(T1))


def test_gfdl_mp_subgrid_condensation_relaxes_to_saturation():
    """a warm supersaturated cloud-free layer with nothing to precipitate: subgrid_z_proc
    condenses (1 - exp(-dt / tau_v2l)) of the linearised excess"""
    t = np.full(4, 290.0)
    den = np.full(4, 1.1)
    qsw, dq = mp.wqs2(t, den)
    qv = qsw * 1.05
    z = np.zeros(4)
    ql = z.copy()
    qv1, t1 = qv.copy(), t.copy()
    mp.subgrid_z_proc(100.0, t1, den, qv1, ql, z.copy(), z.copy(), z.copy(), z.copy())
    assert np.all(ql > 0.0) and np.allclose(qv1 + ql, qv, rtol=1e-15)
    qs_after, _ = mp.wqs2(t1, den)
    assert np.all(qv1 - qs_after < qv - qsw)      # closer to saturation
    assert np.all(t1 > t)                          # latent heating


def test_evap_subl_pdf_conserves_water_and_enthalpy():
    st = moist_state(SHAPE, seed=8)
    T, qv, ql, qi, pm = cols(st, ("T", "qv", "ql", "qi", "pm"))
    ql, qi = np.maximum(ql, 0.0), np.maximum(qi, 0.0)
    z = np.zeros_like(T)
    e = gm.evap_subl_pdf(450.0, pm, T, qv, ql, qi, 0.3 * ql, 0.3 * qi, z + 0.2, z + 0.1, z + 5e7, z + 1e3)
    w0 = qv + ql + qi + 0.3 * ql + 0.3 * qi
    w1 = e["qv"] + e["qlls"] + e["qils"] + e["qlcn"] + e["qicn"]
    assert np.allclose(w1, w0, rtol=1e-13, atol=1e-18)
    # liquid-water static energy cp T - Lv (ql) - Ls (qi) is kept by every phase change
    h0 = om.CP_AIR * T - om.HLV * (ql + 0.3 * ql) - om.HLS * (qi + 0.3 * qi)
    h1 = om.CP_AIR * e["t"] - om.HLV * (e["qlls"] + e["qlcn"]) - om.HLS * (e["qils"] + e["qicn"])
    assert np.allclose(h1, h0, rtol=1e-12)
    assert e["clls"].min() >= 0.0 and e["clls"].max() <= 1.0


def test_radcouple_caps_and_radii():
    st = moist_state(SHAPE, seed=6)
    T, qv, ql, qi, qr, qsn, qg, pm = cols(st, ("T", "qv", "ql", "qi", "qr", "qs", "qg", "pm"))
    ql, qi = np.maximum(ql, 0.0), np.maximum(qi, 0.0)
    cf = np.clip(ql * 500.0, 0.0, 0.7)
    r = gm.radcouple(T, pm, cf, 0.2 * cf, qv, ql, qi, 0.0 * ql, 0.0 * qi, np.maximum(qr, 0), np.maximum(qsn, 0),
                     np.maximum(qg, 0), np.full_like(T, 5e7), np.full_like(T, 1e3))
    for k in ("rad_ql", "rad_qi", "rad_qr", "rad_qs", "rad_qg"):
        assert r[k].min() >= 0.0 and r[k].max() <= gm.QC_MAX
    assert np.all((r["rad_cf"] == 0.0) | (r["rad_cf"] >= 1e-5)) and r["rad_cf"].max() <= 1.0
    assert r["rad_rl"].min() >= 2.5e-6 and r["rad_rl"].max() <= 60e-6
    assert r["rad_ri"].min() >= 5e-6 and r["rad_ri"].max() <= 150e-6


def test_aer_activation_monotone_in_updraft():
    t = np.full(5, 285.0)
    pl = np.full(5, 9.0e4)
    qsw, _ = om.qsat(t, pl)
    zm = np.array([0.0, 500.0, 1000.0, 2000.0, 4000.0])
    n1, _, s1 = gm.aer_activation(pl, t, 0.9 * qsw, zm, np.full(5, 0.2))
    n2, _, s2 = gm.aer_activation(pl, t, 0.9 * qsw, zm, np.full(5, 2.0))
    ntot = sum(m[0] * np.exp(-zm / m[1]) for m in gm.AER_MODES)
    assert np.all(n2 > n1) and np.all(s2 > s1)
    assert np.all(n2 < ntot) and np.all(n1 > 0.0)


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


def test_gf_shallow_conserves_and_finds_clouds():
    """cup_gf_sh on the synthetic columns: column moist static energy and water conserved to
    round-off, vapour non-negative, cloud base at or above the source level and below the
    top, detrained condensate only in the top layer"""
    from oracle import gf_shallow as gf
    st = moist_state(SHAPE, seed=3)
    T, qv, pl, zm, dp = cols(st, ("T", "qv", "pm", "zm", "delp"), n=60)
    kp = np.where(zm < 1000.0, np.arange(T.shape[0])[:, None], T.shape[0] - 1).min(axis=0).astype(float)
    r = gf.cup_gf_sh(450.0, T, qv, pl, zm, dp, kp, np.full(T.shape[1], 25.0))
    act = r["ktop"] >= 0
    assert act.sum() > 0
    assert np.all(r["ktop"][act] < r["kbcon"][act]) and np.all(r["kbcon"][act] <= r["k22"][act])
    h0 = ((om.CP_AIR * T + om.HLV * qv) * dp).sum(0)
    h1 = ((om.CP_AIR * r["t"] + om.HLV * r["qv"]) * dp).sum(0)
    w0 = (qv * dp).sum(0)
    w1 = ((r["qv"] + r["dqlcn"] + r["dqicn"]) * dp).sum(0)
    assert np.allclose(h1, h0, rtol=1e-14) and np.allclose(w1, w0, rtol=1e-14)
    assert r["qv"].min() >= 0.0
    cond = r["dqlcn"] + r["dqicn"]
    for c in np.nonzero(act)[0]:
        nz = np.nonzero(cond[:, c])[0]
        assert set(nz) <= {int(r["ktop"][c])}
