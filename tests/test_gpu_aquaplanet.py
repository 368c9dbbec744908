"""The Aquaplanet configuration's coupled step on the device (BASELINE.json configs[3]:
dycore + moist column physics): one fv_dynamics call followed by the moist physics in
GEOS's GFDL_1M order (Dycore::moist_physics: aer_activation, evap_subl_pdf, the GFDL cloud
microphysics driver, radcouple, on pt, the six moist tracers, the anvil condensate and
cloud fractions, delp, delz, pe, w), against oracle fv_dynamics followed by
oracle/geos_moist.py aquaplanet_physics.  Bar: each field within 1e-9 of its scale (and
the reference's 0.01 % per value); column water plus surface precipitation conserved by
the moist step on the device."""
import importlib

import numpy as np
import pytest

from conftest import metrics_of, oracle_scalars
from oracle import NG
from oracle import fv_dynamics as fvd
from oracle import geos_moist as gm
from oracle import moist as om

pytestmark = pytest.mark.gpu
NL = dict(n_split=6, dt_atmos=900.0, hord_mt=6, hord_vt=6, hord_tm=6, hord_dp=6, hord_tr=6, dddmp=0.2, d2_bg=0.0,
          p_fac=0.05, dz_min=2.0, fill=1)


def test_aquaplanet_step_matches_oracle(pkg, require_gpu):
    state = importlib.import_module(pkg.__name__ + ".state")
    npx, npz, nq, dt = 13, 12, 6, 900.0
    d = pkg.Domain(npx=npx, npz=npz, nq=nq, dt=dt)
    try:
        ak, bk, ks = state.hybrid_levels(npz)
        st = state.jablonowski_williamson(d, ak, bk)
        state.aquaplanet_tracers(d, st, ak, bk)
        d.set_vertical(ak, bk, ks)
        for k, v in st.items():
            d.upload(k, v)
        d.step(1)
        before = {k: d.download(k) for k in ("q", "delp")}
        d.stencil("aquaplanet_physics", [], [dt])
        got = {k: d.download(k) for k in ("pt", "q")}
        prec = sum(d.download(n)[:, 0] for n in ("prec_rain", "prec_snow", "prec_graupel", "prec_ice"))
        ms = metrics_of(d)
        sc = oracle_scalars(d)
        g = fvd.Grid(d.N, 1, 1, ms, sc["corner_w"], sc["da_min_c"], d.nj, d.pitch)
        ref = fvd.fv_dynamics(st, ak, bk, g, dict(NL, nq=nq))
        J, I = slice(NG, NG + d.ny), slice(NG, NG + d.nx)
        gotx = {k: d.download(k) for k in ("qlcn", "qicn", "clls", "clcn", "nactl", "rad_cf", "rad_ql", "rad_ri",
                                           "prec_rain", "prec_snow")}

        def close(a, b, what, floor=1e-30):
            scale = max(np.abs(b).max(), floor)
            assert np.abs(a - b).max() <= 1e-9 * scale + 1e-18, (what, np.abs(a - b).max() / scale)
            np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-9 * scale + 1e-18, err_msg=str(what))

        for s in range(d.nsub):
            c = lambda a: a[..., J, I]
            sp = [c(ref["q"][s][n * npz:(n + 1) * npz]) for n in range(6)]
            o = gm.aquaplanet_physics(dt, c(ref["pt"][s]), *sp, c(ref["delp"][s]), c(ref["delz"][s]),
                                      c(ref["pe"][s]), c(ref["w"][s]))
            close(got["pt"][s][:, J, I], o["t"], ("pt", s))
            for n, k in enumerate(("qv", "ql", "qr", "qi", "qs", "qg")):
                close(got["q"][s][n * npz:(n + 1) * npz][:, J, I], o[k], (k, s))
            for k in ("qlcn", "qicn", "clls", "clcn", "nactl", "rad_cf", "rad_ql", "rad_ri"):
                close(gotx[k][s][:, J, I], o[k], (k, s))
            for k in ("prec_rain", "prec_snow"):   # (melted-out species arrive as round-off)
                cw = (sum(sp) * c(ref["delp"][s])).sum(0).max() / om.GRAV
                close(gotx[k][s][0][J, I], o[k], (k, s), floor=1e-6 * cw)
            # the device moist step conserves column water + precipitation
            w0 = np.einsum("kji,kji->ji", sum(before["q"][s][n * npz:(n + 1) * npz] for n in range(6)),
                           before["delp"][s]) / om.GRAV
            w1 = np.einsum("kji,kji->ji", sum(got["q"][s][n * npz:(n + 1) * npz] for n in range(6)),
                           before["delp"][s]) / om.GRAV + prec[s]
            assert np.abs(w1 - w0)[J, I].max() <= 1e-12 * np.abs(w0).max()
    finally:
        d.close()


def test_aquaplanet_c180_l72_coupled_step(pkg, require_gpu):
    """BASELINE.json config 4's grid, Aquaplanet C180 L72 (all six tiles on one GPU), one
    coupled step on the device: fv_dynamics then the moist physics.  Checked: the state is
    finite and bounded, the six species are non-negative, the moist step conserves column
    water + surface precipitation to 1e-12, and 200 sampled columns equal the oracle moist
    chain (oracle/geos_moist.aquaplanet_physics, column-wise) applied to the HIP dycore's
    output at those columns, at the 1e-9-of-scale bar (and the reference's 0.01 %,
    physics_standalone.py:132-144).  Anchor: aquaplanet.py:99-178 (the C180 L72 run)."""
    state = importlib.import_module(pkg.__name__ + ".state")
    npx, npz, nq, dt = 181, 72, 6, 450.0
    d = pkg.Domain(npx=npx, npz=npz, nq=nq, dt=dt)
    try:
        ak, bk, ks = state.hybrid_levels(npz)
        st = state.jablonowski_williamson(d, ak, bk)
        state.aquaplanet_tracers(d, st, ak, bk)
        d.set_vertical(ak, bk, ks)
        for k, v in st.items():
            d.upload(k, v)
        del st
        d.step(1)
        n = d.N
        J, I = slice(NG, NG + n), slice(NG, NG + n)
        dyn = {k: d.download(k)[..., J, I] for k in ("pt", "q", "delp", "delz", "pe", "w")}
        d.stencil("aquaplanet_physics", [], [dt])
        got = {k: d.download(k)[..., J, I] for k in ("pt", "q")}
        gotx = {k: d.download(k)[..., J, I] for k in ("qlcn", "qicn", "clls", "clcn", "nactl", "rad_cf", "rad_ql",
                                                      "rad_ri")}
        prec = {k: d.download(k)[:, 0][:, J, I] for k in ("prec_rain", "prec_snow", "prec_graupel", "prec_ice")}
        for k, v in list(got.items()) + list(gotx.items()) + list(prec.items()):
            assert np.all(np.isfinite(v)), f"{k} not finite"
        assert 150.0 < got["pt"].min() and got["pt"].max() < 400.0
        sp = lambda a, m: a[:, m * npz:(m + 1) * npz]
        for m in range(6):
            assert sp(got["q"], m).min() >= 0.0, ("negative species", m, sp(got["q"], m).min())
        # column water + precipitation (the moist step does not change delp)
        w0 = sum(sp(dyn["q"], m) for m in range(6))
        w1 = sum(sp(got["q"], m) for m in range(6))
        c0 = np.einsum("skji,skji->sji", w0, dyn["delp"]) / om.GRAV
        c1 = np.einsum("skji,skji->sji", w1, dyn["delp"]) / om.GRAV + sum(prec.values())
        err = np.abs(c1 - c0).max() / np.abs(c0).max()
        assert err <= 1e-12, f"column water + precipitation not conserved: {err:.3e}"
        # 200 sampled columns against the column-wise oracle chain
        r = np.random.default_rng(180)
        cs, cj, ci = r.integers(0, 6, 200), r.integers(0, n, 200), r.integers(0, n, 200)
        col = lambda a: np.ascontiguousarray(a[cs, :, cj, ci].T)  # (nk, 200)
        qs = [col(sp(dyn["q"], m)) for m in range(6)]
        o = gm.aquaplanet_physics(dt, col(dyn["pt"]), *qs, col(dyn["delp"]), col(dyn["delz"]), col(dyn["pe"]),
                                  col(dyn["w"]))

        def close(a, b, what, floor=1e-30):
            scale = max(np.abs(b).max(), floor)
            assert np.abs(a - b).max() <= 1e-9 * scale + 1e-18, (what, np.abs(a - b).max() / scale)
            np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-9 * scale + 1e-18, err_msg=str(what))

        close(col(got["pt"]), o["t"], "pt")
        for m, k in enumerate(("qv", "ql", "qr", "qi", "qs", "qg")):
            close(col(sp(got["q"], m)), o[k], k)
        for k in gotx:
            close(col(gotx[k]), o[k], k)
        cw = (sum(qs) * col(dyn["delp"])).sum(0).max() / om.GRAV
        for k in ("prec_rain", "prec_snow"):
            close(prec[k][cs, cj, ci], o[k], k, floor=1e-6 * cw)
        print("Aquaplanet C180 L72: water conservation", f"{err:.1e}", "precip max",
              {k: float(v.max()) for k, v in prec.items()})
    finally:
        d.close()
