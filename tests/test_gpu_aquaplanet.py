"""The Aquaplanet configuration's coupled step on the device (BASELINE.json configs[3]:
dycore + moist column physics): one fv_dynamics call followed by the moist column step
(Dycore::moist_physics: gfdl_1m on pt, the six moist tracers, delp, delz and the layer
pressure from pe), against oracle fv_dynamics followed by oracle gfdl_1m.  Bar as the
dycore step test: each field within 1e-9 of its mean magnitude; column water plus
surface precipitation conserved by the moist step on the device."""
import importlib

import numpy as np
import pytest

from conftest import metrics_of
from oracle import NG
from oracle import fv_dynamics as fvd
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
        sc = d.scalars()
        g = fvd.Grid(d.N, 1, 1, ms, sc["corner_w"], sc["da_min_c"], d.nj, d.pitch)
        ref = fvd.fv_dynamics(st, ak, bk, g, dict(NL, nq=nq))
        J, I = slice(NG, NG + d.ny), slice(NG, NG + d.nx)
        for s in range(d.nsub):
            pe = ref["pe"][s]
            sp = [ref["q"][s][n * npz:(n + 1) * npz] for n in range(6)]
            (T, *qs), rp = om.gfdl_1m(ref["pt"][s], ref["delp"][s], ref["delz"][s], 0.5 * (pe[1:] + pe[:-1]),
                                      *sp, dt)
            a, b = got["pt"][s][:, J, I], T[:, J, I]
            assert np.abs(a - b).max() <= 1e-9 * np.abs(b).mean(), ("pt", s)
            for n in range(6):
                a = got["q"][s][n * npz:(n + 1) * npz][:, J, I]
                b = qs[n][:, J, I]
                scale = max(np.abs(b).mean(), 1e-30)
                assert np.abs(a - b).max() <= 1e-9 * scale + 1e-18, ("q", n, s)
            # the device moist step conserves column water + precipitation
            w0 = np.einsum("kji,kji->ji", sum(before["q"][s][n * npz:(n + 1) * npz] for n in range(6)),
                           before["delp"][s]) / om.GRAV
            w1 = np.einsum("kji,kji->ji", sum(got["q"][s][n * npz:(n + 1) * npz] for n in range(6)),
                           before["delp"][s]) / om.GRAV + prec[s]
            assert np.abs(w1 - w0)[J, I].max() <= 1e-12 * np.abs(w0).max()
    finally:
        d.close()
