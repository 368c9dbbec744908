"""Held-Suarez forcing (experiment geos_hs, experiments.yaml:8-29)
on the device against the HS94 restatement oracle/held_suarez.py, from the JW06 state.
Bar: 1e-13 relative per field (same expression order; exp/log/sin/cos from ocml vs
glibc differ in the last place)."""
import importlib

import numpy as np
import pytest

from oracle import NG
from oracle.held_suarez import held_suarez as hs_ref

pytestmark = pytest.mark.gpu


def test_held_suarez_forcing_matches_oracle(pkg, require_gpu):
    state = importlib.import_module(pkg.__name__ + ".state")
    npz, dt = 20, 900.0
    d = pkg.Domain(npx=25, npz=npz, nq=1)
    try:
        ak, bk, ks = state.hybrid_levels(npz)
        st = state.jablonowski_williamson(d, ak, bk)
        lat = d.metric("lat")
        # hydrostatic interfaces over a surface pressure that varies with the grid
        ps = 1.0e5 + 1.5e3 * np.cos(3.0 * lat) * np.sin(2.0 * d.metric("lon"))
        st["pe"] = ak[None, :, None, None] + bk[None, :, None, None] * ps[:, None]
        d.set_vertical(ak, bk, ks)
        for k in ("pe", "pt", "u", "v"):
            d.upload(k, st[k])
        d.stencil("held_suarez", ["pe", "pt", "u", "v"], [dt])
        got = {k: d.download(k) for k in ("pt", "u", "v")}
        for s in range(d.nsub):
            pt, u, v = hs_ref(st["pe"][s], st["pt"][s], st["u"][s], st["v"][s], lat[s], d.nx, d.ny, dt)
            J, I = slice(NG, NG + d.ny + 1), slice(NG, NG + d.nx + 1)
            for name, ref in (("pt", pt), ("u", u), ("v", v)):
                a, b = got[name][s][:, J, I], ref[:, J, I]
                err = np.abs(a - b).max() / np.abs(b).max()
                assert err <= 1e-13, (name, s, err)
            # the forcing acts: T relaxes towards T_eq, boundary-layer winds slow down
            assert not np.array_equal(pt[:, J, I], st["pt"][s][:, J, I])
            wind = lambda a, b: np.abs(a[-1, J, I]).sum() + np.abs(b[-1, J, I]).sum()  # noqa: E731
            assert wind(u, v) < wind(st["u"][s], st["v"][s])
    finally:
        d.close()
