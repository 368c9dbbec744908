"""CPU properties of the oracle dycore step (no GPU): the oracle is the parity
checker, so it is held to the properties FV3 guarantees by construction.

* decomposition invariance: 1x1 and 2x2 sub-domains per tile give identical bits
  (halo widths and tile-edge zones are layout independent);
* tile-edge consistency of the C-grid winds produced by d2a2c_vect at a shared edge;
* dry-mass bookkeeping: the remap keeps each column's mass; the global dry mass drifts by
  1.5e-11 of itself per step (with the C-grid tile-edge synchronisation; 2.8e-7 without it,
  checked here too), the residual being the tile-edge PPM fluxes next to the cube corners,
  whose halo inputs each tile fills from its own copy_corners.
"""
import importlib

import numpy as np

from conftest import metrics_of, oracle_scalars
from oracle import NG
from oracle import fv_dynamics as fvd
from oracle import sw_core
from oracle.util import Plane

NL = dict(n_split=6, dt_atmos=900.0, hord_mt=6, hord_vt=6, hord_tm=6, hord_dp=6, hord_tr=6, dddmp=0.2, d2_bg=0.0,
          p_fac=0.05, dz_min=2.0, fill=1, nq=2)


def _setup(pkg, lx, ly, npz=10, npx=13):
    state = importlib.import_module(pkg.__name__ + ".state")
    d = pkg.Domain(npx=npx, npz=npz, nq=2, layout_x=lx, layout_y=ly, host_only=1)
    ak, bk, ks = state.hybrid_levels(npz)
    st = state.jablonowski_williamson(d, ak, bk)
    ms = metrics_of(d)
    sc = oracle_scalars(d)
    g = fvd.Grid(d.N, lx, ly, ms, sc["corner_w"], sc["da_min_c"], d.nj, d.pitch)
    return d, st, ak, bk, ms, g


def test_oracle_step_decomposition_invariant(pkg):
    d1, st1, ak, bk, ms1, g1 = _setup(pkg, 1, 1)
    d2, st2, _, _, ms2, g2 = _setup(pkg, 2, 2)
    o1 = fvd.fv_dynamics(st1, ak, bk, g1, NL)
    o2 = fvd.fv_dynamics(st2, ak, bk, g2, NL)
    n = d2.nx
    for s2, sub in enumerate(g2.subs):
        t, io, jo = sub["tile"], sub["ioff"], sub["joff"]
        for k in ("u", "v", "w", "delz", "pt", "delp", "q", "ua", "va", "omga", "ps", "pe"):
            a = o2[k][s2][:, NG:NG + n, NG:NG + n]
            b = o1[k][t][:, NG + jo:NG + jo + n, NG + io:NG + io + n]
            assert np.array_equal(a, b), f"{k} differs on sub {s2}"


def test_d2a2c_shared_edge_consistent(pkg):
    """uc, ut at a shared tile edge and one cell either side agree between the two tiles."""
    d, st, ak, bk, ms, g = _setup(pkg, 1, 1, npz=2)
    fvd._halo(g, st, [("u", "d"), ("v", "d")])
    N = d.N
    P0 = Plane(g.subs[0], N, N, d.nj, d.pitch)
    P1 = Plane(g.subs[1], N, N, d.nj, d.pitch)
    r0 = sw_core.d2a2c_vect(st["u"][0], st["v"][0], P0, ms[0])
    r1 = sw_core.d2a2c_vect(st["u"][1], st["v"][1], P1, ms[1])
    for idx in (2, 4):  # uc, ut: tile 0 columns N-1..N+1 == tile 1 columns -1..1 (east/west neighbours)
        a = r0[idx][:, NG:NG + N, NG + N - 1:NG + N + 2]
        b = r1[idx][:, NG:NG + N, NG - 1:NG + 2]
        assert np.abs(a - b).max() <= 1e-13 * np.abs(b).max()


def test_oracle_mass_and_column_bookkeeping(pkg):
    d, st, ak, bk, ms, g = _setup(pkg, 1, 1)
    o = fvd.fv_dynamics(st, ak, bk, g, NL)
    n = d.nx

    def mass(dp):
        return sum((dp[s][:, NG:NG + n, NG:NG + n] * ms[s]["area"][NG:NG + n, NG:NG + n]).sum() for s in range(6))
    m0, m1 = mass(st["delp"]), mass(o["delp"])
    assert abs(m1 - m0) / m0 < 3e-11
    # without the tile-edge synchronisation of uc / vc the drift is 2e4 times larger
    o2 = fvd.fv_dynamics(st, ak, bk, g, dict(NL, edge_sync=0))
    assert abs(mass(o2["delp"]) - m0) / m0 > 1e-7
    # after the remap every column sums to ps - ptop and sits on the hybrid levels
    for s in range(6):
        ps = o["ps"][s, 0, NG:NG + n, NG:NG + n]
        col = o["delp"][s][:, NG:NG + n, NG:NG + n].sum(axis=0)
        np.testing.assert_allclose(col, ps - ak[0], rtol=1e-13)
        pe = o["pe"][s][:, NG:NG + n, NG:NG + n]
        np.testing.assert_allclose(pe[1:-1], ak[1:-1, None, None] + bk[1:-1, None, None] * ps[None], rtol=1e-14)
