"""Williamson et al. (1992) shallow-water test case 2 -- steady-state nonlinear zonal
geostrophic flow -- run on the device c_sw / d_sw stencils with the pressure-gradient stencils
and the cubed-sphere halo exchanges, in dyn_core's order (VERDICT r05 next #4a): a published
case with an analytic solution (the initial state), pinning the acoustic dynamics
independently of this package's own oracle.

Shallow water on one layer (npz = 1, FV3's shallow_water mode): delp holds the fluid depth
h (m), pt = 1 and w = 0 ride along.  The pressure gradient of a single layer with the
interface "pressures" pk = (0, h) and geopotentials gz = (phis + g h, phis) is, through FV3's
finite-volume form (Lin 1997; p_grad_c / nh_p_grad, whose expression is linear in gz and pk),

    dt / (h_1 + h_2) [(gz_b1 - gz_t2)(pk_b2 - pk_t1) + (gz_t1 - gz_b2)(pk_b1 - pk_t2)]
      = dt [(phis_1 - phis_2) + g (h_1 - h_2)],

the shallow-water gradient of g (h + h_s) exactly; the non-hydrostatic part (pp = 0) adds
nothing.  One acoustic sub-step, as Dycore::step runs it (dycore.hip acoustic()):

    c_sw -> gz, pk from delpc -> p_grad_c -> uc/vc exchange ('X') -> d_sw ->
    delp / pt / w exchange -> gz, pk from delp -> nh_p_grad -> u/v exchange ('d')

(gz and pk are formed on the host from the downloaded depth: two planes per stage, the
stencils themselves are the product's.)

Set-up (Williamson 1992 section 3.2, alpha = 0: the product's Coriolis parameter is
2 Omega sin(lat)): u = u0 cos(lat), v = 0, g h = g h0 - (a Omega u0 + u0^2 / 2) sin^2(lat),
u0 = 2 pi a / 12 days, g h0 = 2.94e4 m^2 s^-2; D-grid winds projected onto the edges from the
grid corners' positions as state.py does, h at the cell centres.  After 5 days the normalised
l1 / l2 / l_inf errors of h against the initial state.

Bars.  Williamson (1992) asks for the steady state to be held; second-order FV schemes on the
gnomonic cubed sphere hold it to normalised l2 errors of order 1e-4 at about 2 degrees (C48),
with their largest errors at the cube corners (Putman & Lin 2007 section 5, the motivation for
their grid modifications).  Measured here (MI355X): l2 5.2e-4 / 3.5e-4 / 2.5e-4 at C24 / C48 /
C96 and l_inf 2.7e-3 / 2.9e-3 / 3.2e-3 -- a ~9 m height error at the cube corners that sets in
within the first ten sub-steps and does not shrink with resolution (its area does), the cells
N / 8 away from every tile edge converging at first to second order (3.4e-4, 1.3e-4, 7.9e-5).
The bars: the steady state held (no growth from day 1 to day 5), l2 <= 5e-4 and l_inf <= 5e-3
at C48, global l2 falling with resolution, the interior l2 by >= 2x (C24 -> C48) and >= 1.5x
(C48 -> C96), mass moved only through the cube-corner cells (<= 1e-5 over 5 days, second order).
The corner error is the restated algorithm's (product and oracle agree sub-step by sub-step,
test_williamson2_substeps_match_oracle), so it flags the corner forms of d2a2c_vect / a2b_ord4
as this build restates them -- FV3's own source is not available here to compare.
"""
import numpy as np
import pytest

from oracle import NG

pytestmark = pytest.mark.gpu

A = 6371.0e3
G = 9.80665
OMEGA = 2.0 * np.pi / 86164.0
DAY = 86400.0
U0 = 2.0 * np.pi * A / (12.0 * DAY)
GH0 = 2.94e4


def _unit(v):
    n = np.linalg.norm(v, axis=-1, keepdims=True)
    return v / np.where(n > 0.0, n, 1.0)


def _depth(lat):
    return (GH0 - (A * OMEGA * U0 + 0.5 * U0 ** 2) * np.sin(lat) ** 2) / G


def setup_case(d):
    """initial u, v (D grid), h (cell centres) as (nsub, 1, nj, pitch) planes, halos included"""
    H = NG + 1
    xyz = d.corner_xyz()
    nj, pitch = d.nj, d.pitch
    jj, ii = np.meshgrid(np.arange(nj), np.arange(pitch), indexing="ij")
    o = H - NG
    u, v = d.zeros(1), d.zeros(1)
    for s in range(d.nsub):
        P = xyz[s]

        def corner(dj, di):
            return P[np.clip(jj + o + dj, 0, P.shape[0] - 1), np.clip(ii + o + di, 0, P.shape[1] - 1)]

        c00, c10, c01 = corner(0, 0), corner(0, 1), corner(1, 0)
        for out, (pa, pb) in ((u, (c00, c10)), (v, (c00, c01))):
            mid = _unit(pa + pb)
            lat = np.arcsin(np.clip(mid[..., 2], -1.0, 1.0))
            lon = np.arctan2(mid[..., 1], mid[..., 0])
            ev = _unit(pb - pa)
            elon = np.stack([-np.sin(lon), np.cos(lon), np.zeros_like(lon)], -1)
            out[s, 0] = U0 * np.cos(lat) * np.sum(elon * ev, axis=-1)
    h = _depth(d.metric("lat"))[:, None]
    for a in (u, v, h):
        np.nan_to_num(a, copy=False)
    return u, v, h


class ShallowWater:
    """one-layer FV3 dyn_core on the device stencils (see the module docstring)"""

    def __init__(self, d, dt_sub, dddmp=0.0, d2_bg=0.0):
        self.d, self.dt, self.dddmp, self.d2_bg = d, dt_sub, dddmp, d2_bg
        self.phis = d.zeros(1)
        d.upload("phis", self.phis)
        d.upload("_sw_pp", d.zeros(2))
        self.first = True

    def _levels(self, depth, gz, pk):
        self.d.upload(gz, np.concatenate([self.phis + G * depth, self.phis], axis=1))
        self.d.upload(pk, np.concatenate([np.zeros_like(depth), depth], axis=1))

    def substep(self):
        d, dt = self.d, self.dt
        if self.first:
            d.halo_update("u:d,v:d,delp:c,pt:c,w:c")
            self.first = False
        d.stencil("c_sw", ["delp", "pt", "w", "u", "v", "uc", "vc", "ua", "va", "_sw_ut", "_sw_vt", "_sw_delpc",
                           "_sw_ptc", "_sw_wc"], [0.5 * dt])
        self._levels(d.download("_sw_delpc"), "_sw_gzc", "_sw_pkc")
        d.stencil("p_grad_c", ["_sw_delpc", "_sw_pkc", "_sw_gzc", "uc", "vc"], [0.5 * dt])
        d.halo_update("uc:X,vc:X")
        d.stencil("d_sw", ["delp", "pt", "w", "u", "v", "uc", "vc", "ua", "va", "crx", "cry", "xfx", "yfx", "cx",
                           "cy", "mfx", "mfy", "_sw_ke"], [dt, self.dddmp, self.d2_bg, 6, 6, 6, 6])
        d.halo_update("delp:c,pt:c,w:c")
        self._levels(d.download("delp"), "_sw_gz", "_sw_pk")
        d.stencil("nh_p_grad", ["_sw_pp", "_sw_pk", "_sw_gz", "delp", "u", "v"], [dt, 0.0])
        d.halo_update("u:d,v:d")


def norms(h, h0, area, d):
    c = (Ellipsis, slice(NG, NG + d.ny), slice(NG, NG + d.nx))
    err, w, ref = h[c] - h0[c], area[c], h0[c]
    return dict(l1=float((np.abs(err) * w).sum() / (np.abs(ref) * w).sum()),
                l2=float(np.sqrt((err ** 2 * w).sum() / (ref ** 2 * w).sum())),
                linf=float(np.abs(err).max() / np.abs(ref).max()),
                mass=float(abs((h[c] * w).sum() - (ref * w).sum()) / (ref * w).sum()),
                finite=bool(np.all(np.isfinite(h[c]))))


def _interior_l2(h, h0, area, d):
    """l2 of the height error over the cells at least N / 8 cells from every tile edge"""
    c = (Ellipsis, slice(NG, NG + d.ny), slice(NG, NG + d.nx))
    jj, ii = np.meshgrid(np.arange(d.ny), np.arange(d.nx), indexing="ij")
    N = d.N
    m = np.minimum(np.minimum(ii, N - 1 - ii), np.minimum(jj, N - 1 - jj)) >= N // 8
    e, w, ref = (h[c] - h0[c])[:, 0][:, m], area[c][:, 0][:, m], h0[c][:, 0][:, m]
    return float(np.sqrt((e ** 2 * w).sum() / (ref ** 2 * w).sum()))


def run_days(pkg, npx, dt_sub, days=(1.0, 5.0)):
    """{day: norms} of one run, the interior l2 added"""
    d = pkg.Domain(npx=npx, npz=1, nq=1)
    try:
        u, v, h = setup_case(d)
        for n, a in (("u", u), ("v", v), ("delp", h), ("pt", np.ones(d.shape(1))), ("w", d.zeros(1))):
            d.upload(n, a)
        sw = ShallowWater(d, dt_sub)
        area = d.metric("area")[:, None]
        out, done = {}, 0
        for day in days:
            n = int(round(day * DAY / dt_sub))
            while done < n:
                sw.substep()
                done += 1
            hh = d.download("delp")
            r = norms(hh, h, area, d)
            r["l2_interior"] = _interior_l2(hh, h, area, d)
            out[day] = r
        return out
    finally:
        d.close()


def test_williamson2_steady_geostrophic_flow(pkg, require_gpu):
    runs = {c: run_days(pkg, c + 1, dt) for c, dt in ((24, 900.0), (48, 450.0), (96, 225.0))}
    for c, r in runs.items():
        print(f"\nWilliamson 2, alpha = 0, C{c}: day 1 {r[1.0]}\n  day 5 {r[5.0]}")
    r24, r48, r96 = (runs[c][5.0] for c in (24, 48, 96))
    assert all(r["finite"] for r in (r24, r48, r96))
    # the steady state is held: no drift or growth between day 1 and day 5
    for c in runs:
        assert runs[c][5.0]["l2"] <= 1.5 * runs[c][1.0]["l2"], (c, runs[c])
    # accuracy at C48 (measured: l2 3.5e-4, l_inf 2.9e-3)
    assert r48["l2"] <= 5e-4 and r48["linf"] <= 5e-3, r48
    # convergence: global l2 falls with resolution (measured 5.2e-4, 3.5e-4, 2.5e-4: the
    # cube-corner error ~9 m does not shrink, its area does); away from the tile edges the error
    # converges at first to second order (measured 3.4e-4, 1.3e-4, 7.9e-5)
    assert r24["l2"] > r48["l2"] > r96["l2"], (r24["l2"], r48["l2"], r96["l2"])
    assert r24["l2_interior"] / r48["l2_interior"] >= 2.0, (r24["l2_interior"], r48["l2_interior"])
    assert r48["l2_interior"] / r96["l2_interior"] >= 1.5, (r48["l2_interior"], r96["l2_interior"])
    # mass: the flux form moves it only through the cube-corner cells, each tile forming the
    # corner-adjacent fluxes from its own copy_corners fill (as in Williamson 1; measured 8.9e-6,
    # 2.4e-6, 6.1e-7 over 5 days: second order)
    assert r48["mass"] <= 1e-5, r48
    assert r24["mass"] / r48["mass"] >= 3.0 and r48["mass"] / r96["mass"] >= 3.0, (r24["mass"], r48["mass"],
                                                                                    r96["mass"])


def _oracle_substep(g, st, phis, dt, first):
    """the same sub-step on the numpy oracle (oracle/sw_core.py, oracle/nh_core.py, oracle/halo.py)"""
    from oracle import fv_dynamics as fvd
    from oracle import nh_core, sw_core
    from oracle.halo import fill_vector, sync_edges
    if first:
        fvd._halo(g, st, [("u", "d"), ("v", "d"), ("delp", "c"), ("pt", "c"), ("w", "c")])
    def lv(dp, s):
        return np.concatenate([phis[s] + G * dp, phis[s]]), np.concatenate([np.zeros_like(dp), dp])

    for s in range(g.nsub):
        m, sub, P = g.ms[s], g.subs[s], g.P[s]
        c = sw_core.c_sw(st["delp"][s], st["pt"][s], st["u"][s], st["v"][s], st["w"][s], sub, m, g.nx, g.ny, 0.5 * dt)
        gz, pk = lv(c["delpc"], s)
        st["uc"][s], st["vc"][s] = nh_core.p_grad_c(c["uc"], c["vc"], c["delpc"], pk, gz, m, P, 0.5 * dt)
        st["ua"][s], st["va"][s] = c["ua"], c["va"]
    sync_edges(st["uc"], st["vc"], g.layout, "cgrid")
    fill_vector(st["uc"], st["vc"], g.layout, "cgrid")
    for s in range(g.nsub):
        m, sub = g.ms[s], g.subs[s]
        r = sw_core.d_sw(st["delp"][s], st["pt"][s], st["u"][s], st["v"][s], st["w"][s], st["uc"][s], st["vc"][s],
                         st["ua"][s], st["va"][s], sub, m, g.nx, g.ny, dt, (6, 6, 6, 6), 0.0, 0.0, g.da_min_c)
        for name in ("delp", "pt", "w", "u", "v"):
            st[name][s] = r[name]
    fvd._halo(g, st, [("delp", "c"), ("pt", "c"), ("w", "c")])
    for s in range(g.nsub):
        gz, pk = lv(st["delp"][s], s)
        st["u"][s], st["v"][s] = nh_core.nh_p_grad(st["u"][s], st["v"][s], np.zeros_like(gz), gz, st["delp"][s], pk,
                                                   dt, 0.0, g.P[s], g.ms[s], g.corner_w[s])
    fvd._halo(g, st, [("u", "d"), ("v", "d")])


def test_williamson2_substeps_match_oracle(pkg, require_gpu):
    """C12: four shallow-water sub-steps through the device stencils (c_sw, p_grad_c, d_sw,
    nh_p_grad and the exchanges) equal the same sub-steps of the oracle to 1e-11 of each
    field's magnitude -- the W2 norms above are the restated FV3 algorithm's"""
    from conftest import metrics_of, oracle_scalars
    from oracle import fv_dynamics as fvd
    d = pkg.Domain(npx=13, npz=1, nq=1)
    try:
        u, v, h = setup_case(d)
        init = {"u": u, "v": v, "delp": h, "pt": np.ones(d.shape(1)), "w": d.zeros(1)}
        for n, a in init.items():
            d.upload(n, a)
        sw = ShallowWater(d, 3600.0)
        sc = oracle_scalars(d)
        g = fvd.Grid(d.N, 1, 1, metrics_of(d), sc["corner_w"], sc["da_min_c"], d.nj, d.pitch)
        st = {k: a.copy() for k, a in init.items()}
        for k in ("uc", "vc", "ua", "va"):
            st[k] = d.zeros(1)
        phis = d.zeros(1)
        c = (Ellipsis, slice(NG, NG + d.ny), slice(NG, NG + d.nx))
        for it in range(4):
            sw.substep()
            _oracle_substep(g, st, phis, 3600.0, it == 0)
            for k in ("delp", "u", "v"):
                a, b = d.download(k)[c], st[k][c]
                err = np.abs(a - b).max() / np.abs(b).max()
                assert err <= 1e-11, (it, k, err)
            moved = np.abs(st["delp"][c] - h[c]).max()
        assert moved > 1e-3  # the state moved (corner adjustment): the comparison is not of a copy
    finally:
        d.close()
