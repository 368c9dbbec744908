"""Oracle: one fv_dynamics call (non-hydrostatic FV3 as configured by the GEOS
Held-Suarez namelist) composed from the oracle pieces — TEST INFRASTRUCTURE ONLY.

Sequence (FV3 fv_dynamics.F90 -> dyn_core.F90 -> tracer_2d_1l -> Lagrangian_to_Eulerian
-> cubed_to_latlon, the call stack of SURVEY.md §8(a)):

  entry      pkz from the nh state, pt -> virtual potential temperature, dp1 = delp
  dyn_core   n_split acoustic sub-steps of
               c_sw, update_dz_c, riem_solver_c, p_grad_c,
               d_sw, update_dz_d, riem_solver3, pk3/pe halo, nh_p_grad
  tracers    tracer_2d_1l with the accumulated mass fluxes and Courant numbers
  remap      Lagrangian_to_Eulerian (kord 9, T_v in log p)
  exit       T = T_v / (1 + zvir q), omega = delp / delz * w, A-grid winds (c2l_ord4)

All arrays are (nsub, nk, nj, pitch) in the product's HBM layout; sub-domains are
the single-rank Layout order.  The halo fills are the oracle's own (halo.py).
"""
import numpy as np

from . import NG
from . import fv_mapz, nh_core, sw_core, tp_core
from . import grid as og
from .halo import Layout, fill_scalar, fill_vector, sync_edges
from .util import Plane, sh

np.seterr(all="ignore")

GRAV = nh_core.GRAV
RDGAS = nh_core.RDGAS
KAPPA = nh_core.KAPPA
ZVIR = (8314.47 / 18.015) / (8314.47 / 28.965) - 1.0


class Grid:
    """Everything the oracle needs about the decomposition and metrics."""

    def __init__(self, N, lx, ly, ms, corner_w, da_min_c, nj, pitch, da_min=None):
        self.layout = Layout(N, lx, ly)
        self.subs = self.layout.subs()
        self.nx, self.ny = self.layout.nx, self.layout.ny
        self.ms = ms
        self.corner_w = corner_w
        self.da_min_c = da_min_c
        # the smallest cell area (fv_tp_2d's del-n damping, del2_cubed): the oracle grid's own
        self.da_min = og.min_areas(N)[0] if da_min is None else da_min
        self.P = [Plane(s, self.nx, self.ny, nj, pitch) for s in self.subs]

    @property
    def nsub(self):
        return len(self.subs)


SPONGE_DEFAULTS = dict(n_sponge=1, d2_bg_k1=0.20, d2_bg_k2=0.10)


def sponge_defaults(nl):
    """the sponge keys of nl with the product's Namelist defaults (gtfv3.hpp)"""
    return {k: type(v)(nl.get(k, v)) for k, v in SPONGE_DEFAULTS.items()}


def level_groups(cols):
    """contiguous runs of levels with equal d_sw parameters: [(k0, k1, params)]"""
    out = []
    for k, c in enumerate(cols):
        if out and out[-1][2] == c:
            out[-1] = (out[-1][0], k + 1, c)
        else:
            out.append((k, k + 1, c))
    return out


def d_sw_levels(st, s, sub, m, nx, ny, dt, ords, dddmp, groups, da_min_c, da_min, d4_bg=0.0, ke_bg=0.0, divg_d=None,
                corner_w=None):
    """sw_core.d_sw over the whole column of sub-domain s of the state dict st, one call per run
    of levels with equal parameters (groups from level_groups), outputs joined along the level
    axis; heat / diss are zero on the levels that make none"""
    parts = []
    for k0, k1, c in groups:
        ks = slice(k0, k1)
        parts.append(sw_core.d_sw(
            st["delp"][s, ks], st["pt"][s, ks], st["u"][s, ks], st["v"][s, ks], st["w"][s, ks], st["uc"][s, ks],
            st["vc"][s, ks], st["ua"][s, ks], st["va"][s, ks], sub, m, nx, ny, dt, ords, dddmp, c["d2_divg"], da_min_c,
            nord=c["nord"], d4_bg=d4_bg, divg_d=divg_d[ks] if c["nord"] > 0 else None, vtdm4=c["damp_vt"],
            nord_v=c["nord_v"], d_con=c["d_con"], corner_w=corner_w, damp_w=c["damp_w"], nord_w=c["nord_w"],
            damp_t=c["damp_t"], nord_t=c["nord_t"], ke_bg=ke_bg, da_min=da_min))
    r = {name: np.concatenate([p[name] for p in parts])
         for name in ("delp", "pt", "w", "u", "v", "crx", "cry", "xfx", "yfx", "fx", "fy", "ke")}
    for name in ("heat", "diss"):
        r[name] = np.concatenate([p[name] if name in p else np.zeros_like(p["delp"]) for p in parts])
    return r


def _halo(g, st, items):
    """items: list of (name, kind) as in Dycore::halo_update; vector kinds take two names"""
    n = 0
    while n < len(items):
        name, k = items[n]
        if k == "c":
            fill_scalar(st[name], g.layout, "cell")
        elif k == "b":
            fill_scalar(st[name], g.layout, "corner")
        else:
            fill_vector(st[name], st[items[n + 1][0]], g.layout, {"d": "dgrid", "C": "cgrid", "a": "agrid"}[k])
            n += 1
        n += 1


def c2l_ord4(u, v, m, P):
    """cubed_to_latlon, 4th order (FV3 fv_grid_utils c2l_ord4): D-grid (u, v) -> A-grid (ua, va)
    on compute cells; 2nd-order distance-weighted averages on the tile-edge rows/columns."""
    N, I, J = P.N, P.I, P.J
    c1, c2 = 1.125, -0.125
    dx, dy = m["dx"], m["dy"]
    ut = c2 * (sh(u, 0, -1) + sh(u, 0, 2)) + c1 * (u + sh(u, 0, 1))
    vt = c2 * (sh(v, -1, 0) + sh(v, 2, 0)) + c1 * (v + sh(v, 1, 0))
    row = (J == 0) | (J == N - 1)
    vt_e = 2.0 * (v * dy + sh(v, 1, 0) * sh(dy, 1, 0)) / (dy + sh(dy, 1, 0))
    ut_e = 2.0 * (u * dx + sh(u, 0, 1) * sh(dx, 0, 1)) / (dx + sh(dx, 0, 1))
    vt = np.where(row, vt_e, vt)
    ut = np.where(row, ut_e, ut)
    col = (I == 0) | (I == N - 1)
    ut = np.where(col, ut_e, ut)
    vt = np.where(col, vt_e, vt)
    ua = m["a11"] * ut + m["a12"] * vt
    va = m["a21"] * ut + m["a22"] * vt
    comp = P.reg(0, P.nx - 1, 0, P.ny - 1)
    return np.where(comp, ua, 0.0), np.where(comp, va, 0.0)


def fv_dynamics(st, ak, bk, g, nl):
    """One fv_dynamics call.  st: dict name -> array; updated and returned (new dict).

    Required inputs: u, v, w, delz, pt (T), delp, q (nq*npz levels, tracer 0 = sphum), phis.
    nl: dict with n_split, dt_atmos, hord_mt/vt/tm/dp/tr, dddmp, d2_bg, p_fac, dz_min, fill, nq;
    optional damping keys (sw_core.d_sw): nord, d4_bg, vtdm4, nord_v, d_con, delt_max.
    With d_con > 0 the state gains diss_est (the summed dissipation estimate of the call).
    """
    st = {k: v.copy() for k, v in st.items()}
    nsub, nx, ny = g.nsub, g.nx, g.ny
    npz = st["delp"].shape[1]
    k1 = npz + 1
    nq = nl["nq"]
    shp = st["delp"].shape
    shp1 = (nsub, k1) + shp[2:]
    shp0 = (nsub, 1) + shp[2:]
    for name, s_ in (("pe", shp1), ("peln", shp1), ("pk", shp1), ("pkz", shp), ("ps", shp0), ("omga", shp),
                     ("ua", shp), ("va", shp), ("uc", shp), ("vc", shp), ("mfx", shp), ("mfy", shp), ("cx", shp),
                     ("cy", shp), ("zh", shp1), ("ppe", shp1), ("pk3", shp1), ("ws", shp0)):
        if name not in st:
            st[name] = np.zeros(s_)
    bdt = nl["dt_atmos"]
    dt = bdt / nl["n_split"]
    dt2 = 0.5 * dt
    ptop = ak[0]
    dp0 = nh_core.dp_ref(ak, bk)
    comp = [P.reg(0, nx - 1, 0, ny - 1) for P in g.P]
    q0 = st["q"][:, :npz]
    # adiabatic = dry dynamics: no moisture in the virtual temperature (FV3 moist_phys off)
    zvir = 0.0 if nl.get("adiabatic", 0) else ZVIR

    # ---- entry ----
    rdg = -RDGAS * (1.0 / GRAV)
    for s in range(nsub):
        dp1 = zvir * q0[s]
        pk = np.exp(KAPPA * np.log(rdg * st["delp"][s] * st["pt"][s] * (1.0 + dp1) / st["delz"][s]))
        st["pkz"][s] = np.where(comp[s], pk, st["pkz"][s])
        st["pt"][s] = np.where(comp[s], st["pt"][s] * (1.0 + dp1) / pk, st["pt"][s])
    st["dp1"] = st["delp"].copy()
    for name in ("mfx", "mfy", "cx", "cy"):
        st[name][:] = 0.0

    # ---- dyn_core ----
    _halo(g, st, [("u", "d"), ("v", "d"), ("delp", "c"), ("pt", "c"), ("w", "c"), ("phis", "c")])
    zs = [st["phis"][s, 0] * (1.0 / GRAV) for s in range(nsub)]
    for s in range(nsub):
        zc = zs[s]
        z = st["zh"][s]
        z[npz] = np.where(comp[s], zc, z[npz])
        for k in range(npz - 1, -1, -1):
            z[k] = np.where(comp[s], z[k + 1] - st["delz"][s, k], z[k])
    _halo(g, st, [("zh", "c")])
    ords = (nl["hord_mt"], nl["hord_vt"], nl["hord_tm"], nl["hord_dp"])
    nord, d_con = int(nl.get("nord", 0)), float(nl.get("d_con", 0.0))
    # FV3 dyn_core's per-level d_sw parameters (sw_core.column_namelist): nord_v = min(2, nord)
    # unless given, vtdm4 acts only with do_vort_damp, the sponge-layer overrides in the top
    # levels (the product's Namelist defaults: n_sponge 1, d2_bg_k1 0.2, d2_bg_k2 0.1)
    sp = sponge_defaults(nl)
    cols = sw_core.column_namelist(npz, nord=nord, d2_bg=nl["d2_bg"], vtdm4=float(nl.get("vtdm4", 0.0)),
                                   do_vort_damp=bool(nl.get("do_vort_damp", 0)), nord_v=nl.get("nord_v"),
                                   d_con=d_con, **sp)
    groups = level_groups(cols)
    # update_dz_d's height damping: (nord_v, (damp_vt da_min_c)^(nord_v+1)) per interface, the
    # bottom layer's repeated for the surface (FV3 damp(km+1) = damp(km))
    zdamp = [(c["nord_v"], (c["damp_vt"] * g.da_min_c) ** (c["nord_v"] + 1) if c["damp_vt"] > 1e-5 else 0.0)
             for c in cols]
    zdamp = zdamp + zdamp[-1:] if any(z[1] > 0.0 for z in zdamp) else None
    d4_bg, ke_bg = float(nl.get("d4_bg", 0.0)), float(nl.get("ke_bg", 0.0))
    if nord > 0:
        st["divgd"] = np.zeros(shp)
    if d_con > 1e-5:
        heat = np.zeros(shp)
        st["diss_est"] = np.zeros(shp)
    for it in range(nl["n_split"]):
        last = it == nl["n_split"] - 1
        cs = []
        for s in range(nsub):
            m, sub, P = g.ms[s], g.subs[s], g.P[s]
            c = sw_core.c_sw(st["delp"][s], st["pt"][s], st["u"][s], st["v"][s], st["w"][s], sub, m, nx, ny, dt2)
            gzc, ws = nh_core.update_dz_c(c["ut"], c["vt"], st["zh"][s], zs[s], sub, m, nx, ny, dp0, dt2,
                                          nl["dz_min"])
            reg = P.reg(-1, nx, -1, ny)
            pef, gzc = nh_core.riem_solver_c(dt2, c["delpc"], c["ptc"], c["wc"], gzc, st["phis"][s, 0], ws, ptop,
                                             nl["p_fac"], reg)
            uc, vc = nh_core.p_grad_c(c["uc"], c["vc"], c["delpc"], pef, gzc, m, P, dt2)
            st["uc"][s], st["vc"][s], st["ua"][s], st["va"][s] = uc, vc, c["ua"], c["va"]
            if nord > 0:  # c_sw's divergence_corner (from the old D-grid winds and d2a2c's ua, va)
                st["divgd"][s] = sw_core.divergence_corner(st["u"][s], st["v"][s], c["ua"], c["va"], sub, m, nx, ny)
            cs.append(c)
        if nord > 0:
            _halo(g, st, [("divgd", "b")])
        # one value per shared tile-edge point: east / north edges take the neighbour's winds
        # (FV3 mpp_get_boundary; without it the cube-corner circulation of c_sw leaves the two
        # tiles with different winds, hence mass fluxes, next to each corner)
        if nl.get("edge_sync", 1):
            sync_edges(st["uc"], st["vc"], g.layout, "cgrid")
        _halo(g, st, [("uc", "C"), ("vc", "C")])
        ds = []
        for s in range(nsub):
            m, sub, P = g.ms[s], g.subs[s], g.P[s]
            r = d_sw_levels(st, s, sub, m, nx, ny, dt, ords, nl["dddmp"], groups, g.da_min_c, g.da_min, d4_bg, ke_bg,
                            st["divgd"][s] if nord > 0 else None, g.corner_w[s])
            for name in ("delp", "pt", "w", "u", "v"):
                st[name][s] = r[name]
            if d_con > 1e-5:
                heat[s] += r["heat"]
                st["diss_est"][s] += r["diss"]
            st["cx"][s] = np.where(P.reg(0, nx, -NG, ny + NG - 1), st["cx"][s] + r["crx"], st["cx"][s])
            st["cy"][s] = np.where(P.reg(-NG, nx + NG - 1, 0, ny), st["cy"][s] + r["cry"], st["cy"][s])
            st["mfx"][s] = np.where(P.reg(0, nx, 0, ny - 1), st["mfx"][s] + r["fx"], st["mfx"][s])
            st["mfy"][s] = np.where(P.reg(0, nx - 1, 0, ny), st["mfy"][s] + r["fy"], st["mfy"][s])
            ds.append(r)
        _halo(g, st, [("delp", "c"), ("pt", "c")])
        for s in range(nsub):
            m, sub, P = g.ms[s], g.subs[s], g.P[s]
            r = ds[s]
            zh, ws = nh_core.update_dz_d(st["zh"][s], r["crx"], r["cry"], r["xfx"], r["yfx"], zs[s], sub, m, nx, ny,
                                         dp0, dt, nl["hord_tm"], nl["dz_min"], zdamp)
            o = nh_core.riem_solver3(dt, st["delp"][s], st["pt"][s], st["w"][s], zh, zs[s], ws, ptop, nl["p_fac"],
                                     comp[s], last)
            st["w"][s] = o["w"]
            st["delz"][s] = np.where(comp[s], o["delz"], st["delz"][s])
            st["zh"][s] = o["zh"]
            st["ppe"][s] = np.where(comp[s], o["ppe"], st["ppe"][s])
            st["pk3"][s] = np.where(comp[s], o["pk3"], st["pk3"][s])
            st["ws"][s, 0] = np.where(comp[s], ws, st["ws"][s, 0])
            if last:
                for name in ("pe", "peln", "pk"):
                    st[name][s] = np.where(comp[s], o[name], st[name][s])
        _halo(g, st, [("zh", "c"), ("ppe", "c"), ("w", "c")])
        for s in range(nsub):
            P = g.P[s]
            st["pk3"][s] = nh_core.pk3_halo(st["pk3"][s], st["delp"][s], ptop, P)
            if last:
                st["pe"][s] = nh_core.pe_halo(st["pe"][s], st["delp"][s], ptop, P)
        for s in range(nsub):
            m, P = g.ms[s], g.P[s]
            gz = st["zh"][s] * GRAV
            st["u"][s], st["v"][s] = nh_core.nh_p_grad(st["u"][s], st["v"][s], st["ppe"][s], gz, st["delp"][s],
                                                       st["pk3"][s], dt, ptop, P, m, g.corner_w[s])
        if not last:
            _halo(g, st, [("u", "d"), ("v", "d")])

    # ---- d_con: the kinetic energy the damping removed, as heat (dyn_core after the acoustic
    # loop, "Add dissipative heating"), on the top n_con levels (sw_core.heat_levels): the heat
    # source's halo filled, smoothed by del2_cubed (min(3, nord + 1) passes, 0.2 da_min), then
    # dT = heat / (cv_air delp), limited to delt_max * bdt per call (0.1x / 0.5x in the top
    # two layers), added to the potential temperature through pkz ----
    n_con = sw_core.heat_levels(npz, float(nl.get("vtdm4", 0.0)), sp["d2_bg_k1"], sp["d2_bg_k2"],
                                bool(nl.get("convert_ke", 0)))
    if d_con > 1e-5 and n_con > 0:
        fill_scalar(heat, g.layout, "cell")
        for s in range(nsub):
            heat[s, :n_con] = sw_core.del2_cubed(heat[s, :n_con], 0.2 * g.da_min, g.subs[s], g.ms[s], nx, ny,
                                                 min(3, nord + 1))
        cv = RDGAS / KAPPA - RDGAS
        k1k = KAPPA / (1.0 - KAPPA)
        delt = abs(bdt * float(nl.get("delt_max", 1.0)))
        lim = np.full(n_con, delt)
        lim[0] = 0.1 * delt
        if n_con > 1:
            lim[1] = 0.5 * delt
        lim = lim[:, None, None]
        kc = slice(0, n_con)
        for s in range(nsub):
            dp, pt = st["delp"][s, kc], st["pt"][s, kc]
            pkz = np.exp(k1k * np.log(rdg * dp / st["delz"][s, kc] * pt))
            dtmp = heat[s, kc] / (cv * dp)
            st["pt"][s, kc] = np.where(comp[s], pt + np.sign(dtmp) * np.minimum(lim, np.abs(dtmp)) / pkz, pt)

    # ---- tracer transport ----
    st["q"], nsplt = tp_core.tracer_2d_1l(st["q"], st["dp1"], st["mfx"], st["mfy"], st["cx"], st["cy"], g.subs,
                                          g.ms, nx, ny, npz, nq, nl["hord_tr"],
                                          lambda a: fill_scalar(a, g.layout, "cell"))

    # ---- vertical remap ----
    keys = ("pe", "peln", "pk", "pkz", "delp", "delz", "pt", "w", "q", "u", "v", "ps")
    for s in range(nsub):
        sub_st = {k: st[k][s] for k in keys}
        sub_st["ws"] = st["ws"][s, 0]
        o = fv_mapz.lagrangian_to_eulerian(sub_st, ak, bk, ptop, nq, nl["fill"], g.P[s])
        for k in keys:
            st[k][s] = o[k]

    # ---- exit ----
    for s in range(nsub):
        q0s = st["q"][s, :npz]
        st["pt"][s] = np.where(comp[s], st["pt"][s] / (1.0 + zvir * q0s), st["pt"][s])
        st["omga"][s] = np.where(comp[s], st["delp"][s] / st["delz"][s] * st["w"][s], st["omga"][s])
    _halo(g, st, [("u", "d"), ("v", "d")])
    for s in range(nsub):
        st["ua"][s], st["va"][s] = c2l_ord4(st["u"][s], st["v"][s], g.ms[s], g.P[s])
    st["_nsplt"] = nsplt
    return st
