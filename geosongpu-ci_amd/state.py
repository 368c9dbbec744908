"""Synthetic initial states for the dycore path (host-side, numpy).

No checkpoint or dataset can be fetched here, so the benchmark and the step tests
start from analytic states of the documented shape:

* `hybrid_levels(npz)`   — a hybrid sigma-pressure coordinate (ak, bk, ks) with a
  1 Pa model top like GEOS L72 (pure pressure above ~ 200 hPa, terrain-following
  below).  The level *values* are synthetic; the vertical structure matches.
* `jablonowski_williamson(dom, ak, bk)` — the JW06 baroclinic-wave initial state
  (balanced zonal jet + Gaussian zonal-wind perturbation at 20E/40N), the dry
  dycore test FV3 ships as its test_case 12/13, with hydrostatic delz, w = 0 and
  passive tracers.  Winds are projected onto the D-grid edges from the grid
  corners' 3-D positions, scalars evaluated at the cell centres — halos included,
  so the state is complete without a first halo exchange.
"""
import numpy as np

from .domain import NG

GRAV = 9.80665
RDGAS = 8314.47 / 28.965
RADIUS = 6371.0e3
OMEGA = 2.0 * np.pi / 86164.0


def hybrid_levels(npz=72, ptop=1.0, p_sig=2.0e4, ps_ref=1.0e5):
    """(ak, bk, ks): interfaces k = 0 (top) .. npz (surface); pe = ak + bk * ps."""
    s = np.linspace(0.0, 1.0, npz + 1)
    # spacing stretched towards the top and the surface in log-pressure
    x = 0.5 * (1.0 - np.cos(np.pi * s)) * 0.75 + 0.25 * s
    lp = np.log(ptop) + (np.log(ps_ref) - np.log(ptop)) * x
    pref = np.exp(lp)
    pref[0], pref[-1] = ptop, ps_ref
    bk = np.clip((pref - p_sig) / (ps_ref - p_sig), 0.0, None) ** 1.2
    bk[-1] = 1.0
    ak = pref - bk * ps_ref
    ak[-1] = 0.0
    ks = int(np.sum(bk == 0.0)) - 1
    return ak, bk, ks


def _unit(v):
    n = np.linalg.norm(v, axis=-1, keepdims=True)
    return v / np.where(n > 0.0, n, 1.0)


def _latlon(p):
    p = _unit(p)
    return np.arcsin(np.clip(p[..., 2], -1.0, 1.0)), np.arctan2(p[..., 1], p[..., 0])


def _jw_wind(lat, lon, eta, perturb=True):
    u0, eta0 = 35.0, 0.252
    ev = (eta - eta0) * np.pi / 2.0
    u = u0 * np.cos(ev) ** 1.5 * np.sin(2.0 * lat) ** 2
    if not perturb:  # the steady-state test (JW06 section 3.1)
        return u
    # perturbation: Gaussian bump of 1 m/s centred at (20E, 40N), radius a/10
    lonc, latc = np.deg2rad(20.0), np.deg2rad(40.0)
    r = np.arccos(np.clip(np.sin(latc) * np.sin(lat) + np.cos(latc) * np.cos(lat) * np.cos(lon - lonc), -1, 1))
    u = u + np.exp(-(r * 10.0) ** 2)
    return u


def _jw_temp(lat, eta):
    u0, eta0, etat, T0, gam, dT = 35.0, 0.252, 0.2, 288.0, 0.005, 4.8e5
    ev = (eta - eta0) * np.pi / 2.0
    tbar = T0 * eta ** (RDGAS * gam / GRAV) + np.where(eta < etat, dT * (etat - eta) ** 5, 0.0)
    sl, cl = np.sin(lat), np.cos(lat)
    a = (-2.0 * sl ** 6 * (cl ** 2 + 1.0 / 3.0) + 10.0 / 63.0) * 2.0 * u0 * np.cos(ev) ** 1.5
    b = (1.6 * cl ** 3 * (sl ** 2 + 2.0 / 3.0) - np.pi / 4.0) * RADIUS * OMEGA
    return tbar + 0.75 * eta * np.pi * u0 / RDGAS * np.sin(ev) * np.sqrt(np.cos(ev)) * (a + b)


def _jw_phis(lat):
    u0, eta0 = 35.0, 0.252
    ev = (1.0 - eta0) * np.pi / 2.0
    sl, cl = np.sin(lat), np.cos(lat)
    return u0 * np.cos(ev) ** 1.5 * ((-2.0 * sl ** 6 * (cl ** 2 + 1.0 / 3.0) + 10.0 / 63.0) * u0 * np.cos(ev) ** 1.5
                                     + (1.6 * cl ** 3 * (sl ** 2 + 2.0 / 3.0) - np.pi / 4.0) * RADIUS * OMEGA)


def tracer_planes(dom, iq):
    """tracer iq of the synthetic state as (nsub, npz, nj, pitch): specific humidity for
    iq = 0, else a smooth bell pattern shifted in longitude per tracer"""
    lat, lon = dom.metric("lat"), dom.metric("lon")
    if iq == 0:
        t = 1.0e-6 * (1.0 + np.cos(lat))
    else:
        t = 0.5 * (1.0 + np.cos(lat) * np.cos(lon - 0.7 * iq))
    out = np.repeat(t[:, None], dom.npz, axis=1)
    np.nan_to_num(out, copy=False)
    return out


def jablonowski_williamson(dom, ak, bk, ps=1.0e5, tracers=None, perturb=True):
    """dict of host arrays (nsub, nk, nj, pitch): u, v, w, delz, pt, delp, q, phis.
    tracers: how many tracers to put in q (default all dom.nq; large sets go through
    tracer_planes + Domain.upload_levels one tracer at a time).  perturb=False: the
    balanced jet alone (JW06's steady-state test)."""
    nsub, npz = dom.nsub, dom.npz
    nq = max(dom.nq, 1) if tracers is None else max(int(tracers), 1)
    nj, pitch, nx, ny = dom.nj, dom.pitch, dom.nx, dom.ny
    H = NG + 1
    xyz = dom.corner_xyz()  # (nsub, ny+2H+1, nx+2H+1, 3), corner (i, j) at [j+H, i+H]
    lat_c = dom.metric("lat")
    lon_c = dom.metric("lon")
    pe = ak[None, :] + bk[None, :] * ps                 # (1, npz+1)
    pm = 0.5 * (pe[0, 1:] + pe[0, :-1])                 # layer mid pressures
    eta = pm / ps
    out = {n: np.zeros((nsub, npz, nj, pitch)) for n in ("u", "v", "w", "delz", "pt", "delp")}
    out["q"] = np.zeros((nsub, nq * npz, nj, pitch))
    out["phis"] = np.zeros((nsub, 1, nj, pitch))
    dp = (ak[1:] - ak[:-1]) + (bk[1:] - bk[:-1]) * ps
    # plane slots (j, i) for i, j in [-NG, n+NG]; xyz slot = plane slot + (H - NG)
    jj, ii = np.meshgrid(np.arange(nj), np.arange(pitch), indexing="ij")
    o = H - NG
    for s in range(nsub):
        P = xyz[s]

        def corner(dj, di):
            jc = np.clip(jj + o + dj, 0, P.shape[0] - 1)
            ic = np.clip(ii + o + di, 0, P.shape[1] - 1)
            return P[jc, ic]

        c00, c10, c01 = corner(0, 0), corner(0, 1), corner(1, 0)
        for name, (pa, pb) in (("u", (c00, c10)), ("v", (c00, c01))):
            mid = _unit(pa + pb)
            lat, lon = _latlon(mid)
            ev = _unit(pb - pa)  # edge direction
            elon = np.stack([-np.sin(lon), np.cos(lon), np.zeros_like(lon)], -1)
            for k in range(npz):
                uz = _jw_wind(lat, lon, eta[k], perturb)
                out[name][s, k] = uz * np.sum(elon * ev, axis=-1)
        lat, lon = lat_c[s], lon_c[s]
        out["phis"][s, 0] = _jw_phis(lat)
        for k in range(npz):
            t = _jw_temp(lat, eta[k])
            out["pt"][s, k] = t
            out["delp"][s, k] = dp[k]
            out["delz"][s, k] = -RDGAS / GRAV * t * np.log(pe[0, k + 1] / pe[0, k])
        out["q"][s, :npz] = 1.0e-6 * (1.0 + np.cos(lat))[None]
        for iq in range(1, nq):
            out["q"][s, iq * npz:(iq + 1) * npz] = (0.5 * (1.0 + np.cos(lat) * np.cos(lon - 0.7 * iq)))[None]
    # keep the padding columns finite and harmless
    for a in out.values():
        np.nan_to_num(a, copy=False)
    return out


def aquaplanet_tracers(dom, st, ak, bk, ps=1.0e5, rh_sfc=0.8, seed=20250117):
    """Moist tracers for the Aquaplanet configuration (BASELINE.json configs[3]) on a JW06
    state `st` in place: q tracers 0..5 = qv, ql, qr, qi, qs, qg (needs nq >= 6).
    qv from a relative-humidity profile (rh_sfc at the surface decreasing as (p/ps)^2)
    with a Tetens saturation curve (initial-state synthesis only; the physics kernels
    use the GFDL tables), a thin cloud layer where the profile nears saturation, and no
    precipitating species; the remaining tracers keep their passive bells."""
    nq = max(dom.nq, 1)
    if nq < 6:
        raise ValueError("aquaplanet_tracers: nq >= 6 required")
    npz = dom.npz
    pe = ak[:, None, None] + bk[:, None, None] * ps
    pm = 0.5 * (pe[1:] + pe[:-1])
    r = np.random.default_rng(seed)
    for s in range(dom.nsub):
        t = st["pt"][s]
        tc = t - 273.15
        es = 610.78 * np.exp(np.where(tc >= 0.0, 17.27 * tc / (tc + 237.3), 21.875 * tc / (tc + 265.5)))
        qsat = 0.622 * es / np.maximum(pm - 0.378 * es, 1.0)
        rh = rh_sfc * (pm / ps) ** 2 * (1.0 + 0.05 * r.standard_normal(t.shape))
        qv = np.clip(rh, 0.0, 1.02) * qsat
        cloud = np.clip(rh - 0.75, 0.0, None) * 2e-3
        st["q"][s, 0:npz] = qv
        st["q"][s, npz:2 * npz] = np.where(t > 253.0, cloud, 0.0)
        st["q"][s, 2 * npz:3 * npz] = 0.0
        st["q"][s, 3 * npz:4 * npz] = np.where(t <= 253.0, cloud, 0.0)
        st["q"][s, 4 * npz:6 * npz] = 0.0
    return st
