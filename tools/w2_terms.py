"""(CPU, oracle) Williamson 2's balanced state through one small oracle sub-step: the u
tendency split into its kinetic-energy, vorticity-flux and pressure-gradient parts, each
against its analytic counterpart, by distance to the tile edge -- which part of the discrete
balance fails to converge at the tile edges."""
import sys
import importlib
import numpy as np
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
pkg = importlib.import_module("geosongpu-ci_amd")
import test_gpu_williamson2 as w2
from conftest import metrics_of, oracle_scalars
from oracle import NG, nh_core, sw_core
from oracle import fv_dynamics as fvd
from oracle.halo import fill_vector, sync_edges
from oracle.util import sh

G = w2.G
dt = 10.0
for npx in [int(a) for a in sys.argv[1:]] or (13, 25, 49):
    d = pkg.Domain(npx=npx, npz=1, nq=1, host_only=1)
    u, v, h = w2.setup_case(d)
    sc = oracle_scalars(d)
    ms = metrics_of(d)
    g = fvd.Grid(d.N, 1, 1, ms, sc["corner_w"], sc["da_min_c"], d.nj, d.pitch)
    st = dict(u=u.copy(), v=v.copy(), delp=h.copy(), pt=np.ones(d.shape(1)), w=d.zeros(1), uc=d.zeros(1),
              vc=d.zeros(1), ua=d.zeros(1), va=d.zeros(1))
    fvd._halo(g, st, [("u", "d"), ("v", "d"), ("delp", "c"), ("pt", "c"), ("w", "c")])
    for s in range(g.nsub):
        m, sub, P = g.ms[s], g.subs[s], g.P[s]
        c = sw_core.c_sw(st["delp"][s], st["pt"][s], st["u"][s], st["v"][s], st["w"][s], sub, m, g.nx, g.ny, 0.5 * dt)
        dp = c["delpc"]
        gz = np.concatenate([G * dp, 0 * dp])
        pk = np.concatenate([0 * dp, dp])
        st["uc"][s], st["vc"][s] = nh_core.p_grad_c(c["uc"], c["vc"], dp, pk, gz, m, P, 0.5 * dt)
        st["ua"][s], st["va"][s] = c["ua"], c["va"]
    sync_edges(st["uc"], st["vc"], g.layout, "cgrid")
    fill_vector(st["uc"], st["vc"], g.layout, "cgrid")
    xyz = d.corner_xyz()
    H = NG + 1
    N = d.N
    rows = {}
    for s in range(g.nsub):
        m, sub, P = g.ms[s], g.subs[s], g.P[s]
        r = sw_core.d_sw(st["delp"][s], st["pt"][s], st["u"][s], st["v"][s], st["w"][s], st["uc"][s], st["vc"][s],
                         st["ua"][s], st["va"][s], sub, m, g.nx, g.ny, dt, (6, 6, 6, 6), 0.0, 0.0, g.da_min_c)
        ke = r["ke"]
        udx = st["u"][s] * m["dx"]
        term_k = ke - sh(ke, 1, 0)
        term_v = r["u"] - udx - term_k
        # pressure gradient on the updated depth (its halo from this sub-domain's own values is
        # enough for the tendency split: the depth barely moves in dt)
        dpn = r["delp"]
        gzn = np.concatenate([G * dpn, 0 * dpn])
        pkn = np.concatenate([0 * dpn, dpn])
        un, _ = nh_core.nh_p_grad(r["u"], r["v"], np.zeros_like(gzn), gzn, dpn, pkn, dt, 0.0, P, m, g.corner_w[s])
        term_p = un * m["dx"] - r["u"]
        # analytic corner K and G
        P3 = xyz[s]
        o = H - NG
        lat = np.arcsin(np.clip(w2._unit(P3)[..., 2], -1, 1))  # corner (i, j) at [j+H, i+H]
        nj, pitch = d.nj, d.pitch
        Kc = np.zeros((nj, pitch)); Gc = np.zeros((nj, pitch))
        jj = slice(o, o + nj); ii = slice(o, o + pitch)
        latc = lat[jj, ii][:nj, :pitch]
        Kc[:latc.shape[0], :latc.shape[1]] = 0.5 * (w2.U0 * np.cos(latc)) ** 2
        Gc[:latc.shape[0], :latc.shape[1]] = G * w2._depth(latc)
        ek = dt * (Kc - sh(Kc, 1, 0))
        ep = dt * (Gc - sh(Gc, 1, 0))
        for J in range(0, d.ny + 1):
            de = min(J, N - J)
            for I in range(0, d.nx):
                jx, ix = J + NG, I + NG
                den = dt * m["dx"][jx, ix]
                key = min(de, min(I, N - 1 - I), 4)
                rec = rows.setdefault(key, [])
                rec.append((term_k[0, jx, ix] / den, ek[jx, ix] / den, term_p[0, jx, ix] / den, ep[jx, ix] / den,
                            term_v[0, jx, ix] / den))
    print(f"C{npx - 1}: u accelerations (m/s^2), max |discrete - analytic| by edge distance (4 = interior)")
    for key in sorted(rows):
        a = np.array(rows[key])
        tot = a[:, 0] + a[:, 2] + a[:, 4]
        print(f"  dist {key}: KE {np.abs(a[:, 0] - a[:, 1]).max():.3e}  PG {np.abs(a[:, 2] - a[:, 3]).max():.3e}"
              f"  vort-flux residual vs -(K+G) {np.abs(a[:, 4] + a[:, 1] + a[:, 3]).max():.3e}  total {np.abs(tot).max():.3e}"
              f"  (|KE| {np.abs(a[:, 1]).max():.2e} |PG| {np.abs(a[:, 3]).max():.2e})")
    d.close()
