"""Held & Suarez (1994) forcing oracle — TEST INFRASTRUCTURE ONLY.

The Held-Suarez experiment (`geos_hs`, experiments.yaml:8-29; GEOShs.x launched by
held_suarez.py:79-126) drives the dycore with HS94 forcing; GEOS's implementation is
external, so this restates the published forcing:
  T_eq = max(200, [315 - dT_y sin^2(lat) - dth_z log(p/p0) cos^2(lat)] (p/p0)^kappa)
  k_T  = k_a + (k_s - k_a) max(0, (sigma - 0.7)/0.3) cos^4(lat)
  k_v  = k_f max(0, (sigma - 0.7)/0.3)
applied implicitly over dt:  T <- (T + dt k_T T_eq)/(1 + dt k_T),  u <- u/(1 + dt k_v),
with sigma = layer-mean pressure / surface pressure, D-grid winds using the mean sigma
of the two cells sharing the edge.  Same expression order as csrc/misc.hip hs_k.
Parity unpinned (no reference numerics).  Arrays use the HBM layout a[k, j+NG, i+NG].
"""
import numpy as np

from . import NG

from .nh_core import KAPPA  # noqa: E402  rdgas / cp_air = 2/7 (csrc Constants::kappa)


def held_suarez(pe, pt, u, v, lat, nx, ny, dt):
    """pe [npz+1, nj, pitch]; pt, u, v [npz, nj, pitch] (updated copies returned); lat plane."""
    p0, sigb = 1.0e5, 0.7
    ka, ks, kf = 1.0 / (40.0 * 86400.0), 1.0 / (4.0 * 86400.0), 1.0 / 86400.0
    dty, dthz = 60.0, 10.0
    npz = pt.shape[0]
    pt, u, v = pt.copy(), u.copy(), v.copy()
    ps = pe[npz]
    J, I = slice(NG, NG + ny), slice(NG, NG + nx)
    for k in range(npz):
        pm = 0.5 * (pe[k] + pe[k + 1])
        sig = pm / ps
        la = lat[J, I]
        sl, cl = np.sin(la), np.cos(la)
        pmc = pm[J, I]
        teq = np.maximum(200.0, (315.0 - dty * sl * sl - dthz * np.log(pmc / p0) * cl * cl) *
                         np.exp(KAPPA * np.log(pmc / p0)))
        kt = ka + (ks - ka) * np.maximum(0.0, (sig[J, I] - sigb) / (1.0 - sigb)) * cl * cl * cl * cl
        pt[k, J, I] = (pt[k, J, I] + dt * kt * teq) / (1.0 + dt * kt)
        Ju = slice(NG, NG + ny + 1)
        sgu = 0.5 * (sig[Ju, I] + sig[NG - 1:NG + ny, I])
        u[k, Ju, I] = u[k, Ju, I] / (1.0 + dt * (kf * np.maximum(0.0, (sgu - sigb) / (1.0 - sigb))))
        Iv = slice(NG, NG + nx + 1)
        sgv = 0.5 * (sig[J, Iv] + sig[J, NG - 1:NG + nx])
        v[k, J, Iv] = v[k, J, Iv] / (1.0 + dt * (kf * np.maximum(0.0, (sgv - sigb) / (1.0 - sigb))))
    return pt, u, v
