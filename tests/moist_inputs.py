"""Synthetic aquaplanet-like column states for the moist physics tests (fp64, HBM
layout arrays (nsub, nk, nj, pitch)): temperature with a 6.5 K/km lapse rate and a
stratospheric floor, humidity from a relative-humidity profile with supersaturated
patches, cloud water / ice / precipitating species in random columns, and a sprinkle of
small negative values (the neg_adj / fillq2zero paths)."""
import numpy as np

GRAV = 9.80665
RDGAS = 8314.47 / 28.965


def hybrid(nk, ptop=100.0, ps=1.0e5):
    s = np.linspace(0.0, 1.0, nk + 1) ** 1.6
    return ptop + (ps - ptop) * s


def moist_state(shape, seed=5):
    """shape = (nsub, nk, nj, pitch)"""
    from oracle import moist as om
    r = np.random.default_rng(seed)
    nsub, nk, nj, pitch = shape
    pe = hybrid(nk)[None, :, None, None] * (1.0 + 0.02 * r.standard_normal((nsub, 1, nj, pitch)))
    pm = 0.5 * (pe[:, 1:] + pe[:, :-1])
    dp = pe[:, 1:] - pe[:, :-1]
    # temperature: surface 280-305 K, 6.5 K/km lapse rate, floor at 200 K
    tsfc = 280.0 + 25.0 * r.random((nsub, 1, nj, pitch))
    zapprox = -RDGAS * 255.0 / GRAV * np.log(pm / pe[:, -1:])
    T = np.maximum(200.0, tsfc - 6.5e-3 * zapprox) + 0.5 * r.standard_normal(pm.shape)
    dz = -RDGAS / GRAV * T * np.log(pe[:, 1:] / pe[:, :-1])
    zi = np.zeros(pe.shape)
    for k in range(nk - 1, -1, -1):
        zi[:, k] = zi[:, k + 1] - dz[:, k]
    zm = 0.5 * (zi[:, 1:] + zi[:, :-1])
    qs, _ = om.qsat(T, pm, ice=False)
    rh = np.clip(0.3 + 0.8 * (pm / 1e5) + 0.15 * r.standard_normal(pm.shape), 0.05, 1.08)
    qv = rh * qs
    cloud = r.random(pm.shape) < 0.3
    ql = np.where(cloud & (T > 250.0), 1.0e-3 * r.random(pm.shape), 0.0)
    qi = np.where(cloud & (T < 265.0), 2.0e-4 * r.random(pm.shape), 0.0)
    qr = np.where(r.random(pm.shape) < 0.2, 5.0e-4 * r.random(pm.shape), 0.0)
    qsn = np.where((r.random(pm.shape) < 0.2) & (T < 275.0), 3.0e-4 * r.random(pm.shape), 0.0)
    qg = np.where(r.random(pm.shape) < 0.1, 2.0e-4 * r.random(pm.shape), 0.0)
    for q in (ql, qr, qi, qsn, qg):
        neg = r.random(pm.shape) < 0.02
        q[neg] = -1.0e-6 * r.random(neg.sum())
    return dict(T=T, qv=qv, ql=ql, qr=qr, qi=qi, qs=qsn, qg=qg, delp=dp, delz=dz, pm=pm, zm=zm)
