"""GPU parity of the SIM1 Riemann solvers (riem_solver_c, riem_solver3).

Two checks per case:
  * the register-resident level-block kernel (default) against the column-sweep kernel
    (variant 1): bit-identical on every output, including columns where the dz_min
    clamp is active in several blocks (the blocked clamp is speculative);
  * both against the oracle (oracle/nh_core.py, after the dz_min clamp FV3 applies in
    update_dz_c / update_dz_d): |hip - oracle| <= 1e-11 * mean|oracle| (exp / log
    come from ocml on the device and glibc on the host).
Inputs are near-hydrostatic columns (pt chosen so that the nonhydrostatic pressure is
the layer-mean pressure to 1e-3), so the perturbation pressures the solver forms are
well conditioned.
"""
import numpy as np
import pytest

from conftest import rng
from oracle import NG
from oracle import nh_core

pytestmark = pytest.mark.gpu

GRAV, RDGAS, KAPPA = nh_core.GRAV, nh_core.RDGAS, nh_core.KAPPA
PTOP, P_FAC, DZ_MIN = 300.0, 0.05, 2.0


def columns(d, npz, r, thin):
    """delp, pt, w, heights (npz+1), zs, phis on the whole plane of every sub-domain"""
    sh = d.shape(npz)
    delp = 800.0 + 1200.0 * r.random(sh)
    pem = PTOP + np.concatenate([np.zeros(sh[:1] + (1,) + sh[2:]), np.cumsum(delp, axis=1)], axis=1)
    T = 220.0 + 60.0 * r.random(sh)
    dz = -RDGAS * T / GRAV * np.log(pem[:, 1:] / pem[:, :-1])
    if thin:  # layers thinner than dz_min in a scatter of columns and levels
        m = r.random(sh) < 0.03
        dz = np.where(m, -0.5 * r.random(sh), dz)
    zs = 1500.0 * r.random((sh[0], 1) + sh[2:])
    zh = np.concatenate([np.zeros_like(pem[:, :-1]), zs], axis=1)
    for k in range(npz - 1, -1, -1):
        zh[:, k] = zh[:, k + 1] - dz[:, k]
    zh[:, npz] += 0.3 * r.standard_normal(zs.shape[:1] + zs.shape[2:])  # nonzero ws
    pm = delp / np.log(pem[:, 1:] / pem[:, :-1])
    dzc = np.minimum(dz, -1.0)
    pt = np.exp((1.0 - KAPPA) * np.log(pm)) * (-dzc) / (delp / GRAV * RDGAS)
    pt *= 1.0 + 1e-3 * r.standard_normal(sh)
    w = 0.5 * r.standard_normal(sh)
    return dict(delp=delp, pt=pt, w=w, zh=zh, zs=zs, phis=zs * GRAV)


def clamp(h):
    h = h.copy()
    for k in range(h.shape[0] - 2, -1, -1):
        h[k] = np.maximum(h[k], h[k + 1] + DZ_MIN)
    return h


def region(a, ring, nx, ny):
    return a[..., NG - ring:NG + ny + ring, NG - ring:NG + nx + ring]


def close(a, b, what, rtol=1e-11, atol=0.0):
    scale = np.abs(b).mean() + 1e-300
    worst = (np.abs(a - b).max() - atol) / scale
    assert worst <= rtol, f"{what}: max scaled error {worst:.3e}"


@pytest.mark.parametrize("npz,thin", [(12, True), (10, False), (72, True), (7, True), (137, True), (137, False)])
def test_riem_solver_c(pkg, require_gpu, npz, thin):
    d = pkg.Domain(npx=13, npz=npz, nq=1)
    r = rng(100 + npz)
    col = columns(d, npz, r, thin)
    dt2 = 225.0
    for k in ("delp", "pt", "w", "phis"):
        d.upload("rc_" + k, col[k])
    got = {}
    for var in (1, 0):
        d.upload("rc_gz", col["zh"])
        d.stencil("riem_solver_c", ["rc_delp", "rc_pt", "rc_w", "rc_phis", "rc_gz", "rc_pef"],
                  [dt2, PTOP, P_FAC, DZ_MIN, var])
        got[var] = {k: region(d.download(k), 1, d.nx, d.ny) for k in ("rc_gz", "rc_pef")}
    for k in got[0]:
        assert np.array_equal(got[0][k], got[1][k]), f"{k}: blocked kernel differs from the column kernel"
    for s in range(d.nsub):
        gz = clamp(col["zh"][s])
        ws = (col["zs"][s, 0] - col["zh"][s, npz]) * (1.0 / dt2)
        reg = np.ones(gz.shape[1:], dtype=bool)
        pef, gzo = nh_core.riem_solver_c(dt2, col["delp"][s], col["pt"][s], col["w"][s], gz, col["phis"][s, 0], ws,
                                         PTOP, P_FAC, reg)
        close(got[0]["rc_pef"][s], region(pef, 1, d.nx, d.ny), f"sub{s} pef")
        close(got[0]["rc_gz"][s], region(gzo, 1, d.nx, d.ny), f"sub{s} gz")


@pytest.mark.parametrize("npz,last", [(12, 1), (72, 0), (10, 1), (137, 1), (137, 0)])
def test_riem_solver3(pkg, require_gpu, npz, last):
    d = pkg.Domain(npx=13, npz=npz, nq=1)
    r = rng(200 + npz)
    col = columns(d, npz, r, True)
    dt = 450.0
    for k in ("delp", "pt", "phis"):
        d.upload("r3_" + k, col[k])
    outs = ["r3_w", "r3_zh", "r3_delz", "r3_ppe", "r3_pk3", "r3_pe", "r3_peln", "r3_pk", "r3_ws"]
    got = {}
    for var in (1, 0):
        d.upload("r3_w", col["w"])
        d.upload("r3_zh", col["zh"])
        for k in ("r3_pe", "r3_peln", "r3_pk"):
            d.upload(k, np.zeros(d.shape(npz + 1)))
        d.stencil("riem_solver3", ["r3_delp", "r3_pt", "r3_w", "r3_phis", "r3_zh", "r3_delz", "r3_ppe", "r3_pk3",
                                   "r3_pe", "r3_peln", "r3_pk", "r3_ws"], [dt, PTOP, P_FAC, DZ_MIN, last, var])
        got[var] = {k: region(d.download(k), 0, d.nx, d.ny) for k in outs}
    for k in outs:
        assert np.array_equal(got[0][k], got[1][k]), f"{k}: blocked kernel differs from the column kernel"
    for s in range(d.nsub):
        zh = clamp(col["zh"][s])
        ws = (col["zs"][s, 0] - col["zh"][s, npz]) * (1.0 / dt)
        reg = np.ones(zh.shape[1:], dtype=bool)
        o = nh_core.riem_solver3(dt, col["delp"][s], col["pt"][s], col["w"][s], zh, col["zs"][s, 0], ws, PTOP, P_FAC,
                                 reg, bool(last))
        g = {k[3:]: v[s] for k, v in got[0].items()}
        close(g["ws"][0], region(ws, 0, d.nx, d.ny), f"sub{s} ws")
        close(g["w"], region(o["w"], 0, d.nx, d.ny), f"sub{s} w", atol=1e-12)
        for k in ("zh", "delz", "pk3"):
            close(g[k], region(o[k], 0, d.nx, d.ny), f"sub{s} {k}")
        close(g["ppe"], region(o["ppe"], 0, d.nx, d.ny), f"sub{s} ppe", rtol=1e-9)
        if last:
            for k in ("pe", "peln", "pk"):
                close(g[k], region(o[k], 0, d.nx, d.ny), f"sub{s} {k}")
