"""Oracle: FV3 non-hydrostatic pieces (nh_core / nh_utils / a2b_edge / dyn_core
helpers) in fp64 numpy — TEST INFRASTRUCTURE ONLY.

update_dz_c, update_dz_d (+ edge_profile), riem_solver_c / riem_solver3 with the
SIM1 semi-implicit column solver (a_imp = 1), p_grad_c, a2b_ord4, nh_p_grad,
pk3_halo, pe_halo.  Arrays are per sub-domain planes with a leading level axis:
cell fields (npz, nj, pitch), interface fields (npz+1, nj, pitch), level 0 = top.
Fortran index f -> tile-global g = f - 1.
"""
import numpy as np

from . import NG
from .tp_core import copy_corners, fv_tp_2d
from .util import Plane, sh

np.seterr(all="ignore")

GRAV = 9.80665
RDGAS = 8314.47 / 28.965
KAPPA = 1.0 / 3.5
R3 = 1.0 / 3.0


def dp_ref(ak, bk):
    return (ak[1:] - ak[:-1]) + (bk[1:] - bk[:-1]) * 1.0e5


# ---------------- update_dz_c ----------------

def update_dz_c(ut, vt, gz, zs, sub, m, nx, ny, dp0, dt, dz_min):
    """gz: heights at interfaces (npz+1, ...) with halo; ut/vt: c_sw area fluxes.
    Returns updated gz (cells [-1,nx]x[-1,ny]) and ws."""
    km = ut.shape[0]
    P = Plane(sub, nx, ny, gz.shape[-2], gz.shape[-1])
    top_ratio = dp0[0] / (dp0[1] + dp0[0])
    bot_ratio = dp0[km - 1] / (dp0[km - 2] + dp0[km - 1])
    area = m["area"]
    out = gz.copy()
    reg = P.reg(-1, nx, -1, ny)
    for k in range(km + 1):
        if k == 0:
            xfx = ut[0] + (ut[0] - ut[1]) * top_ratio
            yfx = vt[0] + (vt[0] - vt[1]) * top_ratio
        elif k == km:
            xfx = ut[km - 1] + (ut[km - 1] - ut[km - 2]) * bot_ratio
            yfx = vt[km - 1] + (vt[km - 1] - vt[km - 2]) * bot_ratio
        else:
            int_ratio = 1.0 / (dp0[k - 1] + dp0[k])
            xfx = (dp0[k] * ut[k - 1] + dp0[k - 1] * ut[k]) * int_ratio
            yfx = (dp0[k] * vt[k - 1] + dp0[k - 1] * vt[k]) * int_ratio
        g1 = copy_corners(gz[k:k + 1], sub, 1)[0]
        g2 = copy_corners(gz[k:k + 1], sub, 2)[0]
        fx = xfx * np.where(xfx > 0.0, sh(g1, -1, 0), g1)
        fy = yfx * np.where(yfx > 0.0, sh(g2, 0, -1), g2)
        new = (g2 * area + fx - sh(fx, 1, 0) + fy - sh(fy, 0, 1)) / (area + xfx - sh(xfx, 1, 0) + yfx - sh(yfx, 0, 1))
        out[k] = np.where(reg, new, gz[k])
    ws = np.where(reg, (zs - out[km]) * (1.0 / dt), 0.0)
    for k in range(km - 1, -1, -1):
        out[k] = np.where(reg, np.maximum(out[k], out[k + 1] + dz_min), out[k])
    return out, ws


# ---------------- SIM1 column solver ----------------

def sim1_solver(dt, gama, kappa, dm2, pm2, pem, w2, dz2, pt2, ws, p_fac, rgas=RDGAS):
    """All arrays (km, ...) columns; pem (km+1, ...).  Returns pe (km+1) perturbation, w2, dz2."""
    km = dm2.shape[0]
    t1g = gama * 2.0 * dt * dt
    rdt = 1.0 / dt
    capa1 = kappa - 1.0
    pl = np.exp(gama * np.log(-dm2 / dz2 * rgas * pt2)) - pm2
    w1 = w2.copy()
    g_rat = np.zeros_like(dm2)
    bb = np.zeros_like(dm2)
    dd = np.zeros_like(dm2)
    g_rat[:km - 1] = dm2[:km - 1] / dm2[1:]
    bb[:km - 1] = 2.0 * (1.0 + g_rat[:km - 1])
    dd[:km - 1] = 3.0 * (pl[:km - 1] + g_rat[:km - 1] * pl[1:])
    pp = np.zeros((km + 1,) + dm2.shape[1:])
    gam = np.zeros_like(dm2)
    bet = bb[0].copy()
    pp[0] = 0.0
    pp[1] = dd[0] / bet
    bb[km - 1] = 2.0
    dd[km - 1] = 3.0 * pl[km - 1]
    for k in range(1, km):
        gam[k] = g_rat[k - 1] / bet
        bet = bb[k] - gam[k]
        pp[k + 1] = (dd[k] - pp[k]) / bet
    for k in range(km - 1, 0, -1):
        pp[k] = pp[k] - gam[k] * pp[k + 1]
    aa = np.zeros_like(dm2)
    for k in range(1, km):
        aa[k] = t1g / (dz2[k - 1] + dz2[k]) * (pem[k] + pp[k])
    w2 = w2.copy()
    bet = dm2[0] - aa[1]
    w2[0] = (dm2[0] * w1[0] + dt * pp[1]) / bet
    for k in range(1, km - 1):
        gam[k] = aa[k] / bet
        bet = dm2[k] - (aa[k] + aa[k + 1] + aa[k] * gam[k])
        w2[k] = (dm2[k] * w1[k] + dt * (pp[k + 1] - pp[k]) - aa[k] * w2[k - 1]) / bet
    p1 = t1g / dz2[km - 1] * (pem[km] + pp[km])
    gam[km - 1] = aa[km - 1] / bet
    bet = dm2[km - 1] - (aa[km - 1] + p1 + aa[km - 1] * gam[km - 1])
    w2[km - 1] = (dm2[km - 1] * w1[km - 1] + dt * (pp[km] - pp[km - 1]) - p1 * ws - aa[km - 1] * w2[km - 2]) / bet
    for k in range(km - 2, -1, -1):
        w2[k] = w2[k] - gam[k + 1] * w2[k + 1]
    pe = np.zeros_like(pp)
    for k in range(km):
        pe[k + 1] = pe[k] + dm2[k] * (w2[k] - w1[k]) * rdt
    dz2 = dz2.copy()
    p1 = (pe[km - 1] + 2.0 * pe[km]) * R3
    dz2[km - 1] = -dm2[km - 1] * rgas * pt2[km - 1] * np.exp(capa1 * np.log(np.maximum(p_fac * pm2[km - 1], p1 + pm2[km - 1])))
    for k in range(km - 2, -1, -1):
        p1 = (pe[k] + bb[k] * pe[k + 1] + g_rat[k] * pe[k + 2]) * R3 - g_rat[k] * p1
        dz2[k] = -dm2[k] * rgas * pt2[k] * np.exp(capa1 * np.log(np.maximum(p_fac * pm2[k], p1 + pm2[k])))
    return pe, w2, dz2


def riem_solver_c(dt, delpc, ptc, wc, gz, hs, ws, ptop, p_fac, reg):
    """C-grid Riemann solve on the columns of mask `reg`.  gz: heights in, geopotential out."""
    km = delpc.shape[0]
    gama = 1.0 / (1.0 - KAPPA)
    dm = delpc.copy()
    pem = np.zeros((km + 1,) + dm.shape[1:])
    pem[0] = ptop
    for k in range(1, km + 1):
        pem[k] = pem[k - 1] + dm[k - 1]
    dz2 = gz[1:] - gz[:-1]
    pm2 = dm / np.log(pem[1:] / pem[:-1])
    dm = dm * (1.0 / GRAV)
    pe2, w2, dz2 = sim1_solver(dt, gama, KAPPA, dm, pm2, pem, wc.copy(), dz2, ptc, ws, p_fac)
    pef = np.zeros_like(pem)
    pef[0] = ptop
    pef[1:] = pe2[1:] + pem[1:]
    gzo = np.zeros_like(gz)
    gzo[km] = hs
    for k in range(km - 1, -1, -1):
        gzo[k] = gzo[k + 1] - dz2[k] * GRAV
    pef = np.where(reg, pef, 0.0)
    gzo = np.where(reg, gzo, gz)
    return pef, gzo


def riem_solver3(dt, delp, pt, w, zh, zs, ws, ptop, p_fac, reg, last_call=True):
    """Full-step Riemann solve: returns w, delz, zh, ppe (perturbation), pk3, pe, peln, pk."""
    km = delp.shape[0]
    gama = 1.0 / (1.0 - KAPPA)
    peln1 = np.log(ptop)
    ptk = np.exp(KAPPA * peln1)
    dm = delp.copy()
    pem = np.zeros((km + 1,) + dm.shape[1:])
    peln2 = np.zeros_like(pem)
    pk3 = np.zeros_like(pem)
    pem[0] = ptop
    peln2[0] = peln1
    pk3[0] = ptk
    for k in range(1, km + 1):
        pem[k] = pem[k - 1] + dm[k - 1]
        peln2[k] = np.log(pem[k])
        pk3[k] = np.exp(KAPPA * peln2[k])
    pm2 = dm / (peln2[1:] - peln2[:-1])
    dm = dm * (1.0 / GRAV)
    dz2 = zh[1:] - zh[:-1]
    pe2, w2, dz2 = sim1_solver(dt, gama, KAPPA, dm, pm2, pem, w.copy(), dz2, pt, ws, p_fac)
    zho = np.zeros_like(zh)
    zho[km] = zs
    for k in range(km - 1, -1, -1):
        zho[k] = zho[k + 1] - dz2[k]
    r = reg
    return dict(w=np.where(r, w2, w), delz=np.where(r, dz2, 0.0), zh=np.where(r, zho, zh),
                ppe=np.where(r, pe2, 0.0), pk3=np.where(r, pk3, 0.0), pe=np.where(r, pem, 0.0),
                peln=np.where(r, peln2, 0.0), pk=np.where(r, pk3, 0.0))


# ---------------- p_grad_c ----------------

def p_grad_c(uc, vc, delpc, pkc, gz, m, P, dt2):
    nx, ny = P.nx, P.ny
    wk = delpc
    rdxc, rdyc = m["rdxc"], m["rdyc"]
    gzu, gzl = gz[:-1], gz[1:]     # k, k+1
    pku, pkl = pkc[:-1], pkc[1:]
    du = dt2 * rdxc / (sh(wk, -1, 0) + wk) * ((sh(gzl, -1, 0) - gzu) * (pkl - sh(pku, -1, 0))
                                             + (sh(gzu, -1, 0) - gzl) * (sh(pkl, -1, 0) - pku))
    dv = dt2 * rdyc / (sh(wk, 0, -1) + wk) * ((sh(gzl, 0, -1) - gzu) * (pkl - sh(pku, 0, -1))
                                             + (sh(gzu, 0, -1) - gzl) * (sh(pkl, 0, -1) - pku))
    uco = np.where(P.reg(0, nx, 0, ny - 1), uc + du, uc)
    vco = np.where(P.reg(0, nx - 1, 0, ny), vc + dv, vc)
    return uco, vco


# ---------------- edge_profile + update_dz_d ----------------

def edge_profile(q, dp0):
    """interface values (km+1, ...) of q (km, ...), non-uniform grid, limiter = 0"""
    km = q.shape[0]
    qe = np.zeros((km + 1,) + q.shape[1:])
    gam = np.zeros((km + 1,) + q.shape[1:])
    g0 = dp0[1] / dp0[0]
    xt1 = 2.0 * g0 * (g0 + 1.0)
    bet = g0 * (g0 + 0.5)
    qe[0] = (xt1 * q[0] + q[1]) / bet
    gam[0] = (1.0 + g0 * (g0 + 1.5)) / bet
    gk = g0
    for k in range(1, km):
        gk = dp0[k - 1] / dp0[k]
        bet = 2.0 + 2.0 * gk - gam[k - 1]
        qe[k] = (3.0 * (q[k - 1] + gk * q[k]) - qe[k - 1]) / bet
        gam[k] = gk / bet
    a_bot = 1.0 + gk * (gk + 1.5)
    xt1 = 2.0 * gk * (gk + 1.0)
    xt2 = gk * (gk + 0.5) - a_bot * gam[km - 1]
    qe[km] = (xt1 * q[km - 1] + q[km - 2] - a_bot * qe[km - 1]) / xt2
    for k in range(km - 1, -1, -1):
        qe[k] = qe[k] - gam[k] * qe[k + 1]
    return qe


def update_dz_d_transport(zh, crx, cry, xfx, yfx, sub, m, nx, ny, dp0, hord):
    """the interface heights zh transported with the interface-level Courant numbers and
    area fluxes (edge_profile, fv_tp_2d, flux-form update); compute cells updated, the
    rest of the plane unchanged.  FV3 update_dz_d before its dz_min clamp."""
    P = Plane(sub, nx, ny, zh.shape[-2], zh.shape[-1])
    rx = P.reg(0, nx, -NG, ny + NG - 1)
    ry = P.reg(-NG, nx + NG - 1, 0, ny)
    crx_e = np.where(rx, edge_profile(crx, dp0), 0.0)
    xfx_e = np.where(rx, edge_profile(xfx, dp0), 0.0)
    cry_e = np.where(ry, edge_profile(cry, dp0), 0.0)
    yfx_e = np.where(ry, edge_profile(yfx, dp0), 0.0)
    area = m["area"]
    ra_x = np.where(P.reg(0, nx - 1, -NG, ny + NG - 1), area + xfx_e - sh(xfx_e, 1, 0), 0.0)
    ra_y = np.where(P.reg(-NG, nx + NG - 1, 0, ny - 1), area + yfx_e - sh(yfx_e, 0, 1), 0.0)
    fx, fy = fv_tp_2d(zh, crx_e, cry_e, xfx_e, yfx_e, ra_x, ra_y, sub, m, nx, ny, hord)
    comp = P.reg(0, nx - 1, 0, ny - 1)
    new = (zh * area + fx - sh(fx, 1, 0) + fy - sh(fy, 0, 1)) / (ra_x + ra_y - area)
    return np.where(comp, new, zh)


def update_dz_d(zh, crx, cry, xfx, yfx, zs, sub, m, nx, ny, dp0, dt, hord, dz_min, damp=None):
    """FV3 nh_utils update_dz_d: the heights transported (update_dz_d_transport), plus, on the
    interfaces whose damp_vt > 1e-5, del6_vt_flux's diffusive fluxes of the old heights with
    coefficient (damp_vt da_min_c)^(nord_v+1) (`damp`: per interface level (nord_v, coefficient
    or 0); FV3 damp(km+1) = damp(km)), zh += div(fx2, fy2) rarea; then the dz_min clamp and ws"""
    km = crx.shape[0]
    P = Plane(sub, nx, ny, zh.shape[-2], zh.shape[-1])
    comp = P.reg(0, nx - 1, 0, ny - 1)
    out = update_dz_d_transport(zh, crx, cry, xfx, yfx, sub, m, nx, ny, dp0, hord)
    if damp is not None:
        from .sw_core import deln_flux
        for k, (nord_v, coef) in enumerate(damp):
            if coef > 0.0:
                fx2, fy2 = deln_flux(nord_v, coef, zh[k], sub, m, nx, ny)
                out[k] = np.where(comp, out[k] + (fx2 - sh(fx2, 1, 0) + fy2 - sh(fy2, 0, 1)) * m["rarea"], out[k])
    ws = np.where(comp, (zs - out[km]) * (1.0 / dt), 0.0)
    for k in range(km - 1, -1, -1):
        out[k] = np.where(comp, np.maximum(out[k], out[k + 1] + dz_min), out[k])
    return out, ws


# ---------------- halo pressure helpers ----------------

def pk3_halo(pk3, delp, ptop, P):
    """p**kappa on the 2-wide halo ring from the (halo-updated) delp"""
    nx, ny = P.nx, P.ny
    ring = (P.reg(-2, nx + 1, -2, ny + 1)) & ~P.reg(0, nx - 1, 0, ny - 1)
    pei = np.full(delp.shape[1:], ptop)
    out = pk3.copy()
    for k in range(delp.shape[0]):
        pei = pei + delp[k]
        out[k + 1] = np.where(ring, np.exp(KAPPA * np.log(pei)), pk3[k + 1])
    return out


def pe_halo(pe, delp, ptop, P):
    nx, ny = P.nx, P.ny
    ring = P.reg(-1, nx, -1, ny) & ~P.reg(0, nx - 1, 0, ny - 1)
    out = pe.copy()
    out[0] = np.where(ring, ptop, pe[0])
    acc = np.full(delp.shape[1:], ptop)
    for k in range(delp.shape[0]):
        acc = acc + delp[k]
        out[k + 1] = np.where(ring, acc, pe[k + 1])
    return out


# ---------------- a2b_ord4 + nh_p_grad ----------------

B1, B2 = 7.0 / 12.0, -1.0 / 12.0
A1, A2 = 0.5625, -0.0625
AC1, AC2 = 2.0 / 3.0, -1.0 / 6.0


def a2b_ord4(q, P, m, corner_w):
    """cell -> corner 4th-order interpolation with cubed-sphere edge/corner treatment.
    q: (nk, nj, pitch); returns corner values on local [0,nx]x[0,ny] (zeros elsewhere)."""
    N, io, jo, nx, ny = P.N, P.io, P.jo, P.nx, P.ny
    I, J = P.I, P.J
    dxa, dya = m["dxa"], m["dya"]
    qx = np.zeros_like(q)
    qy = np.zeros_like(q)
    # qx: interior then tile edges
    rows = (J >= max(0, jo - 2)) & (J <= min(N - 1, jo + ny + 1))
    gen = B2 * (sh(q, -2, 0) + sh(q, 1, 0)) + B1 * (sh(q, -1, 0) + q)
    qx = np.where(rows & (I >= max(2, io)) & (I <= min(N - 2, io + nx)), gen, qx)
    gr_w = sh(dxa, 1, 0) / dxa          # at I = 0: dxa(1)/dxa(0)
    qx0 = 0.5 * ((2.0 + gr_w) * (sh(q, -1, 0) + q) - (sh(q, -2, 0) + sh(q, 1, 0))) / (1.0 + gr_w)
    gr_e = sh(dxa, -2, 0) / sh(dxa, -1, 0)  # at I = N: dxa(N-2)/dxa(N-1)
    qxN = 0.5 * ((2.0 + gr_e) * (sh(q, -1, 0) + q) - (sh(q, -2, 0) + sh(q, 1, 0))) / (1.0 + gr_e)
    qx = np.where(rows & (I == 0), qx0, qx)
    qx = np.where(rows & (I == N), qxN, qx)
    # I = 1: uses qx(0) and qx(2)
    g1 = sh(dxa, 0, 0) / sh(dxa, -1, 0)  # at I = 1: dxa(1)/dxa(0)
    qx1 = (3.0 * (g1 * sh(q, -1, 0) + q) - (g1 * sh(qx, -1, 0) + sh(qx, 1, 0))) / (2.0 + 2.0 * g1)
    gN1 = sh(dxa, -1, 0) / dxa           # at I = N-1: dxa(N-2)/dxa(N-1)
    qxN1 = (3.0 * (sh(q, -1, 0) + gN1 * q) - (gN1 * sh(qx, 1, 0) + sh(qx, -1, 0))) / (2.0 + 2.0 * gN1)
    qx = np.where(rows & (I == 1), qx1, qx)
    qx = np.where(rows & (I == N - 1), qxN1, qx)
    # qy
    cols = (I >= max(0, io - 2)) & (I <= min(N - 1, io + nx + 1))
    gen = B2 * (sh(q, 0, -2) + sh(q, 0, 1)) + B1 * (sh(q, 0, -1) + q)
    qy = np.where(cols & (J >= max(2, jo)) & (J <= min(N - 2, jo + ny)), gen, qy)
    gr_s = sh(dya, 0, 1) / dya
    qy0 = 0.5 * ((2.0 + gr_s) * (sh(q, 0, -1) + q) - (sh(q, 0, -2) + sh(q, 0, 1))) / (1.0 + gr_s)
    gr_n = sh(dya, 0, -2) / sh(dya, 0, -1)
    qyN = 0.5 * ((2.0 + gr_n) * (sh(q, 0, -1) + q) - (sh(q, 0, -2) + sh(q, 0, 1))) / (1.0 + gr_n)
    qy = np.where(cols & (J == 0), qy0, qy)
    qy = np.where(cols & (J == N), qyN, qy)
    g1 = dya / sh(dya, 0, -1)
    qy1 = (3.0 * (g1 * sh(q, 0, -1) + q) - (g1 * sh(qy, 0, -1) + sh(qy, 0, 1))) / (2.0 + 2.0 * g1)
    gN1 = sh(dya, 0, -1) / dya
    qyN1 = (3.0 * (sh(q, 0, -1) + gN1 * q) - (gN1 * sh(qy, 0, 1) + sh(qy, 0, -1))) / (2.0 + 2.0 * gN1)
    qy = np.where(cols & (J == 1), qy1, qy)
    qy = np.where(cols & (J == N - 1), qyN1, qy)

    qout = np.zeros_like(q)

    def put(Ig, Jg, val):
        jj, ii = P.slot(Ig, Jg)
        qout[:, jj, ii] = val

    def g(arr, Ig, Jg):
        jj, ii = P.slot(Ig, Jg)
        return arr[..., jj, ii]

    pairs = [
        [(0, 0, 1, 1), (-1, 0, -2, 1), (0, -1, 1, -2)],
        [(N - 1, 0, N - 2, 1), (N - 1, -1, N - 2, -2), (N, 0, N + 1, 1)],
        [(N - 1, N - 1, N - 2, N - 2), (N, N - 1, N + 1, N - 2), (N - 1, N, N - 2, N + 1)],
        [(0, N - 1, 1, N - 2), (-1, N - 1, -2, N - 2), (0, N, 1, N + 1)],
    ]
    cpos = [(0, 0), (N, 0), (N, N), (0, N)]
    for c, (cx, cy) in enumerate(cpos):
        if not P.owns(cx, cy):
            continue
        acc = None
        for r in range(3):
            i1, j1, i2, j2 = pairs[c][r]
            q1, q2 = g(q, i1, j1), g(q, i2, j2)
            e = q1 + corner_w[c, r] * (q1 - q2)
            acc = e if acc is None else acc + e
        put(cx, cy, acc * R3)
    # W/E edge columns
    edge_rows = (J >= max(2, jo)) & (J <= min(N - 2, jo + ny))
    colv = A2 * (sh(qx, 0, -2) + sh(qx, 0, 1)) + A1 * (sh(qx, 0, -1) + qx)
    qout = np.where(edge_rows & ((I == 0) | (I == N)), colv, qout)
    rowv = A2 * (sh(qy, -2, 0) + sh(qy, 1, 0)) + A1 * (sh(qy, -1, 0) + qy)
    edge_cols = (I >= max(2, io)) & (I <= min(N - 2, io + nx))
    qout = np.where(edge_cols & ((J == 0) | (J == N)), rowv, qout)
    # points next to the cube corners along the edges
    for (Ig, Jg, a, b, c_, d_) in ((0, 1, (0, 0), (0, 1), (0, 0), (0, 2)), (0, N - 1, (0, N - 2), (0, N - 1), (0, N - 2), (0, N)),
                                   (N, 1, (N, 0), (N, 1), (N, 0), (N, 2)), (N, N - 1, (N, N - 2), (N, N - 1), (N, N - 2), (N, N))):
        if P.owns(Ig, Jg) and ((Jg == 1 and jo == 0) or (Jg == N - 1 and jo + ny == N)) and (Ig == 0 and io == 0 or Ig == N and io + nx == N):
            put(Ig, Jg, AC1 * (g(qx, *a) + g(qx, *b)) + AC2 * (g(qout, *c_) + g(qout, *d_)))
    for (Ig, Jg, a, b, c_, d_) in ((1, 0, (0, 0), (1, 0), (0, 0), (2, 0)), (N - 1, 0, (N - 2, 0), (N - 1, 0), (N - 2, 0), (N, 0)),
                                   (1, N, (0, N), (1, N), (0, N), (2, N)), (N - 1, N, (N - 2, N), (N - 1, N), (N - 2, N), (N, N))):
        if P.owns(Ig, Jg) and ((Ig == 1 and io == 0) or (Ig == N - 1 and io + nx == N)) and (Jg == 0 and jo == 0 or Jg == N and jo + ny == N):
            put(Ig, Jg, AC1 * (g(qy, *a) + g(qy, *b)) + AC2 * (g(qout, *c_) + g(qout, *d_)))
    # interior: average of the x-then-y and y-then-x interpolants
    irows = (J >= max(2, jo)) & (J <= min(N - 2, jo + ny))
    icols = (I >= max(1, io)) & (I <= min(N - 1, io + nx))
    qxx = np.where(irows & icols, A2 * (sh(qx, 0, -2) + sh(qx, 0, 1)) + A1 * (sh(qx, 0, -1) + qx), 0.0)
    qxx1 = AC1 * (sh(qx, 0, -1) + qx) + AC2 * (sh(qout, 0, -1) + sh(qxx, 0, 1))
    qxx = np.where(icols & (J == 1), qxx1, qxx)
    qxxN = AC1 * (sh(qx, 0, -1) + qx) + AC2 * (sh(qout, 0, 1) + sh(qxx, 0, -1))
    qxx = np.where(icols & (J == N - 1), qxxN, qxx)
    jrows = (J >= max(1, jo)) & (J <= min(N - 1, jo + ny))
    jcols = (I >= max(2, io)) & (I <= min(N - 2, io + nx))
    qyy = np.where(jrows & jcols, A2 * (sh(qy, -2, 0) + sh(qy, 1, 0)) + A1 * (sh(qy, -1, 0) + qy), 0.0)
    qyy1 = AC1 * (sh(qy, -1, 0) + qy) + AC2 * (sh(qout, -1, 0) + sh(qyy, 1, 0))
    qyy = np.where(jrows & (I == 1), qyy1, qyy)
    qyyN = AC1 * (sh(qy, -1, 0) + qy) + AC2 * (sh(qout, 1, 0) + sh(qyy, -1, 0))
    qyy = np.where(jrows & (I == N - 1), qyyN, qyy)
    inner = jrows & icols
    qout = np.where(inner, 0.5 * (qxx + qyy), qout)
    return np.where(P.reg(0, nx, 0, ny), qout, 0.0)


def nh_p_grad(u, v, pp, gz, delp, pk, dt, ptop, P, m, corner_w):
    """u, v arrive multiplied by dx, dy (from d_sw); returns the new winds.
    pp: non-hydrostatic perturbation (npz+1), gz: geopotential (npz+1), pk: p**kappa (npz+1)."""
    km = delp.shape[0]
    nx, ny = P.nx, P.ny
    ptk = np.exp(KAPPA * np.log(ptop))
    ppb = a2b_ord4(pp, P, m, corner_w)
    pkb = a2b_ord4(pk, P, m, corner_w)
    gzb = a2b_ord4(gz, P, m, corner_w)
    ppb[0] = 0.0
    pkb[0] = ptk
    wk1 = a2b_ord4(delp, P, m, corner_w)
    wk = pkb[1:] - pkb[:-1]
    gu, gl = gzb[:-1], gzb[1:]
    ku, kl = pkb[:-1], pkb[1:]
    pu, pl = ppb[:-1], ppb[1:]
    du1 = dt / (wk + sh(wk, 1, 0)) * ((gl - sh(gu, 1, 0)) * (sh(kl, 1, 0) - ku) + (gu - sh(gl, 1, 0)) * (kl - sh(ku, 1, 0)))
    un = (u + du1 + dt / (wk1 + sh(wk1, 1, 0)) * ((gl - sh(gu, 1, 0)) * (sh(pl, 1, 0) - pu)
                                                 + (gu - sh(gl, 1, 0)) * (pl - sh(pu, 1, 0)))) * m["rdx"]
    dv1 = dt / (wk + sh(wk, 0, 1)) * ((gl - sh(gu, 0, 1)) * (sh(kl, 0, 1) - ku) + (gu - sh(gl, 0, 1)) * (kl - sh(ku, 0, 1)))
    vn = (v + dv1 + dt / (wk1 + sh(wk1, 0, 1)) * ((gl - sh(gu, 0, 1)) * (sh(pl, 0, 1) - pu)
                                                 + (gu - sh(gl, 0, 1)) * (pl - sh(pu, 0, 1)))) * m["rdy"]
    uo = np.where(P.reg(0, nx - 1, 0, ny), un, u)
    vo = np.where(P.reg(0, nx, 0, ny - 1), vn, v)
    return uo, vo
