"""Oracle: FV3 sw_core — c_sw (with d2a2c_vect and, for nord > 0, divergence_corner) and
d_sw (divergence damping nord = 0 .. 3 with the del-2 Smagorinsky-type coefficient, del-2n
vorticity damping damp_vt / nord_v, the del-n mass-flux damping of delp (damp_vt / nord_v) and
the mass-weighted del-n damping of pt (damp_t / nord_t) inside fv_tp_2d (tp_core deln_flux),
the w damping (damp_w / nord_w) with its heat, the d_con conversion of the damped kinetic
energy into heat and the dissipation estimate diss_est) in fp64 numpy, with the per-level
parameters of FV3 dyn_core's k loop -- the sponge-layer overrides in the top three levels
included (column_namelist).  TEST INFRASTRUCTURE ONLY.

Restated from the FV3 C-D grid shallow-water solver (Lin & Rood 1997; Harris &
Lin 2013; FV3 sw_core.F90 structure).  Fortran 1-based indices f are written
here as 0-based tile-global g = f - 1 (npx -> N).  Arrays per sub-domain are
(nk, nj, pitch) planes, a[k, j+NG, i+NG].
"""
import numpy as np

from . import NG
from .tp_core import copy_corners, fv_tp_2d

np.seterr(all="ignore")  # NaN/inf only arise outside the compared regions
from .util import Plane, sh

A1, A2 = 0.5625, -0.0625
C1, C2, C3 = -2.0 / 14.0, 11.0 / 14.0, 5.0 / 14.0
BIG = 1.0e8


def _ei4(u0, u1, u2, u3, d0, d1, d2, d3):
    """edge_interpolate4"""
    t1 = d0 + d1
    t2 = d2 + d3
    return 0.5 * (((t1 + d1) * u1 - d1 * u0) / t1 + ((t2 + d2) * u2 - d2 * u3) / t2)


def d2a2c_vect(u, v, P, m):
    """D-grid (u,v) -> A-grid (ua,va) and C-grid (uc,vc), contravariant ut, vt."""
    N, nx, ny, io, jo = P.N, P.nx, P.ny, P.io, P.jo
    I, J = P.I, P.J
    cosa_s, rsin2 = m["cosa_s"], m["rsin2"]
    utmp = np.full_like(u, BIG)
    vtmp = np.full_like(v, BIG)
    # interior
    rows = (J >= max(3, jo - 1)) & (J <= min(N - 4, jo + ny)) & (P.li >= -NG) & (P.li <= nx + NG - 1)
    utmp = np.where(rows, A2 * (sh(u, 0, -1) + sh(u, 0, 2)) + A1 * (u + sh(u, 0, 1)), utmp)
    cols = (I >= max(3, io - 1)) & (I <= min(N - 4, io + nx)) & (P.lj >= -NG) & (P.lj <= ny + NG - 1)
    vtmp = np.where(cols, A2 * (sh(v, -1, 0) + sh(v, 2, 0)) + A1 * (v + sh(v, 1, 0)), vtmp)
    u2 = 0.5 * (u + sh(u, 0, 1))
    v2 = 0.5 * (v + sh(v, 1, 0))
    allc = (P.li >= -NG) & (P.li <= nx + NG - 1)
    allr = (P.lj >= -NG) & (P.lj <= ny + NG - 1)
    # tile-edge zones (npt = 4: three cells each side, matching the halo width so the
    # zone reads the same from both tiles), applied wherever this sub-domain's halo reaches them
    # (FV3: `js==1 .or. jsd<npt` etc.), so the result does not depend on the layout
    jsd, jed, isd, ied = jo - NG, jo + ny + NG - 1, io - NG, io + nx + NG - 1
    msk = allc & (J >= jsd) & (J <= 2)  # south edge rows
    utmp = np.where(msk, u2, utmp)
    vtmp = np.where(msk, v2, vtmp)
    msk = allc & (J >= N - 3) & (J <= jed)  # north edge rows
    utmp = np.where(msk, u2, utmp)
    vtmp = np.where(msk, v2, vtmp)
    midrows = (J >= max(3, jsd)) & (J <= min(N - 4, jed))
    msk = midrows & (I >= isd) & (I <= 2)  # west edge columns
    utmp = np.where(msk, u2, utmp)
    vtmp = np.where(msk, v2, vtmp)
    msk = midrows & (I >= N - 3) & (I <= ied)  # east edge columns
    utmp = np.where(msk, u2, utmp)
    vtmp = np.where(msk, v2, vtmp)
    del allr
    ua = np.zeros_like(u)
    va = np.zeros_like(v)
    reg = P.reg(-2, nx + 1, -2, ny + 1)
    ua = np.where(reg, (utmp - vtmp * cosa_s) * rsin2, ua)
    va = np.where(reg, (vtmp - utmp * cosa_s) * rsin2, va)

    def setp(arr, Ig, Jg, val):
        if 0 <= Jg - jo + NG < P.nj and 0 <= Ig - io + NG < P.pitch:
            arr[:, Jg - jo + NG, Ig - io + NG] = val

    def getp(arr, Ig, Jg):
        return arr[:, Jg - jo + NG, Ig - io + NG]

    sw, se = P.owns(0, 0), P.owns(N, 0)
    ne, nw = P.owns(N, N), P.owns(0, N)
    # corner fixes (reads of generic values only)
    ut0, vt0, ua0, va0 = utmp.copy(), vtmp.copy(), ua.copy(), va.copy()
    if sw:
        for Ig in (-3, -2, -1):
            setp(utmp, Ig, -1, -getp(vt0, -1, -Ig - 1))
        for Jg in (-3, -2, -1):
            setp(vtmp, -1, Jg, -getp(ut0, -Jg - 1, -1))
        setp(ua, -2, -1, -getp(va0, -1, 1))
        setp(ua, -1, -1, -getp(va0, -1, 0))
        setp(va, -1, -2, -getp(ua0, 1, -1))
        setp(va, -1, -1, -getp(ua0, 0, -1))
    if se:
        for i in (0, 1, 2):
            setp(utmp, N + i, -1, getp(vt0, N, i))
        for Jg in (-3, -2, -1):
            setp(vtmp, N, Jg, getp(ut0, N + Jg, -1))
        setp(ua, N, -1, getp(va0, N, 0))
        setp(ua, N + 1, -1, getp(va0, N, 1))
        setp(va, N, -1, getp(ua0, N - 1, -1))
        setp(va, N, -2, getp(ua0, N - 2, -1))
    if ne:
        for i in (0, 1, 2):
            setp(utmp, N + i, N, -getp(vt0, N, N - 1 - i))
        for j in (0, 1, 2):
            setp(vtmp, N, N + j, -getp(ut0, N - j - 1, N))
        setp(ua, N, N, -getp(va0, N, N - 1))
        setp(ua, N + 1, N, -getp(va0, N, N - 2))
        setp(va, N, N, -getp(ua0, N - 1, N))
        setp(va, N, N + 1, -getp(ua0, N - 2, N))
    if nw:
        for Ig in (-3, -2, -1):
            setp(utmp, Ig, N, getp(vt0, -1, N + Ig))
        for j in (0, 1, 2):
            setp(vtmp, -1, N + j, getp(ut0, j, N))
        setp(ua, -2, N, getp(va0, -1, N - 2))
        setp(ua, -1, N, getp(va0, -1, N - 1))
        setp(va, -1, N, getp(ua0, 0, N))
        setp(va, -1, N + 1, getp(ua0, 1, N))

    cosa_u, rsin_u, cosa_v, rsin_v = m["cosa_u"], m["rsin_u"], m["cosa_v"], m["rsin_v"]
    dxa, dya, s1, s2, s3, s4 = m["dxa"], m["dya"], m["sin_sg1"], m["sin_sg2"], m["sin_sg3"], m["sin_sg4"]
    # x: uc, ut at y-edges, local i in [-1, nx+1], j in [-1, ny]
    reg = P.reg(-1, nx + 1, -1, ny)
    gen = A2 * (sh(utmp, -2, 0) + sh(utmp, 1, 0)) + A1 * (sh(utmp, -1, 0) + utmp)
    e_m1 = C1 * sh(utmp, -2, 0) + C2 * sh(utmp, -1, 0) + C3 * utmp  # g = -1 and g = N-1
    e_p1 = C1 * sh(utmp, 1, 0) + C2 * utmp + C3 * sh(utmp, -1, 0)  # g = 1
    e_np1 = C3 * sh(utmp, -1, 0) + C2 * utmp + C1 * sh(utmp, 1, 0)  # g = N+1
    with np.errstate(all="ignore"):
        e0 = _ei4(sh(ua, -2, 0), sh(ua, -1, 0), ua, sh(ua, 1, 0), sh(dxa, -2, 0), sh(dxa, -1, 0), dxa, sh(dxa, 1, 0))
    uc = np.zeros_like(u)
    uc = np.where(reg, gen, uc)
    uc = np.where(reg & ((I == -1) | (I == N - 1)), e_m1, uc)
    uc = np.where(reg & (I == 1), e_p1, uc)
    uc = np.where(reg & (I == N + 1), e_np1, uc)
    edge = reg & ((I == 0) | (I == N))
    uc = np.where(edge, e0 * np.where(e0 > 0.0, sh(s3, -1, 0), s1), uc)
    ut = np.zeros_like(u)
    ut = np.where(reg, (uc - v * cosa_u) * rsin_u, ut)
    ut = np.where(edge, e0, ut)
    # y: vc, vt at x-edges, local i in [-1, nx], j in [-1, ny+1]
    reg = P.reg(-1, nx, -1, ny + 1)
    gen = A2 * (sh(vtmp, 0, -2) + sh(vtmp, 0, 1)) + A1 * (sh(vtmp, 0, -1) + vtmp)
    e_m1 = C1 * sh(vtmp, 0, -2) + C2 * sh(vtmp, 0, -1) + C3 * vtmp
    e_p1 = C1 * sh(vtmp, 0, 1) + C2 * vtmp + C3 * sh(vtmp, 0, -1)
    with np.errstate(all="ignore"):
        e0 = _ei4(sh(va, 0, -2), sh(va, 0, -1), va, sh(va, 0, 1), sh(dya, 0, -2), sh(dya, 0, -1), dya, sh(dya, 0, 1))
    vc = np.zeros_like(v)
    vc = np.where(reg, gen, vc)
    vc = np.where(reg & ((J == -1) | (J == N - 1)), e_m1, vc)
    vc = np.where(reg & ((J == 1) | (J == N + 1)), e_p1, vc)
    edge = reg & ((J == 0) | (J == N))
    vc = np.where(edge, e0 * np.where(e0 > 0.0, sh(s4, 0, -1), s2), vc)
    vt = np.zeros_like(v)
    vt = np.where(reg, (vc - u * cosa_v) * rsin_v, vt)
    vt = np.where(edge, e0, vt)
    return ua, va, uc, vc, ut, vt


def c_sw(delp, pt, u, v, w, sub, m, nx, ny, dt2):
    """FV3 c_sw (non-hydrostatic, nord = 0): returns delpc, ptc, wc, uc, vc, ua, va, ut, vt
    (ut, vt scaled to dt2 * area fluxes)."""
    P = Plane(sub, nx, ny, u.shape[-2], u.shape[-1])
    N, I, J = P.N, P.I, P.J
    ua, va, uc, vc, ut, vt = d2a2c_vect(u, v, P, m)
    s1, s2, s3, s4 = m["sin_sg1"], m["sin_sg2"], m["sin_sg3"], m["sin_sg4"]
    c1_, c2_, c3_, c4_ = m["cos_sg1"], m["cos_sg2"], m["cos_sg3"], m["cos_sg4"]
    dx, dy = m["dx"], m["dy"]
    reg = P.reg(-1, nx + 1, -1, ny)
    ut = np.where(reg, np.where(ut > 0.0, dt2 * ut * dy * sh(s3, -1, 0), dt2 * ut * dy * s1), ut)
    reg = P.reg(-1, nx, -1, ny + 1)
    vt = np.where(reg, np.where(vt > 0.0, dt2 * vt * dx * sh(s4, 0, -1), dt2 * vt * dx * s2), vt)
    # first-order upwind transport of delp, pt, w (fill_4corners via copy_corners)
    dpx, ptx, wx = (copy_corners(a, sub, 1) for a in (delp, pt, w))
    dpy, pty, wy = (copy_corners(a, sub, 2) for a in (delp, pt, w))
    fx1 = np.where(ut > 0.0, sh(dpx, -1, 0), dpx)
    fx = np.where(ut > 0.0, sh(ptx, -1, 0), ptx)
    fx2 = np.where(ut > 0.0, sh(wx, -1, 0), wx)
    fx1 = ut * fx1
    fx = fx1 * fx
    fx2 = fx1 * fx2
    fy1 = np.where(vt > 0.0, sh(dpy, 0, -1), dpy)
    fy = np.where(vt > 0.0, sh(pty, 0, -1), pty)
    fy2 = np.where(vt > 0.0, sh(wy, 0, -1), wy)
    fy1 = vt * fy1
    fy = fy1 * fy
    fy2 = fy1 * fy2
    rarea = m["rarea"]
    reg = P.reg(-1, nx, -1, ny)
    delpc = np.zeros_like(delp)
    ptc = np.zeros_like(pt)
    wc = np.zeros_like(w)
    dpc_ = dpy + (fx1 - sh(fx1, 1, 0) + fy1 - sh(fy1, 0, 1)) * rarea
    delpc = np.where(reg, dpc_, delpc)
    ptc = np.where(reg, (pty * dpy + (fx - sh(fx, 1, 0) + fy - sh(fy, 0, 1)) * rarea) / dpc_, ptc)
    wc = np.where(reg, (wy * dpy + (fx2 - sh(fx2, 1, 0) + fy2 - sh(fy2, 0, 1)) * rarea) / dpc_, wc)
    # kinetic energy at cell centres from upwind C-grid winds
    kpos = np.where(I == 0, uc * s1 + v * c1_, np.where(I == N, uc * s1 + v * c1_, uc))
    ucE, vE = sh(uc, 1, 0), sh(v, 1, 0)
    kneg = np.where(I == -1, ucE * s3 + vE * c3_, np.where(I == N - 1, ucE * s3 + vE * c3_, ucE))
    ke = np.where(ua > 0.0, kpos, kneg)
    vpos = np.where(J == 0, vc * s2 + u * c2_, np.where(J == N, vc * s2 + u * c2_, vc))
    vcN, uN = sh(vc, 0, 1), sh(u, 0, 1)
    vneg = np.where(J == -1, vcN * s4 + uN * c4_, np.where(J == N - 1, vcN * s4 + uN * c4_, vcN))
    vort = np.where(va > 0.0, vpos, vneg)
    dt4 = 0.5 * dt2
    ke = np.where(reg, dt4 * (ua * ke + va * vort), 0.0)
    # circulation -> absolute vorticity at cell corners
    fxc = uc * m["dxc"]
    fyc = vc * m["dyc"]
    vortc = sh(fxc, 0, -1) - fxc - sh(fyc, -1, 0) + fyc
    fy_w = sh(fyc, -1, 0)
    vortc = np.where(P.at(0, 0), vortc + fy_w, vortc)
    vortc = np.where(P.at(N, 0), vortc - fyc, vortc)
    vortc = np.where(P.at(N, N), vortc - fyc, vortc)
    vortc = np.where(P.at(0, N), vortc + fy_w, vortc)
    vortc = m["fC"] + m["rarea_c"] * vortc
    # vorticity flux + KE gradient update of uc, vc
    cosa_u, sina_u, cosa_v, sina_v = m["cosa_u"], m["sina_u"], m["cosa_v"], m["sina_v"]
    fy1v = np.where((I == 0) | (I == N), dt2 * v, dt2 * (v - uc * cosa_u) / sina_u)
    fyv = np.where(fy1v > 0.0, vortc, sh(vortc, 0, 1))
    fx1v = np.where((J == 0) | (J == N), dt2 * u, dt2 * (u - vc * cosa_v) / sina_v)
    fxv = np.where(fx1v > 0.0, vortc, sh(vortc, 1, 0))
    ucn = uc + fy1v * fyv + m["rdxc"] * (sh(ke, -1, 0) - ke)
    vcn = vc - fx1v * fxv + m["rdyc"] * (sh(ke, 0, -1) - ke)
    uc = np.where(P.reg(0, nx, 0, ny - 1), ucn, uc)
    vc = np.where(P.reg(0, nx - 1, 0, ny), vcn, vc)
    return dict(delpc=delpc, ptc=ptc, wc=wc, uc=uc, vc=vc, ua=ua, va=va, ut=ut, vt=vt)


# ----------------------------------------------------------------------------------
# d_sw

def _ppm_stag_x(q, c_cfl, spacing, P, ord_, i0, i1, j0, j1):
    """xtp_u: PPM flux of a field stored at x-edge columns (cells) along i, interface = corner i."""
    from .tp_core import xppm
    return xppm(q, c_cfl, spacing, P.io, P.N, ord_, i0, i1, j0, j1)


def d_sw_ut_vt(uc, vc, P, m, dt):
    """contravariant C-grid winds ut, vt with tile-edge and cube-corner treatment"""
    N, I, J, io, jo, nx, ny = P.N, P.I, P.J, P.io, P.jo, P.nx, P.ny
    cosa_u, rsin_u, cosa_v, rsin_v = m["cosa_u"], m["rsin_u"], m["cosa_v"], m["rsin_v"]
    s1, s2, s3, s4 = m["sin_sg1"], m["sin_sg2"], m["sin_sg3"], m["sin_sg4"]
    ut = np.zeros_like(uc)
    vt = np.zeros_like(vc)
    reg = P.reg(-1, nx + 1, -NG, ny + NG - 1) & (J != -1) & (J != 0) & (J != N - 1) & (J != N)
    ut = np.where(reg, (uc - 0.25 * cosa_u * (sh(vc, -1, 0) + vc + sh(vc, -1, 1) + sh(vc, 0, 1))) * rsin_u, ut)
    reg = P.reg(-NG, nx + NG - 1, -1, ny + 1) & (J != 0) & (J != N)
    vt = np.where(reg, (vc - 0.25 * cosa_v * (sh(uc, 0, -1) + sh(uc, 1, -1) + uc + sh(uc, 1, 0))) * rsin_v, vt)
    # direct edge values
    colr = (P.lj >= -NG) & (P.lj <= ny + NG - 1)
    ut = np.where(colr & ((I == 0) | (I == N)), np.where(uc * dt > 0.0, uc / sh(s3, -1, 0), uc / s1), ut)
    rowr = (P.li >= -NG) & (P.li <= nx + NG - 1)
    vt = np.where(rowr & ((J == 0) | (J == N)), np.where(vc * dt > 0.0, vc / sh(s4, 0, -1), vc / s2), vt)
    ut1, vt1 = ut.copy(), vt.copy()
    # edge-adjacent cross terms
    rows = (J >= max(2, jo)) & (J <= min(N - 2, jo + ny))
    vt_edge = vc - 0.25 * cosa_v * (sh(ut1, 0, -1) + sh(ut1, 1, -1) + ut1 + sh(ut1, 1, 0))
    vt = np.where(rows & ((I == -1) | (I == 0) | (I == N - 1) | (I == N)), vt_edge, vt)
    cols = (I >= max(2, io)) & (I <= min(N - 2, io + nx))
    ut_edge = uc - 0.25 * cosa_u * (sh(vt1, -1, 0) + vt1 + sh(vt1, -1, 1) + sh(vt1, 0, 1))
    ut = np.where(cols & ((J == -1) | (J == 0) | (J == N - 1) | (J == N)), ut_edge, ut)
    # cube corners: 2x2 solves (reflections of the south-west formulas)
    for (cx, cy) in ((0, 0), (N, 0), (N, N), (0, N)):
        if not P.owns(cx, cy):
            continue
        fx = -1 if cx == N else 1
        fy = -1 if cy == N else 1

        def L(l, axis):  # edge-line index
            return l if (fx if axis == 0 else fy) == 1 else N - l

        def C(c, axis):  # cell index
            return c if (fx if axis == 0 else fy) == 1 else N - 1 - c

        def g(arr, i, j):
            jj, ii = P.slot(i, j)
            return arr[..., jj, ii]

        def UT(a, b):
            return g(ut1, L(a, 0), C(b, 1))

        def VT(a, b):
            return g(vt1, C(a, 0), L(b, 1))

        def UC(a, b):
            return g(uc, L(a, 0), C(b, 1))

        def VC(a, b):
            return g(vc, C(a, 0), L(b, 1))

        def CU(a, b):
            return g(cosa_u, L(a, 0), C(b, 1))

        def CV(a, b):
            return g(cosa_v, C(a, 0), L(b, 1))

        d1 = 1.0 / (1.0 - 0.0625 * CU(1, -1) * CV(0, -1))
        n_ut_a = (UC(1, -1) - 0.25 * CU(1, -1) * (VT(0, 0) + VT(1, 0) + VT(1, -1) + VC(0, -1)
                                                  - 0.25 * CV(0, -1) * (UT(0, -1) + UT(0, -2) + UT(1, -2)))) * d1
        d2 = 1.0 / (1.0 - 0.0625 * CU(-1, 0) * CV(-1, 1))
        n_vt_a = (VC(-1, 1) - 0.25 * CV(-1, 1) * (UT(0, 0) + UT(0, 1) + UT(-1, 1) + UC(-1, 0)
                                                  - 0.25 * CU(-1, 0) * (VT(-1, 0) + VT(-2, 0) + VT(-2, 1)))) * d2
        d3 = 1.0 / (1.0 - 0.0625 * CU(1, 0) * CV(0, 1))
        n_ut_b = (UC(1, 0) - 0.25 * CU(1, 0) * (VT(0, 0) + VT(1, 0) + VT(1, 1) + VC(0, 1)
                                                - 0.25 * CV(0, 1) * (UT(0, 0) + UT(0, 1) + UT(1, 1)))) * d3
        n_vt_b = (VC(0, 1) - 0.25 * CV(0, 1) * (UT(0, 0) + UT(0, 1) + UT(1, 1) + UC(1, 0)
                                                - 0.25 * CU(1, 0) * (VT(0, 0) + VT(1, 0) + VT(1, 1)))) * d3
        jj, ii = P.slot(L(1, 0), C(-1, 1)); ut[:, jj, ii] = n_ut_a
        jj, ii = P.slot(C(-1, 0), L(1, 1)); vt[:, jj, ii] = n_vt_a
        jj, ii = P.slot(L(1, 0), C(0, 1)); ut[:, jj, ii] = n_ut_b
        jj, ii = P.slot(C(0, 0), L(1, 1)); vt[:, jj, ii] = n_vt_b
    return ut, vt


def column_namelist(npz, nord=0, d2_bg=0.0, vtdm4=0.0, do_vort_damp=False, nord_v=None, d_con=0.0, n_sponge=-1,
                    d2_bg_k1=0.0, d2_bg_k2=0.0):
    """The per-level d_sw parameters of FV3 dyn_core's k loop (dyn_core.F90 before the d_sw
    call; the same rule as pyFV3 dyn_core get_column_namelist), one dict per level (0 = top):
    nord, d2_divg, nord_v, damp_vt, nord_w, damp_w, nord_t, damp_t, d_con.

    Every level: nord_v = min(2, nord) (nord_v given: the GTFV3_CONFIG extension),
    d2_divg = min(0.2, d2_bg), damp_vt = vtdm4 with do_vort_damp (else 0), w and pt take
    nord_v / damp_vt.  Sponge layers (npz > 1, n_sponge >= 0), no special damping of pt:
      level 0:  nord 0, d2_divg = max(0.01, d2_bg, d2_bg_k1), w del-2 with damp_w = d2_divg,
                with do_vort_damp vorticity / delp del-2 with damp_vt = d2_divg / 2, d_con 0;
      level max(1, n_sponge-2) (d2_bg_k2 > 0.01): the same with d2_divg = max(d2_bg, d2_bg_k2);
      level max(2, n_sponge-1) (d2_bg_k2 > 0.05): nord 0, d2_divg = max(d2_bg, 0.2 d2_bg_k2),
      w del-2, d_con 0 (levels 1 and 2 for n_sponge <= 3).
    npz = 1 or n_sponge < 0: d2_divg = d2_bg on every level."""
    nv = min(2, nord) if nord_v is None else int(nord_v)
    dvt = float(vtdm4) if do_vort_damp else 0.0
    base = dict(nord=int(nord), d2_divg=min(0.20, d2_bg), nord_v=nv, damp_vt=dvt, nord_w=nv, damp_w=dvt, nord_t=nv,
                damp_t=dvt, d_con=float(d_con))
    cols = [dict(base) for _ in range(npz)]
    if npz == 1 or n_sponge < 0:
        for c in cols:
            c["d2_divg"] = d2_bg
        return cols

    def sponge(c, d2, vort):
        c.update(nord=0, d2_divg=d2, nord_w=0, damp_w=d2, d_con=0.0)
        if vort and do_vort_damp:
            c.update(nord_v=0, damp_vt=0.5 * d2)
    # dyn_core's levels (1-based) k == 1, k == max(2, n_sponge - 1), k == max(3, n_sponge)
    k2, k3 = max(1, n_sponge - 2), max(2, n_sponge - 1)
    sponge(cols[0], max(0.01, d2_bg, d2_bg_k1), True)
    if npz > k2 and d2_bg_k2 > 0.01:
        sponge(cols[k2], max(d2_bg, d2_bg_k2), True)
    if npz > k3 and d2_bg_k2 > 0.05:
        sponge(cols[k3], max(d2_bg, 0.2 * d2_bg_k2), False)
    return cols


def heat_levels(npz, vtdm4=0.0, d2_bg_k1=0.0, d2_bg_k2=0.0, convert_ke=False):
    """FV3 dyn_core n_con: the levels (from the top) whose dissipated kinetic energy heats the
    air -- all with convert_ke or vtdm4 > 1e-4 (the namelist vtdm4, do_vort_damp or not), else
    the sponge levels d2_bg_k1 / d2_bg_k2 switch on (0, 1 or 2)"""
    if convert_ke or vtdm4 > 1e-4:
        return npz
    if d2_bg_k1 < 1e-3:
        return 0
    if d2_bg_k2 < 1e-3:
        return 1
    return 2


def d_sw(delp, pt, u, v, w, uc, vc, ua, va, sub, m, nx, ny, dt, ords, dddmp, d2_bg, da_min_c, nord=0,
         d4_bg=0.0, divg_d=None, vtdm4=0.0, nord_v=0, d_con=0.0, corner_w=None, damp_w=0.0, nord_w=0,
         damp_t=0.0, nord_t=0, ke_bg=0.0, da_min=None):
    """FV3 d_sw for the given levels at once (one parameter set: the caller splits the column by
    column_namelist).  ords = (hord_mt, hord_vt, hord_tm, hord_dp).
    Returns dict: delp, pt, w (updated), u, v (times dx / dy: finished by the pressure
    gradient), crx, cry, xfx, yfx (advective), fx, fy (mass fluxes, delp's diffusive fluxes
    included), and with d_con > 0 or damp_w > 0 the heat source and the dissipation-estimate
    increment of this call (heat, diss).
    Damping: nord = 0 del-2 divergence damping (dddmp, d2_bg = d2_divg); nord = 1..3 the
    del-(2 nord + 2) damping of the corner divergence divg_d (c_sw's, halo filled) with d4_bg
    plus the del-2 Smagorinsky-type term; vtdm4 (= damp_vt) > 1e-5 del-(2 nord_v + 2) vorticity
    damping fluxes added to u, v and, > 1e-4, del-(2 nord_v + 2) diffusive fluxes of delp added
    to the mass fluxes (coefficient from da_min); damp_t > 1e-4 the mass-weighted
    del-(2 nord_t + 2) fluxes of pt added to pt's fluxes; damp_w > 1e-5 w's del-(2 nord_w + 2)
    increment dw (w = w / delp + dw) and its heat ke_bg |dt| - dw (w + dw / 2); d_con > 0 the
    damped kinetic energy returned as heat."""
    hord_mt, hord_vt, hord_tm, hord_dp = ords
    P = Plane(sub, nx, ny, u.shape[-2], u.shape[-1])
    N, I, J, io, jo = P.N, P.I, P.J, P.io, P.jo
    if (vtdm4 > 1e-4 or damp_t > 1e-4) and da_min is None:
        raise ValueError("d_sw: the delp / pt del-n damping needs da_min")
    ut, vt = d_sw_ut_vt(uc, vc, P, m, dt)
    s1, s2, s3, s4 = m["sin_sg1"], m["sin_sg2"], m["sin_sg3"], m["sin_sg4"]
    dx, dy, rdxa, rdya, area, rarea = m["dx"], m["dy"], m["rdxa"], m["rdya"], m["area"], m["rarea"]
    z = np.zeros_like(u)
    # advective Courant numbers / area fluxes
    reg = P.reg(0, nx, -NG, ny + NG - 1)
    xf = dt * ut
    crx = np.where(reg, np.where(xf > 0.0, xf * sh(rdxa, -1, 0), xf * rdxa), z)
    xfx = np.where(reg, np.where(xf > 0.0, dy * xf * sh(s3, -1, 0), dy * xf * s1), z)
    reg = P.reg(-NG, nx + NG - 1, 0, ny)
    yf = dt * vt
    cry = np.where(reg, np.where(yf > 0.0, yf * sh(rdya, 0, -1), yf * rdya), z)
    yfx = np.where(reg, np.where(yf > 0.0, dx * yf * sh(s4, 0, -1), dx * yf * s2), z)
    ra_y = np.where(P.reg(-NG, nx + NG - 1, 0, ny - 1), area + yfx - sh(yfx, 0, 1), z)
    ra_x = np.where(P.reg(0, nx - 1, -NG, ny + NG - 1), area + xfx - sh(xfx, 1, 0), z)
    # mass fluxes (fv_tp_2d(delp, ..., nord = nord_v, damp_c = damp_vt): the diffusive fluxes
    # of delp added inside fv_tp_2d, so the flux capacitor and w / pt see them)
    fx, fy = fv_tp_2d(delp, crx, cry, xfx, yfx, ra_x, ra_y, sub, m, nx, ny, hord_dp)
    xreg, yreg = P.reg(0, nx, 0, ny - 1), P.reg(0, nx - 1, 0, ny)
    if vtdm4 > 1e-4:
        fx2, fy2 = deln_flux(nord_v, (vtdm4 * da_min) ** (nord_v + 1), delp, sub, m, nx, ny)
        fx = np.where(xreg, fx + fx2, fx)
        fy = np.where(yreg, fy + fy2, fy)
    comp = P.reg(0, nx - 1, 0, ny - 1)
    # w damping (non-hydrostatic d_sw, before w's transport): dw and its heat
    heat_w = dw = None
    if damp_w > 1e-5:
        dd8 = ke_bg * abs(dt)
        fx2, fy2 = deln_flux(nord_w, (damp_w * da_min_c) ** (nord_w + 1), w, sub, m, nx, ny)
        dw = np.where(comp, (fx2 - sh(fx2, 1, 0) + fy2 - sh(fy2, 0, 1)) * rarea, 0.0)
        heat_w = np.where(comp, dd8 - dw * (w + 0.5 * dw), 0.0)
    # w
    gx, gy = fv_tp_2d(w, crx, cry, xfx, yfx, ra_x, ra_y, sub, m, nx, ny, hord_vt, fx, fy)
    w_new = np.where(comp, delp * w + (gx - sh(gx, 1, 0) + gy - sh(gy, 0, 1)) * rarea, w)
    # pt (fv_tp_2d(pt, ..., mass = delp, nord = nord_t, damp_c = damp_t)), delp
    gx, gy = fv_tp_2d(pt, crx, cry, xfx, yfx, ra_x, ra_y, sub, m, nx, ny, hord_tm, fx, fy)
    if damp_t > 1e-4:
        damp2 = 0.5 * (damp_t * da_min) ** (nord_t + 1)
        fx2, fy2 = deln_flux(nord_t, None, pt, sub, m, nx, ny)
        gx = np.where(xreg, gx + damp2 * (sh(delp, -1, 0) + delp) * fx2, gx)
        gy = np.where(yreg, gy + damp2 * (sh(delp, 0, -1) + delp) * fy2, gy)
    pt_new = pt * delp + (gx - sh(gx, 1, 0) + gy - sh(gy, 0, 1)) * rarea
    dp_new = delp + (fx - sh(fx, 1, 0) + fy - sh(fy, 0, 1)) * rarea
    pt_new = np.where(comp, pt_new / dp_new, pt)
    dp_new = np.where(comp, dp_new, delp)
    w_new = np.where(comp, w_new / dp_new, w_new)
    if dw is not None:
        w_new = np.where(comp, w_new + dw, w_new)

    # kinetic energy at corners (B-grid contravariant winds, upwind PPM of u and v)
    dt5, dt4 = 0.5 * dt, 0.25 * dt
    cosa, rsina = m["cosa"], m["rsina"]
    Ilo, Ihi = max(1, io), min(N - 1, io + nx)
    Jlo, Jhi = max(1, jo), min(N - 1, jo + ny)
    inner = (I >= Ilo) & (I <= Ihi) & (J >= Jlo) & (J <= Jhi)
    allx = P.reg(0, nx, 0, ny)
    vb = np.where(inner, dt5 * (sh(vc, -1, 0) + vc - (sh(uc, 0, -1) + uc) * cosa) * rsina, z)
    vb_we = dt4 * (-sh(vt, -2, 0) + 3.0 * (sh(vt, -1, 0) + vt) - sh(vt, 1, 0))
    vb = np.where(allx & ((I == 0) | (I == N)), vb_we, vb)
    vb_sn = dt5 * (sh(vt, -1, 0) + vt)
    vb = np.where((I >= Ilo) & (I <= Ihi) & allx & ((J == 0) | (J == N)), vb_sn, vb)
    # ytp_v: PPM of v along j with Courant vb*rdy(upwind)
    rdy = m["rdy"]
    cfl = np.where(vb > 0.0, vb * sh(rdy, 0, -1), vb * rdy)
    from .tp_core import yppm
    ub_flux = z.copy()
    ub_flux[:, NG:NG + ny + 1, NG:NG + nx + 1] = yppm(v, cfl, dy, jo, N, hord_mt, 0, nx, 0, ny)
    ke = np.where(allx, vb * ub_flux, z)
    ub = np.where(inner, dt5 * (sh(uc, 0, -1) + uc - (sh(vc, -1, 0) + vc) * cosa) * rsina, z)
    ub_we = dt5 * (sh(ut, 0, -1) + ut)
    ub = np.where((J >= Jlo) & (J <= Jhi) & allx & ((I == 0) | (I == N)), ub_we, ub)
    ub_sn = dt4 * (-sh(ut, 0, -2) + 3.0 * (sh(ut, 0, -1) + ut) - sh(ut, 0, 1))
    ub = np.where(allx & ((J == 0) | (J == N)), ub_sn, ub)
    rdx = m["rdx"]
    cfl = np.where(ub > 0.0, ub * sh(rdx, -1, 0), ub * rdx)
    from .tp_core import xppm
    vb_flux = z.copy()
    vb_flux[:, NG:NG + ny + 1, NG:NG + nx + 1] = xppm(u, cfl, dx, io, N, hord_mt, 0, nx, 0, ny)
    ke = np.where(allx, 0.5 * (ke + ub * vb_flux), z)
    dt6 = dt / 6.0

    def g(arr, i, j):
        jj, ii = P.slot(i, j)
        return arr[:, jj, ii]

    def put(arr, i, j, val):
        jj, ii = P.slot(i, j)
        arr[:, jj, ii] = val
    if P.owns(0, 0):
        put(ke, 0, 0, dt6 * ((g(ut, 0, 0) + g(ut, 0, -1)) * g(u, 0, 0) + (g(vt, 0, 0) + g(vt, -1, 0)) * g(v, 0, 0)
                             + (g(ut, 0, 0) + g(vt, 0, 0)) * g(u, -1, 0)))
    if P.owns(N, 0):
        put(ke, N, 0, dt6 * ((g(ut, N, 0) + g(ut, N, -1)) * g(u, N - 1, 0) + (g(vt, N, 0) + g(vt, N - 1, 0)) * g(v, N, 0)
                             + (g(ut, N, 0) - g(vt, N - 1, 0)) * g(u, N, 0)))
    if P.owns(N, N):
        put(ke, N, N, dt6 * ((g(ut, N, N) + g(ut, N, N - 1)) * g(u, N - 1, N)
                             + (g(vt, N, N) + g(vt, N - 1, N)) * g(v, N, N - 1)
                             + (g(ut, N, N - 1) + g(vt, N - 1, N)) * g(u, N, N)))
    if P.owns(0, N):
        put(ke, 0, N, dt6 * ((g(ut, 0, N) + g(ut, 0, N - 1)) * g(u, 0, N) + (g(vt, 0, N) + g(vt, -1, N)) * g(v, 0, N - 1)
                             + (g(ut, 0, N - 1) - g(vt, 0, N)) * g(u, -1, N)))

    # relative vorticity (cell mean): the Smagorinsky coefficient and the vorticity damping
    # use it before the transport
    udx = u * dx
    vdy = v * dy
    wk = np.where(P.reg(-NG, nx + NG - 1, -NG, ny + NG - 1), rarea * (udx - sh(udx, 0, 1) + sh(vdy, 1, 0) - vdy), z)
    if nord > 0:
        vd = divergence_damping_nord(divg_d, wk, sub, m, nx, ny, dt, nord, dddmp, d2_bg, d4_bg, da_min_c, corner_w)
        ke = np.where(allx, ke + vd, ke)
        return _d_sw_finish(dict(delp=dp_new, pt=pt_new, w=w_new, crx=crx, cry=cry, xfx=xfx, yfx=yfx, fx=fx, fy=fy,
                                 ut=ut, vt=vt), ke, vd, wk, u, v, udx, vdy, dp_new, sub, m, nx, ny, crx, cry, xfx, yfx,
                            ra_x, ra_y, hord_vt, da_min_c, vtdm4, nord_v, d_con, P, heat_w)
    # divergence damping (nord = 0)
    ptc = z.copy()
    regp = P.reg(-1, nx, 0, ny)
    ptc_edge = np.where(vc > 0.0, u * m["dyc"] * sh(s4, 0, -1), u * m["dyc"] * s2)
    ptc_gen = (u - 0.5 * (sh(va, 0, -1) + va) * m["cosa_v"]) * m["dyc"] * m["sina_v"]
    ptc = np.where(regp, np.where((J == 0) | (J == N), ptc_edge, ptc_gen), ptc)
    vrt = z.copy()
    regv = (I >= Ilo) & (I <= Ihi) & P.reg(-1, nx, -1, ny)
    vrt = np.where(regv, (v - 0.5 * (sh(ua, -1, 0) + ua) * m["cosa_u"]) * m["dxc"] * m["sina_u"], vrt)
    vrt_edge = np.where(uc > 0.0, v * m["dxc"] * sh(s3, -1, 0), v * m["dxc"] * s1)
    vrt = np.where(P.reg(-1, nx, -1, ny) & ((I == 0) | (I == N)), vrt_edge, vrt)
    delpc = np.where(allx, sh(vrt, 0, -1) - vrt + sh(ptc, -1, 0) - ptc, z)
    vS = sh(vrt, 0, -1)
    delpc = np.where(P.at(0, 0), delpc - vS, delpc)
    delpc = np.where(P.at(N, 0), delpc - vS, delpc)
    delpc = np.where(P.at(N, N), delpc + vrt, delpc)
    delpc = np.where(P.at(0, N), delpc + vrt, delpc)
    delpc = m["rarea_c"] * delpc
    damp = da_min_c * np.maximum(d2_bg, np.minimum(0.20, dddmp * np.abs(delpc * dt)))
    vd = np.where(allx, damp * delpc, z)
    ke = np.where(allx, ke + damp * delpc, ke)
    return _d_sw_finish(dict(delp=dp_new, pt=pt_new, w=w_new, crx=crx, cry=cry, xfx=xfx, yfx=yfx, fx=fx, fy=fy,
                             ut=ut, vt=vt), ke, vd, wk, u, v, udx, vdy, dp_new, sub, m, nx, ny, crx, cry, xfx, yfx,
                        ra_x, ra_y, hord_vt, da_min_c, vtdm4, nord_v, d_con, P, heat_w)


def _d_sw_finish(out, ke, vd, wk, u, v, udx, vdy, dp_new, sub, m, nx, ny, crx, cry, xfx, yfx, ra_x, ra_y, hord_vt,
                 da_min_c, vtdm4, nord_v, d_con, P, heat_w=None):
    """vorticity transport and the momentum update, then the vorticity damping fluxes and the
    d_con heat (FV3 d_sw's last part); heat_w: the w damping's heat (None: no w damping)"""
    z = np.zeros_like(u)
    vort = np.where(P.reg(-NG, nx + NG - 1, -NG, ny + NG - 1), wk + m["f0"], z)
    fxv, fyv = fv_tp_2d(vort, crx, cry, xfx, yfx, ra_x, ra_y, sub, m, nx, ny, hord_vt)
    u_new = np.where(P.reg(0, nx - 1, 0, ny), udx + ke - sh(ke, 1, 0) + fyv, u)
    v_new = np.where(P.reg(0, nx, 0, ny - 1), vdy + ke - sh(ke, 0, 1) - fxv, v)
    fx2 = fy2 = z
    if vtdm4 > 1e-5:
        damp4 = (vtdm4 * da_min_c) ** (nord_v + 1)
        fx2, fy2 = del6_vt_flux(nord_v, damp4, wk, sub, m, nx, ny)
    if d_con > 1e-5:
        out["heat"], out["diss"] = damping_heat(u_new, v_new, vd, fx2, fy2, dp_new, m, P, d_con, heat_w)
    elif heat_w is not None:  # the sponge levels (d_con_k = 0): the w damping's heat alone
        out["heat"], out["diss"] = heat_w, heat_w.copy()
    if vtdm4 > 1e-5:
        u_new = np.where(P.reg(0, nx - 1, 0, ny), u_new + fy2, u_new)
        v_new = np.where(P.reg(0, nx, 0, ny - 1), v_new - fx2, v_new)
    out.update(u=u_new, v=v_new, ke=ke, vd=vd, wk=wk)
    return out


# ----------------------------------------------------------------------------------
# higher-order divergence damping, vorticity damping, d_con heating (FV3 sw_core.F90
# d_sw / divergence_corner / del6_vt_flux and fv_grid_utils fill_corners, as described in
# Harris et al. 2021 "A scientific description of the GFDL FV3 dynamical core" section 6
# (damping) and restated from the FV3 module structure: literal index formulas, 0-based
# tile-global indices g = f - 1)

def divergence_corner(u, v, ua, va, sub, m, nx, ny):
    """FV3 divergence_corner (c_sw, nord > 0): the divergence of the D-grid winds on the dual
    cell around each compute corner (i, j in [0, n]), times rarea_c; zero elsewhere."""
    P = Plane(sub, nx, ny, u.shape[-2], u.shape[-1])
    N, I, J = P.N, P.I, P.J
    s1, s2, s3, s4 = m["sin_sg1"], m["sin_sg2"], m["sin_sg3"], m["sin_sg4"]
    c1, c2, c3, c4 = m["cos_sg1"], m["cos_sg2"], m["cos_sg3"], m["cos_sg4"]
    # uf on x-edges (u positions), vf on y-edges (v positions)
    sx = m["dyc"] * 0.5 * (sh(s4, 0, -1) + s2)
    uf_gen = (u - 0.25 * (sh(va, 0, -1) + va) * (sh(c4, 0, -1) + c2)) * sx
    uf = np.where((J == 0) | (J == N), u * sx, uf_gen)
    sy = m["dxc"] * 0.5 * (sh(s3, -1, 0) + s1)
    vf_gen = (v - 0.25 * (sh(ua, -1, 0) + ua) * (sh(c3, -1, 0) + c1)) * sy
    vf = np.where((I == 0) | (I == N), v * sy, vf_gen)
    dd = sh(vf, 0, -1) - vf + sh(uf, -1, 0) - uf
    vS = sh(vf, 0, -1)
    dd = np.where(P.at(0, 0) | P.at(N, 0), dd - vS, dd)
    dd = np.where(P.at(N, N) | P.at(0, N), dd + vf, dd)
    return np.where(P.reg(0, nx, 0, ny), m["rarea_c"] * dd, 0.0)


def fill_corners_bgrid(q, sub, direction, nx, ny):
    """FV3 fill_corners(q, FILL=XDir|YDir, BGRID=.true.) on a copy of a corner-point field:
    the cube-corner halo points from the rotated ones (only corners this sub-domain holds)"""
    out = q.copy()
    N, io, jo = sub["N"], sub["ioff"], sub["joff"]

    def slot(I, J):
        return J - jo + NG, I - io + NG

    def ok(I, J):
        jj, ii = slot(I, J)
        return 0 <= jj < q.shape[-2] and 0 <= ii < q.shape[-1]

    def setp(I, J, Is, Js):
        if ok(I, J) and ok(Is, Js):
            a, b = slot(I, J)
            c, d = slot(Is, Js)
            out[..., a, b] = q[..., c, d]
    own = lambda I, J: io <= I <= io + nx and jo <= J <= jo + ny
    sw, se, ne, nw = [own(I, J) for (I, J) in ((0, 0), (N, 0), (N, N), (0, N))]
    for j in range(1, NG + 1):
        for i in range(1, NG + 1):
            if direction == 1:
                if sw: setp(-i, -j, -j, i)
                if se: setp(N + i, -j, N + j, i)
                if ne: setp(N + i, N + j, N + j, N - i)
                if nw: setp(-i, N + j, -j, N - i)
            else:
                if sw: setp(-j, -i, i, -j)
                if se: setp(N + j, -i, N - i, -j)
                if ne: setp(N + j, N + i, N - i, N + j)
                if nw: setp(-j, N + i, i, N + j)
    return out


def fill_corners_dgrid(x, y, sub, nx, ny, sign=-1.0):
    """FV3 fill_corners(x, y, DGRID=.true., VECTOR=.true.) on copies: the D-grid pair's
    cube-corner halo values (x on x-edges, y on y-edges) from the other component, the
    south-west and north-east corners with the vector sign"""
    xo, yo = x.copy(), y.copy()
    N, io, jo = sub["N"], sub["ioff"], sub["joff"]
    nj, ni = x.shape[-2:]

    def slot(I, J):
        return J - jo + NG, I - io + NG

    def ok(I, J):
        jj, ii = slot(I, J)
        return 0 <= jj < nj and 0 <= ii < ni
    own = lambda I, J: io <= I <= io + nx and jo <= J <= jo + ny
    sw, se, ne, nw = [own(I, J) for (I, J) in ((0, 0), (N, 0), (N, N), (0, N))]

    def cp(dst, src, I, J, Is, Js, f):
        if ok(I, J) and ok(Is, Js):
            a, b = slot(I, J)
            c, d = slot(Is, Js)
            dst[..., a, b] = f * src[..., c, d]
    for j in range(1, NG + 1):
        for i in range(1, NG + 1):
            if sw: cp(xo, y, -i, -j, -j, i - 1, sign)
            if se: cp(xo, y, N - 1 + i, -j, N + j, i - 1, 1.0)
            if ne: cp(xo, y, N - 1 + i, N + j, N + j, N - i, sign)
            if nw: cp(xo, y, -i, N + j, -j, N - i, 1.0)
    for j in range(1, NG + 1):
        for i in range(1, NG + 1):
            if sw: cp(yo, x, -i, -j, j - 1, -i, sign)
            if se: cp(yo, x, N + i, -j, N - j, -i, 1.0)
            if ne: cp(yo, x, N + i, N - 1 + j, N - j, N + i, sign)
            if nw: cp(yo, x, -i, N - 1 + j, j - 1, N + i, 1.0)
    return xo, yo


def _divg_u(m):
    return m["sina_v"] * m["dyc"] / m["dx"]


def _divg_v(m):
    return m["sina_u"] * m["dxc"] / m["dy"]


def _del6_u(m):
    return m["sina_v"] * m["dx"] / m["dyc"]


def _del6_v(m):
    return m["sina_u"] * m["dy"] / m["dxc"]


def divergence_damping_nord(divg_d, wk, sub, m, nx, ny, dt, nord, dddmp, d2_bg, d4_bg, da_min_c, corner_w):
    """d_sw's nord > 0 branch: the corner damping term damp2 * delpc + dd8 * del^(2 nord) divg_d
    (added to ke by the caller).  divg_d: the corner divergence of c_sw with its halo filled;
    wk: the relative vorticity at cell centres (halo included) for the Smagorinsky-type del-2
    coefficient (a2b_ord4 to the corners) when dddmp > 0."""
    from .nh_core import a2b_ord4
    P = Plane(sub, nx, ny, divg_d.shape[-2], divg_d.shape[-1])
    N = P.N
    delpc = np.where(P.reg(0, nx, 0, ny), divg_d, 0.0)
    dgu, dgv = _divg_u(m), _divg_v(m)
    dd = divg_d.copy()
    corner_sub = any(P.owns(I, J) for (I, J) in ((0, 0), (N, 0), (N, N), (0, N)))
    for n in range(1, nord + 1):
        nt = nord - n
        fill_c = nt != 0 and corner_sub
        d_x = fill_corners_bgrid(dd, sub, 1, nx, ny) if fill_c else dd
        vc = np.where(P.reg(-1 - nt, nx + nt, -nt, ny + nt), (sh(d_x, 1, 0) - d_x) * dgu, 0.0)
        d_y = fill_corners_bgrid(dd, sub, 2, nx, ny) if fill_c else dd
        uc = np.where(P.reg(-nt, nx + nt, -1 - nt, ny + nt), (sh(d_y, 0, 1) - d_y) * dgv, 0.0)
        if fill_c:
            vc, uc = fill_corners_dgrid(vc, uc, sub, nx, ny)
        new = sh(uc, 0, -1) - uc + sh(vc, -1, 0) - vc
        uS = sh(uc, 0, -1)
        new = np.where(P.at(0, 0) | P.at(N, 0), new - uS, new)
        new = np.where(P.at(N, N) | P.at(0, N), new + uc, new)
        reg = P.reg(-nt, nx + nt, -nt, ny + nt)
        dd = np.where(reg, new * m["rarea_c"], 0.0)
    if dddmp < 1e-5:
        vort = np.zeros_like(dd)
    else:
        vc_ = a2b_ord4(wk, P, m, corner_w)
        vort = abs(dt) * np.sqrt(delpc ** 2 + vc_ ** 2)
    dd8 = (da_min_c * d4_bg) ** (nord + 1)
    damp2 = da_min_c * np.maximum(d2_bg, np.minimum(0.20, dddmp * vort))
    return np.where(P.reg(0, nx, 0, ny), damp2 * delpc + dd8 * dd, 0.0)


def del6_vt_flux(nord, damp, q, sub, m, nx, ny):
    """FV3 del6_vt_flux: del-(2 nord + 2) diffusive fluxes (fx2 on y-edges, fy2 on x-edges) of
    the cell field q (the relative vorticity) with coefficient damp (the loops of deln_flux)"""
    return deln_flux(nord, damp, q, sub, m, nx, ny)


def deln_flux(nord, damp, q, sub, m, nx, ny):
    """FV3 tp_core deln_flux's diffusive fluxes: fx2 on y-edges over [-nord, nx+nord] x
    [-nord, ny-1+nord], fy2 on x-edges (zero elsewhere), from d2 = damp q on
    [-1-nord, n+nord] (damp None: d2 = q, the mass-weighted form whose caller adds
    0.5 damp (mass(i-1) + mass(i)) fx2), the cube-corner halo of d2 read through copy_corners
    for nord > 0, then nord passes d2 = div(fluxes) rarea / fluxes of d2 with the opposite
    sign, each one ring narrower"""
    P = Plane(sub, nx, ny, q.shape[-2], q.shape[-1])
    d6u, d6v, rarea = _del6_u(m), _del6_v(m), m["rarea"]
    d2 = np.where(P.reg(-1 - nord, nx + nord, -1 - nord, ny + nord), q if damp is None else damp * q, 0.0)
    dx_ = copy_corners(d2, sub, 1) if nord > 0 else d2
    fx2 = np.where(P.reg(-nord, nx + nord, -nord, ny - 1 + nord), d6v * (sh(dx_, -1, 0) - dx_), 0.0)
    dy_ = copy_corners(d2, sub, 2) if nord > 0 else d2
    fy2 = np.where(P.reg(-nord, nx - 1 + nord, -nord, ny + nord), d6u * (sh(dy_, 0, -1) - dy_), 0.0)
    for n in range(1, nord + 1):
        nt = nord - n
        d2 = np.where(P.reg(-nt - 1, nx + nt, -nt - 1, ny + nt),
                      (fx2 - sh(fx2, 1, 0) + fy2 - sh(fy2, 0, 1)) * rarea, 0.0)
        dx_ = copy_corners(d2, sub, 1)
        fx2 = np.where(P.reg(-nt, nx + nt, -nt, ny - 1 + nt), d6v * (dx_ - sh(dx_, -1, 0)), 0.0)
        dy_ = copy_corners(d2, sub, 2)
        fy2 = np.where(P.reg(-nt, nx - 1 + nt, -nt, ny + nt), d6u * (dy_ - sh(dy_, 0, -1)), 0.0)
    return fx2, fy2


def damping_heat(u, v, vd, fx2, fy2, delp, m, P, d_con, heat_w=None):
    """d_sw's d_con branch: the kinetic energy the divergence damping (corner term vd) and the
    vorticity damping (fluxes fx2, fy2) remove, as a heat source delp * (heat_w - 0.25 d_con ...)
    and the dissipation estimate increment (heat_w - rsin2 ...), on compute cells; heat_w: the w
    damping's heat (None: 0).  u, v: the updated D-grid winds times dx, dy before the
    vorticity-damping fluxes are added."""
    hw = 0.0 if heat_w is None else heat_w
    nx, ny = P.nx, P.ny
    ub = (vd - sh(vd, 1, 0) + fy2) * m["rdx"]
    fy = u * m["rdx"]
    gy = fy * ub
    vb = (vd - sh(vd, 0, 1) - fx2) * m["rdy"]
    fx = v * m["rdy"]
    gx = fx * vb
    u2 = fy + sh(fy, 0, 1)
    du2 = ub + sh(ub, 0, 1)
    v2 = fx + sh(fx, 1, 0)
    dv2 = vb + sh(vb, 1, 0)
    t = (ub ** 2 + sh(ub, 0, 1) ** 2 + vb ** 2 + sh(vb, 1, 0) ** 2) + 2.0 * (gy + sh(gy, 0, 1) + gx + sh(gx, 1, 0)) \
        - m["cosa_s"] * (u2 * dv2 + v2 * du2 + du2 * dv2)
    comp = P.reg(0, nx - 1, 0, ny - 1)
    heat = np.where(comp, delp * (hw - 0.25 * d_con * m["rsin2"] * t), 0.0)
    diss = np.where(comp, hw - m["rsin2"] * t, 0.0)
    return heat, diss


def del2_cubed(q, cd, sub, m, nx, ny, nmax):
    """FV3 del2_cubed (dyn_core's smoothing of the heat source; pyFV3 HyperdiffusionDamping):
    min(3, nmax) del-2 passes on a cell field whose halo was filled once, pass n over the
    region [-nt, n-1+nt] (nt = ntimes - n): at the cube corners this sub-domain owns the corner
    cell and its two halo neighbours are first set to their mean; fx on y-edges
    del6_v (q(i-1) - q(i)) and fy on x-edges del6_u (q(j-1) - q(j)) (copy_corners for nt > 0);
    q += cd rarea (fx - fx(i+1) + fy - fy(j+1)).  Returns the smoothed copy."""
    P = Plane(sub, nx, ny, q.shape[-2], q.shape[-1])
    N = P.N
    q = q.copy()
    d6u, d6v, rarea = _del6_u(m), _del6_v(m), m["rarea"]
    r3 = 1.0 / 3.0
    # (corner cell, its west / east halo neighbour, its south / north halo neighbour)
    corners = []
    if P.owns(0, 0):
        corners.append(((0, 0), (-1, 0), (0, -1)))
    if P.owns(N, 0):
        corners.append(((N - 1, 0), (N, 0), (N - 1, -1)))
    if P.owns(N, N):
        corners.append(((N - 1, N - 1), (N, N - 1), (N - 1, N)))
    if P.owns(0, N):
        corners.append(((0, N - 1), (-1, N - 1), (0, N)))
    ntimes = min(3, nmax)
    for n in range(1, ntimes + 1):
        nt = ntimes - n
        for c0, c1, c2 in corners:
            a, b, c = P.slot(*c0), P.slot(*c1), P.slot(*c2)
            avg = (q[:, a[0], a[1]] + q[:, b[0], b[1]] + q[:, c[0], c[1]]) * r3
            q[:, a[0], a[1]] = avg
            q[:, b[0], b[1]] = avg
            q[:, c[0], c[1]] = avg
        qx = copy_corners(q, sub, 1) if nt > 0 else q
        fx = np.where(P.reg(-nt, nx + nt, -nt, ny - 1 + nt), d6v * (sh(qx, -1, 0) - qx), 0.0)
        qy = copy_corners(q, sub, 2) if nt > 0 else q
        fy = np.where(P.reg(-nt, nx - 1 + nt, -nt, ny + nt), d6u * (sh(qy, 0, -1) - qy), 0.0)
        q = np.where(P.reg(-nt, nx - 1 + nt, -nt, ny - 1 + nt),
                     q + cd * rarea * (fx - sh(fx, 1, 0) + fy - sh(fy, 0, 1)), q)
    return q
