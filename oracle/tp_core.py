"""Oracle: FV3 tp_core (fv_tp_2d, xppm/yppm, copy_corners) and fv_tracer2d
(tracer_2d_1l) in vectorised fp64 numpy — TEST INFRASTRUCTURE ONLY.

Restated from Lin & Rood (1996) and the FV3 tp_core / fv_tracer2d structure
(see oracle/__init__.py for the parity status).  Arrays: a[k, j+NG, i+NG] for one
sub-domain; `sub` = dict(ioff, joff, N); `m` = dict of metric planes (nj, pitch).
Operation order follows the Fortran expressions.
"""
import numpy as np

from . import NG

P1, P2 = 7.0 / 12.0, -1.0 / 12.0
C1, C2, C3 = -2.0 / 14.0, 11.0 / 14.0, 5.0 / 14.0


def copy_corners(q, sub, direction):
    """FV3 fv_grid_utils copy_corners, literal Fortran index formulas (1-based,
    npx = N+1), applied to a copy of q.  Only the cube corners this sub owns."""
    out = q.copy()
    N, io, jo = sub["N"], sub["ioff"], sub["joff"]
    npx = npy = N + 1
    ng = NG

    def L(fi, fj):  # Fortran (i,j) -> array slot
        return fj - 1 - jo + NG, fi - 1 - io + NG

    def inside(fi, fj):
        jj, ii = L(fi, fj)
        return 0 <= jj < q.shape[-2] and 0 <= ii < q.shape[-1]

    def setc(fi, fj, si, sj):
        if inside(fi, fj) and inside(si, sj):
            a, b = L(fi, fj)
            c, d = L(si, sj)
            out[..., a, b] = q[..., c, d]

    # a sub-domain owns a cube corner iff the corner's halo cells fall inside its plane
    for j in range(1 - ng, 1):
        for i in range(1 - ng, 1):
            if direction == 1:
                setc(i, j, j, 1 - i)
            else:
                setc(i, j, 1 - j, i)
    for j in range(1 - ng, 1):
        for i in range(npx, npx + ng):
            if direction == 1:
                setc(i, j, npy - j, i - npx + 1)
            else:
                setc(i, j, npy + j - 1, npx - i)
    for j in range(npy, npy + ng):
        for i in range(npx, npx + ng):
            if direction == 1:
                setc(i, j, j, 2 * npx - 1 - i)
            else:
                setc(i, j, 2 * npy - 1 - j, i)
    for j in range(npy, npy + ng):
        for i in range(1 - ng, 1):
            if direction == 1:
                setc(i, j, npy - j, i - 1 + npx)
            else:
                setc(i, j, j + 1 - npx, npy - i)
    return out


def _al(Q, DX, g, dg, N):
    qm2, qm1, q0, qp1 = Q(dg - 2), Q(dg - 1), Q(dg), Q(dg + 1)
    gg = g + dg
    base = P1 * (qm1 + q0) + P2 * (qm2 + qp1)
    e1 = C1 * qm2 + C2 * qm1 + C3 * q0
    e2 = C3 * qm1 + C2 * q0 + C1 * qp1
    dm2, dm1, d0, dp1 = DX(dg - 2), DX(dg - 1), DX(dg), DX(dg + 1)
    with np.errstate(all="ignore"):
        e0 = 0.5 * (((2.0 * dm1 + dm2) * qm1 - dm1 * qm2) / (dm2 + dm1) + ((2.0 * d0 + dp1) * q0 - d0 * qp1) / (d0 + dp1))
    out = np.where((gg == -1) | (gg == N - 1), e1, base)
    out = np.where((gg == 1) | (gg == N + 1), e2, out)
    out = np.where((gg == 0) | (gg == N), e0, out)
    return out


def xppm(q, c, dxa, off, N, ord_, i0, i1, j0, j1):
    """PPM flux (hord 5/6) at interfaces i in [i0,i1] along the last axis, rows j in [j0,j1].
    Returns array (nk, j1-j0+1, i1-i0+1)."""
    R = slice(j0 + NG, j1 + NG + 1)

    def Q(di):
        return q[:, R, i0 + NG + di: i1 + NG + 1 + di]

    def DX(di):
        return dxa[R, i0 + NG + di: i1 + NG + 1 + di]

    g = np.arange(i0, i1 + 1) + off
    alm, al0, alp = _al(Q, DX, g, -1, N), _al(Q, DX, g, 0, N), _al(Q, DX, g, 1, N)
    qm, q0 = Q(-1), Q(0)
    blm = alm - qm
    brm = al0 - qm
    b0m = blm + brm
    bl0 = al0 - q0
    br0 = alp - q0
    b00 = bl0 + br0
    if ord_ == 5:
        sm = blm * brm < 0.0
        s0 = bl0 * br0 < 0.0
    else:
        sm = 3.0 * np.abs(b0m) < np.abs(blm - brm)
        s0 = 3.0 * np.abs(b00) < np.abs(bl0 - br0)
    smooth = sm | s0
    cc = c[:, R, i0 + NG: i1 + NG + 1]
    fpos = (1.0 - cc) * (brm - cc * b0m)
    fneg = (1.0 + cc) * (bl0 + cc * b00)
    return np.where(cc > 0.0, qm + np.where(smooth, fpos, 0.0), q0 + np.where(smooth, fneg, 0.0))


def yppm(q, c, dya, off, N, ord_, i0, i1, j0, j1):
    """PPM flux at interfaces j in [j0,j1] (x-edges), columns i in [i0,i1]; returns (nk, nj, ni)."""
    qt = np.swapaxes(q, -1, -2)
    ct = np.swapaxes(c, -1, -2)
    dt = np.swapaxes(dya, -1, -2)
    f = xppm(qt, ct, dt, off, N, ord_, j0, j1, i0, i1)
    return np.swapaxes(f, -1, -2)


def _put(dst, val, i0, i1, j0, j1):
    dst[:, j0 + NG: j1 + NG + 1, i0 + NG: i1 + NG + 1] = val


def _get(a, i0, i1, j0, j1):
    if a.ndim == 2:
        return a[j0 + NG: j1 + NG + 1, i0 + NG: i1 + NG + 1]
    return a[:, j0 + NG: j1 + NG + 1, i0 + NG: i1 + NG + 1]


def fv_tp_2d(q, crx, cry, xfx, yfx, ra_x, ra_y, sub, m, nx, ny, ord_=6, mfx=None, mfy=None):
    """FV3 fv_tp_2d: returns (fx, fy) full planes (y-edge / x-edge fluxes)."""
    N = sub["N"]
    io, jo = sub["ioff"], sub["joff"]
    area, dxa, dya = m["area"], m["dxa"], m["dya"]
    z = np.zeros_like(q)
    # y sweep first on the y-corner-filled field
    qy = copy_corners(q, sub, 2)
    fy2 = z.copy()
    _put(fy2, yppm(qy, cry, dya, jo, N, ord_, -NG, nx + NG - 1, 0, ny), -NG, nx + NG - 1, 0, ny)
    fyy = yfx * fy2
    qi = z.copy()
    _put(qi, (_get(qy, -NG, nx + NG - 1, 0, ny - 1) * _get(area, -NG, nx + NG - 1, 0, ny - 1)
              + _get(fyy, -NG, nx + NG - 1, 0, ny - 1) - _get(fyy, -NG, nx + NG - 1, 1, ny))
         / _get(ra_y, -NG, nx + NG - 1, 0, ny - 1), -NG, nx + NG - 1, 0, ny - 1)
    fx = z.copy()
    _put(fx, xppm(qi, crx, dxa, io, N, ord_, 0, nx, 0, ny - 1), 0, nx, 0, ny - 1)
    # x sweep on the x-corner-filled field
    qx = copy_corners(q, sub, 1)
    fx2 = z.copy()
    _put(fx2, xppm(qx, crx, dxa, io, N, ord_, 0, nx, -NG, ny + NG - 1), 0, nx, -NG, ny + NG - 1)
    fxx = xfx * fx2
    qj = z.copy()
    _put(qj, (_get(qx, 0, nx - 1, -NG, ny + NG - 1) * _get(area, 0, nx - 1, -NG, ny + NG - 1)
              + _get(fxx, 0, nx - 1, -NG, ny + NG - 1) - _get(fxx, 1, nx, -NG, ny + NG - 1))
         / _get(ra_x, 0, nx - 1, -NG, ny + NG - 1), 0, nx - 1, -NG, ny + NG - 1)
    fy = z.copy()
    _put(fy, yppm(qj, cry, dya, jo, N, ord_, 0, nx - 1, 0, ny), 0, nx - 1, 0, ny)
    mx = xfx if mfx is None else mfx
    my = yfx if mfy is None else mfy
    fxo = z.copy()
    fyo = z.copy()
    _put(fxo, 0.5 * (_get(fx, 0, nx, 0, ny - 1) + _get(fx2, 0, nx, 0, ny - 1)) * _get(mx, 0, nx, 0, ny - 1),
         0, nx, 0, ny - 1)
    _put(fyo, 0.5 * (_get(fy, 0, nx - 1, 0, ny) + _get(fy2, 0, nx - 1, 0, ny)) * _get(my, 0, nx - 1, 0, ny),
         0, nx - 1, 0, ny)
    return fxo, fyo


# ---------------- fv_tracer2d: tracer_2d_1l ----------------

def tracer_fluxes(cx, cy, m, nx, ny):
    """xfx/yfx from Courant numbers (upwind-side dxa*dy*sin_sg)."""
    xfx = np.zeros_like(cx)
    yfx = np.zeros_like(cy)
    i0, i1, j0, j1 = 0, nx, -NG, ny + NG - 1
    c = _get(cx, i0, i1, j0, j1)
    pos = c * _get(m["dxa"], i0 - 1, i1 - 1, j0, j1) * _get(m["dy"], i0, i1, j0, j1) * _get(m["sin_sg3"], i0 - 1, i1 - 1, j0, j1)
    neg = c * _get(m["dxa"], i0, i1, j0, j1) * _get(m["dy"], i0, i1, j0, j1) * _get(m["sin_sg1"], i0, i1, j0, j1)
    _put(xfx, np.where(c > 0.0, pos, neg), i0, i1, j0, j1)
    i0, i1, j0, j1 = -NG, nx + NG - 1, 0, ny
    c = _get(cy, i0, i1, j0, j1)
    pos = c * _get(m["dya"], i0, i1, j0 - 1, j1 - 1) * _get(m["dx"], i0, i1, j0, j1) * _get(m["sin_sg4"], i0, i1, j0 - 1, j1 - 1)
    neg = c * _get(m["dya"], i0, i1, j0, j1) * _get(m["dx"], i0, i1, j0, j1) * _get(m["sin_sg2"], i0, i1, j0, j1)
    _put(yfx, np.where(c > 0.0, pos, neg), i0, i1, j0, j1)
    return xfx, yfx


def tracer_cmax(cx, cy, m, nx, ny, npz):
    a = np.maximum(np.abs(_get(cx, 0, nx - 1, 0, ny - 1)), np.abs(_get(cy, 0, nx - 1, 0, ny - 1)))
    k = np.arange(npz)[:, None, None]
    a = np.where(k + 1 < npz // 6, a, a + 1.0 - _get(m["sin_sg5"], 0, nx - 1, 0, ny - 1))
    return a.reshape(npz, -1).max(axis=1)


def tracer_2d_1l(q, dp1, mfx, mfy, cx, cy, subs, ms, nx, ny, npz, nq, ord_, halo_fill):
    """q: (nsub, nq*npz, nj, pitch); per-sub lists of metrics; halo_fill(q) fills q halos in place.
    Mirrors FV3 tracer_2d_1l with global cmax (mp_reduce_max over all sub-domains)."""
    nsub = q.shape[0]
    dp1 = dp1.copy()
    cx, cy, mfx, mfy = cx.copy(), cy.copy(), mfx.copy(), mfy.copy()
    xfx, yfx = [], []
    cmax = np.zeros(npz)
    for s in range(nsub):
        a, b = tracer_fluxes(cx[s], cy[s], ms[s], nx, ny)
        xfx.append(a)
        yfx.append(b)
        cmax = np.maximum(cmax, tracer_cmax(cx[s], cy[s], ms[s], nx, ny, npz))
    nsplt = (1.0 + cmax).astype(int)
    nmax = int(nsplt.max())
    frac = np.where(nsplt > 1, 1.0 / nsplt, 1.0)[:, None, None]
    for s in range(nsub):
        for arr in (cx[s], xfx[s], cy[s], yfx[s], mfx[s], mfy[s]):
            sel = nsplt > 1
            arr[sel] = arr[sel] * frac[sel]
    ra_x, ra_y = [], []
    for s in range(nsub):
        area = ms[s]["area"]
        rx = np.zeros_like(cx[s])
        ry = np.zeros_like(cy[s])
        _put(rx, _get(area, 0, nx - 1, -NG, ny + NG - 1) + _get(xfx[s], 0, nx - 1, -NG, ny + NG - 1)
             - _get(xfx[s], 1, nx, -NG, ny + NG - 1), 0, nx - 1, -NG, ny + NG - 1)
        _put(ry, _get(area, -NG, nx + NG - 1, 0, ny - 1) + _get(yfx[s], -NG, nx + NG - 1, 0, ny - 1)
             - _get(yfx[s], -NG, nx + NG - 1, 1, ny), -NG, nx + NG - 1, 0, ny - 1)
        ra_x.append(rx)
        ra_y.append(ry)
    q = q.copy()
    halo_fill(q)
    for it in range(nmax):
        active = (it < nsplt)
        dp2s = []
        for s in range(nsub):
            dp2 = np.zeros_like(dp1[s])
            _put(dp2, _get(dp1[s], 0, nx - 1, 0, ny - 1) + (_get(mfx[s], 0, nx - 1, 0, ny - 1) - _get(mfx[s], 1, nx, 0, ny - 1)
                 + _get(mfy[s], 0, nx - 1, 0, ny - 1) - _get(mfy[s], 0, nx - 1, 1, ny)) * _get(ms[s]["rarea"], 0, nx - 1, 0, ny - 1),
                 0, nx - 1, 0, ny - 1)
            dp2s.append(dp2)
        for s in range(nsub):
            for iq in range(nq):
                qq = q[s, iq * npz:(iq + 1) * npz]
                fx, fy = fv_tp_2d(qq, cx[s], cy[s], xfx[s], yfx[s], ra_x[s], ra_y[s], subs[s], ms[s], nx, ny, ord_,
                                  mfx[s], mfy[s])
                new = (_get(qq, 0, nx - 1, 0, ny - 1) * _get(dp1[s], 0, nx - 1, 0, ny - 1)
                       + (_get(fx, 0, nx - 1, 0, ny - 1) - _get(fx, 1, nx, 0, ny - 1) + _get(fy, 0, nx - 1, 0, ny - 1)
                          - _get(fy, 0, nx - 1, 1, ny)) * _get(ms[s]["rarea"], 0, nx - 1, 0, ny - 1)) \
                    / _get(dp2s[s], 0, nx - 1, 0, ny - 1)
                old = _get(qq, 0, nx - 1, 0, ny - 1)
                _put(qq, np.where(active[:, None, None], new, old), 0, nx - 1, 0, ny - 1)
        if it + 1 < nmax:
            for s in range(nsub):
                dp1[s] = np.where(True, dp2s[s], dp1[s])
            halo_fill(q)
    return q, nsplt
