"""Oracle: FV3 fv_mapz — vertical Lagrangian-to-Eulerian remap (Lin 2004) in fp64
numpy, vectorised over columns.  TEST INFRASTRUCTURE ONLY.

cs_profile (PPM sub-grid reconstruction with kord = 9 Huynh constraint and
cs_limiters), map1_ppm (exact integration over target layers), fillz, and the
per-column sequence of Lagrangian_to_Eulerian for the non-hydrostatic dycore with
kord_tm < 0 (T_v remapped in log-p).  Columns are the trailing axes; level axis 0.
0-based: interface e = Fortran k-1 (top edge of layer e), layer l = Fortran k-1.
"""
import numpy as np

np.seterr(all="ignore")

GRAV = 9.80665
RDGAS = 8314.47 / 28.965
RVGAS = 8314.47 / 18.015
KAPPA = 1.0 / 3.5
ZVIR = RVGAS / RDGAS - 1.0
R3 = 1.0 / 3.0
R23 = 2.0 / 3.0


def cs_limiters(a, AL, AR, A6, extm, iv):
    """in place on column arrays (...)"""
    if iv == 0:
        neg = a <= 0.0
        cond = ~neg & (np.abs(AR - AL) < -A6)
        with np.errstate(all="ignore"):
            lm = a + 0.25 * (AR - AL) ** 2 / A6 + A6 * (1.0 / 12.0)
        cond = cond & (lm < 0.0)
        c1 = cond & (a < AR) & (a < AL)
        c2 = cond & ~c1 & (AR > AL)
        c3 = cond & ~c1 & ~c2
        flat = neg | c1
        nA6_2 = 3.0 * (AL - a)
        nA6_3 = 3.0 * (AR - a)
        AL_n = np.where(flat, a, np.where(c3, AR - nA6_3, AL))
        AR_n = np.where(flat, a, np.where(c2, AL - nA6_2, AR))
        A6_n = np.where(flat, 0.0, np.where(c2, nA6_2, np.where(c3, nA6_3, A6)))
        return AL_n, AR_n, A6_n
    if iv == 1:
        flat = (a - AL) * (a - AR) >= 0.0
    else:
        flat = extm
    da1 = AR - AL
    da2 = da1 * da1
    a6da = A6 * da1
    lo = ~flat & (a6da < -da2)
    hi = ~flat & ~lo & (a6da > da2)
    A6lo = 3.0 * (AL - a)
    A6hi = 3.0 * (AR - a)
    AL_n = np.where(flat, a, np.where(hi, AR - A6hi, AL))
    AR_n = np.where(flat, a, np.where(lo, AL - A6lo, AR))
    A6_n = np.where(flat, 0.0, np.where(lo, A6lo, np.where(hi, A6hi, A6)))
    return AL_n, AR_n, A6_n


def cs_profile(a, dp, iv, qs=None):
    """a, dp: (km, ...) -> (AL, AR, A6) each (km, ...); kord = 9."""
    km = a.shape[0]
    q = np.zeros((km + 1,) + a.shape[1:])
    gam = np.zeros((km + 1,) + a.shape[1:])
    if iv == -2:
        gam[1] = 0.5
        q[0] = 1.5 * a[0]
        for e in range(1, km - 1):
            grat = dp[e - 1] / dp[e]
            bet = 2.0 + grat + grat - gam[e]
            q[e] = (3.0 * (a[e - 1] + a[e]) - q[e - 1]) / bet
            gam[e + 1] = grat / bet
        grat = dp[km - 2] / dp[km - 1]
        q[km - 1] = (3.0 * (a[km - 2] + a[km - 1]) - grat * qs - q[km - 2]) / (2.0 + grat + grat - gam[km - 1])
        q[km] = qs
        for e in range(km - 2, -1, -1):
            q[e] = q[e] - gam[e + 1] * q[e + 1]
    else:
        grat = dp[1] / dp[0]
        bet = grat * (grat + 0.5)
        q[0] = ((grat + grat) * (grat + 1.0) * a[0] + a[1]) / bet
        gam[0] = (1.0 + grat * (grat + 1.5)) / bet
        d4 = grat
        for e in range(1, km):
            d4 = dp[e - 1] / dp[e]
            bet = 2.0 + d4 + d4 - gam[e - 1]
            q[e] = (3.0 * (a[e - 1] + d4 * a[e]) - q[e - 1]) / bet
            gam[e] = d4 / bet
        a_bot = 1.0 + d4 * (d4 + 1.5)
        q[km] = (2.0 * d4 * (d4 + 1.0) * a[km - 1] + a[km - 2] - a_bot * q[km - 1]) / (d4 * (d4 + 0.5) - a_bot * gam[km - 1])
        for e in range(km - 1, -1, -1):
            q[e] = q[e] - gam[e] * q[e + 1]
    # large-scale constraints
    q[1] = np.minimum(q[1], np.maximum(a[0], a[1]))
    q[1] = np.maximum(q[1], np.minimum(a[0], a[1]))
    g = np.zeros_like(q)  # g[e] = a[e] - a[e-1], e = 1..km-1
    g[1:km] = a[1:km] - a[0:km - 1]
    for e in range(2, km - 1):
        both = g[e - 1] * g[e + 1] > 0.0
        c_both = np.maximum(np.minimum(q[e], np.maximum(a[e - 1], a[e])), np.minimum(a[e - 1], a[e]))
        c_max = np.maximum(q[e], np.minimum(a[e - 1], a[e]))
        c_min = np.minimum(q[e], np.maximum(a[e - 1], a[e]))
        if iv == 0:
            c_min = np.maximum(0.0, c_min)
        q[e] = np.where(both, c_both, np.where(g[e - 1] > 0.0, c_max, c_min))
    q[km - 1] = np.minimum(q[km - 1], np.maximum(a[km - 2], a[km - 1]))
    q[km - 1] = np.maximum(q[km - 1], np.minimum(a[km - 2], a[km - 1]))
    AL = q[:km].copy()
    AR = q[1:].copy()
    A6 = np.zeros_like(a)
    extm = np.zeros(a.shape, dtype=bool)
    for l in range(km):
        if l == 0 or l == km - 1:
            extm[l] = (AL[l] - a[l]) * (AR[l] - a[l]) > 0.0
        else:
            extm[l] = g[l] * g[l + 1] < 0.0
    # top layer
    if iv == 0:
        AL[0] = np.maximum(0.0, AL[0])
    elif iv == -1:
        AL[0] = np.where(AL[0] * a[0] <= 0.0, 0.0, AL[0])
    A6[0] = 3.0 * (2.0 * a[0] - (AL[0] + AR[0]))
    AL[0], AR[0], A6[0] = cs_limiters(a[0], AL[0], AR[0], A6[0], extm[0], 1)
    A6[1] = 3.0 * (2.0 * a[1] - (AL[1] + AR[1]))
    AL[1], AR[1], A6[1] = cs_limiters(a[1], AL[1], AR[1], A6[1], extm[1], 2)
    for l in range(2, km - 2):
        flat = (extm[l] & extm[l - 1]) | (extm[l] & extm[l + 1])
        a6 = 6.0 * a[l] - 3.0 * (AL[l] + AR[l])
        chk = ~flat & (np.abs(a6) > np.abs(AL[l] - AR[l]))
        pmp_1 = a[l] - 2.0 * g[l + 1]
        lac_1 = pmp_1 + 1.5 * g[l + 2]
        al_n = np.minimum(np.maximum(AL[l], np.minimum(np.minimum(a[l], pmp_1), lac_1)),
                          np.maximum(np.maximum(a[l], pmp_1), lac_1))
        pmp_2 = a[l] + 2.0 * g[l]
        lac_2 = pmp_2 - 1.5 * g[l - 1]
        ar_n = np.minimum(np.maximum(AR[l], np.minimum(np.minimum(a[l], pmp_2), lac_2)),
                          np.maximum(np.maximum(a[l], pmp_2), lac_2))
        AL[l] = np.where(flat, a[l], np.where(chk, al_n, AL[l]))
        AR[l] = np.where(flat, a[l], np.where(chk, ar_n, AR[l]))
        A6[l] = np.where(flat, 0.0, np.where(chk, 6.0 * a[l] - 3.0 * (AL[l] + AR[l]), a6))
        if iv == 0:
            AL[l], AR[l], A6[l] = cs_limiters(a[l], AL[l], AR[l], A6[l], extm[l], 0)
    if iv == 0:
        AR[km - 1] = np.maximum(0.0, AR[km - 1])
    elif iv == -1:
        AR[km - 1] = np.where(AR[km - 1] * a[km - 1] <= 0.0, 0.0, AR[km - 1])
    for l in (km - 2, km - 1):
        A6[l] = 3.0 * (2.0 * a[l] - (AL[l] + AR[l]))
        AL[l], AR[l], A6[l] = cs_limiters(a[l], AL[l], AR[l], A6[l], extm[l], 2 if l == km - 2 else 1)
    return AL, AR, A6


def map1_ppm(pe1, a, pe2, iv, qs=None):
    """remap layer means a (km, ncol) from source edges pe1 (km+1, ncol) to pe2 (kn+1, ncol).
    Vectorised over columns; per column the Fortran two-pointer walk (k0, l, m) and the
    sequential qsum accumulation order are reproduced exactly."""
    km = a.shape[0]
    dp1 = pe1[1:] - pe1[:-1]
    AL, AR, A6 = cs_profile(a, dp1, iv, qs)
    kn = pe2.shape[0] - 1
    ncol = a.shape[1]
    cols = np.arange(ncol)
    out = np.zeros((kn, ncol))
    k0 = np.zeros(ncol, dtype=np.int64)
    for k in range(kn):
        top, bot = pe2[k], pe2[k + 1]
        l = np.minimum(np.maximum(k0, (pe1[1:] < top).sum(axis=0)), km - 1)
        p1l, p1l1, dpl = pe1[l, cols], pe1[l + 1, cols], dp1[l, cols]
        ALl, ARl, A6l = AL[l, cols], AR[l, cols], A6[l, cols]
        pl = (top - p1l) / dpl
        inside = bot <= p1l1
        pr = (bot - p1l) / dpl
        vA = ALl + 0.5 * (A6l + ARl - ALl) * (pr + pl) - A6l * R3 * (pr * (pr + pl) + pl * pl)
        qsum = (p1l1 - top) * (ALl + 0.5 * (A6l + ARl - ALl) * (1.0 + pl) - A6l * (R3 * (1.0 + pl * (1.0 + pl))))
        m = np.minimum(np.maximum(l + 1, (pe1[1:] < bot).sum(axis=0)), km - 1)
        for mm in range(km):
            add = (~inside) & (mm > l) & (mm < m)
            qsum = np.where(add, qsum + dp1[mm] * a[mm], qsum)
        dp = bot - pe1[m, cols]
        esl = dp / dp1[m, cols]
        qsum = qsum + dp * (AL[m, cols] + 0.5 * esl * (AR[m, cols] - AL[m, cols] + A6[m, cols] * (1.0 - R23 * esl)))
        out[k] = np.where(inside, vA, qsum / (bot - top))
        k0 = np.where(inside, l, m)
    return out


def fillz(q, dp):
    """FV3 fillz on (km, ncol) columns (one tracer), vectorised over columns"""
    q = q.copy()
    km = q.shape[0]
    neg = q[0] < 0.0
    q[1] = np.where(neg, q[1] + q[0] * dp[0] / dp[1], q[1])
    q[0] = np.where(neg, 0.0, q[0])
    zfix = np.zeros(q.shape[1], dtype=bool)
    for k in range(1, km - 1):
        n = q[k] < 0.0
        zfix |= n
        up = n & (q[k - 1] > 0.0)
        dq = np.minimum(q[k - 1] * dp[k - 1], -q[k] * dp[k])
        q[k - 1] = np.where(up, q[k - 1] - dq / dp[k - 1], q[k - 1])
        q[k] = np.where(up, q[k] + dq / dp[k], q[k])
        dn = n & (q[k] < 0.0) & (q[k + 1] > 0.0)
        dq = np.minimum(q[k + 1] * dp[k + 1], -q[k] * dp[k])
        q[k + 1] = np.where(dn, q[k + 1] - dq / dp[k + 1], q[k + 1])
        q[k] = np.where(dn, q[k] + dq / dp[k], q[k])
    k = km - 1
    b = (q[k] < 0.0) & (q[k - 1] > 0.0)
    zfix |= b
    qup = q[k - 1] * dp[k - 1]
    qly = -q[k] * dp[k]
    dup = np.minimum(qly, qup)
    q[k - 1] = np.where(b, q[k - 1] - dup / dp[k - 1], q[k - 1])
    q[k] = np.where(b, q[k] + dup / dp[k], q[k])
    dm = q[1:] * dp[1:]
    sum0 = np.zeros(q.shape[1])
    for kk in range(km - 1):
        sum0 = sum0 + dm[kk]
    sum1 = np.zeros(q.shape[1])
    for kk in range(km - 1):
        sum1 = sum1 + np.maximum(0.0, dm[kk])
    fix = zfix & (sum0 > 0.0)
    fac = sum0 / sum1
    for kk in range(1, km):
        q[kk] = np.where(fix, np.maximum(0.0, fac * dm[kk - 1] / dp[kk]), q[kk])
    return q


def lagrangian_to_eulerian(st, ak, bk, ptop, nq, fill, P):
    """Remap one sub-domain's state dict (planes with level axis) in place-like fashion.
    st keys: pe (km+1, with 1-halo), delp, delz, pt (theta_v), w, q (nq*km), u, v, ws, peln, pk, pkz, ps.
    Returns a new dict."""
    from . import NG
    nx, ny = P.nx, P.ny
    km = st["delp"].shape[0]
    rrg = -RDGAS / GRAV
    k1k = KAPPA / (1.0 - KAPPA)
    out = {k: v.copy() for k, v in st.items()}
    j0, i0 = NG, NG
    sl = (slice(None), slice(j0, j0 + ny), slice(i0, i0 + nx))

    def col(a):  # (k, ny, nx) -> (k, ncol)
        return a[sl].reshape(a.shape[0], -1)

    def put(name, vals, nk):
        arr = out[name]
        arr[sl] = vals.reshape(nk, ny, nx)

    pe1 = col(st["pe"])
    delp, delz, pt, w = col(st["delp"]), col(st["delz"]), col(st["pt"]), col(st["w"])
    ncol = pe1.shape[1]
    pt = pt * np.exp(k1k * np.log(rrg * delp / delz * pt))
    delz = -delz / delp
    psn = pe1[km]
    pe2 = np.zeros_like(pe1)
    pe2[0] = ptop
    pe2[km] = pe1[km]
    for k in range(1, km):
        pe2[k] = ak[k] + bk[k] * pe1[km]
    dp2 = pe2[1:] - pe2[:-1]
    peln1 = col(st["peln"])
    pn2 = np.zeros_like(pe1)
    pn2[0] = peln1[0]
    pn2[km] = peln1[km]
    pn2[1:km] = np.log(pe2[1:km])
    # T_v in log p (kord_tm < 0, iv = 1)
    ptn = map1_ppm(peln1, pt, pn2, 1)
    qs = col(st["q"]) if nq else None
    qn = []
    for iq in range(nq):
        qq = map1_ppm(pe1, qs[iq * km:(iq + 1) * km], pe2, 0)
        if fill:
            qq = fillz(qq, dp2)
        qn.append(qq)
    ws = st["ws"][NG:NG + ny, NG:NG + nx].reshape(-1)
    wn = map1_ppm(pe1, w, pe2, -2, ws)
    dzn = map1_ppm(pe1, delz, pe2, 1)
    dzn = -dzn * dp2
    pkn = np.exp(KAPPA * pn2)
    pkzn = np.exp(KAPPA * np.log(rrg * dp2 / dzn * ptn))
    put("pt", ptn, km)
    put("delp", dp2, km)
    put("delz", dzn, km)
    put("w", wn, km)
    put("pk", pkn, km + 1)
    put("peln", pn2, km + 1)
    put("pkz", pkzn, km)
    out["ps"][0, NG:NG + ny, NG:NG + nx] = psn.reshape(ny, nx)
    if nq:
        put("q", np.concatenate(qn, axis=0), nq * km)
    # u on x-edges (rows j in [0, ny]), v on y-edges (cols i in [0, nx])
    pe = st["pe"]
    pu_j = pe[:, NG - 1:NG + ny, NG:NG + nx]      # cell rows j-1 for edge rows 0..ny
    pu_0 = pe[:, NG:NG + ny + 1, NG:NG + nx]      # cell rows j
    pe0 = np.zeros_like(pu_0)
    pe0[0] = pu_0[0]
    pe0[1:] = 0.5 * (pu_j[1:] + pu_0[1:])
    pe3 = np.zeros_like(pu_0)
    for k in range(km + 1):
        bkh = 0.5 * bk[k]
        pe3[k] = ak[k] + bkh * (pu_j[km] + pu_0[km])
    u = st["u"][:, NG:NG + ny + 1, NG:NG + nx]
    un = map1_ppm(pe0.reshape(km + 1, -1), u.reshape(km, -1), pe3.reshape(km + 1, -1), -1)
    out["u"][:, NG:NG + ny + 1, NG:NG + nx] = un.reshape(km, ny + 1, nx)
    pv_i = pe[:, NG:NG + ny, NG - 1:NG + nx]
    pv_0 = pe[:, NG:NG + ny, NG:NG + nx + 1]
    pe0 = np.zeros_like(pv_0)
    pe0[0] = pv_0[0]
    pe3 = np.zeros_like(pv_0)
    pe3[0] = ak[0]
    for k in range(1, km + 1):
        bkh = 0.5 * bk[k]
        pe0[k] = 0.5 * (pv_i[k] + pv_0[k])
        pe3[k] = ak[k] + bkh * (pv_i[km] + pv_0[km])
    v = st["v"][:, NG:NG + ny, NG:NG + nx + 1]
    vn = map1_ppm(pe0.reshape(km + 1, -1), v.reshape(km, -1), pe3.reshape(km + 1, -1), -1)
    out["v"][:, NG:NG + ny, NG:NG + nx + 1] = vn.reshape(km, ny, nx + 1)
    # Eulerian interface pressures
    pen = out["pe"].copy()
    for k in range(1, km):
        pen[k, NG:NG + ny, NG:NG + nx] = ak[k] + bk[k] * pe[km, NG:NG + ny, NG:NG + nx]
    out["pe"] = pen
    del ncol
    return out
