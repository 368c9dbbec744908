"""Moist column physics oracle — TEST INFRASTRUCTURE ONLY.

Numpy fp64 restatement of the moist column kernels of csrc/moist.hip, arrays [k, ...]
with k = 0 at the model top (the HBM layout's level order), columns in the trailing
axes.  The reference runs GEOS moist physics (GFDL 1M driver chain, buoyancy,
fillq2zero, ...: geos_documentation/moist/GFDL_1M.drawio:70-618, the standalone
experiments.yaml:42-110) from external repositories; none of that code is in the
reference, so this restates the published algorithms and is **parity unpinned**:

  saturation tables  GFDL MP qs_table form: es(T) = e00 exp((dc * ln(T/T0) + L0 (T-T0)/(T T0))/Rv),
                     integrated Clausius-Clapeyron with constant heat capacities, over water
                     (dc = cp_vap - c_liq) and over ice below T0 (dc = cp_vap - c_ice); tabulated
                     every 0.1 K from T0 - 160 K and read with linear interpolation
                     (GFDL_1M.drawio qs_table*, "wqs1 / iqs1")
  fillq2zero         column fill of negative water by rescaling the positive values so the
                     column mass sum(q dp) is kept (GEOS Moist FILLQ2ZERO)
  gfdl_1m            one column step of a GFDL-1M-style single-moment scheme (Lin et al. 1983,
                     Chen & Lin 2013): neg_adj, terminal velocities of rain / snow / graupel /
                     ice, implicit_fall sedimentation (GFDL_1M.drawio terminal_fall /
                     implicit_fall), Kessler autoconversion + accretion, Klemp-Wilhelmson rain
                     evaporation (revap_racc), saturation adjustment of cloud water,
                     homogeneous freezing below T0-40 K, ice deposition / sublimation,
                     melting of ice, snow and graupel (subgrid_z_proc / icloud)
  buoyancy           GEOS BUOYANCY: g (h_parcel - h*_env) / (cp T (1 + gamma)) with the parcel
                     moist static energy of the lowest layer, CAPE / CIN, and the LCL level index
                     of a dry-adiabatically lifted lowest-layer parcel (integer: bit-exact)

Same expression order as the HIP kernels; exp/log/pow differ in the last place between
ocml and glibc, so the HIP-vs-oracle bar is relative 1e-12 (bit-exact for the index field).
"""
import math

import numpy as np

GRAV = 9.80665
RDGAS = 8314.47 / 28.965
RVGAS = 8314.47 / 18.015
CP_AIR = 3.5 * RDGAS
EPS = RDGAS / RVGAS
CP_VAP = 4.0 * RVGAS
C_LIQ = 4185.5
C_ICE = 1972.0
HLV = 2.5e6
HLF = 3.3358e5
HLS = HLV + HLF
T_ICE = 273.16
E00 = 611.21
DC_VAP = CP_VAP - C_LIQ
D2ICE = CP_VAP - C_ICE
LV0 = HLV - DC_VAP * T_ICE
LI2 = HLS - D2ICE * T_ICE
KAPPA = RDGAS / CP_AIR

TABLE_T0 = T_ICE - 160.0
TABLE_N = 2621
TABLE_DT = 0.1

# GFDL / Lin (1983) fall-speed constants
VCONR, NORMR = 2503.23638966667, 25132741228.7183
VCONS, NORMS = 6.6280504, 942477796.076938
VCONG, NORMG = 87.2382675, 5026548245.74367
RHO_SFC = 1.2
VR_MIN, VR_MAX = 1.0e-3, 12.0
VS_MAX, VG_MAX, VI_MAX = 2.0, 12.0, 1.0
QMIN_FALL = 1.0e-8

# process constants (documented in csrc/moist.hip)
C_AUT, QL_CRIT = 1.0e-3, 5.0e-4     # Kessler autoconversion (1/s, kg/kg)
C_ACC = 2.2                          # Kessler accretion (1/s)
T_HOM = T_ICE - 40.0                 # homogeneous freezing
TAU_DEP = 600.0                      # ice deposition / sublimation relaxation time (s)
TAU_MLT = 600.0                      # melting relaxation time (s)


def es_water(t):
    """scalar, with the C library's exp/log (the HIP build tabulates on the host with the
    same libm, so the tables are bit-identical)"""
    fac0 = (t - T_ICE) / (t * T_ICE)
    return E00 * math.exp((DC_VAP * math.log(t / T_ICE) + LV0 * fac0) / RVGAS)


def es_ice(t):
    fac0 = (t - T_ICE) / (t * T_ICE)
    return E00 * math.exp((D2ICE * math.log(t / T_ICE) + LI2 * fac0) / RVGAS)


def tables():
    """(es over water, es over ice below T_ICE / water above) at TABLE_T0 + n TABLE_DT, and
    their forward differences (GFDL qs_table / qs_table2 with des = table(n+1) - table(n))."""
    t = [TABLE_T0 + TABLE_DT * float(n) for n in range(TABLE_N)]
    tw = np.array([es_water(x) for x in t])
    ti = np.array([es_ice(x) if x < T_ICE else es_water(x) for x in t])
    dw = np.append(tw[1:] - tw[:-1], 0.0)
    di = np.append(ti[1:] - ti[:-1], 0.0)
    return tw, ti, dw, di


_TAB = None


def _tab():
    global _TAB
    if _TAB is None:
        _TAB = tables()
    return _TAB


def es_lookup(t, ice):
    """table read: ap1 = 10 (T - T0), it = floor, es = table[it] + (ap1 - it) des[it]
    (T clamped to the table range)."""
    tw, ti, dw, di = _tab()
    tab, des = (ti, di) if ice else (tw, dw)
    tt = np.clip(t, TABLE_T0, TABLE_T0 + TABLE_DT * (TABLE_N - 2))
    ap1 = (tt - TABLE_T0) * 10.0
    it = ap1.astype(np.int64)
    return tab[it] + (ap1 - it) * des[it], des[it] * 10.0


def qsat(t, p, ice=False):
    """saturation specific humidity and its temperature derivative (GEOS form
    qs = eps es / (p - (1 - eps) es))."""
    es, desdt = es_lookup(t, ice)
    den = p - (1.0 - EPS) * es
    qs = EPS * es / den
    dqs = EPS * desdt * p / (den * den)
    return qs, dqs


def fillq2zero(q, dp):
    """q [k, ...] (copy returned), dp [k, ...]; also returns the filled amount -sum(min(q,0) dp)."""
    tpw = np.zeros(q.shape[1:])
    neg = np.zeros_like(tpw)
    tpw2 = np.zeros_like(tpw)
    for k in range(q.shape[0]):        # sequential sums, as the column kernel adds them
        tpw = tpw + q[k] * dp[k]
        neg = neg + np.minimum(q[k], 0.0) * dp[k]
        tpw2 = tpw2 + np.maximum(q[k], 0.0) * dp[k]
    qp = np.maximum(q, 0.0)
    fac = np.where(tpw2 > 0.0, np.maximum(tpw, 0.0) / np.where(tpw2 > 0.0, tpw2, 1.0), 0.0)
    out = qp * fac[None]
    return out, -neg


def fall_speeds(den, qr, qs, qg, qi):
    rhof = np.sqrt(np.minimum(10.0, RHO_SFC / den))
    vr = np.where(qr > QMIN_FALL,
                  np.minimum(VR_MAX, np.maximum(VR_MIN, VCONR * rhof * np.exp(0.2 * np.log(np.maximum(qr, QMIN_FALL) * den / NORMR)))),
                  VR_MIN)
    vs = np.where(qs > QMIN_FALL,
                  np.minimum(VS_MAX, VCONS * rhof * np.exp(0.0625 * np.log(np.maximum(qs, QMIN_FALL) * den / NORMS))), 0.0)
    vg = np.where(qg > QMIN_FALL,
                  np.minimum(VG_MAX, VCONG * rhof * np.sqrt(np.sqrt(np.sqrt(np.maximum(qg, QMIN_FALL) * den / NORMG)))), 0.0)
    vi = np.where(qi > QMIN_FALL,
                  np.minimum(VI_MAX, 3.29 * np.exp(0.16 * np.log(np.maximum(qi, QMIN_FALL) * den))), 0.0)
    return vr, vs, vg, vi


def implicit_fall(q, vt, dp, dz, dt):
    """GFDL implicit_fall: q [k, ...] mixing ratio, vt fall speed (m/s), dp (Pa), dz (m, >0).
    Returns the new q and the surface flux (kg/m2 over dt)."""
    nk = q.shape[0]
    dd = dt * vt
    m = q * dp / GRAV                       # layer mass (kg/m2)
    qm = np.empty_like(q)
    qm[0] = m[0] / (dz[0] + dd[0])
    for k in range(1, nk):
        qm[k] = (m[k] + dd[k - 1] * qm[k - 1]) / (dz[k] + dd[k])
    mout = qm * dz                          # new layer mass
    flux = dd[nk - 1] * qm[nk - 1]          # out of the bottom
    return mout * GRAV / dp, flux


def gfdl_1m(T, dp, dz, pm, qv, ql, qr, qi, qs, qg, dt):
    """One column step; all inputs [k, ...] (dz negative, FV3 delz).  Returns the updated
    (T, qv, ql, qr, qi, qs, qg) and the surface precipitation (rain, snow, graupel, ice)
    in kg/m2 over dt."""
    T, qv, ql, qr, qi, qs, qg = (np.array(x, dtype=np.float64, copy=True) for x in (T, qv, ql, qr, qi, qs, qg))
    lcp, icp, scp = HLV / CP_AIR, HLF / CP_AIR, HLS / CP_AIR
    # 1. neg_adj: negative species back to vapour, with the latent heat
    for q, lat in ((ql, lcp), (qr, lcp), (qi, scp), (qs, scp), (qg, scp)):
        neg = np.minimum(q, 0.0)
        qv += neg
        T -= neg * lat
        q -= neg
    # 2-3. fall speeds and implicit sedimentation (top to bottom)
    thick = -dz
    den = dp / (GRAV * thick)
    vr, vs, vg, vi = fall_speeds(den, qr, qs, qg, qi)
    qi, pi_ = implicit_fall(qi, vi, dp, thick, dt)
    qs, ps_ = implicit_fall(qs, vs, dp, thick, dt)
    qg, pg_ = implicit_fall(qg, vg, dp, thick, dt)
    qr, pr_ = implicit_fall(qr, vr, dp, thick, dt)
    # 4. warm rain: autoconversion, accretion, evaporation of rain
    aut = np.minimum(ql, dt * C_AUT * np.maximum(ql - QL_CRIT, 0.0))
    ql = ql - aut
    qr = qr + aut
    acc = np.minimum(ql, dt * C_ACC * ql * np.exp(0.875 * np.log(np.maximum(qr, 1.0e-30))))
    acc = np.where(qr > 0.0, acc, 0.0)
    ql = ql - acc
    qr = qr + acc
    qsw, dqsw = qsat(T, pm, ice=False)
    rq = den * qr
    cvent = 1.6 + 124.9 * np.exp(0.2046 * np.log(np.maximum(rq, 1.0e-30)))
    erate = (1.0 - qv / qsw) * cvent * np.exp(0.525 * np.log(np.maximum(rq, 1.0e-30))) / \
        (den * (5.4e5 + 2.55e8 / (pm * qsw)))
    evap = np.where((qv < qsw) & (qr > 0.0),
                    np.minimum(np.minimum(qr, dt * erate), (qsw - qv) / (1.0 + lcp * dqsw)), 0.0)
    qr = qr - evap
    qv = qv + evap
    T = T - evap * lcp
    # 5. saturation adjustment of cloud water (one Newton step)
    qsw, dqsw = qsat(T, pm, ice=False)
    dq = (qv - qsw) / (1.0 + lcp * dqsw)
    dq = np.where(dq > 0.0, dq, np.maximum(dq, -ql))
    qv = qv - dq
    ql = ql + dq
    T = T + dq * lcp
    # 6. homogeneous freezing of cloud water
    frz = np.where(T < T_HOM, ql, 0.0)
    ql = ql - frz
    qi = qi + frz
    T = T + frz * icp
    # 7. ice deposition / sublimation (relaxation towards ice saturation, T < T0)
    qsi, dqsi = qsat(T, pm, ice=True)
    fdep = 1.0 - np.exp(-dt / TAU_DEP)
    ddep = fdep * (qv - qsi) / (1.0 + scp * dqsi)
    ddep = np.where(T < T_ICE, np.where(ddep > 0.0, ddep, np.maximum(ddep, -qi)), 0.0)
    qv = qv - ddep
    qi = qi + ddep
    T = T + ddep * scp
    # 8. melting above T0: ice -> cloud water, snow and graupel -> rain
    fmlt = 1.0 - np.exp(-dt / TAU_MLT)
    for which in ("i", "s", "g"):
        q = {"i": qi, "s": qs, "g": qg}[which]
        cap = np.maximum(T - T_ICE, 0.0) / icp
        mlt = np.where(T > T_ICE, np.minimum(fmlt * q, cap), 0.0)
        q -= mlt
        if which == "i":
            ql = ql + mlt
        else:
            qr = qr + mlt
        T = T - mlt * icp
    return (T, qv, ql, qr, qi, qs, qg), (pr_, ps_, pg_, pi_)


def buoyancy(T, qv, pm, zm):
    """GEOS BUOYANCY on [k, ...] (k = 0 top): returns (buoy [k, ...], cape, cin, klcl)
    with zm the layer-mid heights (m).  klcl: index of the lowest level (counting from the
    top) at which a lowest-layer parcel lifted dry-adiabatically is saturated; -1 if none."""
    nk = T.shape[0]
    kb = nk - 1
    qs, dqs = qsat(T, pm, ice=False)
    hp = CP_AIR * T[kb] + GRAV * zm[kb] + HLV * qv[kb]
    gam = HLV / CP_AIR * dqs
    hs = CP_AIR * T + GRAV * zm + HLV * qs
    by = GRAV * (hp[None] - hs) / (CP_AIR * T * (1.0 + gam))
    cape = np.zeros_like(hp)
    cin = np.zeros_like(hp)
    free = np.zeros(hp.shape, dtype=bool)
    for k in range(kb - 1, -1, -1):          # bottom-up above the parcel level
        dzk = zm[k] - zm[k + 1]
        free = free | (by[k] > 0.0)
        cape = cape + np.where(by[k] > 0.0, by[k] * dzk, 0.0)
        cin = cin + np.where((by[k] < 0.0) & ~free, by[k] * dzk, 0.0)
    klcl = np.full(hp.shape, -1.0)
    tp0, pp0, qp0 = T[kb], pm[kb], qv[kb]
    for k in range(kb, -1, -1):
        tpar = tp0 * np.exp(KAPPA * np.log(pm[k] / pp0))
        qsp, _ = qsat(tpar, pm[k], ice=False)
        klcl = np.where((klcl < 0.0) & (qp0 >= qsp), float(k), klcl)
    return by, cape, cin, klcl
