"""Moist column physics oracle, common pieces — TEST
INFRASTRUCTURE ONLY (the checker of csrc/moist.hip; never on the product path).

Numpy fp64, arrays [k, ...] with k = 0 at the model top (the HBM layout's level order),
columns in the trailing axes.  The reference runs GEOS moist physics (GFDL 1M driver
chain, buoyancy, fillq2zero, ...: geos_documentation/moist/GFDL_1M.drawio:70-618, the
standalone experiments.yaml:42-110) from external repositories; none of that code is in
the reference, so this restates the published algorithms and is **parity unpinned**:

  saturation tables  GFDL MP qs_table form: es(T) = e00 exp((dc * ln(T/T0) + L0 (T-T0)/(T T0))/Rv),
                     Clausius-Clapeyron integrated with constant heat capacities (Emanuel 1994
                     eq. 4.4.13), over water (dc = cp_vap - c_liq) and over ice below T0
                     (dc = cp_vap - c_ice); tabulated every 0.1 K from T0 - 160 K and read with
                     linear interpolation (GFDL_1M.drawio qs_table*, "wqs1 / iqs1")
  fillq2zero         column fill of negative water by rescaling the positive values so the
                     column mass sum(q dp) is kept (GEOS Moist FILLQ2ZERO)
  buoyancy           GEOS BUOYANCY: g (h_parcel - h*_env) / (cp T (1 + gamma)) with the parcel
                     moist static energy of the lowest layer (Emanuel 1994 §6.1), CAPE / CIN,
                     and the LCL level index of a dry-adiabatically lifted lowest-layer parcel
                     (integer: bit-exact)

The GFDL cloud microphysics driver is oracle/gfdl_mp.py, the GEOS pieces around it
(evap_subl_pdf, radcouple, aer_activation) oracle/geos_moist.py.  The HIP kernels follow
these expressions; exp/log/pow differ in the last place between ocml and glibc, so the
HIP-vs-oracle bar is relative (bit-exact for the table reads and the index field).
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
