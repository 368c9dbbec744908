"""GFDL single-moment cloud microphysics, one column driver
— TEST INFRASTRUCTURE ONLY (the checker of csrc/moist.hip; never on the product path).

Restated from the published scheme, not from the HIP kernels: six species (vapour,
cloud water, rain, cloud ice, snow, graupel) with Marshall-Palmer exponential size
distributions and the bulk process rates of Lin, Farley & Orville (1983, JCAM 22),
Rutledge & Hobbs (1984), Lord et al. (1984), with the GFDL modifications of Chen & Lin
(2013, J. Climate 26) and Zhou, Harris et al. (2019, JAMES 11): moist heat capacity
(cvm) with temperature-dependent latent heats, time-split sub-steps of at most MP_TIME,
sedimentation as a Lagrangian remap of a PPM profile in height, and the heat carried by
falling condensate.  The call structure is GEOS's (the reference's call graph
geos_documentation/moist/GFDL_1M.drawio):

  gfdl_cloud_microphys_driver :122 -> mpdrv :418 per column
     neg_adj                               negative species -> their source, with latent heat
     fall_speed                            terminal velocities of ice, snow, graupel
     terminal_fall :436                    melting of falling ice species, then
        lagrangian_fall_ppm :507           sedimentation of qi, qs, qg (cs_profile :615,
                                           cs_limiters: monotone PPM in height)
        sedi_heat                          heat of the falling condensate
     warm_rain :477                        two half steps of revap_racc (rain evaporation +
                                           accretion of cloud water), rain sedimentation and
                                           sedi_heat between them, then autoconversion
     icloud :501                           ice-phase processes (pimlt, pifr, psacw, psaut,
                                           psaci, pgaut, pgacw, smlt, gmlt) then
        subgrid_z_proc                     condensation / evaporation of cloud water,
                                           deposition / sublimation of ice, snow, graupel

Arrays are [k, ...] with k = 0 at the model top (the HBM level order); everything is
elementwise over the trailing column axes except the sedimentation remap, which walks
each column.  The reference holds no GFDL numerics (they live in GEOS repositories the
CI fetches): **parity unpinned** — the HIP kernels are checked against this module at
the reference's own moist bar (0.01 %, physics_standalone.py:132-144) and, tighter, at
1e-9 of each field's scale (exp / log / pow come from ocml on the GPU, glibc here).
"""
import math

import numpy as np

from .moist import GRAV, RDGAS, RVGAS, CP_AIR, T_ICE, C_LIQ, C_ICE, HLV, HLF, es_lookup

# ---- heat capacities and latent heats (constant-volume, the non-hydrostatic dycore) ----
CV_AIR = CP_AIR - RDGAS
CV_VAP = 3.0 * RVGAS
D0_VAP = CV_VAP - C_LIQ          # d(Lv)/dT at constant volume
DC_ICE = C_LIQ - C_ICE           # d(Lf)/dT
LV00 = HLV - D0_VAP * T_ICE      # Lv(T) = LV00 + D0_VAP T
LI00 = HLF - DC_ICE * T_ICE      # Lf(T) = LI00 + DC_ICE T

# ---- size distributions (Lin et al. 1983 Table 1; Rutledge & Hobbs 1984) ----
PIE = math.pi
RNZR, RNZS, RNZG = 8.0e6, 3.0e6, 4.0e6      # intercepts (m-4)
RHOR, RHOS, RHOG = 1.0e3, 1.0e2, 4.0e2      # densities (kg m-3)
ALIN, CLIN = 842.0, 4.8                     # rain / snow fall-speed coefficients
GCON = 40.74 * math.sqrt(1.2)               # graupel
SFCRHO = 1.2                                # reference surface air density
VDIFU, TCOND, VISK = 2.11e-5, 2.36e-2, 1.259e-5   # vapour diffusivity, conductivity, viscosity
ACT_S, ACT_R, ACT_G = PIE * RNZS * RHOS, PIE * RNZR * RHOR, PIE * RNZG * RHOG
SCM3 = (VISK / VDIFU) ** (1.0 / 3.0)
# collection and evaporation coefficients (Lin et al. 1983 eqs. 20-22, 52; gamma function
# values at the distribution exponents)
CRACW = PIE * RNZR * ALIN * math.gamma(3.8) / (4.0 * ACT_R ** 0.95)
CSACW = PIE * RNZS * CLIN * math.gamma(3.25) / (4.0 * ACT_S ** 0.8125)
CGACW = PIE * RNZG * math.gamma(3.5) * GCON / (4.0 * ACT_G ** 0.875)
CREVP = (2.0 * PIE * VDIFU * TCOND * RVGAS * RNZR,
         0.78 / math.sqrt(ACT_R),
         0.31 * SCM3 * math.gamma(2.9) * math.sqrt(ALIN / VISK) / ACT_R ** 0.725,
         TCOND * RVGAS,
         HLV * HLV * VDIFU)

# ---- namelist-style parameters (GFDL MP defaults as GEOS sets them) ----
MP_TIME = 150.0                  # longest microphysics sub-step (s)
TAU_IMLT, TAU_SMLT, TAU_GMLT = 600.0, 900.0, 600.0   # melting time scales (s)
TAU_L2V, TAU_V2L, TAU_I2V = 300.0, 150.0, 300.0      # cloud water evaporation / condensation, ice sublimation
TAU_I2S = 1000.0                 # ice -> snow autoconversion
QI0_CRIT, QS0_CRIT = 1.0e-4, 1.0e-3                  # ice -> snow, snow -> graupel thresholds
C_PSACI, C_PAUT = 0.02, 0.55     # ice accretion by snow efficiency, autoconversion scale
QL0_AUT = 5.0e-4                 # cloud water autoconversion threshold
T_WFR = T_ICE - 40.0             # homogeneous freezing
QRMIN, QCMIN, QVMIN = 1.0e-8, 1.0e-12, 1.0e-20
DZ_MIN_FALL = 1.0e-2             # smallest Lagrangian layer (m)
VI_MAX, VS_MAX, VG_MAX, VR_MAX = 1.0, 2.0, 12.0, 12.0
VR_MIN = 1.0e-3
R3, R23 = 1.0 / 3.0, 2.0 / 3.0


# ------------------------------------------------------------------------------ helpers
def cvm_of(qv, ql, qr, qi, qs, qg):
    """moist heat capacity at constant volume per unit moist-air mass"""
    return CV_AIR + qv * CV_VAP + (qr + ql) * C_LIQ + (qi + qs + qg) * C_ICE


def lhl(t):
    return LV00 + D0_VAP * t


def lhi(t):
    return LI00 + DC_ICE * t


def wqs2(t, den):
    """saturation mixing ratio over water in density form es(T) / (Rv T rho) and dqs/dT
    (GFDL wqs2; es from the 0.1 K table of oracle/moist.py, qs_table2)"""
    es, des = es_lookup(t, False)
    q = es / (RVGAS * t * den)
    return q, (des - es / t) / (RVGAS * t * den)


def iqs2(t, den):
    """same over ice below T_ICE (GFDL iqs2, qs_table)"""
    es, des = es_lookup(t, True)
    q = es / (RVGAS * t * den)
    return q, (des - es / t) / (RVGAS * t * den)


# ------------------------------------------------------------------------------ neg_adj
def neg_adj(t, dp, qv, ql, qr, qi, qs, qg):
    """GFDL neg_adj: negative ice species borrow down the chain ice -> snow -> graupel ->
    vapour, liquid rain -> cloud water -> vapour (with the latent heat of the phase change),
    negative vapour borrows from the layer below (column water kept).  In place."""
    nk = t.shape[0]
    for k in range(nk):
        cvm = cvm_of(qv[k], ql[k], qr[k], qi[k], qs[k], qg[k])
        lcpk = lhl(t[k]) / cvm
        icpk = lhi(t[k]) / cvm
        # ice phase
        m = qi[k] < 0.0
        qs[k] = np.where(m, qs[k] + qi[k], qs[k])
        qi[k] = np.where(m, 0.0, qi[k])
        m = qs[k] < 0.0
        qg[k] = np.where(m, qg[k] + qs[k], qg[k])
        qs[k] = np.where(m, 0.0, qs[k])
        m = qg[k] < 0.0
        dq = np.where(m, qg[k], 0.0)
        qv[k] = qv[k] + dq
        t[k] = t[k] - dq * (lcpk + icpk)
        qg[k] = np.where(m, 0.0, qg[k])
        # liquid phase
        m = qr[k] < 0.0
        ql[k] = np.where(m, ql[k] + qr[k], ql[k])
        qr[k] = np.where(m, 0.0, qr[k])
        m = ql[k] < 0.0
        dq = np.where(m, ql[k], 0.0)
        qv[k] = qv[k] + dq
        t[k] = t[k] - dq * lcpk
        ql[k] = np.where(m, 0.0, ql[k])
    # negative vapour: borrow from below (moist mass dp kept)
    for k in range(nk - 1):
        m = qv[k] < 0.0
        qv[k + 1] = np.where(m, qv[k + 1] + qv[k] * dp[k] / dp[k + 1], qv[k + 1])
        qv[k] = np.where(m, 0.0, qv[k])
    k = nk - 1
    m = (qv[k] < 0.0) & (qv[k - 1] > 0.0)
    dq = np.minimum(-qv[k] * dp[k], qv[k - 1] * dp[k - 1])
    dq = np.where(m, dq, 0.0)
    qv[k - 1] = qv[k - 1] - dq / dp[k - 1]
    qv[k] = qv[k] + dq / dp[k]


# ------------------------------------------------------------------------------ fall speeds
def fall_speed(den, qs, qi, qg):
    """terminal velocities (m/s, positive down): ice after Heymsfield & Donner (1990),
    snow and graupel from the Lin et al. (1983) mass-weighted distribution averages with the
    density correction sqrt(rho_sfc / rho)"""
    rhof = np.sqrt(np.minimum(10.0, SFCRHO / den))
    qi_ = np.maximum(qi, QCMIN)
    vti = np.where(qi > QCMIN, np.minimum(VI_MAX, 3.29 * np.exp(0.16 * np.log(qi_ * den))), 0.0)
    qs_ = np.maximum(qs, QCMIN)
    vts = np.where(qs > QCMIN, np.minimum(VS_MAX, 6.6280504 * rhof * np.exp(0.0625 * np.log(qs_ * den / 942477796.076938))), 0.0)
    qg_ = np.maximum(qg, QCMIN)
    vtg = np.where(qg > QCMIN, np.minimum(VG_MAX, 87.2382675 * rhof * np.sqrt(np.sqrt(np.sqrt(qg_ * den / 5026548245.74367)))), 0.0)
    return vti, vts, vtg


def rain_speed(den, qr):
    rhof = np.sqrt(np.minimum(10.0, SFCRHO / den))
    qr_ = np.maximum(qr, QRMIN)
    return np.where(qr > QRMIN,
                    np.minimum(VR_MAX, np.maximum(VR_MIN, 2503.23638966667 * rhof *
                                                  np.exp(0.2 * np.log(qr_ * den / 25132741228.7183)))), 0.0)


# ------------------------------------------------------------------------------ PPM in height
def cs_profile_mono(a, dz):
    """Edge values and curvature of a monotone PPM profile of the layer means a[k] (layer
    thicknesses dz[k] > 0, k = 0 top) — GFDL MP cs_profile with cs_limiters (mono): the
    4th-order edge values of the tridiagonal system (Colella & Woodward 1984 eq. 1.6 on a
    non-uniform grid), bounded by the neighbouring means, then the monotonicity limiter.
    Per column (1-D arrays).  Returns (aL, aR, a6)."""
    n = a.shape[0]
    q = np.empty(n + 1)
    gam = np.empty(n)
    # top edge: extrapolation from the first two layers
    grat = dz[1] / dz[0]
    bet = grat * (grat + 0.5)
    q[0] = ((grat + grat) * (grat + 1.0) * a[0] + a[1]) / bet
    gam[0] = (1.0 + grat * (grat + 1.5)) / bet
    for k in range(1, n):
        d4 = dz[k - 1] / dz[k]
        bet = 2.0 + d4 + d4 - gam[k - 1]
        q[k] = (3.0 * (a[k - 1] + d4 * a[k]) - q[k - 1]) / bet
        gam[k] = d4 / bet
    d4 = dz[n - 2] / dz[n - 1]
    a_bot = 1.0 + d4 * (d4 + 1.5)
    q[n] = (2.0 * d4 * (d4 + 1.0) * a[n - 1] + a[n - 2] - a_bot * q[n - 1]) / (d4 * (d4 + 0.5) - a_bot * gam[n - 1])
    for k in range(n - 1, -1, -1):
        q[k] = q[k] - gam[k] * q[k + 1]
    # edges bounded by the adjacent means; non-negative
    for k in range(1, n):
        q[k] = min(max(q[k], min(a[k - 1], a[k])), max(a[k - 1], a[k]))
    q[0] = max(q[0], 0.0)
    q[n] = max(q[n], 0.0)
    aL = q[:-1].copy()
    aR = q[1:].copy()
    a6 = np.empty(n)
    for k in range(n):
        # monotonicity (cs_limiters, mono): flatten extrema, steepen overshooting parabolas
        da1 = aR[k] - aL[k]
        if (a[k] - aL[k]) * (a[k] - aR[k]) >= 0.0:
            aL[k] = a[k]
            aR[k] = a[k]
            a6[k] = 0.0
            continue
        a6[k] = 3.0 * (2.0 * a[k] - (aL[k] + aR[k]))
        if a6[k] * da1 < -da1 * da1:
            a6[k] = 3.0 * (aL[k] - a[k])
            aR[k] = aL[k] - a6[k]
        elif a6[k] * da1 > da1 * da1:
            a6[k] = 3.0 * (aR[k] - a[k])
            aL[k] = aR[k] - a6[k]
    return aL, aR, a6


def lagrangian_fall_ppm(ze, zt, dp, q):
    """GFDL lagrangian_fall_ppm, one column: the layers [ze(k+1), ze(k)] (heights, k = 0 top,
    ze decreasing) fall to [zt(k+1), zt(k)]; the species' mass per unit height is profiled
    (monotone PPM) on the fallen layers and integrated back over the fixed layers.  Returns
    the new mixing ratio and the mass flux m1[k] through the bottom of layer k (kg m-2 over
    the step, GRAV-scaled as dp: the surface precipitation is m1[-1] / GRAV)."""
    n = q.shape[0]
    qm0 = q * dp                               # layer "mass" (Pa units)
    dz = zt[:-1] - zt[1:]
    a = qm0 / dz                               # per unit height on the fallen layers
    aL, aR, a6 = cs_profile_mono(a, dz)
    qm = np.zeros(n)
    k0 = 0
    for k in range(n):
        top, bot = ze[k], ze[k + 1]
        done = False
        for m in range(k0, n):
            if top <= zt[m] and top >= zt[m + 1]:
                pl = (zt[m] - top) / dz[m]
                if zt[m + 1] <= bot:
                    # the fixed layer lies inside fallen layer m
                    pr = (zt[m] - bot) / dz[m]
                    qm[k] = (aL[m] + 0.5 * (a6[m] + aR[m] - aL[m]) * (pr + pl) - a6[m] * R3 * (pr * (pr + pl) + pl * pl)) * (top - bot)
                    k0 = m
                else:
                    s = (top - zt[m + 1]) * (aL[m] + 0.5 * (a6[m] + aR[m] - aL[m]) * (1.0 + pl) - a6[m] * (R3 * (1.0 + pl * (1.0 + pl))))
                    for mm in range(m + 1, n):
                        if bot < zt[mm + 1]:
                            s = s + qm0[mm]              # whole fallen layer
                        else:
                            dzz = zt[mm] - bot
                            esl = dzz / dz[mm]
                            s = s + dzz * (aL[mm] + 0.5 * esl * (aR[mm] - aL[mm] + a6[mm] * (1.0 - R23 * esl)))
                            k0 = mm
                            break
                    qm[k] = s
                done = True
                break
        if not done:
            qm[k] = 0.0
    m1 = np.empty(n)
    acc = 0.0
    for k in range(n):
        acc = acc + qm0[k] - qm[k]
        m1[k] = acc
    return qm / dp, m1


def fallen_edges(ze, vt, dts):
    """Lagrangian interface heights after a fall of dts with layer speeds vt (k = 0 top):
    interior interfaces move with the mean of the two layers' speeds, the top stays, the
    bottom moves with the last layer's; kept strictly decreasing (DZ_MIN_FALL)."""
    n = vt.shape[0]
    zt = np.empty(n + 1)
    zt[0] = ze[0]
    for k in range(1, n):
        zt[k] = ze[k] - 0.5 * dts * (vt[k - 1] + vt[k])
    zt[n] = ze[n] - dts * vt[n - 1]
    for k in range(n):
        if zt[k + 1] >= zt[k]:
            zt[k + 1] = zt[k] - DZ_MIN_FALL
    return zt


def sedi_heat(t, dp, m1, dz, qv, ql, qr, qi, qs, qg, cw):
    """GFDL sedi_heat, one column: the condensate falling into layer k (flux m1[k-1], Pa
    units) arrives with heat capacity cw at the temperature of the layer above plus the
    potential energy it lost, g |dz| / 2 per unit mass; in place"""
    n = t.shape[0]
    for k in range(1, n):
        dgz = -0.5 * GRAV * dz[k]          # dz < 0
        cv0 = dp[k] * cvm_of(qv[k], ql[k], qr[k], qi[k], qs[k], qg[k]) + cw * (m1[k] - m1[k - 1])
        t[k] = (cv0 * t[k] + m1[k - 1] * (cw * t[k - 1] + dgz)) / (cv0 + cw * m1[k - 1])


# ------------------------------------------------------------------------------ processes
def terminal_fall(dts, t, dp, dz, ze, den, qv, ql, qr, qi, qs, qg):
    """melting of falling cloud ice / snow / graupel in layers above freezing (relaxation with
    the available heat), then sedimentation of qi, qs, qg (lagrangian_fall_ppm) with
    sedi_heat.  One column, in place; returns the surface (ice, snow, graupel) precipitation
    in kg m-2 over dts."""
    # melting of the falling ice species where T > T_ICE (into cloud water / rain)
    fi = 1.0 - math.exp(-dts / TAU_IMLT)
    fs = 1.0 - math.exp(-dts / TAU_SMLT)
    fg = 1.0 - math.exp(-dts / TAU_GMLT)
    for k in range(t.shape[0]):
        if t[k] > T_ICE:
            for which, f in (("i", fi), ("s", fs), ("g", fg)):
                q = {"i": qi, "s": qs, "g": qg}[which]
                cvm = cvm_of(qv[k], ql[k], qr[k], qi[k], qs[k], qg[k])
                icpk = lhi(t[k]) / cvm
                mlt = min(f * q[k], (t[k] - T_ICE) / icpk)
                if mlt > 0.0:
                    q[k] = q[k] - mlt
                    if which == "i":
                        ql[k] = ql[k] + mlt
                    else:
                        qr[k] = qr[k] + mlt
                    t[k] = t[k] - mlt * icpk
    vti, vts, vtg = fall_speed(den, qs, qi, qg)
    out = []
    for q, vt in ((qi, vti), (qs, vts), (qg, vtg)):
        if np.any(q > QCMIN):
            zt = fallen_edges(ze, vt, dts)
            qn, m1 = lagrangian_fall_ppm(ze, zt, dp, q)
            q[:] = qn
            sedi_heat(t, dp, m1, dz, qv, ql, qr, qi, qs, qg, C_ICE)
            out.append(m1[-1] / GRAV)
        else:
            out.append(0.0)
    return tuple(out)


def revap_racc(dt, t, den, qv, ql, qr, qi, qs, qg):
    """evaporation of rain in subsaturated air (Lin et al. 1983 eq. 52, ventilated) and the
    accretion of cloud water by rain (eq. 51), elementwise over a layer (in place)"""
    cvm = cvm_of(qv, ql, qr, qi, qs, qg)
    lcpk = lhl(t) / cvm
    qsat, dqsdt = wqs2(t, den)
    dqv = qsat - qv
    qden = np.maximum(qr, QRMIN) * den
    t2 = t * t
    ev = CREVP[0] * t2 * dqv * (CREVP[1] * np.sqrt(qden) + CREVP[2] * np.exp(0.725 * np.log(qden))) / \
        (CREVP[3] * t2 + CREVP[4] * qsat * den)
    evap = np.minimum(np.minimum(qr, dt * ev), dqv / (1.0 + lcpk * dqsdt))
    evap = np.where((dqv > QVMIN) & (qr > QRMIN), evap, 0.0)
    qr -= evap
    qv += evap
    t -= evap * lcpk
    # accretion of cloud water by rain
    denfac = np.sqrt(SFCRHO / den)
    sink = dt * denfac * CRACW * np.exp(0.95 * np.log(np.maximum(qr, QRMIN) * den))
    sink = sink / (1.0 + sink) * ql
    sink = np.where((qr > QRMIN) & (ql > QCMIN), sink, 0.0)
    ql -= sink
    qr += sink


def warm_rain(dts, t, dp, dz, ze, den, qv, ql, qr, qi, qs, qg):
    """two half steps of revap_racc around the rain sedimentation (lagrangian_fall_ppm +
    sedi_heat), then the autoconversion of cloud water (Kessler-type with the threshold
    QL0_AUT, rate c_paut (ql - ql0)^2 / (ql + ...) form of GFDL praut).  One column, in
    place; returns the surface rain (kg m-2 over dts)."""
    dt5 = 0.5 * dts
    revap_racc(dt5, t, den, qv, ql, qr, qi, qs, qg)
    vtr = rain_speed(den, qr)
    rain = 0.0
    if np.any(qr > QRMIN):
        zt = fallen_edges(ze, vtr, dts)
        qn, m1 = lagrangian_fall_ppm(ze, zt, dp, qr)
        qr[:] = qn
        sedi_heat(t, dp, m1, dz, qv, ql, qr, qi, qs, qg, C_LIQ)
        rain = m1[-1] / GRAV
    revap_racc(dt5, t, den, qv, ql, qr, qi, qs, qg)
    # autoconversion cloud water -> rain
    dq = ql - QL0_AUT
    aut = dts * C_PAUT * 1.0e-3 * dq * dq / (dq + 1.0e-3)
    aut = np.where(dq > 0.0, np.minimum(aut, dq), 0.0)
    ql -= aut
    qr += aut
    return rain


def icloud(dts, t, den, qv, ql, qr, qi, qs, qg):
    """ice-phase processes of one layer set (elementwise, in place), each with its latent
    heat at the current moist heat capacity:
      pimlt  cloud ice melting above T_ICE (relaxation, heat limited)
      pifr   homogeneous freezing of cloud water below T_WFR
      psacw  accretion of cloud water by snow (rimed onto snow below T_ICE)
      psaut  ice -> snow autoconversion above QI0_CRIT (time scale TAU_I2S, T dependent)
      psaci  accretion of cloud ice by snow (efficiency exp(0.05 Tc) C_PSACI)
      pgaut  snow -> graupel above QS0_CRIT (T dependent)
      pgacw  accretion of cloud water by graupel
      smlt / gmlt   melting of snow / graupel above T_ICE into rain
    then subgrid_z_proc."""
    denfac = np.sqrt(SFCRHO / den)
    tc = t - T_ICE
    # pimlt
    cvm = cvm_of(qv, ql, qr, qi, qs, qg)
    icpk = lhi(t) / cvm
    mlt = np.minimum(qi * (1.0 - math.exp(-dts / TAU_IMLT)), np.maximum(tc, 0.0) / icpk)
    mlt = np.where(tc > 0.0, mlt, 0.0)
    qi -= mlt
    ql += mlt
    t -= mlt * icpk
    # pifr
    cvm = cvm_of(qv, ql, qr, qi, qs, qg)
    icpk = lhi(t) / cvm
    frz = np.where(t < T_WFR, ql, 0.0)
    ql -= frz
    qi += frz
    t += frz * icpk
    tc = t - T_ICE
    cold = tc < 0.0
    # psacw (below freezing: riming; above, it is shed as rain)
    fac = dts * denfac * CSACW * np.exp(0.8125 * np.log(np.maximum(qs, QCMIN) * den))
    psacw = np.where((qs > QCMIN) & (ql > QCMIN), fac / (1.0 + fac) * ql, 0.0)
    ql -= psacw
    cvm = cvm_of(qv, ql, qr, qi, qs, qg)
    icpk = lhi(t) / cvm
    qs += np.where(cold, psacw, 0.0)
    qr += np.where(cold, 0.0, psacw)
    t += np.where(cold, psacw * icpk, 0.0)
    # psaut
    qim = QI0_CRIT / den
    aut = np.where(cold & (qi > qim),
                   (1.0 - np.exp(-dts * np.exp(0.025 * tc) / TAU_I2S)) * (qi - qim), 0.0)
    qi -= aut
    qs += aut
    # psaci
    fac = dts * denfac * CSACW * C_PSACI * np.exp(0.05 * tc + 0.8125 * np.log(np.maximum(qs, QCMIN) * den))
    saci = np.where(cold & (qs > QCMIN) & (qi > QCMIN), fac / (1.0 + fac) * qi, 0.0)
    qi -= saci
    qs += saci
    # pgaut
    gaut = np.where(cold & (qs > QS0_CRIT), dts * 1.0e-3 * np.exp(0.09 * tc) * (qs - QS0_CRIT), 0.0)
    gaut = np.minimum(gaut, np.maximum(qs, 0.0))
    qs -= gaut
    qg += gaut
    # pgacw
    fac = dts * CGACW * np.exp(0.875 * np.log(np.maximum(qg, QCMIN) * den)) * denfac
    gacw = np.where((qg > QCMIN) & (ql > QCMIN), fac / (1.0 + fac) * ql, 0.0)
    ql -= gacw
    cvm = cvm_of(qv, ql, qr, qi, qs, qg)
    icpk = lhi(t) / cvm
    qg += np.where(cold, gacw, 0.0)
    qr += np.where(cold, 0.0, gacw)
    t += np.where(cold, gacw * icpk, 0.0)
    # smlt, gmlt
    for q, tau in ((qs, TAU_SMLT), (qg, TAU_GMLT)):
        cvm = cvm_of(qv, ql, qr, qi, qs, qg)
        icpk = lhi(t) / cvm
        tc = t - T_ICE
        m = np.minimum(q * (1.0 - math.exp(-dts / tau)), np.maximum(tc, 0.0) / icpk)
        m = np.where((tc > 0.0) & (q > QCMIN), m, 0.0)
        q -= m
        qr += m
        t -= m * icpk
    subgrid_z_proc(dts, t, den, qv, ql, qr, qi, qs, qg)


def subgrid_z_proc(dts, t, den, qv, ql, qr, qi, qs, qg):
    """phase changes with vapour (elementwise, in place):
      cloud water  evaporation towards saturation (1 - exp(-dt/TAU_L2V)) and condensation of
                   supersaturation (1 - exp(-dt/TAU_V2L)), linearised saturation adjustment
      cloud ice    deposition / sublimation towards ice saturation below T_ICE (TAU_I2V)
      snow, graupel sublimation in ice-subsaturated air (same time scale, limited by the
                   species)"""
    # cloud water
    cvm = cvm_of(qv, ql, qr, qi, qs, qg)
    lcpk = lhl(t) / cvm
    qsw, dwsdt = wqs2(t, den)
    dq0 = (qv - qsw) / (1.0 + lcpk * dwsdt)
    cond = np.where(dq0 > 0.0, dq0 * (1.0 - math.exp(-dts / TAU_V2L)),
                    np.maximum(dq0 * (1.0 - math.exp(-dts / TAU_L2V)), -ql))
    cond = np.where((dq0 > 0.0) & (t < T_WFR), 0.0, cond)   # no liquid condensation below T_WFR
    qv -= cond
    ql += cond
    t += cond * lcpk
    # ice deposition / sublimation and snow / graupel sublimation
    fdep = 1.0 - math.exp(-dts / TAU_I2V)
    cvm = cvm_of(qv, ql, qr, qi, qs, qg)
    tcpk = (lhl(t) + lhi(t)) / cvm
    qsi, dqsidt = iqs2(t, den)
    dq = (qv - qsi) / (1.0 + tcpk * dqsidt)
    cold = t < T_ICE
    dep = np.where(dq > 0.0, fdep * dq, np.maximum(fdep * dq, -qi))
    dep = np.where(cold, dep, 0.0)
    qv -= dep
    qi += dep
    t += dep * tcpk
    for q in (qs, qg):
        cvm = cvm_of(qv, ql, qr, qi, qs, qg)
        tcpk = (lhl(t) + lhi(t)) / cvm
        qsi, dqsidt = iqs2(t, den)
        dq = (qsi - qv) / (1.0 + tcpk * dqsidt)
        sub = np.where((dq > 0.0) & (q > QCMIN), np.minimum(q, fdep * dq), 0.0)
        q -= sub
        qv += sub
        t -= sub * tcpk


# ------------------------------------------------------------------------------ driver
def mpdrv(t, dp, dz, qv, ql, qr, qi, qs, qg, dt):
    """One microphysics step on columns [k, ncol] (copies returned): ntimes = ceil(dt /
    MP_TIME) sub-steps of neg_adj, terminal_fall, warm_rain, icloud.  dz < 0 (FV3 delz),
    dp the moist layer pressure thickness.  Returns ((t, qv, ql, qr, qi, qs, qg), (rain,
    snow, graupel, ice)) with the surface precipitation in kg m-2 over dt."""
    t, qv, ql, qr, qi, qs, qg = (np.array(x, dtype=np.float64, copy=True) for x in (t, qv, ql, qr, qi, qs, qg))
    dp = np.asarray(dp, dtype=np.float64)
    dz = np.asarray(dz, dtype=np.float64)
    nk = t.shape[0]
    cols = t.shape[1:]
    ntimes = max(1, int(math.ceil(dt / MP_TIME - 1.0e-9)))
    dts = dt / ntimes
    den = -dp / (GRAV * dz)
    ze = np.zeros((nk + 1,) + cols)
    for k in range(nk - 1, -1, -1):
        ze[k] = ze[k + 1] - dz[k]
    prec = [np.zeros(cols) for _ in range(4)]   # rain, snow, graupel, ice
    for _ in range(ntimes):
        neg_adj(t, dp, qv, ql, qr, qi, qs, qg)
        for idx in np.ndindex(*cols):
            sl = (slice(None),) + idx
            c = [a[sl] for a in (t, qv, ql, qr, qi, qs, qg)]
            pi, ps, pg = terminal_fall(dts, c[0], dp[sl], dz[sl], ze[sl], den[sl], *c[1:])
            pr = warm_rain(dts, c[0], dp[sl], dz[sl], ze[sl], den[sl], *c[1:])
            prec[0][idx] += pr
            prec[1][idx] += ps
            prec[2][idx] += pg
            prec[3][idx] += pi
        icloud(dts, t, den, qv, ql, qr, qi, qs, qg)
    return (t, qv, ql, qr, qi, qs, qg), tuple(prec)
