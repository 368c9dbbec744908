"""Shallow cumulus mass-flux scheme (GEOS cup_gf_sh, the shallow plume of Grell & Freitas
2014) -- TEST INFRASTRUCTURE ONLY (the checker of csrc/moist.hip cup_gf_sh_k; never on the
product path).  SURVEY.md §8a row A13 names cup_gf_sh among the GEOS moist standalones
(experiments.yaml:42-110); its source is external to the reference, so this restates the
published method (Grell 1993 for the cloud model, Grell & Freitas 2014, ACP 14, for the
scale-aware shallow plume; Grant 2001 for the convective-velocity closure), column by column
on [k, ...] arrays (k = 0 top), and is **parity unpinned**:

  source level   k22: the level of largest moist static energy h = cp T + g z + Lv qv between
                 the lowest level and the PBL top kpbl; the parcel starts with h(k22) + cp DT_PERT
  cloud base     kbcon: the first level above k22 where the parcel's h reaches the saturation
                 moist static energy h* = cp T + g z + Lv qsat(T, p) of the environment, no more
                 than DP_BASE above the source; none -> no convection
  updraft        entraining plume from the cloud base up: h_c and total water q_c mix with the
                 environment at the rate EPS_ENT (per metre, trapezoidal in the layer), the
                 normalised mass flux grows with (EPS_ENT - DEL_DET) per metre; in-cloud vapour
                 q* + gamma / (1 + gamma) (h_c - h*) / Lv (the linearised moist adiabat), condensate
                 the excess of q_c over it
  cloud top      ktop: the last level going up where h_c >= h*, within DP_DEPTH of the cloud base;
                 at least one level above the base, else no convection
  closure        cloud-base mass flux mb = C_MB rho(k22) w*, with the convective velocity
                 w* = (g / T h_flux / (rho cp) z_pbl)^(1/3) (Grant 2001); no convection for
                 h_flux <= 0; mb is then limited so no layer's vapour turns negative
  tendencies     flux form: the updraft eddy flux E = M (phi_c - phi) of h and of the total water
                 through the upper interface of every layer from k22 to just below ktop (zero
                 at ktop: the plume detrains there), d(phi)/dt = g (E_below - E_above) / dp;
                 the condensate carried into the top layer is detrained as convective cloud
                 (liquid / ice by the ice fraction), the rest of the water change is vapour,
                 dT = (dh - Lv dqv) / cp: column h and water are conserved exactly
  cloud fraction the convective cloud of every cloud layer: M / (rho W_UP), at most CF_MAX

The HIP kernel follows these expressions; the index fields (k22, kbcon, ktop) are bit-exact.
"""
import numpy as np

from .moist import GRAV, RDGAS, CP_AIR, HLV, T_ICE, qsat
from .geos_moist import ice_fraction

DT_PERT = 0.5            # parcel temperature excess at the source (K)
DP_BASE = 1.5e4          # the cloud base within 150 hPa of the source level
DP_DEPTH = 3.0e4         # shallow: cloud top within 300 hPa of the base
EPS_ENT = 1.0e-3         # lateral entrainment (1/m)
DEL_DET = 0.75e-3        # lateral detrainment (1/m)
C_MB = 0.03              # cloud-base mass flux per rho w*
W_UP = 1.0               # updraft velocity for the cloud fraction (m/s)
CF_MAX = 0.3


def cup_gf_sh(dt, t, qv, pl, zm, dp, kpbl, hfx):
    """Columns [k, ...] (k = 0 top): t (K), qv, pl (Pa), zm (m), dp (Pa); kpbl (level index of
    the PBL top, counted from the top), hfx (surface sensible heat flux, W m-2) per column.
    Returns dict t, qv, dqlcn, dqicn (detrained convective condensate), cf (convective cloud
    fraction), mb (kg m-2 s-1), k22, kbcon, ktop (level indices, -1 without convection)."""
    t = np.array(t, dtype=np.float64, copy=True)
    qv = np.array(qv, dtype=np.float64, copy=True)
    nk = t.shape[0]
    cols = t.shape[1:]
    out_l = np.zeros_like(t)
    out_i = np.zeros_like(t)
    cf = np.zeros_like(t)
    mb_o = np.zeros(cols)
    k22_o = np.full(cols, -1.0)
    kb_o = np.full(cols, -1.0)
    kt_o = np.full(cols, -1.0)
    qs, dqs = qsat(t, pl, ice=False)
    h = CP_AIR * t + GRAV * zm + HLV * qv
    hs = CP_AIR * t + GRAV * zm + HLV * qs
    gam = HLV / CP_AIR * dqs
    rho = pl / (RDGAS * t)
    for idx in np.ndindex(*cols):
        c = (slice(None),) + idx
        tc, qc_, hc_, hsc, gc, rc = t[c], qv[c], h[c], hs[c], gam[c], rho[c]
        plc, zc, dpc = pl[c], zm[c], dp[c]
        kp = int(kpbl[idx])
        # source level: largest h from the bottom up to the PBL top
        k22 = nk - 1
        for k in range(nk - 2, kp - 1, -1):
            if hc_[k] > hc_[k22]:
                k22 = k
        hp = hc_[k22] + CP_AIR * DT_PERT
        qp = qc_[k22]
        # cloud base
        kb = -1
        for k in range(k22, -1, -1):
            if plc[k] < plc[k22] - DP_BASE:
                break
            if hp >= hsc[k]:
                kb = k
                break
        if kb < 1 or hfx[idx] <= 0.0:
            continue
        # entraining updraft from the cloud base up
        hcl = np.zeros(nk)
        qtl = np.zeros(nk)
        zu = np.zeros(nk)
        qcl = np.zeros(nk)
        hcl[kb], qtl[kb], zu[kb] = hp, qp, 1.0
        kt = kb
        for k in range(kb - 1, -1, -1):
            if plc[k] < plc[kb] - DP_DEPTH:
                break
            dz = zc[k] - zc[k + 1]
            a = 0.5 * EPS_ENT * dz
            hn = (hcl[k + 1] * (1.0 - a) + 2.0 * a * hc_[k]) / (1.0 + a)
            if hn < hsc[k]:
                break
            hcl[k] = hn
            qtl[k] = (qtl[k + 1] * (1.0 - a) + 2.0 * a * qc_[k]) / (1.0 + a)
            zu[k] = zu[k + 1] * (1.0 + (EPS_ENT - DEL_DET) * dz)
            kt = k
        if kt == kb:
            continue
        # sub-cloud layers carry the source air with the base mass flux
        for k in range(k22, kb, -1):
            hcl[k], qtl[k], zu[k] = hp, qp, 1.0
        # in-cloud vapour and condensate (cloud layers)
        for k in range(kt, kb + 1):
            qsat_c = (qs[c][k] + gc[k] / (1.0 + gc[k]) * (hcl[k] - hsc[k]) / HLV)
            qcl[k] = max(qtl[k] - qsat_c, 0.0)
        # eddy fluxes per unit mb through the upper interface of layers kt+1 .. k22
        eh = np.zeros(nk + 1)
        eq = np.zeros(nk + 1)
        for k in range(kt + 1, k22 + 1):
            eh[k] = zu[k] * (hcl[k] - hc_[k])
            eq[k] = zu[k] * (qtl[k] - qc_[k])
        dh = np.zeros(nk)
        dq = np.zeros(nk)
        for k in range(kt, k22 + 1):
            dh[k] = GRAV * (eh[k + 1] - eh[k]) / dpc[k]
            dq[k] = GRAV * (eq[k + 1] - eq[k]) / dpc[k]
        # condensate detrained in the top layer (carried through its lower interface)
        dc = GRAV * zu[kt + 1] * qcl[kt + 1] / dpc[kt]
        dqv = dq.copy()
        dqv[kt] = dq[kt] - dc
        # closure (convective velocity) and the vapour limiter
        zi = zc[kp]
        wst = np.cbrt(GRAV / tc[nk - 1] * hfx[idx] / (rc[nk - 1] * CP_AIR) * zi)
        mb = C_MB * rc[k22] * wst
        for k in range(kt, k22 + 1):
            if dqv[k] < 0.0:
                mb = min(mb, 0.9 * qc_[k] / (-dt * dqv[k]))
        if not mb > 0.0:
            continue
        for k in range(kt, k22 + 1):
            dqk = mb * dqv[k]
            qv[c][k] = qc_[k] + dt * dqk
            t[c][k] = tc[k] + dt * (mb * dh[k] - HLV * dqk) / CP_AIR
        fi = ice_fraction(t[c][kt])
        out_i[c][kt] = dt * mb * dc * fi
        out_l[c][kt] = dt * mb * dc * (1.0 - fi)
        for k in range(kt, kb + 1):
            cf[c][k] = min(CF_MAX, mb * zu[k] / (rc[k] * W_UP))
        mb_o[idx] = mb
        k22_o[idx], kb_o[idx], kt_o[idx] = float(k22), float(kb), float(kt)
    return dict(t=t, qv=qv, dqlcn=out_l, dqicn=out_i, cf=cf, mb=mb_o, k22=k22_o, kbcon=kb_o, ktop=kt_o)
