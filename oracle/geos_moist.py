"""GEOS moist pieces around the GFDL microphysics — TEST
INFRASTRUCTURE ONLY (the checker of csrc/moist.hip; never on the product path).

The reference's GEOS GFDL_1M run sequence (geos_documentation/moist/GFDL_1M.drawio) calls,
around gfdl_cloud_microphys_driver, the "evap_subl_pdf loop" (MELTFRZ, EVAP3, SUBL3,
hystpdf with ice_fraction / Bergeron partition), RADCOUPLE with LDRADIUS4, and the
standalone experiments add aer_activation (experiments.yaml:42-110).  None of their
source is in the reference, so each is restated here from the published method it
implements, elementwise over [k, ...] arrays (pointwise in the column):

  ice_fraction       liquid / ice partition of new condensate, linear in T between
                     T_ICE - 40 K (all ice) and T_ICE (all liquid)
  meltfrz            relaxation freezing of cloud water (by the ice fraction, time scale
                     TAU_FRZ) below T_ICE, melting of cloud ice above (TAU_MLT)
  evap3 / subl3      evaporation of convective (anvil) cloud water / sublimation of its ice
                     in air drier than the critical humidity: diffusion-limited growth
                     equation (Pruppacher & Klett 1997 eq. 13-28), rate proportional to
                     (RHcr - RH) / ((K1 + K2) r^2) with the droplet radius of ldradius4
  hystpdf            large-scale condensation from a uniform sub-grid PDF of total water
                     (half width (1 - RHcr) qsat, Sundqvist / Smith 1990 form): cloud fraction
                     and condensate from the PDF, the condensate change applied with the
                     latent heat (three Newton-linearised iterations), new condensate split
                     by ice_fraction, evaporation taken from liquid first
  radcouple          the radiation's view of the clouds (GEOS RADCOUPLE): total cloud
                     fraction, in-cloud water contents capped at 0.01 kg/kg, effective radii
  ldradius4          effective radius: liquid from the volume-mean radius of the droplet
                     number (x 1.1 effective / volume ratio), ice after Wyser (1998)
  aer_activation     droplet activation of a three-mode lognormal aerosol, Abdul-Razzak &
                     Ghan (2000, JGR 105) maximum supersaturation and activated fraction; ice
                     nuclei after Meyers et al. (1992)

**Parity unpinned** (no GEOS numerics in the reference); the HIP kernels are checked
against this module at the reference's moist bar (0.01 %, physics_standalone.py:132-144)
and at 1e-9 of each field's scale.
"""
import math

import numpy as np

from .moist import GRAV, RDGAS, RVGAS, CP_AIR, T_ICE, HLV, HLF, HLS, EPS, qsat

TAU_FRZ, TAU_MLT = 450.0, 450.0
RHO_W, RHO_I = 1000.0, 917.0
K_COND, DIFFU = 2.4e-2, 2.2e-5          # thermal conductivity (W m-1 K-1), vapour diffusivity at 1000 hPa
A_EFF_L, A_EFF_I = 0.8, 0.5             # anvil evaporation / sublimation efficiencies
NN_LAND, NN_OCEAN = 150.0e6, 30.0e6
QC_MAX = 0.01                            # radcouple cap of in-cloud water contents


def ice_fraction(t):
    return np.clip((T_ICE - t) / 40.0, 0.0, 1.0)


def rhcrit(pl):
    """critical relative humidity of the sub-grid PDF: 0.80 below 750 hPa, rising
    quadratically towards 0.99 at the model top"""
    x = np.clip((75000.0 - pl) / 75000.0, 0.0, 1.0)
    return 0.80 + 0.19 * x * x


def meltfrz(dt, t, ql, qi):
    """in place"""
    fqi = ice_fraction(t)
    frz = np.where(t <= T_ICE, ql * fqi * (1.0 - math.exp(-dt / TAU_FRZ)), 0.0)
    mlt = np.where(t > T_ICE, qi * (1.0 - math.exp(-dt / TAU_MLT)), 0.0)
    ql += mlt - frz
    qi += frz - mlt
    t += (frz - mlt) * (HLF / CP_AIR)


def ldradius4(pl, t, qc, nnl, nni, itype):
    """effective radius (m) of liquid (itype 1) or ice (itype 2) with in-cloud water qc
    (kg/kg), pressure pl (Pa), droplet / crystal numbers (m-3)"""
    rho = pl / (RDGAS * t)
    wc = rho * np.maximum(qc, 0.0)                                   # kg m-3
    if itype == 1:
        nnx = np.maximum(nnl, 1.0e7)
        r = 1.1 * np.cbrt(3.0 * wc / (4.0 * math.pi * RHO_W * nnx))
        return np.minimum(60.0e-6, np.maximum(2.5e-6, r))
    wcg = np.maximum(1.0e3 * wc, 1.0e-12)                             # g m-3
    bb = np.where((t > T_ICE) | (qc <= 0.0), -2.0,
                  -2.0 + np.log10(wcg / 50.0) * (1.0e-3 * np.power(np.maximum(T_ICE - t, 0.0), 1.5)))
    bb = np.minimum(np.maximum(bb, -6.0), -2.0)
    r = 377.4 + 203.3 * bb + 37.91 * bb * bb + 2.3696 * bb * bb * bb   # microns
    return np.minimum(150.0e-6, np.maximum(5.0e-6, 1.0e-6 * r))


def evap3(dt, rhcr, pl, t, qv, ql, qi, f, nl, ni):
    """in place; returns the evaporated amount"""
    qs, _ = qsat(t, pl, ice=False)
    es = pl * qs / (EPS + (1.0 - EPS) * qs)
    rhx = np.minimum(qv / qs, 1.0)
    k1 = HLV * HLV * RHO_W / (K_COND * RVGAS * t * t)
    k2 = RVGAS * t * RHO_W / (DIFFU * (1.0e5 / pl) * es)
    qcm = np.where((f > 0.0) & (ql > 0.0), ql / np.where(f > 0.0, f, 1.0), 0.0)
    rad = ldradius4(pl, t, qcm, nl, ni, 1)
    teff = np.where(rhx < rhcr, (rhcr - rhx) / ((k1 + k2) * rad * rad), 0.0)
    ev = np.minimum(A_EFF_L * ql * dt * teff, ql)
    ev = np.where(ql > 0.0, ev, 0.0)
    qv += ev
    ql -= ev
    t -= ev * (HLV / CP_AIR)
    return ev


def subl3(dt, rhcr, pl, t, qv, ql, qi, f, nl, ni):
    """in place; returns the sublimated amount"""
    qs, _ = qsat(t, pl, ice=True)
    es = pl * qs / (EPS + (1.0 - EPS) * qs)
    rhx = np.minimum(qv / qs, 1.0)
    k1 = HLS * HLS * RHO_I / (K_COND * RVGAS * t * t)
    k2 = RVGAS * t * RHO_I / (DIFFU * (1.0e5 / pl) * es)
    qcm = np.where((f > 0.0) & (qi > 0.0), qi / np.where(f > 0.0, f, 1.0), 0.0)
    rad = ldradius4(pl, t, qcm, nl, ni, 2)
    teff = np.where(rhx < rhcr, (rhcr - rhx) / ((k1 + k2) * rad * rad), 0.0)
    sb = np.minimum(A_EFF_I * qi * dt * teff, qi)
    sb = np.where(qi > 0.0, sb, 0.0)
    qv += sb
    qi -= sb
    t -= sb * (HLS / CP_AIR)
    return sb


def hystpdf(rhcr, pl, t, qv, ql, qi, clf):
    """in place (t, qv, ql, qi, clf): uniform-PDF large-scale condensation"""
    for _ in range(3):
        qs, dqs = qsat(t, pl, ice=False)
        sig = (1.0 - rhcr) * qs
        qt = qv + ql + qi
        full = qt - sig >= qs
        none = qt + sig <= qs
        cf = np.where(full, 1.0, np.where(none, 0.0, (qt + sig - qs) / (2.0 * sig)))
        qcn = np.where(full, qt - qs, np.where(none, 0.0, (qt + sig - qs) * (qt + sig - qs) / (4.0 * sig)))
        fqi = ice_fraction(t)
        lat = HLV / CP_AIR + fqi * (HLF / CP_AIR)
        dqc = (qcn - (ql + qi)) / (1.0 + lat * dqs * cf)
        # condensation split by the ice fraction; evaporation from liquid first, then ice
        dl = np.where(dqc > 0.0, dqc * (1.0 - fqi), np.maximum(dqc, -ql))
        di = np.where(dqc > 0.0, dqc * fqi, np.maximum(dqc - dl, -qi))
        ql += dl
        qi += di
        qv -= dl + di
        t += dl * (HLV / CP_AIR) + di * (HLS / CP_AIR)
        clf[...] = cf


def evap_subl_pdf(dt, pl, t, qv, qlls, qils, qlcn, qicn, clls, clcn, nactl, nacti):
    """GEOS evap_subl_pdf loop on layer arrays (copies returned, same names)"""
    t, qv, qlls, qils, qlcn, qicn, clls, clcn = (np.array(x, dtype=np.float64, copy=True)
                                                  for x in (t, qv, qlls, qils, qlcn, qicn, clls, clcn))
    rhcr = rhcrit(pl)
    meltfrz(dt, t, qlcn, qicn)
    meltfrz(dt, t, qlls, qils)
    evap3(dt, rhcr, pl, t, qv, qlcn, qicn, clcn, nactl, nacti)
    subl3(dt, rhcr, pl, t, qv, qlcn, qicn, clcn, nactl, nacti)
    # anvil fraction shrinks with its condensate
    clcn = np.where(qlcn + qicn > 0.0, clcn, 0.0)
    hystpdf(rhcr, pl, t, qv, qlls, qils, clls)
    return dict(t=t, qv=qv, qlls=qlls, qils=qils, qlcn=qlcn, qicn=qicn, clls=clls, clcn=clcn)


def radcouple(t, pl, cf, af, qv, qlls, qils, qlcn, qicn, qr, qs, qg, nl, ni):
    """GEOS RADCOUPLE: returns dict rad_qv, rad_ql, rad_qi, rad_qr, rad_qs, rad_qg, rad_cf,
    rad_rl, rad_ri"""
    rcf = np.clip(cf + af, 0.0, 1.0)
    cloudy = rcf >= 1.0e-5
    div = np.where(cloudy, rcf, 1.0)

    def incloud(x):
        return np.where(cloudy & (x >= 1.0e-8), x / div, 0.0)

    rql = np.minimum(incloud(qlls + qlcn), QC_MAX)
    rqi = np.minimum(incloud(qils + qicn), QC_MAX)
    rqr = np.minimum(incloud(qr), QC_MAX)
    rqs = np.minimum(incloud(qs), QC_MAX)
    rqg = np.minimum(incloud(qg), QC_MAX)
    rcf = np.where(cloudy, rcf, 0.0)
    rl = ldradius4(pl, t, rql, nl, ni, 1)
    ri = ldradius4(pl, t, rqi, nl, ni, 2)
    return dict(rad_qv=np.array(qv, dtype=np.float64), rad_ql=rql, rad_qi=rqi, rad_qr=rqr, rad_qs=rqs,
                rad_qg=rqg, rad_cf=rcf, rad_rl=rl, rad_ri=ri)


# ---- aerosol activation (Abdul-Razzak & Ghan 2000), three lognormal modes ----
# (number at the surface m-3, scale height m, dry geometric mean radius m, geometric sd, kappa)
AER_MODES = ((1.0e9, 2000.0, 0.02e-6, 1.6, 0.6),     # Aitken
             (3.0e8, 2000.0, 0.08e-6, 1.8, 0.6),     # accumulation (sulfate)
             (1.0e6, 1000.0, 1.00e-6, 2.0, 1.2))     # coarse (sea salt)
MW, MA = 0.018015, 0.028965                           # kg mol-1
RGAS_U = 8.314462618
SURF_T = 0.0761                                       # water surface tension (N m-1)
W_MIN = 0.1                                           # minimum updraft (m s-1)


def aer_activation(pl, t, qv, zm, w):
    """droplet (nactl) and ice-nucleus (nacti) number concentrations, m-3"""
    wv = np.maximum(w, 0.0) + W_MIN
    es = pl * qsat(t, pl, ice=False)[0] / (EPS + (1.0 - EPS) * qsat(t, pl, ice=False)[0])
    a_k = 2.0 * SURF_T * MW / (RHO_W * RGAS_U * t)                      # Kelvin coefficient (m)
    alpha = GRAV * MW * HLV / (CP_AIR * RGAS_U * t * t) - GRAV * MA / (RGAS_U * t)
    gamma = RGAS_U * t / (es * MW) + MW * HLV * HLV / (CP_AIR * pl * MA * t)
    dv = DIFFU * (1.0e5 / pl)
    gg = 1.0 / (RHO_W * RGAS_U * t / (es * dv * MW) + HLV * RHO_W / (K_COND * t) * (HLV * MW / (RGAS_U * t) - 1.0))
    aw = alpha * wv / gg
    zeta = 2.0 * a_k / 3.0 * np.sqrt(aw)
    ssum = np.zeros_like(t)
    sms, nns, lss = [], [], []
    for (n0, h, rd, sg, kap) in AER_MODES:
        nn = n0 * np.exp(-np.maximum(zm, 0.0) / h)
        sm = 2.0 / math.sqrt(kap) * (a_k / (3.0 * rd)) ** 1.5
        ls = math.log(sg)
        eta = aw ** 1.5 / (2.0 * math.pi * RHO_W * gamma * nn)
        f = 0.5 * math.exp(2.5 * ls * ls)
        g = 1.0 + 0.25 * ls
        ssum = ssum + (f * (zeta / eta) ** 1.5 + g * (sm * sm / (eta + 3.0 * zeta)) ** 0.75) / (sm * sm)
        sms.append(sm)
        nns.append(nn)
        lss.append(ls)
    smax = 1.0 / np.sqrt(ssum)
    from scipy.special import erfc
    nact = np.zeros_like(t)
    for sm, nn, ls in zip(sms, nns, lss):
        u = 2.0 * np.log(sm / smax) / (3.0 * math.sqrt(2.0) * ls)
        nact = nact + nn * 0.5 * erfc(u)
    # ice nuclei (Meyers et al. 1992) from the supersaturation over ice, below T_ICE - 5 K
    qsi, _ = qsat(t, pl, ice=True)
    si = np.clip(qv / qsi - 1.0, -0.2, 0.25)
    nacti = np.where(t < T_ICE - 5.0, 1.0e3 * np.exp(-0.639 + 12.96 * si), 0.0)
    return nact, nacti, smax


Z_PBL = 1000.0
HFX_SURF = 15.0   # the Aquaplanet coupling's uniform surface sensible heat flux (W m-2)


def moist_prep(pe, dz):
    """layer pressure from the interfaces, layer-mid heights from delz (surface at 0) and the
    PBL-top level index (the highest level whose mid height is below Z_PBL)"""
    nk = dz.shape[0]
    pl = 0.5 * (pe[:-1] + pe[1:])
    zm = np.empty_like(dz)
    zb = np.zeros(dz.shape[1:])
    kp = np.full(dz.shape[1:], float(nk - 1))
    for k in range(nk - 1, -1, -1):
        zt = zb - dz[k]
        zm[k] = 0.5 * (zt + zb)
        kp = np.where(zm[k] < Z_PBL, float(k), kp)
        zb = zt
    return pl, zm, kp


def aquaplanet_physics(dt, t, qv, ql, qr, qi, qs, qg, dp, dz, pe, w, qlcn=None, qicn=None, clls=None, clcn=None,
                       hfx=HFX_SURF):
    """GEOS moist run order on column arrays [k, ...]: aer_activation, cup_gf_sh (the shallow
    cumulus, oracle/gf_shallow.py), evap_subl_pdf, the GFDL microphysics driver
    (oracle/gfdl_mp.py mpdrv), radcouple.  Returns a dict of
    the updated state (t, qv, ql, qr, qi, qs, qg, qlcn, qicn, clls, clcn), the surface
    precipitation (prec_rain, prec_snow, prec_graupel, prec_ice), nactl, nacti and the
    radiation fields rad_*."""
    from . import gf_shallow, gfdl_mp
    z = np.zeros_like(t)
    qlcn = z if qlcn is None else qlcn
    qicn = z if qicn is None else qicn
    clls = z if clls is None else clls
    clcn = z if clcn is None else clcn
    pl, zm, kpbl = moist_prep(pe, dz)
    nactl, nacti, _ = aer_activation(pl, t, qv, zm, w)
    g = gf_shallow.cup_gf_sh(dt, t, qv, pl, zm, dp, kpbl, np.full(t.shape[1:], hfx))
    t, qv = g["t"], g["qv"]
    qlcn = qlcn + g["dqlcn"]
    qicn = qicn + g["dqicn"]
    clcn = np.maximum(clcn, g["cf"])
    e = evap_subl_pdf(dt, pl, t, qv, ql, qi, qlcn, qicn, clls, clcn, nactl, nacti)
    (t1, qv1, ql1, qr1, qi1, qs1, qg1), prec = gfdl_mp.mpdrv(e["t"], dp, dz, e["qv"], e["qlls"], qr, e["qils"],
                                                             qs, qg, dt)
    r = radcouple(t1, pl, e["clls"], e["clcn"], qv1, ql1, qi1, e["qlcn"], e["qicn"], qr1, qs1, qg1, nactl, nacti)
    out = dict(t=t1, qv=qv1, ql=ql1, qr=qr1, qi=qi1, qs=qs1, qg=qg1, qlcn=e["qlcn"], qicn=e["qicn"],
               clls=e["clls"], clcn=e["clcn"], prec_rain=prec[0], prec_snow=prec[1], prec_graupel=prec[2],
               prec_ice=prec[3], nactl=nactl, nacti=nacti, gf_mb=g["mb"], gf_k22=g["k22"], gf_kbcon=g["kbcon"],
               gf_ktop=g["ktop"])
    out.update(r)
    return out
