// moist.hip — moist column physics for gfx950.
//
// The GEOS moist schemes the Aquaplanet configuration runs (GFDL_1M run sequence:
// aer_activation, the evap_subl_pdf loop, gfdl_cloud_microphys_driver, RADCOUPLE;
// buoyancy, fillq2zero: geos_documentation/moist/GFDL_1M.drawio:70-618,
// experiments.yaml:42-110) live outside the reference.  The oracles restate the published
// algorithms independently of this file (oracle/gfdl_mp.py: Lin et al. 1983, Chen & Lin
// 2013, Zhou et al. 2019; oracle/geos_moist.py: Abdul-Razzak & Ghan 2000, Wyser 1998, ...)
// and these kernels follow them expression by expression; parity unpinned by reference data.
//
// Decomposition: the K axis is never split.  Column schemes (the GFDL driver,
// fillq2zero, buoyancy) run one lane per column, i-fastest, so every level access of a
// wavefront is one coalesced 64-wide row; the GEOS pieces are pointwise, one lane per
// (column, level).  Saturation vapour pressure comes from 0.1 K tables built on the host
// with the C library's exp/log (bit-identical to the oracle's tables) and read with linear
// interpolation (GFDL wqs1 / iqs1 style).
#include <algorithm>
#include <cmath>
#include <map>
#include <mutex>
#include <vector>

#include "blockscan.hpp"
#include "kernels_moist.hpp"
#include "stencil_common.hpp"

namespace gtfv3 {
namespace moist {

constexpr double GRAV = Constants::grav;
constexpr double RDGAS = Constants::rdgas;
constexpr double RVGAS = Constants::rvgas;
constexpr double CP_AIR = Constants::cp_air;
constexpr double EPS = RDGAS / RVGAS;
constexpr double CP_VAP = 4.0 * RVGAS;
constexpr double C_LIQ = 4185.5;
constexpr double C_ICE = 1972.0;
constexpr double HLV = 2.5e6;
constexpr double HLF = 3.3358e5;
constexpr double HLS = HLV + HLF;
constexpr double T_ICE = 273.16;
constexpr double E00 = 611.21;
constexpr double DC_VAP = CP_VAP - C_LIQ;
constexpr double D2ICE = CP_VAP - C_ICE;
constexpr double LV0 = HLV - DC_VAP * T_ICE;
constexpr double LI2 = HLS - D2ICE * T_ICE;
constexpr double KAPPA = RDGAS / CP_AIR;

constexpr double TABLE_T0 = T_ICE - 160.0;
constexpr int TABLE_N = 2621;
constexpr double TABLE_DT = 0.1;

// GFDL / Lin (1983) fall-speed constants (Marshall-Palmer exponential distributions)
constexpr double VCONR = 2503.23638966667, NORMR = 25132741228.7183;
constexpr double VCONS = 6.6280504, NORMS = 942477796.076938;
constexpr double VCONG = 87.2382675, NORMG = 5026548245.74367;
constexpr double VR_MIN = 1.0e-3, VR_MAX = 12.0, VS_MAX = 2.0, VG_MAX = 12.0, VI_MAX = 1.0;

struct Tables {
  const double *tw, *ti, *dw, *di;
};

// table read (oracle es_lookup): T clamped to the table, linear interpolation
__device__ __forceinline__ void es_lookup(const double* tab, const double* des, double t, double& es, double& desdt) {
  const double tt = fmin(fmax(t, TABLE_T0), TABLE_T0 + TABLE_DT * (TABLE_N - 2));
  const double ap1 = (tt - TABLE_T0) * 10.0;
  const int it = (int)ap1;
  es = tab[it] + (ap1 - it) * des[it];
  desdt = des[it] * 10.0;
}

__device__ __forceinline__ void qsat(const Tables& T, bool ice, double t, double p, double& qs, double& dqs) {
  double es, desdt;
  es_lookup(ice ? T.ti : T.tw, ice ? T.di : T.dw, t, es, desdt);
  const double den = p - (1.0 - EPS) * es;
  qs = EPS * es / den;
  dqs = EPS * desdt * p / (den * den);
}

struct Col3 {
  const Dims& d;
  int s, nk;
  long o;
  __device__ __forceinline__ long at(int k) const { return ((long)s * nk + k) * d.plane + o; }
};

__device__ __forceinline__ bool col_point(const Dims& d, int& s, long& o) {
  const int i = blockIdx.x * BX + threadIdx.x, j = blockIdx.y * BY + threadIdx.y;
  s = blockIdx.z;
  o = pidx(d, i, j);
  return i < d.nx && j < d.ny;
}

// ---- saturation specific humidity (pointwise) ----
__global__ void __launch_bounds__(256) qsat_k(Dims d, int nk, Tables tb, const double* __restrict__ t,
                                              const double* __restrict__ p, double* __restrict__ qsw,
                                              double* __restrict__ qsi, double* __restrict__ dqsw) {
  const int i = blockIdx.x * BX + threadIdx.x, j = blockIdx.y * BY + threadIdx.y;
  if (i >= d.nx || j >= d.ny) return;
  const long x = (long)blockIdx.z * d.plane + pidx(d, i, j);
  double qs, dq, qi, dqi;
  qsat(tb, false, t[x], p[x], qs, dq);
  qsat(tb, true, t[x], p[x], qi, dqi);
  qsw[x] = qs;
  dqsw[x] = dq;
  qsi[x] = qi;
}

// ---- fillq2zero (column) ----
__global__ void __launch_bounds__(256) fillq2zero_k(Dims d, int nk, double* __restrict__ q,
                                                    const double* __restrict__ dp, double* __restrict__ fill) {
  int s;
  long o;
  if (!col_point(d, s, o)) return;
  const Col3 c{d, s, nk, o};
  double tpw = 0.0, neg = 0.0, tpw2 = 0.0;
  for (int k = 0; k < nk; ++k) {
    const double qk = q[c.at(k)], dk = dp[c.at(k)];
    tpw = tpw + qk * dk;
    neg = neg + fmin(qk, 0.0) * dk;
    tpw2 = tpw2 + fmax(qk, 0.0) * dk;
  }
  const double fac = tpw2 > 0.0 ? fmax(tpw, 0.0) / tpw2 : 0.0;
  for (int k = 0; k < nk; ++k) q[c.at(k)] = fmax(q[c.at(k)], 0.0) * fac;
  fill[(long)s * d.plane + o] = -neg;
}

// ---- GFDL cloud microphysics, one column per lane (oracle/gfdl_mp.py mpdrv) ----
//
// The column driver of GEOS's gfdl_cloud_microphys_driver (GFDL_1M.drawio :122-618):
// ntimes sub-steps of neg_adj, terminal_fall (melting of falling ice species, Lagrangian
// PPM sedimentation of ice / snow / graupel with sedi_heat), warm_rain (revap_racc half
// steps around the rain sedimentation, autoconversion) and icloud (+ subgrid_z_proc).
// Every expression and its operand order follow oracle/gfdl_mp.py.  The sedimentation
// remap walks the column with data-dependent indices, so its working columns (interface
// heights, fallen heights, the PPM profile, masses, fluxes) live in HBM scratch planes
// at the lane's column (coalesced across the wave's consecutive columns), not in
// registers; everything pointwise streams the fields in place.
constexpr double CV_AIR = CP_AIR - RDGAS;
constexpr double CV_VAP = 3.0 * RVGAS;
constexpr double D0_VAP = CV_VAP - C_LIQ;
constexpr double DC_ICE = C_LIQ - C_ICE;
constexpr double LV00 = HLV - D0_VAP * T_ICE;
constexpr double LI00 = HLF - DC_ICE * T_ICE;
constexpr double SFCRHO = 1.2;
constexpr double QI0_CRIT = 1.0e-4, QS0_CRIT = 1.0e-3;
constexpr double C_PSACI = 0.02, C_PAUT = 0.55, QL0_AUT = 5.0e-4;
constexpr double T_WFR = T_ICE - 40.0;
constexpr double QRMIN = 1.0e-8, QCMIN = 1.0e-12, QVMIN = 1.0e-20;
constexpr double DZ_MIN_FALL = 1.0e-2;
constexpr double TAU_I2S = 1000.0;
constexpr double MP_R3 = 1.0 / 3.0, MP_R23 = 2.0 / 3.0;
constexpr int MP_NSCR = 9;  // scratch columns of nk+1 levels per sub-domain

// host-computed coefficients (oracle/gfdl_mp.py module constants; exp(-dts / tau) factors)
struct MpConst {
  double cracw, csacw, cgacw, crevp[5];
  double e_imlt, e_smlt, e_gmlt, e_l2v, e_v2l, e_i2v;
};

struct MpArgs {
  Dims d;
  int nk, qsub, ntimes;
  double dts;
  Tables tb;
  MpConst k;
  double *T, *qv, *ql, *qr, *qi, *qs, *qg;
  const double *dp, *dz;
  double* scr;  // MP_NSCR * (nk+1) planes per sub-domain
  double *pr, *ps, *pg, *pi;
};

// strided column
struct MCol {
  double* p;
  long st;
  __device__ __forceinline__ double& operator[](int k) const { return p[(long)k * st]; }
};

__device__ __forceinline__ double lhl_(double t) { return LV00 + D0_VAP * t; }
__device__ __forceinline__ double lhi_(double t) { return LI00 + DC_ICE * t; }
__device__ __forceinline__ double cvm_(double qv, double ql, double qr, double qi, double qs, double qg) {
  return CV_AIR + qv * CV_VAP + (qr + ql) * C_LIQ + (qi + qs + qg) * C_ICE;
}
// exp / log of the processes: ocml (the column driver) or fastmath.hpp's (~1 ulp; the
// level-block form)
template <bool FM>
__device__ __forceinline__ double mexp(double x) { return FM ? fm_exp(x) : exp(x); }
template <bool FM>
__device__ __forceinline__ double mlog(double x) { return FM ? fm_log(x) : log(x); }

// density-form saturation mixing ratio and its T derivative (oracle wqs2 / iqs2)
__device__ __forceinline__ void qs2(const Tables& tb, bool ice, double t, double den, double& q, double& dq) {
  double es, des;
  es_lookup(ice ? tb.ti : tb.tw, ice ? tb.di : tb.dw, t, es, des);
  q = es / (RVGAS * t * den);
  dq = (des - es / t) / (RVGAS * t * den);
}

// Every column pass below is a function whose arrays are __restrict__ parameters (the
// lane's column at stride P): a level's loads may then be issued before the previous
// level's stores complete, instead of each level waiting out a store -> load round trip
// through memory (the passes are otherwise chains of dependent HBM / L2 latencies).
// Recurrences carry their previous level in registers; values and operation order are
// those of oracle/gfdl_mp.py.
#define RP double* __restrict__
#define CRP const double* __restrict__

__device__ __forceinline__ void mp_neg_adj(int n, long P, RP t, RP qv, RP ql, RP qr, RP qi, RP qs, RP qg, CRP dp) {
  for (int k = 0; k < n; ++k) {
    const long x = (long)k * P;
    double tt = t[x], v = qv[x], l = ql[x], r = qr[x], ii = qi[x], sn = qs[x], g = qg[x];
    const double cvm = cvm_(v, l, r, ii, sn, g);
    const double lcpk = lhl_(tt) / cvm, icpk = lhi_(tt) / cvm;
    if (ii < 0.0) { sn = sn + ii; ii = 0.0; }
    if (sn < 0.0) { g = g + sn; sn = 0.0; }
    {
      const double dq = g < 0.0 ? g : 0.0;
      v = v + dq;
      tt = tt - dq * (lcpk + icpk);
      if (g < 0.0) g = 0.0;
    }
    if (r < 0.0) { l = l + r; r = 0.0; }
    {
      const double dq = l < 0.0 ? l : 0.0;
      v = v + dq;
      tt = tt - dq * lcpk;
      if (l < 0.0) l = 0.0;
    }
    t[x] = tt; qv[x] = v; ql[x] = l; qr[x] = r; qi[x] = ii; qs[x] = sn; qg[x] = g;
  }
  // negative vapour borrows from below (the level below carried in a register)
  double cur = qv[0];
  for (int k = 0; k < n - 1; ++k) {
    double nxt = qv[(long)(k + 1) * P];
    if (cur < 0.0) {
      nxt = nxt + cur * dp[(long)k * P] / dp[(long)(k + 1) * P];
      qv[(long)k * P] = 0.0;
      cur = 0.0;
    }
    if (k + 1 < n - 1) qv[(long)(k + 1) * P] = nxt;
    else {
      // bottom: qb = nxt (level n-1), qa = cur (level n-2)
      const double qb = nxt, qa = cur;
      double dq = fmin(-qb * dp[(long)k * P + P], qa * dp[(long)k * P]);
      if (!(qb < 0.0 && qa > 0.0)) dq = 0.0;
      qv[(long)k * P] = qa - dq / dp[(long)k * P];
      qv[(long)(k + 1) * P] = qb + dq / dp[(long)(k + 1) * P];
    }
    cur = nxt;
  }
}

// melting of the falling ice species in layers above freezing (oracle terminal_fall)
__device__ __forceinline__ void mp_melt(int n, long P, const MpConst& kc, RP t, CRP qv, RP ql, RP qr, RP qi, RP qs,
                                        RP qg) {
  for (int k = 0; k < n; ++k) {
    const long x = (long)k * P;
    double tt = t[x];
    if (!(tt > T_ICE)) continue;
    double v = qv[x], l = ql[x], r = qr[x], ii = qi[x], sn = qs[x], g = qg[x];
#pragma unroll
    for (int w = 0; w < 3; ++w) {
      double& q = w == 0 ? ii : (w == 1 ? sn : g);
      const double fq = w == 0 ? kc.e_imlt : (w == 1 ? kc.e_smlt : kc.e_gmlt);
      const double icpk = lhi_(tt) / cvm_(v, l, r, ii, sn, g);
      const double mlt = fmin(fq * q, (tt - T_ICE) / icpk);
      if (mlt > 0.0) {
        q = q - mlt;
        if (w == 0) l = l + mlt;
        else r = r + mlt;
        tt = tt - mlt * icpk;
      }
    }
    t[x] = tt; ql[x] = l; qr[x] = r; qi[x] = ii; qs[x] = sn; qg[x] = g;
  }
}

// fall speeds of species w (0 ice, 1 snow, 2 graupel, 3 rain) into vt; returns whether
// any level holds more than the species' threshold
__device__ __forceinline__ bool mp_speeds(int n, long P, int w, CRP q, CRP den, RP vt) {
  bool any = false;
  for (int k = 0; k < n; ++k) {
    const long x = (long)k * P;
    const double dn = den[x], qq = q[x];
    const double rhof = sqrt(fmin(10.0, SFCRHO / dn));
    double v;
    if (w == 3) {
      const double q_ = fmax(qq, QRMIN);
      v = qq > QRMIN ? fmin(VR_MAX, fmax(VR_MIN, VCONR * rhof * exp(0.2 * log(q_ * dn / NORMR)))) : 0.0;
      any = any || qq > QRMIN;
    } else {
      const double q_ = fmax(qq, QCMIN);
      if (w == 0) v = qq > QCMIN ? fmin(VI_MAX, 3.29 * exp(0.16 * log(q_ * dn))) : 0.0;
      else if (w == 1) v = qq > QCMIN ? fmin(VS_MAX, VCONS * rhof * exp(0.0625 * log(q_ * dn / NORMS))) : 0.0;
      else v = qq > QCMIN ? fmin(VG_MAX, VCONG * rhof * sqrt(sqrt(sqrt(q_ * dn / NORMG)))) : 0.0;
      any = any || qq > QCMIN;
    }
    vt[x] = v;
  }
  return any;
}

// fallen interface heights (oracle fallen_edges; the monotone fix carried in one pass: each
// raw height depends only on ze and vt, the fix of k+1 on the fixed k)
__device__ __forceinline__ void mp_fallen_edges(int n, long P, double dts, CRP ze, CRP vt, RP zt) {
  double zp = ze[0];
  zt[0] = zp;
  double vprev = vt[0];
  for (int k = 1; k <= n; ++k) {
    const long x = (long)k * P;
    double z;
    if (k < n) {
      const double v = vt[x];
      z = ze[x] - 0.5 * dts * (vprev + v);
      vprev = v;
    } else {
      z = ze[x] - dts * vprev;
    }
    if (z >= zp) z = zp - DZ_MIN_FALL;
    zt[x] = z;
    zp = z;
  }
}

// Lagrangian sedimentation of q (oracle lagrangian_fall_ppm + cs_profile_mono); the flux
// out of the bottom of each layer into m1; returns m1[n-1]
__device__ __forceinline__ double mp_lagrangian_fall(int n, long P, CRP ze, CRP zt, CRP dp, RP q, RP qm0, RP a,
                                                     RP qe, RP gam, RP qm, RP m1) {
  for (int k = 0; k < n; ++k) {
    const long x = (long)k * P;
    const double m0 = q[x] * dp[x];
    qm0[x] = m0;
    a[x] = m0 / (zt[x] - zt[x + P]);
  }
  // cs_profile: forward elimination (carries: q, gam, a and dz of the level above)
  {
    const double z0 = zt[0], z1 = zt[P], z2 = zt[2 * P];
    const double dz0 = z0 - z1, dz1 = z1 - z2;
    const double a0 = a[0], a1 = a[P];
    const double grat = dz1 / dz0;
    const double bet = grat * (grat + 0.5);
    double qp = ((grat + grat) * (grat + 1.0) * a0 + a1) / bet;
    double gp = (1.0 + grat * (grat + 1.5)) / bet;
    qe[0] = qp;
    gam[0] = gp;
    double dzp = dz0, ap = a0, zb = z1;
    double zn_n = z2, ak_n = a1;  // the level's loads, issued one level ahead
    for (int k = 1; k < n; ++k) {
      const long x = (long)k * P;
      const double zn = zn_n, ak = ak_n;
      if (k + 1 < n) {
        zn_n = zt[x + 2 * P];
        ak_n = a[x + P];
      }
      const double dzk = zb - zn;
      const double d4 = dzp / dzk;
      const double bt = 2.0 + d4 + d4 - gp;
      qp = (3.0 * (ap + d4 * ak) - qp) / bt;
      gp = d4 / bt;
      qe[x] = qp;
      gam[x] = gp;
      dzp = dzk;
      ap = ak;
      zb = zn;
    }
    // bottom edge: dz(n-2) / dz(n-1) (dzp is dz(n-1); dz(n-2) recomputed from zt)
    const long xn = (long)n * P;
    const double d4 = (zt[xn - 2 * P] - zt[xn - P]) / dzp;
    const double a_bot = 1.0 + d4 * (d4 + 1.5);
    qe[xn] = (2.0 * d4 * (d4 + 1.0) * ap + a[xn - 2 * P] - a_bot * qp) / (d4 * (d4 + 0.5) - a_bot * gp);
  }
  // back substitution (on the unbounded values), each edge bounded by its neighbouring
  // means as it is finalised; both end edges non-negative
  {
    const long xn = (long)n * P;
    double x = qe[xn];
    qe[xn] = fmax(x, 0.0);
    double anext = a[xn - P];
    double qe_n = qe[xn - P], g_n = gam[xn - P], ap_n = n >= 2 ? a[xn - 2 * P] : 0.0;  // one level ahead
    for (int k = n - 1; k >= 0; --k) {
      const long y = (long)k * P;
      const double qek = qe_n, gk = g_n, apk = ap_n;
      if (k >= 1) {
        qe_n = qe[y - P];
        g_n = gam[y - P];
        ap_n = k >= 2 ? a[y - 2 * P] : 0.0;
      }
      x = qek - gk * x;
      if (k >= 1) {
        const double ap = apk;
        qe[y] = fmin(fmax(x, fmin(ap, anext)), fmax(ap, anext));
        anext = ap;
      } else {
        qe[y] = fmax(x, 0.0);
      }
    }
  }
  // (the monotone limiter of cs_limiters is applied to each fallen layer's profile where the
  // integration forms it: no stored aL / aR / a6 planes)
  // integrate the fallen profile over the fixed layers: one streaming sweep over the fallen
  // layers m with the target (fixed) layer k dynamic -- the pieces of every target in the
  // same order and with the same expressions as the two-pointer search, whose every step
  // was a dependent memory round trip; the fallen layer's heights, edges, mean and mass are
  // loaded one layer ahead of their use
  {
    auto prof_v = [&](double l0, double r0, double av, double& l, double& r, double& a6v) {
      l = l0;
      r = r0;
      const double da1 = r - l;
      if ((av - l) * (av - r) >= 0.0) {
        l = av; r = av; a6v = 0.0;
      } else {
        a6v = 3.0 * (2.0 * av - (l + r));
        if (a6v * da1 < -da1 * da1) {
          a6v = 3.0 * (l - av);
          r = l - a6v;
        } else if (a6v * da1 > da1 * da1) {
          a6v = 3.0 * (r - av);
          l = r - a6v;
        }
      }
    };
    int k = 0;
    bool open = false;
    double sm = 0.0;
    double top = ze[0], bot = ze[P];
    double ztm = zt[0], ztm1 = zt[P], qeL = qe[0], qeR = qe[P], am = a[0], q0m = qm0[0];
    for (int m = 0; m < n; ++m) {
      const long yn = (long)(m + 1) * P;
      const bool more = m + 1 < n;
      const double zt2 = more ? zt[yn + P] : 0.0, qe2 = more ? qe[yn + P] : 0.0;
      const double an = more ? a[yn] : 0.0, q0n = more ? qm0[yn] : 0.0;
      double l, r, a6v;
      prof_v(qeL, qeR, am, l, r, a6v);
      while (k < n) {
        if (open) {
          if (bot < ztm1) {  // the whole fallen layer
            sm = sm + q0m;
            break;
          }
          const double dzz = ztm - bot;  // the last (partial) piece
          const double esl = dzz / (ztm - ztm1);
          sm = sm + dzz * (l + 0.5 * esl * (r - l + a6v * (1.0 - MP_R23 * esl)));
          qm[(long)k * P] = sm;
          open = false;
          ++k;
          top = bot;
          bot = k < n ? ze[(long)(k + 1) * P] : 0.0;
          continue;
        }
        if (!(top <= ztm && top >= ztm1)) break;
        const double dzm = ztm - ztm1;
        const double pl = (ztm - top) / dzm;
        if (ztm1 <= bot) {  // the target inside this fallen layer
          const double pr = (ztm - bot) / dzm;
          qm[(long)k * P] = (l + 0.5 * (a6v + r - l) * (pr + pl) - a6v * MP_R3 * (pr * (pr + pl) + pl * pl)) * (top - bot);
          ++k;
          top = bot;
          bot = k < n ? ze[(long)(k + 1) * P] : 0.0;
          continue;
        }
        sm = (top - ztm1) * (l + 0.5 * (a6v + r - l) * (1.0 + pl) - a6v * (MP_R3 * (1.0 + pl * (1.0 + pl))));
        open = true;
        break;
      }
      ztm = ztm1; ztm1 = zt2; qeL = qeR; qeR = qe2; am = an; q0m = q0n;
    }
    if (open) {  // the target ran past the last fallen layer: its whole-layer sum
      qm[(long)k * P] = sm;
      ++k;
    }
    for (; k < n; ++k) qm[(long)k * P] = 0.0;  // (no piece: as the search leaves them)
  }
  double acc = 0.0;
  for (int k = 0; k < n; ++k) {
    const long x = (long)k * P;
    const double qmk = qm[x];
    acc = acc + qm0[x] - qmk;
    m1[x] = acc;
    q[x] = qmk / dp[x];
  }
  return acc;
}

__device__ __forceinline__ void mp_sedi_heat(int n, long P, double cw, RP t, CRP dp, CRP dz, CRP m1, CRP qv, CRP ql,
                                             CRP qr, CRP qi, CRP qs, CRP qg) {
  double tp = t[0], mp = m1[0];
  for (int k = 1; k < n; ++k) {
    const long x = (long)k * P;
    const double mk = m1[x];
    const double dgz = -0.5 * GRAV * dz[x];
    const double cv0 = dp[x] * cvm_(qv[x], ql[x], qr[x], qi[x], qs[x], qg[x]) + cw * (mk - mp);
    const double tn = (cv0 * t[x] + mp * (cw * tp + dgz)) / (cv0 + cw * mp);
    t[x] = tn;
    tp = tn;
    mp = mk;
  }
}

template <bool FM = false>
__device__ __forceinline__ void mp_revap_racc(const Tables& tb, const MpConst& kc, double dt, double den, double& t, double& qv,
                              double& ql, double& qr, double qi, double qs, double qg) {
  const double cvm = cvm_(qv, ql, qr, qi, qs, qg);
  const double lcpk = lhl_(t) / cvm;
  double qsat, dqsdt;
  qs2(tb, false, t, den, qsat, dqsdt);
  const double dqv = qsat - qv;
  const double qden = fmax(qr, QRMIN) * den;
  const double t2 = t * t;
  const double ev = kc.crevp[0] * t2 * dqv * (kc.crevp[1] * sqrt(qden) + kc.crevp[2] * mexp<FM>(0.725 * mlog<FM>(qden))) /
                    (kc.crevp[3] * t2 + kc.crevp[4] * qsat * den);
  double evap = fmin(fmin(qr, dt * ev), dqv / (1.0 + lcpk * dqsdt));
  if (!(dqv > QVMIN && qr > QRMIN)) evap = 0.0;
  qr = qr - evap;
  qv = qv + evap;
  t = t - evap * lcpk;
  const double denfac = sqrt(SFCRHO / den);
  double sink = dt * denfac * kc.cracw * mexp<FM>(0.95 * mlog<FM>(fmax(qr, QRMIN) * den));
  sink = sink / (1.0 + sink) * ql;
  if (!(qr > QRMIN && ql > QCMIN)) sink = 0.0;
  ql = ql - sink;
  qr = qr + sink;
}

__device__ __forceinline__ void mp_revap_pass(int n, long P, const Tables& tb, const MpConst& kc, double dt, CRP den,
                                              RP t, RP qv, RP ql, RP qr, CRP qi, CRP qs, CRP qg) {
  // software pipelined as mp_icloud_pass
  double nt = t[0], nv = qv[0], nl = ql[0], nr = qr[0], ni = qi[0], ns = qs[0], ng = qg[0], nd = den[0];
  for (int k = 0; k < n; ++k) {
    const long x = (long)k * P;
    double tt = nt, v = nv, l = nl, r = nr;
    const double ii = ni, sn = ns, g = ng, dn = nd;
    if (k + 1 < n) {
      const long y = x + P;
      nt = t[y]; nv = qv[y]; nl = ql[y]; nr = qr[y]; ni = qi[y]; ns = qs[y]; ng = qg[y]; nd = den[y];
    }
    mp_revap_racc(tb, kc, dt, dn, tt, v, l, r, ii, sn, g);
    t[x] = tt; qv[x] = v; ql[x] = l; qr[x] = r;
  }
}

__device__ __forceinline__ void mp_autoconv(int n, long P, double dts, RP ql, RP qr) {
  for (int k = 0; k < n; ++k) {
    const long x = (long)k * P;
    const double l = ql[x];
    const double dq = l - QL0_AUT;
    double aut = dts * C_PAUT * 1.0e-3 * dq * dq / (dq + 1.0e-3);
    aut = dq > 0.0 ? fmin(aut, dq) : 0.0;
    ql[x] = l - aut;
    qr[x] = qr[x] + aut;
  }
}

template <bool FM = false>
__device__ __forceinline__ void mp_icloud(const Tables& tb, const MpConst& kc, double dts, double den, double& t, double& qv,
                          double& ql, double& qr, double& qi, double& qs, double& qg) {
  const double denfac = sqrt(SFCRHO / den);
  double tc = t - T_ICE;
  {  // pimlt
    const double icpk = lhi_(t) / cvm_(qv, ql, qr, qi, qs, qg);
    double mlt = fmin(qi * kc.e_imlt, fmax(tc, 0.0) / icpk);
    if (!(tc > 0.0)) mlt = 0.0;
    qi = qi - mlt; ql = ql + mlt; t = t - mlt * icpk;
  }
  {  // pifr
    const double icpk = lhi_(t) / cvm_(qv, ql, qr, qi, qs, qg);
    const double frz = t < T_WFR ? ql : 0.0;
    ql = ql - frz; qi = qi + frz; t = t + frz * icpk;
  }
  tc = t - T_ICE;
  const bool cold = tc < 0.0;
  {  // psacw
    const double fac = dts * denfac * kc.csacw * mexp<FM>(0.8125 * mlog<FM>(fmax(qs, QCMIN) * den));
    const double psacw = (qs > QCMIN && ql > QCMIN) ? fac / (1.0 + fac) * ql : 0.0;
    ql = ql - psacw;
    const double icpk = lhi_(t) / cvm_(qv, ql, qr, qi, qs, qg);
    qs = qs + (cold ? psacw : 0.0);
    qr = qr + (cold ? 0.0 : psacw);
    t = t + (cold ? psacw * icpk : 0.0);
  }
  {  // psaut
    const double qim = QI0_CRIT / den;
    const double aut = (cold && qi > qim) ? (1.0 - mexp<FM>(-dts * mexp<FM>(0.025 * tc) / TAU_I2S)) * (qi - qim) : 0.0;
    qi = qi - aut; qs = qs + aut;
  }
  {  // psaci
    const double fac = dts * denfac * kc.csacw * C_PSACI * mexp<FM>(0.05 * tc + 0.8125 * mlog<FM>(fmax(qs, QCMIN) * den));
    const double saci = (cold && qs > QCMIN && qi > QCMIN) ? fac / (1.0 + fac) * qi : 0.0;
    qi = qi - saci; qs = qs + saci;
  }
  {  // pgaut
    double gaut = (cold && qs > QS0_CRIT) ? dts * 1.0e-3 * mexp<FM>(0.09 * tc) * (qs - QS0_CRIT) : 0.0;
    gaut = fmin(gaut, fmax(qs, 0.0));
    qs = qs - gaut; qg = qg + gaut;
  }
  {  // pgacw
    const double fac = dts * kc.cgacw * mexp<FM>(0.875 * mlog<FM>(fmax(qg, QCMIN) * den)) * denfac;
    const double gacw = (qg > QCMIN && ql > QCMIN) ? fac / (1.0 + fac) * ql : 0.0;
    ql = ql - gacw;
    const double icpk = lhi_(t) / cvm_(qv, ql, qr, qi, qs, qg);
    qg = qg + (cold ? gacw : 0.0);
    qr = qr + (cold ? 0.0 : gacw);
    t = t + (cold ? gacw * icpk : 0.0);
  }
  for (int w = 0; w < 2; ++w) {  // smlt, gmlt
    double& q = w == 0 ? qs : qg;
    const double e = w == 0 ? kc.e_smlt : kc.e_gmlt;
    const double icpk = lhi_(t) / cvm_(qv, ql, qr, qi, qs, qg);
    const double tcm = t - T_ICE;
    double m = fmin(q * e, fmax(tcm, 0.0) / icpk);
    if (!(tcm > 0.0 && q > QCMIN)) m = 0.0;
    q = q - m; qr = qr + m; t = t - m * icpk;
  }
  // subgrid_z_proc
  {
    const double lcpk = lhl_(t) / cvm_(qv, ql, qr, qi, qs, qg);
    double qsw, dwsdt;
    qs2(tb, false, t, den, qsw, dwsdt);
    const double dq0 = (qv - qsw) / (1.0 + lcpk * dwsdt);
    double cond = dq0 > 0.0 ? dq0 * kc.e_v2l : fmax(dq0 * kc.e_l2v, -ql);
    if (dq0 > 0.0 && t < T_WFR) cond = 0.0;
    qv = qv - cond; ql = ql + cond; t = t + cond * lcpk;
  }
  const double fdep = kc.e_i2v;
  {
    const double tcpk = (lhl_(t) + lhi_(t)) / cvm_(qv, ql, qr, qi, qs, qg);
    double qsi, dqsidt;
    qs2(tb, true, t, den, qsi, dqsidt);
    const double dq = (qv - qsi) / (1.0 + tcpk * dqsidt);
    double dep = dq > 0.0 ? fdep * dq : fmax(fdep * dq, -qi);
    if (!(t < T_ICE)) dep = 0.0;
    qv = qv - dep; qi = qi + dep; t = t + dep * tcpk;
  }
  for (int w = 0; w < 2; ++w) {
    double& q = w == 0 ? qs : qg;
    const double tcpk = (lhl_(t) + lhi_(t)) / cvm_(qv, ql, qr, qi, qs, qg);
    double qsi, dqsidt;
    qs2(tb, true, t, den, qsi, dqsidt);
    const double dq = (qsi - qv) / (1.0 + tcpk * dqsidt);
    const double sub = (dq > 0.0 && q > QCMIN) ? fmin(q, fdep * dq) : 0.0;
    q = q - sub; qv = qv + sub; t = t - sub * tcpk;
  }
}

__device__ __forceinline__ void mp_icloud_pass(int n, long P, const Tables& tb, const MpConst& kc, double dts,
                                               CRP den, RP t, RP qv, RP ql, RP qr, RP qi, RP qs, RP qg) {
  // the next level's inputs are loaded while this level computes (software pipelined)
  double nt = t[0], nv = qv[0], nl = ql[0], nr = qr[0], ni = qi[0], ns = qs[0], ng = qg[0], nd = den[0];
  for (int k = 0; k < n; ++k) {
    const long x = (long)k * P;
    double tt = nt, v = nv, l = nl, r = nr, ii = ni, sn = ns, g = ng;
    const double dn = nd;
    if (k + 1 < n) {
      const long y = x + P;
      nt = t[y]; nv = qv[y]; nl = ql[y]; nr = qr[y]; ni = qi[y]; ns = qs[y]; ng = qg[y]; nd = den[y];
    }
    mp_icloud(tb, kc, dts, dn, tt, v, l, r, ii, sn, g);
    t[x] = tt; qv[x] = v; ql[x] = l; qr[x] = r; qi[x] = ii; qs[x] = sn; qg[x] = g;
  }
}

__global__ void __launch_bounds__(256) mpdrv_k(MpArgs a) {
  int s;
  long o;
  if (!col_point(a.d, s, o)) return;
  const long P = a.d.plane;
  const int n = a.nk;
  const double dts = a.dts;
  const MpConst& kc = a.k;
  double* t = a.T + (long)s * n * P + o;
  const long qo = (long)s * a.qsub * P + o;
  double *qv = a.qv + qo, *ql = a.ql + qo, *qr = a.qr + qo, *qi = a.qi + qo, *qs = a.qs + qo, *qg = a.qg + qo;
  const double* dp = a.dp + (long)s * n * P + o;
  const double* dz = a.dz + (long)s * n * P + o;
  double* sb = a.scr + (long)s * MP_NSCR * (n + 1) * P + o;
  const long SB = (long)(n + 1) * P;
  double *ze = sb, *zt = sb + SB, *den = sb + 2 * SB, *aa = sb + 3 * SB, *gam = sb + 4 * SB, *qe = sb + 5 * SB;
  double *vt = sb + 6 * SB, *m1 = sb + 7 * SB, *qm0 = sb + 8 * SB;
  double* qm = vt;  // the fall speeds are consumed (fallen heights) before the remap writes qm
  {
    double z = 0.0;
    ze[(long)n * P] = z;
    for (int k = n - 1; k >= 0; --k) {
      z = z - dz[(long)k * P];
      ze[(long)k * P] = z;
    }
    for (int k = 0; k < n; ++k) den[(long)k * P] = -dp[(long)k * P] / (GRAV * dz[(long)k * P]);
  }
  double prr = 0.0, prs = 0.0, prg = 0.0, pri = 0.0;
  for (int it = 0; it < a.ntimes; ++it) {
    mp_neg_adj(n, P, t, qv, ql, qr, qi, qs, qg, dp);
    // terminal_fall: melting, then ice, snow, graupel
    mp_melt(n, P, kc, t, qv, ql, qr, qi, qs, qg);
    double pf0 = 0.0, pf1 = 0.0, pf2 = 0.0;
#pragma unroll 1
    for (int w = 0; w < 3; ++w) {
      double* q = w == 0 ? qi : (w == 1 ? qs : qg);
      double pfw = 0.0;
      if (mp_speeds(n, P, w, q, den, vt)) {
        mp_fallen_edges(n, P, dts, ze, vt, zt);
        const double m = mp_lagrangian_fall(n, P, ze, zt, dp, q, qm0, aa, qe, gam, qm, m1);
        mp_sedi_heat(n, P, C_ICE, t, dp, dz, m1, qv, ql, qr, qi, qs, qg);
        pfw = m / GRAV;
      }
      if (w == 0) pf0 = pfw;
      else if (w == 1) pf1 = pfw;
      else pf2 = pfw;
    }
    // warm_rain
    const double dt5 = 0.5 * dts;
    mp_revap_pass(n, P, a.tb, kc, dt5, den, t, qv, ql, qr, qi, qs, qg);
    double pr_ = 0.0;
    if (mp_speeds(n, P, 3, qr, den, vt)) {
      mp_fallen_edges(n, P, dts, ze, vt, zt);
      const double m = mp_lagrangian_fall(n, P, ze, zt, dp, qr, qm0, aa, qe, gam, qm, m1);
      mp_sedi_heat(n, P, C_LIQ, t, dp, dz, m1, qv, ql, qr, qi, qs, qg);
      pr_ = m / GRAV;
    }
    mp_revap_pass(n, P, a.tb, kc, dt5, den, t, qv, ql, qr, qi, qs, qg);
    mp_autoconv(n, P, dts, ql, qr);
    prr = prr + pr_;
    prs = prs + pf1;
    prg = prg + pf2;
    pri = pri + pf0;
    mp_icloud_pass(n, P, a.tb, kc, dts, den, t, qv, ql, qr, qi, qs, qg);
  }
  const long p2 = (long)s * P + o;
  a.pr[p2] = prr;
  a.ps[p2] = prs;
  a.pg[p2] = prg;
  a.pi[p2] = pri;
}
#undef RP
#undef CRP

// ---- GFDL cloud microphysics, level-block form (default where a shape is instantiated) ----
//
// The column driver above keeps one lane per column and its nine working columns in HBM:
// ~3000 waves at C180, every pass a chain of dependent memory round trips (9.2 ms per C180
// step, 0.026 of the HBM roofline).  Here a column's levels sit in NB blocks of M on NB
// consecutive lanes of one DPP row (blockscan.hpp, as riem_scan_k / remap_blk_k), the whole
// state (T, six species, dp, dz) in registers for all ntimes sub-steps, read and written
// once; every lane works on every process:
//   * the pointwise processes (neg_adj's phase borrowing, melting, revap_racc, autoconversion,
//     icloud + subgrid_z_proc) per level, the same scalar functions as the column driver;
//   * neg_adj's vapour borrowing and fallen_edges' monotone fix are serial chains that
//     almost never act: each block runs its chain from the incoming value its upper
//     neighbour hands down by DPP, and the hand-over repeats until no incoming value changes
//     (one round when no block's chain reaches its bottom; results identical to the serial
//     walk);
//   * the Lagrangian sedimentation: fallen heights and layer densities pointwise, cs_profile's
//     edge system (the bottom edge eliminated into the last row, as remap_blk_k) by
//     tri_solve with Moebius-scan pivots, the edge bounds and the monotone limiter pointwise,
//     and the integration over the fixed layers through the mass function Q(z) (the fallen
//     column's mass above height z: block running sums + scanned offsets, each fixed
//     interface's Q evaluated by the block whose fallen range holds it, into LDS; a layer's
//     mass is Q(bottom) - Q(top), from block-local values when both lie in one block);
//     the fluxes m1 by a block scan and sedi_heat as an affine recurrence (scan_aff).
// The same expressions as the column driver, associated differently in the sums and the
// recurrences: agreement with the oracle to rounding (tests/test_gpu_moist.py bars), not bit
// for bit.  Shapes: NB M >= nk with the column's last two levels in one block.
constexpr int MB_WAVES = 4;
typedef unsigned int MbU2 __attribute__((ext_vector_type(2)));
template <int M, int NB>
__global__ void __launch_bounds__(64 * MB_WAVES) mpdrv_blk_k(MpArgs a) {
  constexpr int NC = 64 / NB, KX = NB * M;
  __shared__ double lze[MB_WAVES][NC][KX + 1];  // fixed interface heights (surface 0)
  __shared__ double lq[MB_WAVES][NC][KX + 1];   // block-local Q at fixed interface k
  __shared__ int lown[MB_WAVES][NC][KX + 1];    // the block whose fallen range holds interface k
  __shared__ double loff[MB_WAVES][NC][NB];     // Q at each block's top
  const Dims d = a.d;
  const int n = a.nk;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int b = lane & (NB - 1), cl = lane / NB;
  const int ncol = d.nx * d.ny;
  const int c0 = (blockIdx.x * MB_WAVES + wv) * NC;
  if (c0 >= ncol) return;  // whole wavefront (no barrier follows)
  int c = c0 + cl;
  const bool valid = c < ncol;
  if (!valid) c = ncol - 1;
  const int s = blockIdx.z;
  const long P = d.plane, o = pidx(d, c % d.nx, c / d.nx);
  const int g0 = b * M;
  const int nv = min(max(n - g0, 0), M);  // real levels of this block
  const bool lastb = b == (n - 1) / M;     // holds levels n - 2 and n - 1 (launcher)
  const double dts = a.dts;
  const MpConst& kc = a.k;
  const unsigned long long cmask = NB == 64 ? ~0ull : ((1ull << NB) - 1) << (cl * NB);
  // buffer resources per field (the sub-domain's nk planes), one VGPR offset per lane (the
  // lane's column at its block's first level) plus the level (inside the range-checked vector
  // offset: a partial block's levels past the bottom read 0 and drop their stores)
  const uint32_t PB = (uint32_t)P * 8u;
  const uint32_t vb = (uint32_t)(o + (long)g0 * P) * 8u;
  auto rsrc = [&](const double* base) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, (int)(n * PB), 0x00020000);
  };
  const long qo = (long)s * a.qsub * P;
  const auto rT = rsrc(a.T + (long)s * n * P), rV = rsrc(a.qv + qo), rL = rsrc(a.ql + qo), rR = rsrc(a.qr + qo);
  const auto rI = rsrc(a.qi + qo), rS = rsrc(a.qs + qo), rG = rsrc(a.qg + qo);
  const auto rP = rsrc(a.dp + (long)s * n * P), rZ = rsrc(a.dz + (long)s * n * P);
  auto ld = [&](__amdgpu_buffer_rsrc_t r, int m) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, vb + (uint32_t)m * PB, 0, 0));
  };
  auto st = [&](__amdgpu_buffer_rsrc_t r, int m, double v) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(MbU2, v), r, vb + (uint32_t)m * PB, 0, 0);
  };
  double t[M], qv[M], ql[M], qr[M], qi[M], qs[M], qg[M], dp[M], dz[M], den[M];
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const bool r = m < nv;
    t[m] = r ? ld(rT, m) : T_ICE;
    qv[m] = r ? ld(rV, m) : 0.0;
    ql[m] = r ? ld(rL, m) : 0.0;
    qr[m] = r ? ld(rR, m) : 0.0;
    qi[m] = r ? ld(rI, m) : 0.0;
    qs[m] = r ? ld(rS, m) : 0.0;
    qg[m] = r ? ld(rG, m) : 0.0;
    dp[m] = r ? ld(rP, m) : 1.0;
    dz[m] = r ? ld(rZ, m) : -1.0;
    den[m] = -dp[m] / (GRAV * dz[m]);
  }
  // fixed interface heights: the block's own sums from its bottom, the blocks below by a scan
  {
    double zl[M], z = 0.0;
#pragma unroll
    for (int m = M - 1; m >= 0; --m) {
      z = m < nv ? z - dz[m] : z;
      zl[m] = z;
    }
    const double incl = scan_sum<NB, false>(z, b);
    const double below_ = blk_next(incl);
    const double below = b == NB - 1 ? 0.0 : below_;
#pragma unroll
    for (int m = 0; m < M; ++m)
      if (m < nv) lze[wv][cl][g0 + m] = below + zl[m];
    if (lastb) lze[wv][cl][n] = 0.0;
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
  auto zeF = [&](int k) { return lze[wv][cl][k]; };

  // one Lagrangian fall of species q (w: 0 ice, 1 snow, 2 graupel, 3 rain) with sedi_heat;
  // returns the flux out of the column's bottom (in the lane holding level n - 1)
  auto fall = [&](double (&q)[M], int w, double cw) -> double {
    const double thr = w == 3 ? QRMIN : QCMIN;
    double vt[M];
    bool lany = false;
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const double dn = den[m], qq = q[m];
      const double rhof = sqrt(fmin(10.0, SFCRHO / dn));
      double v;
      if (w == 3) {
        const double q_ = fmax(qq, QRMIN);
        v = qq > QRMIN ? fmin(VR_MAX, fmax(VR_MIN, VCONR * rhof * fm_exp(0.2 * fm_log(q_ * dn / NORMR)))) : 0.0;
      } else if (w == 0) {
        const double q_ = fmax(qq, QCMIN);
        v = qq > QCMIN ? fmin(VI_MAX, 3.29 * fm_exp(0.16 * fm_log(q_ * dn))) : 0.0;
      } else if (w == 1) {
        const double q_ = fmax(qq, QCMIN);
        v = qq > QCMIN ? fmin(VS_MAX, VCONS * rhof * fm_exp(0.0625 * fm_log(q_ * dn / NORMS))) : 0.0;
      } else {
        const double q_ = fmax(qq, QCMIN);
        v = qq > QCMIN ? fmin(VG_MAX, VCONG * rhof * sqrt(sqrt(sqrt(q_ * dn / NORMG)))) : 0.0;
      }
      vt[m] = v;
      lany = lany || (m < nv && qq > thr);
      __builtin_amdgcn_sched_barrier(0);
    }
    const bool cany = (__ballot(lany) & cmask) != 0;  // the column holds this species
    if (__ballot(cany) == 0) return 0.0;               // (wave-uniform)
    // fallen interface heights, raw: interface g0 + m is the top of local layer m
    const double vpv_ = blk_prev(vt[M - 1]);
    const double vpv = b == 0 ? 0.0 : vpv_;
    double zr[M], zbr = 0.0;
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const int g = g0 + m;
      const double vp = m == 0 ? vpv : vt[m > 0 ? m - 1 : 0];
      const double ze = m < nv ? zeF(g) : 0.0;
      zr[m] = g == 0 ? ze : ze - 0.5 * dts * (vp + vt[m]);
      if (lastb && m == nv - 1) zbr = zeF(n) - dts * vt[m];
    }
    // monotone fix (each interface strictly below the one above), as a chain from the
    // incoming fixed height of interface g0 - 1
    double zf[M], zfb = 0.0;
    auto chain = [&](double zin) {
      double zp = zin;
#pragma unroll
      for (int m = 0; m < M; ++m) {
        double z = zr[m];
        if (g0 + m > 0 && m < nv && z >= zp) z = zp - DZ_MIN_FALL;
        zf[m] = z;
        zp = m < nv ? z : zp;
      }
      double z = zbr;
      if (z >= zp) z = zp - DZ_MIN_FALL;
      zfb = z;
    };
    const double zin0_ = blk_prev(zr[M - 1]);
    double zin = b == 0 ? 0.0 : zin0_;
    chain(zin);
#pragma unroll 1
    for (int r = 0; r < NB; ++r) {
      const double zn_ = blk_prev(zf[M - 1]);
      const double zn = b == 0 ? 0.0 : zn_;
      const bool ch = zn != zin;
      if (__ballot(ch) == 0) break;
      zin = zn;
      chain(zin);
    }
    // fallen thicknesses and densities per height
    const double zfn_ = blk_next(zf[0]);
    double dzf[M], qm0[M], aa[M];
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const double zlo = m + 1 < M ? zf[m + 1 < M ? m + 1 : 0] : zfn_;
      const double zb = (lastb && m == nv - 1) ? zfb : zlo;
      dzf[m] = m < nv ? zf[m] - zb : 1.0;
      qm0[m] = q[m] * dp[m];
      aa[m] = qm0[m] / dzf[m];
    }
    const double am1_ = blk_prev(aa[M - 1]), dzm1_ = blk_prev(dzf[M - 1]);
    const double am1 = b == 0 ? 0.0 : am1_, dzm1 = b == 0 ? 1.0 : dzm1_;
    auto Aw = [&](int m) { return m < 0 ? am1 : aa[m]; };
    auto Dw = [&](int m) { return m < 0 ? dzm1 : dzf[m]; };
    // the bottom edge's row (last block; levels n - 2, n - 1 both in it)
    double abot = 1.0, dbot = 1.0, rbot = 0.0, d4b = 0.0;
#pragma unroll
    for (int m = 1; m < M; ++m)
      if (m == nv - 1) {
        d4b = dzf[m - 1] / dzf[m];
        abot = 1.0 + d4b * (d4b + 1.5);
        dbot = d4b * (d4b + 0.5);
        rbot = 2.0 * d4b * (d4b + 1.0) * aa[m] + aa[m - 1];
      }
    auto row = [&](int m, double& am, double& dg, double& cm) {
      const int e = g0 + m;
      if (m >= nv) {
        am = 0.0; dg = 1.0; cm = 0.0;
        return;
      }
      if (e == 0) {
        const double grat = dzf[1 < M ? 1 : 0] / dzf[0];
        am = 0.0;
        dg = grat * (grat + 0.5);
        cm = 1.0 + grat * (grat + 1.5);
        return;
      }
      const double d4 = Dw(m - 1) / dzf[m];
      am = 1.0;
      dg = 2.0 + d4 + d4;
      cm = d4;
      if (lastb && m == nv - 1) {
        dg = dg - cm * abot / dbot;
        cm = 0.0;
      }
    };
    auto rhs = [&](int m) -> double {
      const int e = g0 + m;
      if (m >= nv) return 0.0;
      if (e == 0) {
        const double grat = dzf[1 < M ? 1 : 0] / dzf[0];
        return (grat + grat) * (grat + 1.0) * aa[0] + aa[1 < M ? 1 : 0];
      }
      const double d4 = Dw(m - 1) / dzf[m];
      double r = 3.0 * (Aw(m - 1) + d4 * aa[m]);
      if (lastb && m == nv - 1) r = r - d4 * rbot / dbot;
      return r;
    };
    double qe[M];
    tri_solve<M, NB, true>(row, rhs, qe, b, b == NB - 1);
    double qlast = qe[0];
#pragma unroll
    for (int m = 0; m < M; ++m)
      if (m == nv - 1) qlast = qe[m];
    const double qbot = fmax((rbot - abot * qlast) / dbot, 0.0);
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const double a0 = Aw(m - 1), a1 = aa[m];
      qe[m] = g0 + m == 0 ? fmax(qe[m], 0.0) : fmin(fmax(qe[m], fmin(a0, a1)), fmax(a0, a1));
    }
    const double qen_ = blk_next(qe[0]);
    // running mass of the fallen block, block offsets
    double C[M + 1];
    C[0] = 0.0;
#pragma unroll
    for (int m = 0; m < M; ++m) C[m + 1] = C[m] + (m < nv ? qm0[m] : 0.0);
    const double offx = blk_prev(scan_sum<NB, true>(C[M], b));
    loff[wv][cl][b] = b == 0 ? 0.0 : offx;
    // fixed interfaces in the block's fallen range (the last real layer takes the rest)
    int k = g0 < n ? g0 : n;
    if (b == 0) k = 0;
    else
      while (k <= n && zeF(k) > zf[0]) ++k;
#pragma unroll
    for (int m = 0; m < M; ++m) {
      if (m >= nv) continue;
      // the monotone profile of fallen layer m (cs_limiters, mono)
      const double av = aa[m];
      double l = qe[m];
      double r = m + 1 < M ? qe[m + 1 < M ? m + 1 : 0] : qen_;
      if (lastb && m == nv - 1) r = qbot;
      double a6v;
      const double da1 = r - l;
      if ((av - l) * (av - r) >= 0.0) {
        l = av; r = av; a6v = 0.0;
      } else {
        a6v = 3.0 * (2.0 * av - (l + r));
        if (a6v * da1 < -da1 * da1) {
          a6v = 3.0 * (l - av);
          r = l - a6v;
        } else if (a6v * da1 > da1 * da1) {
          a6v = 3.0 * (r - av);
          l = r - a6v;
        }
      }
      const bool lastlayer = lastb && m == nv - 1;
      const double ztop = zf[m];
      const double zlow = m + 1 < M ? zf[m + 1 < M ? m + 1 : 0] : zfn_;
      const double rdz = 1.0 / dzf[m];
      while (k <= n) {
        const double z = zeF(k);
        if (!lastlayer && z <= zlow) break;
        const double y = ztop - z, x = y * rdz;
        lq[wv][cl][k] = C[m] + y * (l + 0.5 * (a6v + r - l) * x - a6v * MP_R3 * x * x);
        lown[wv][cl][k] = b;
        ++k;
      }
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    // fixed layer masses, fluxes through their bottoms, new mixing ratios
    double qm[M], f[M], racc = 0.0;
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const int kk = g0 + m;
      double v = 0.0;
      if (m < nv) {
        const int o0 = lown[wv][cl][kk], o1 = lown[wv][cl][kk + 1];
        const double q0 = lq[wv][cl][kk], q1 = lq[wv][cl][kk + 1];
        v = o0 == o1 ? q1 - q0 : (loff[wv][cl][o1] - loff[wv][cl][o0]) + (q1 - q0);
      }
      qm[m] = v;
      racc = racc + (m < nv ? qm0[m] - v : 0.0);
      f[m] = racc;
    }
    const double m1x = blk_prev(scan_sum<NB, true>(racc, b));
    const double m1o = b == 0 ? 0.0 : m1x;
#pragma unroll
    for (int m = 0; m < M; ++m) f[m] = m1o + f[m];
    // sedi_heat: t_k = (cv0 t_k + m1_{k-1} (cw t'_{k-1} + dgz)) / (cv0 + cw m1_{k-1}), affine
    // in t'_{k-1}
    const double m1p_ = blk_prev(f[M - 1]);
    double qn[M], A[M], B[M];
#pragma unroll
    for (int m = 0; m < M; ++m) qn[m] = m < nv ? qm[m] / dp[m] : 0.0;
    Aff blk{1.0, 0.0};
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const int g = g0 + m;
      const double mp = m == 0 ? m1p_ : f[m > 0 ? m - 1 : 0];
      double qvv = qv[m], qll = ql[m], qrr = qr[m], qii = qi[m], qss = qs[m], qgg = qg[m];
      if (w == 0) qii = qn[m];
      else if (w == 1) qss = qn[m];
      else if (w == 2) qgg = qn[m];
      else qrr = qn[m];
      const double dgz = -0.5 * GRAV * dz[m];
      const double cv0 = dp[m] * cvm_(qvv, qll, qrr, qii, qss, qgg) + cw * (f[m] - mp);
      const double dd = cv0 + cw * mp;
      double Am = cw * mp / dd, Bm = (cv0 * t[m] + mp * dgz) / dd;
      if (g == 0) { Am = 0.0; Bm = t[m]; }
      if (m >= nv) { Am = 1.0; Bm = 0.0; }
      A[m] = Am;
      B[m] = Bm;
      blk = Aff{Am * blk.A, __builtin_fma(Am, blk.B, Bm)};
    }
    const Aff F = scan_aff<NB, true>(blk, b);
    const double tin_ = blk_prev(F.B);
    double tc = b == 0 ? 0.0 : tin_;
    double bottom = 0.0;
#pragma unroll
    for (int m = 0; m < M; ++m) {
      tc = __builtin_fma(A[m], tc, B[m]);
      if (cany && m < nv) {
        t[m] = tc;
        q[m] = qn[m];
      }
      if (m == nv - 1) bottom = f[m];
    }
    return cany && lastb ? bottom : 0.0;
  };

  double prr = 0.0, prs = 0.0, prg = 0.0, pri = 0.0;
#pragma unroll 1
  for (int it = 0; it < a.ntimes; ++it) {
    // ---- neg_adj: phase borrowing per level, then negative vapour borrows from below
#pragma unroll
    for (int m = 0; m < M; ++m) {
      double tt = t[m], v = qv[m], l = ql[m], r = qr[m], ii = qi[m], sn = qs[m], g = qg[m];
      const double cvm = cvm_(v, l, r, ii, sn, g);
      const double lcpk = lhl_(tt) / cvm, icpk = lhi_(tt) / cvm;
      if (ii < 0.0) { sn = sn + ii; ii = 0.0; }
      if (sn < 0.0) { g = g + sn; sn = 0.0; }
      {
        const double dq = g < 0.0 ? g : 0.0;
        v = v + dq;
        tt = tt - dq * (lcpk + icpk);
        if (g < 0.0) g = 0.0;
      }
      if (r < 0.0) { l = l + r; r = 0.0; }
      {
        const double dq = l < 0.0 ? l : 0.0;
        v = v + dq;
        tt = tt - dq * lcpk;
        if (l < 0.0) l = 0.0;
      }
      t[m] = tt; qv[m] = v; ql[m] = l; qr[m] = r; qi[m] = ii; qs[m] = sn; qg[m] = g;
    }
    {
      double vq[M], cout = 0.0;
      const double dpin_ = blk_prev(dp[M - 1]);
      const double dpin = b == 0 ? 1.0 : dpin_;
      // the block's chain from the incoming value of level g0 - 1 (after its own borrow)
      auto chain = [&](double cin) {
        double cur = cin, dprev = dpin;
#pragma unroll
        for (int m = 0; m < M; ++m) {
          const int g = g0 + m;
          double v = qv[m];
          if (g >= 1 && m < nv && cur < 0.0) v = v + cur * dprev / dp[m];
          vq[m] = v;
          cur = m < nv ? v : cur;
          dprev = dp[m];
        }
        cout = cur;
      };
      double cin = 0.0;
      chain(cin);
#pragma unroll 1
      for (int r = 0; r < NB; ++r) {
        const double cn_ = blk_prev(cout);
        const double cn = b == 0 ? 0.0 : cn_;
        const bool ch = (cn < 0.0 || cin < 0.0) && cn != cin;
        if (__ballot(ch) == 0) break;
        cin = cn;
        chain(cin);
      }
      // levels 0 .. n - 2 that went negative passed their vapour down
#pragma unroll
      for (int m = 0; m < M; ++m) qv[m] = (g0 + m <= n - 2 && vq[m] < 0.0) ? 0.0 : vq[m];
      // bottom: the last level borrows from the one above
#pragma unroll
      for (int m = 1; m < M; ++m)
        if (lastb && m == nv - 1) {
          const double qb = qv[m], qa = qv[m - 1];
          double dq = fmin(-qb * dp[m], qa * dp[m - 1]);
          if (!(qb < 0.0 && qa > 0.0)) dq = 0.0;
          qv[m - 1] = qa - dq / dp[m - 1];
          qv[m] = qb + dq / dp[m];
        }
    }
    // ---- terminal_fall: melting of the falling ice species, then ice, snow, graupel
#pragma unroll
    for (int m = 0; m < M; ++m) {
      double tt = t[m];
      if (!(tt > T_ICE)) continue;
      double v = qv[m], l = ql[m], r = qr[m], ii = qi[m], sn = qs[m], g = qg[m];
#pragma unroll
      for (int w = 0; w < 3; ++w) {
        double& q = w == 0 ? ii : (w == 1 ? sn : g);
        const double fq = w == 0 ? kc.e_imlt : (w == 1 ? kc.e_smlt : kc.e_gmlt);
        const double icpk = lhi_(tt) / cvm_(v, l, r, ii, sn, g);
        const double mlt = fmin(fq * q, (tt - T_ICE) / icpk);
        if (mlt > 0.0) {
          q = q - mlt;
          if (w == 0) l = l + mlt;
          else r = r + mlt;
          tt = tt - mlt * icpk;
        }
      }
      t[m] = tt; ql[m] = l; qr[m] = r; qi[m] = ii; qs[m] = sn; qg[m] = g;
      __builtin_amdgcn_sched_barrier(0);
    }
    const double pf0 = fall(qi, 0, C_ICE);
    const double pf1 = fall(qs, 1, C_ICE);
    const double pf2 = fall(qg, 2, C_ICE);
    // ---- warm_rain
    const double dt5 = 0.5 * dts;
#pragma unroll
    for (int m = 0; m < M; ++m) {
      mp_revap_racc<true>(a.tb, kc, dt5, den[m], t[m], qv[m], ql[m], qr[m], qi[m], qs[m], qg[m]);
      __builtin_amdgcn_sched_barrier(0);  // one level at a time (register pressure)
    }
    const double pr_ = fall(qr, 3, C_LIQ);
#pragma unroll
    for (int m = 0; m < M; ++m) {
      mp_revap_racc<true>(a.tb, kc, dt5, den[m], t[m], qv[m], ql[m], qr[m], qi[m], qs[m], qg[m]);
      __builtin_amdgcn_sched_barrier(0);  // one level at a time (register pressure)
    }
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const double l = ql[m];
      const double dq = l - QL0_AUT;
      double aut = dts * C_PAUT * 1.0e-3 * dq * dq / (dq + 1.0e-3);
      aut = dq > 0.0 ? fmin(aut, dq) : 0.0;
      ql[m] = l - aut;
      qr[m] = qr[m] + aut;
    }
    prr = prr + pr_ / GRAV;
    prs = prs + pf1 / GRAV;
    prg = prg + pf2 / GRAV;
    pri = pri + pf0 / GRAV;
    // ---- icloud
#pragma unroll
    for (int m = 0; m < M; ++m) {
      mp_icloud<true>(a.tb, kc, dts, den[m], t[m], qv[m], ql[m], qr[m], qi[m], qs[m], qg[m]);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if (!valid) return;
#pragma unroll
  for (int m = 0; m < M; ++m) {
    if (m >= nv) continue;
    st(rT, m, t[m]); st(rV, m, qv[m]); st(rL, m, ql[m]); st(rR, m, qr[m]);
    st(rI, m, qi[m]); st(rS, m, qs[m]); st(rG, m, qg[m]);
  }
  if (lastb) {
    const long p2 = (long)s * P + o;
    a.pr[p2] = prr;
    a.ps[p2] = prs;
    a.pg[p2] = prg;
    a.pi[p2] = pri;
  }
}

// ---- GEOS pieces around the microphysics (oracle/geos_moist.py), pointwise ----
constexpr double RHO_W = 1000.0, RHO_I = 917.0;
constexpr double K_COND = 2.4e-2, DIFFU = 2.2e-5;
constexpr double A_EFF_L = 0.8, A_EFF_I = 0.5;
constexpr double QC_MAX = 0.01;
constexpr double PI_ = 3.14159265358979323846;

__device__ __forceinline__ double ice_fraction(double t) { return fmin(fmax((T_ICE - t) / 40.0, 0.0), 1.0); }
__device__ __forceinline__ double rhcrit(double pl) {
  const double x = fmin(fmax((75000.0 - pl) / 75000.0, 0.0), 1.0);
  return 0.80 + 0.19 * x * x;
}
__device__ double ldradius4(double pl, double t, double qc, double nnl, int itype) {
  const double rho = pl / (RDGAS * t);
  const double wc = rho * fmax(qc, 0.0);
  if (itype == 1) {
    const double nnx = fmax(nnl, 1.0e7);
    const double r = 1.1 * cbrt(3.0 * wc / (4.0 * PI_ * RHO_W * nnx));
    return fmin(60.0e-6, fmax(2.5e-6, r));
  }
  const double wcg = fmax(1.0e3 * wc, 1.0e-12);
  double bb = (t > T_ICE || qc <= 0.0) ? -2.0
                                       : -2.0 + log10(wcg / 50.0) * (1.0e-3 * pow(fmax(T_ICE - t, 0.0), 1.5));
  bb = fmin(fmax(bb, -6.0), -2.0);
  const double r = 377.4 + 203.3 * bb + 37.91 * bb * bb + 2.3696 * bb * bb * bb;
  return fmin(150.0e-6, fmax(5.0e-6, 1.0e-6 * r));
}

struct EspArgs {
  Dims d;
  int nk;
  double dt, e_frz, e_mlt;
  Tables tb;
  double *T, *qv, *qlls, *qils, *qlcn, *qicn, *clls, *clcn;
  long qv_sub, ql_sub, qi_sub;  // levels per sub-domain of qv / qlls / qils (tracer slices)
  const double *pl, *nactl, *nacti;
};

__device__ __forceinline__ void meltfrz(double e_frz, double e_mlt, double& t, double& ql, double& qi) {
  const double fqi = ice_fraction(t);
  const double frz = t <= T_ICE ? ql * fqi * e_frz : 0.0;
  const double mlt = t > T_ICE ? qi * e_mlt : 0.0;
  ql = ql + (mlt - frz);
  qi = qi + (frz - mlt);
  t = t + (frz - mlt) * (HLF / CP_AIR);
}

__global__ void __launch_bounds__(256) evap_subl_pdf_k(EspArgs a) {
  const Dims& d = a.d;
  const int i = blockIdx.x * BX + threadIdx.x, j = blockIdx.y * BY + threadIdx.y;
  if (i >= d.nx || j >= d.ny) return;
  const int z = blockIdx.z, s = z / a.nk, k = z % a.nk;
  const long o = pidx(d, i, j);
  const long x = (long)z * d.plane + o;
  const long xv = ((long)s * a.qv_sub + k) * d.plane + o;
  const long xl = ((long)s * a.ql_sub + k) * d.plane + o;
  const long xi = ((long)s * a.qi_sub + k) * d.plane + o;
  const double pl = a.pl[x], nl = a.nactl[x];
  double t = a.T[x], qv = a.qv[xv], qlls = a.qlls[xl], qils = a.qils[xi], qlcn = a.qlcn[x], qicn = a.qicn[x];
  double clls = a.clls[x], clcn = a.clcn[x];
  const double rhcr = rhcrit(pl);
  meltfrz(a.e_frz, a.e_mlt, t, qlcn, qicn);
  meltfrz(a.e_frz, a.e_mlt, t, qlls, qils);
  {  // evap3 (anvil liquid)
    double qs, dqs;
    qsat(a.tb, false, t, pl, qs, dqs);
    const double es = pl * qs / (EPS + (1.0 - EPS) * qs);
    const double rhx = fmin(qv / qs, 1.0);
    const double k1 = HLV * HLV * RHO_W / (K_COND * RVGAS * t * t);
    const double k2 = RVGAS * t * RHO_W / (DIFFU * (1.0e5 / pl) * es);
    const double qcm = (clcn > 0.0 && qlcn > 0.0) ? qlcn / clcn : 0.0;
    const double rad = ldradius4(pl, t, qcm, nl, 1);
    const double teff = rhx < rhcr ? (rhcr - rhx) / ((k1 + k2) * rad * rad) : 0.0;
    double ev = fmin(A_EFF_L * qlcn * a.dt * teff, qlcn);
    if (!(qlcn > 0.0)) ev = 0.0;
    qv = qv + ev; qlcn = qlcn - ev; t = t - ev * (HLV / CP_AIR);
  }
  {  // subl3 (anvil ice)
    double qs, dqs;
    qsat(a.tb, true, t, pl, qs, dqs);
    const double es = pl * qs / (EPS + (1.0 - EPS) * qs);
    const double rhx = fmin(qv / qs, 1.0);
    const double k1 = HLS * HLS * RHO_I / (K_COND * RVGAS * t * t);
    const double k2 = RVGAS * t * RHO_I / (DIFFU * (1.0e5 / pl) * es);
    const double qcm = (clcn > 0.0 && qicn > 0.0) ? qicn / clcn : 0.0;
    const double rad = ldradius4(pl, t, qcm, nl, 2);
    const double teff = rhx < rhcr ? (rhcr - rhx) / ((k1 + k2) * rad * rad) : 0.0;
    double sb = fmin(A_EFF_I * qicn * a.dt * teff, qicn);
    if (!(qicn > 0.0)) sb = 0.0;
    qv = qv + sb; qicn = qicn - sb; t = t - sb * (HLS / CP_AIR);
  }
  if (!(qlcn + qicn > 0.0)) clcn = 0.0;
  for (int it = 0; it < 3; ++it) {  // hystpdf
    double qs, dqs;
    qsat(a.tb, false, t, pl, qs, dqs);
    const double sig = (1.0 - rhcr) * qs;
    const double qt = qv + qlls + qils;
    const bool full = qt - sig >= qs, none = qt + sig <= qs;
    const double cf = full ? 1.0 : (none ? 0.0 : (qt + sig - qs) / (2.0 * sig));
    const double qcn = full ? qt - qs : (none ? 0.0 : (qt + sig - qs) * (qt + sig - qs) / (4.0 * sig));
    const double fqi = ice_fraction(t);
    const double lat = HLV / CP_AIR + fqi * (HLF / CP_AIR);
    const double dqc = (qcn - (qlls + qils)) / (1.0 + lat * dqs * cf);
    const double dl = dqc > 0.0 ? dqc * (1.0 - fqi) : fmax(dqc, -qlls);
    const double di = dqc > 0.0 ? dqc * fqi : fmax(dqc - dl, -qils);
    qlls = qlls + dl;
    qils = qils + di;
    qv = qv - (dl + di);
    t = t + (dl * (HLV / CP_AIR) + di * (HLS / CP_AIR));
    clls = cf;
  }
  a.T[x] = t; a.qv[xv] = qv; a.qlls[xl] = qlls; a.qils[xi] = qils; a.qlcn[x] = qlcn; a.qicn[x] = qicn;
  a.clls[x] = clls; a.clcn[x] = clcn;
}

struct RadArgs {
  Dims d;
  int nk;
  long qv_sub, ql_sub, qi_sub, qr_sub, qs_sub, qg_sub;
  const double *T, *pl, *cf, *af, *qv, *qlls, *qils, *qlcn, *qicn, *qr, *qs, *qg, *nl;
  double *rqv, *rql, *rqi, *rqr, *rqs, *rqg, *rcf, *rrl, *rri;
};

__global__ void __launch_bounds__(256) radcouple_k(RadArgs a) {
  const Dims& d = a.d;
  const int i = blockIdx.x * BX + threadIdx.x, j = blockIdx.y * BY + threadIdx.y;
  if (i >= d.nx || j >= d.ny) return;
  const int z = blockIdx.z, s = z / a.nk, k = z % a.nk;
  const long o = pidx(d, i, j);
  const long x = (long)z * d.plane + o;
  auto sp = [&](long sub) { return ((long)s * sub + k) * d.plane + o; };
  double rcf = fmin(fmax(a.cf[x] + a.af[x], 0.0), 1.0);
  const bool cloudy = rcf >= 1.0e-5;
  const double div = cloudy ? rcf : 1.0;
  auto incloud = [&](double v) { return (cloudy && v >= 1.0e-8) ? v / div : 0.0; };
  const double rql = fmin(incloud(a.qlls[sp(a.ql_sub)] + a.qlcn[x]), QC_MAX);
  const double rqi = fmin(incloud(a.qils[sp(a.qi_sub)] + a.qicn[x]), QC_MAX);
  a.rqr[x] = fmin(incloud(a.qr[sp(a.qr_sub)]), QC_MAX);
  a.rqs[x] = fmin(incloud(a.qs[sp(a.qs_sub)]), QC_MAX);
  a.rqg[x] = fmin(incloud(a.qg[sp(a.qg_sub)]), QC_MAX);
  a.rql[x] = rql;
  a.rqi[x] = rqi;
  a.rcf[x] = cloudy ? rcf : 0.0;
  a.rqv[x] = a.qv[sp(a.qv_sub)];
  const double t = a.T[x], pl = a.pl[x], nl = a.nl[x];
  a.rrl[x] = ldradius4(pl, t, rql, nl, 1);
  a.rri[x] = ldradius4(pl, t, rqi, nl, 2);
}

// Abdul-Razzak & Ghan (2000) activation of three lognormal modes + Meyers (1992) ice nuclei
struct AerMode {
  double n0, h, rd, sg, kap;
};
constexpr AerMode kAerModes[3] = {{1.0e9, 2000.0, 0.02e-6, 1.6, 0.6},
                                  {3.0e8, 2000.0, 0.08e-6, 1.8, 0.6},
                                  {1.0e6, 1000.0, 1.00e-6, 2.0, 1.2}};
constexpr double MW = 0.018015, MA = 0.028965, RGAS_U = 8.314462618, SURF_T = 0.0761, W_MIN = 0.1;

// per-mode constants of the activation, formed on the host as the oracle forms them
// (math.log / math.exp / math.sqrt of the mode parameters)
struct AerModeC {
  double n0, h, rd3, sk, ls, f, g;  // rd3 = 3 rd, sk = 2 / sqrt(kap), ls = log(sg), f, g
};
struct AerArgs {
  Dims d;
  int nk;
  long qv_sub;
  Tables tb;
  const double *pl, *T, *qv, *zm, *w;
  double *nactl, *nacti, *smax;
  AerModeC mode[3];
};

__global__ void __launch_bounds__(256) aer_activation_k(AerArgs a) {
  const Dims& d = a.d;
  const int i = blockIdx.x * BX + threadIdx.x, j = blockIdx.y * BY + threadIdx.y;
  if (i >= d.nx || j >= d.ny) return;
  const int z = blockIdx.z, s = z / a.nk, k = z % a.nk;
  const long o = pidx(d, i, j);
  const long x = (long)z * d.plane + o;
  const double pl = a.pl[x], t = a.T[x], zm = a.zm[x];
  const double qv = a.qv[((long)s * a.qv_sub + k) * d.plane + o];
  const double wv = fmax(a.w[x], 0.0) + W_MIN;
  double qs, dqs;
  qsat(a.tb, false, t, pl, qs, dqs);
  const double es = pl * qs / (EPS + (1.0 - EPS) * qs);
  const double a_k = 2.0 * SURF_T * MW / (RHO_W * RGAS_U * t);
  const double alpha = GRAV * MW * HLV / (CP_AIR * RGAS_U * t * t) - GRAV * MA / (RGAS_U * t);
  const double gamma = RGAS_U * t / (es * MW) + MW * HLV * HLV / (CP_AIR * pl * MA * t);
  const double dv = DIFFU * (1.0e5 / pl);
  const double gg = 1.0 / (RHO_W * RGAS_U * t / (es * dv * MW) + HLV * RHO_W / (K_COND * t) * (HLV * MW / (RGAS_U * t) - 1.0));
  const double aw = alpha * wv / gg;
  const double zeta = 2.0 * a_k / 3.0 * sqrt(aw);
  // x^1.5 as x sqrt(x) and x^0.75 as sqrt(x) sqrt(sqrt(x)) (within a few ulp of pow, which
  // cost ~60 % of the kernel); the mode constants come from the host; modes with the same
  // scale height share one exp
  auto p15 = [](double x) { return x * sqrt(x); };
  auto p075 = [](double x) {
    const double r = sqrt(x);
    return r * sqrt(r);
  };
  const double zp = fmax(zm, 0.0);
  const double aw15 = p15(aw);
  double ssum = 0.0, sm[3], nn[3], ls[3];
  double ex = 0.0;
#pragma unroll
  for (int m = 0; m < 3; ++m) {
    const AerModeC md = a.mode[m];
    if (m == 0 || md.h != a.mode[m > 0 ? m - 1 : 0].h) ex = exp(-zp / md.h);
    nn[m] = md.n0 * ex;
    sm[m] = md.sk * p15(a_k / md.rd3);
    ls[m] = md.ls;
    const double eta = aw15 / (2.0 * PI_ * RHO_W * gamma * nn[m]);
    ssum = ssum + (md.f * p15(zeta / eta) + md.g * p075(sm[m] * sm[m] / (eta + 3.0 * zeta))) / (sm[m] * sm[m]);
  }
  const double smax = 1.0 / sqrt(ssum);
  double nact = 0.0;
#pragma unroll
  for (int m = 0; m < 3; ++m) {
    const double u = 2.0 * log(sm[m] / smax) / (3.0 * sqrt(2.0) * ls[m]);
    nact = nact + nn[m] * 0.5 * erfc(u);
  }
  double qsi, dqsi;
  qsat(a.tb, true, t, pl, qsi, dqsi);
  const double si = fmin(fmax(qv / qsi - 1.0, -0.2), 0.25);
  a.nactl[x] = nact;
  a.nacti[x] = t < T_ICE - 5.0 ? 1.0e3 * exp(-0.639 + 12.96 * si) : 0.0;
  a.smax[x] = smax;
}

// ---- shallow cumulus (GEOS cup_gf_sh; oracle/gf_shallow.py), one lane per column ----
// Source level, cloud base, entraining plume and cloud top are column walks; the plume's
// moist static energy, total water, normalised mass flux and condensate live in HBM scratch
// columns between the walk and the flux-form tendencies.  Same expressions and order as the
// oracle; the level indices k22 / kbcon / ktop come out bit-exact.
constexpr double GF_DT_PERT = 0.5, GF_DP_BASE = 1.5e4, GF_DP_DEPTH = 3.0e4, GF_EPS = 1.0e-3, GF_DEL = 0.75e-3;
constexpr double GF_C_MB = 0.03, GF_W_UP = 1.0, GF_CF_MAX = 0.3;
constexpr int GF_NSCR = 4;

struct GfArgs {
  Dims d;
  int nk;
  long qsub;
  double dt;
  Tables tb;
  double *T, *qv;
  const double *pl, *zm, *dp, *kpbl, *hfx;
  double *qlcn, *qicn, *cf, *mb, *k22, *kbcon, *ktop;
  double* scr;  // GF_NSCR * nk planes per sub-domain
};

__global__ void __launch_bounds__(256) cup_gf_sh_k(GfArgs a) {
  int s;
  long o;
  if (!col_point(a.d, s, o)) return;
  const long P = a.d.plane;
  const int n = a.nk;
  double* __restrict__ T = a.T + (long)s * n * P + o;
  double* __restrict__ QV = a.qv + (long)s * a.qsub * P + o;
  const double* __restrict__ PL = a.pl + (long)s * n * P + o;
  const double* __restrict__ ZM = a.zm + (long)s * n * P + o;
  const double* __restrict__ DP = a.dp + (long)s * n * P + o;
  double* __restrict__ HC = a.scr + (long)s * GF_NSCR * n * P + o;
  double* __restrict__ QT = HC + (long)n * P;
  double* __restrict__ ZU = QT + (long)n * P;
  double* __restrict__ QC = ZU + (long)n * P;
  const long p2 = (long)s * P + o;
  const double kpd = a.kpbl[p2], hf = a.hfx[p2];
  a.mb[p2] = 0.0;
  a.k22[p2] = -1.0;
  a.kbcon[p2] = -1.0;
  a.ktop[p2] = -1.0;
  for (int k = 0; k < n; ++k) a.cf[(long)(s * n + k) * P + o] = 0.0;
  auto L = [&](int k) { return (long)k * P; };
  // environment at level k: h, h*, qsat, gamma
  auto env = [&](int k, double& h, double& hs, double& qs, double& gm) {
    const double t = T[L(k)];
    double dqs;
    qsat(a.tb, false, t, PL[L(k)], qs, dqs);
    h = CP_AIR * t + GRAV * ZM[L(k)] + HLV * QV[L(k)];
    hs = CP_AIR * t + GRAV * ZM[L(k)] + HLV * qs;
    gm = HLV / CP_AIR * dqs;
  };
  const int kp = (int)kpd;
  double hx, hsx, qsx, gx;
  env(n - 1, hx, hsx, qsx, gx);
  int k22 = n - 1;
  double h22 = hx;
  for (int k = n - 2; k >= kp; --k) {
    env(k, hx, hsx, qsx, gx);
    if (hx > h22) {
      k22 = k;
      h22 = hx;
    }
  }
  const double hp = h22 + CP_AIR * GF_DT_PERT;
  const double qp = QV[L(k22)];
  const double pl22 = PL[L(k22)];
  int kb = -1;
  for (int k = k22; k >= 0; --k) {
    if (PL[L(k)] < pl22 - GF_DP_BASE) break;
    env(k, hx, hsx, qsx, gx);
    if (hp >= hsx) {
      kb = k;
      break;
    }
  }
  if (kb < 1 || hf <= 0.0) return;
  HC[L(kb)] = hp;
  QT[L(kb)] = qp;
  ZU[L(kb)] = 1.0;
  int kt = kb;
  const double plb = PL[L(kb)];
  {
    double hcp = hp, qtp = qp, zup = 1.0, zp = ZM[L(kb)];
    for (int k = kb - 1; k >= 0; --k) {
      if (PL[L(k)] < plb - GF_DP_DEPTH) break;
      const double zk = ZM[L(k)];
      const double dz = zk - zp;
      const double aa = 0.5 * GF_EPS * dz;
      env(k, hx, hsx, qsx, gx);
      const double hn = (hcp * (1.0 - aa) + 2.0 * aa * hx) / (1.0 + aa);
      if (hn < hsx) break;
      const double qn = (qtp * (1.0 - aa) + 2.0 * aa * QV[L(k)]) / (1.0 + aa);
      const double zn = zup * (1.0 + (GF_EPS - GF_DEL) * dz);
      HC[L(k)] = hn;
      QT[L(k)] = qn;
      ZU[L(k)] = zn;
      hcp = hn;
      qtp = qn;
      zup = zn;
      zp = zk;
      kt = k;
    }
  }
  if (kt == kb) return;
  for (int k = k22; k > kb; --k) {
    HC[L(k)] = hp;
    QT[L(k)] = qp;
    ZU[L(k)] = 1.0;
  }
  for (int k = kt; k <= kb; ++k) {
    env(k, hx, hsx, qsx, gx);
    const double qsat_c = qsx + gx / (1.0 + gx) * (HC[L(k)] - hsx) / HLV;
    QC[L(k)] = fmax(QT[L(k)] - qsat_c, 0.0);
  }
  // flux-form tendencies per unit mb (the eddy flux through the upper interface of layer k
  // is zero at kt and below k22)
  auto eflux = [&](int k, double& eh, double& eq) {
    if (k <= kt || k > k22) {
      eh = 0.0;
      eq = 0.0;
      return;
    }
    double h, hs, qs, gm;
    env(k, h, hs, qs, gm);
    const double zu = ZU[L(k)];
    eh = zu * (HC[L(k)] - h);
    eq = zu * (QT[L(k)] - QV[L(k)]);
  };
  const double dc = GRAV * ZU[L(kt + 1)] * QC[L(kt + 1)] / DP[L(kt)];
  const double dt = a.dt;
  // closure and the vapour limiter
  const double tb = T[L(n - 1)];
  const double rhob = PL[L(n - 1)] / (RDGAS * tb);
  const double zi = ZM[L(kp)];
  const double wst = cbrt(GRAV / tb * hf / (rhob * CP_AIR) * zi);
  double mb = GF_C_MB * (PL[L(k22)] / (RDGAS * T[L(k22)])) * wst;
  {
    double eha, eqa, ehb, eqb;
    eflux(kt, eha, eqa);
    for (int k = kt; k <= k22; ++k) {
      eflux(k + 1, ehb, eqb);
      double dqv = GRAV * (eqb - eqa) / DP[L(k)];
      if (k == kt) dqv = dqv - dc;
      if (dqv < 0.0) mb = fmin(mb, 0.9 * QV[L(k)] / (-dt * dqv));
      eha = ehb;
      eqa = eqb;
    }
  }
  if (!(mb > 0.0)) return;
  // cloud fraction (initial-state density), then the tendencies (fluxes from the initial
  // state: each level's two interface fluxes are formed before the level is updated)
  for (int k = kt; k <= kb; ++k) {
    const double rho = PL[L(k)] / (RDGAS * T[L(k)]);
    a.cf[(long)(s * n + k) * P + o] = fmin(GF_CF_MAX, mb * ZU[L(k)] / (rho * GF_W_UP));
  }
  {
    double eha, eqa, ehb, eqb;
    eflux(kt, eha, eqa);
    for (int k = kt; k <= k22; ++k) {
      eflux(k + 1, ehb, eqb);
      const double dh = GRAV * (ehb - eha) / DP[L(k)];
      double dq = GRAV * (eqb - eqa) / DP[L(k)];
      if (k == kt) dq = dq - dc;
      const double dqk = mb * dq;
      const double t0 = T[L(k)], q0 = QV[L(k)];
      QV[L(k)] = q0 + dt * dqk;
      T[L(k)] = t0 + dt * (mb * dh - HLV * dqk) / CP_AIR;
      eha = ehb;
      eqa = eqb;
    }
  }
  const double fi = fmin(fmax((T_ICE - T[L(kt)]) / 40.0, 0.0), 1.0);
  const long xt = (long)(s * n + kt) * P + o;
  a.qicn[xt] = a.qicn[xt] + dt * mb * dc * fi;
  a.qlcn[xt] = a.qlcn[xt] + dt * mb * dc * (1.0 - fi);
  a.mb[p2] = mb;
  a.k22[p2] = (double)k22;
  a.kbcon[p2] = (double)kb;
  a.ktop[p2] = (double)kt;
}

// layer pressure from the interfaces, layer-mid heights from delz (surface at 0), and the
// PBL-top level index: the highest level whose mid height is below Z_PBL
constexpr double Z_PBL = 1000.0;
__global__ void __launch_bounds__(256) moist_prep_k(Dims d, int nk, const double* __restrict__ pe,
                                                     const double* __restrict__ dz, double* __restrict__ pl,
                                                     double* __restrict__ zm, double* __restrict__ kpbl) {
  int s;
  long o;
  if (!col_point(d, s, o)) return;
  const long P = d.plane;
  const long b = (long)s * nk * P + o, be = (long)s * (nk + 1) * P + o;
  double zb = 0.0;
  int kp = nk - 1;
  for (int k = nk - 1; k >= 0; --k) {
    const double zt = zb - dz[b + k * P];
    const double z = 0.5 * (zt + zb);
    zm[b + k * P] = z;
    pl[b + k * P] = 0.5 * (pe[be + k * P] + pe[be + (k + 1) * P]);
    if (z < Z_PBL) kp = k;
    zb = zt;
  }
  kpbl[(long)s * P + o] = (double)kp;
}

// ---- buoyancy, CAPE / CIN, LCL index (one bottom-up pass) ----
__global__ void __launch_bounds__(256) buoyancy_k(Dims d, int nk, Tables tb, const double* __restrict__ t,
                                                  const double* __restrict__ qv, const double* __restrict__ pm,
                                                  const double* __restrict__ zm, double* __restrict__ by,
                                                  double* __restrict__ cape, double* __restrict__ cin,
                                                  double* __restrict__ klcl) {
  int s;
  long o;
  if (!col_point(d, s, o)) return;
  const Col3 c{d, s, nk, o};
  const int kb = nk - 1;
  const double tb0 = t[c.at(kb)], pb0 = pm[c.at(kb)], qb0 = qv[c.at(kb)], zb0 = zm[c.at(kb)];
  const double hp = CP_AIR * tb0 + GRAV * zb0 + HLV * qb0;
  double ca = 0.0, ci = 0.0, kl = -1.0, zprev = zb0;
  bool fr = false;
  for (int k = kb; k >= 0; --k) {
    const long x = c.at(k);
    const double tk = t[x], pk = pm[x], zk = zm[x];
    double qs, dqs;
    qsat(tb, false, tk, pk, qs, dqs);
    const double gam = HLV / CP_AIR * dqs;
    const double hs = CP_AIR * tk + GRAV * zk + HLV * qs;
    const double b = GRAV * (hp - hs) / (CP_AIR * tk * (1.0 + gam));
    by[x] = b;
    if (k < kb) {
      const double dzk = zk - zprev;
      fr = fr || b > 0.0;
      ca = ca + (b > 0.0 ? b * dzk : 0.0);
      ci = ci + ((b < 0.0 && !fr) ? b * dzk : 0.0);
    }
    zprev = zk;
    const double tpar = tb0 * exp(KAPPA * log(pk / pb0));
    double qsp, dqsp;
    qsat(tb, false, tpar, pk, qsp, dqsp);
    if (kl < 0.0 && qb0 >= qsp) kl = (double)k;
  }
  const long p2 = (long)s * d.plane + o;
  cape[p2] = ca;
  cin[p2] = ci;
  klcl[p2] = kl;
}

// host tables, one device copy per HIP device
double es_w(double t) {
  const double fac0 = (t - T_ICE) / (t * T_ICE);
  return E00 * std::exp((DC_VAP * std::log(t / T_ICE) + LV0 * fac0) / RVGAS);
}
double es_i(double t) {
  const double fac0 = (t - T_ICE) / (t * T_ICE);
  return E00 * std::exp((D2ICE * std::log(t / T_ICE) + LI2 * fac0) / RVGAS);
}

Tables device_tables() {
  static std::mutex mu;
  static std::map<int, double*> cache;
  int dev = 0;
  HIP_CHECK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(dev);
  if (it == cache.end()) {
    std::vector<double> h(4 * TABLE_N, 0.0);
    double *tw = h.data(), *ti = tw + TABLE_N, *dw = ti + TABLE_N, *di = dw + TABLE_N;
    for (int n = 0; n < TABLE_N; ++n) {
      const double t = TABLE_T0 + TABLE_DT * (double)n;
      tw[n] = es_w(t);
      ti[n] = t < T_ICE ? es_i(t) : es_w(t);
    }
    for (int n = 0; n + 1 < TABLE_N; ++n) {
      dw[n] = tw[n + 1] - tw[n];
      di[n] = ti[n + 1] - ti[n];
    }
    double* dptr = nullptr;
    HIP_CHECK(hipMalloc(&dptr, sizeof(double) * h.size()));
    HIP_CHECK(hipMemcpy(dptr, h.data(), sizeof(double) * h.size(), hipMemcpyHostToDevice));
    it = cache.emplace(dev, dptr).first;
  }
  double* p = it->second;
  return Tables{p, p + TABLE_N, p + 2 * TABLE_N, p + 3 * TABLE_N};
}

inline dim3 colgrid(const Dims& d) { return dim3(cdiv(d.nx, BX), cdiv(d.ny, BY), d.nsub); }
inline dim3 ptgrid(const Dims& d, int nk) { return dim3(cdiv(d.nx, BX), cdiv(d.ny, BY), d.nsub * nk); }

// GFDL MP coefficients on the host, as oracle/gfdl_mp.py forms them
MpConst mp_const(double dts) {
  const double PIE = 3.14159265358979323846;
  const double RNZR = 8.0e6, RNZS = 3.0e6, RNZG = 4.0e6, RHOR = 1.0e3, RHOS = 1.0e2, RHOG = 4.0e2;
  const double ALIN = 842.0, CLIN = 4.8, GCON = 40.74 * std::sqrt(1.2);
  const double VDIFU = 2.11e-5, TCOND = 2.36e-2, VISK = 1.259e-5;
  const double ACT_S = PIE * RNZS * RHOS, ACT_R = PIE * RNZR * RHOR, ACT_G = PIE * RNZG * RHOG;
  const double SCM3 = std::pow(VISK / VDIFU, 1.0 / 3.0);
  MpConst k{};
  k.cracw = PIE * RNZR * ALIN * std::tgamma(3.8) / (4.0 * std::pow(ACT_R, 0.95));
  k.csacw = PIE * RNZS * CLIN * std::tgamma(3.25) / (4.0 * std::pow(ACT_S, 0.8125));
  k.cgacw = PIE * RNZG * std::tgamma(3.5) * GCON / (4.0 * std::pow(ACT_G, 0.875));
  k.crevp[0] = 2.0 * PIE * VDIFU * TCOND * RVGAS * RNZR;
  k.crevp[1] = 0.78 / std::sqrt(ACT_R);
  k.crevp[2] = 0.31 * SCM3 * std::tgamma(2.9) * std::sqrt(ALIN / VISK) / std::pow(ACT_R, 0.725);
  k.crevp[3] = TCOND * RVGAS;
  k.crevp[4] = HLV * HLV * VDIFU;
  k.e_imlt = 1.0 - std::exp(-dts / 600.0);
  k.e_smlt = 1.0 - std::exp(-dts / 900.0);
  k.e_gmlt = 1.0 - std::exp(-dts / 600.0);
  k.e_l2v = 1.0 - std::exp(-dts / 300.0);
  k.e_v2l = 1.0 - std::exp(-dts / 150.0);
  k.e_i2v = 1.0 - std::exp(-dts / 300.0);
  return k;
}


}  // namespace moist

void moist_qsat(const Ctx& c, int nk, const double* t, const double* p, double* qsw, double* qsi, double* dqsw) {
  const Dims& d = c.d;
  GT_LAUNCH(moist::qsat_k, dim3(cdiv(d.nx, BX), cdiv(d.ny, BY), d.nsub * nk), dim3(BX, BY), 0, c.st, d, nk,
            moist::device_tables(), t, p, qsw, qsi, dqsw);
  HIP_LAUNCH_CHECK();
}

void fillq2zero(const Ctx& c, int nk, double* q, const double* dp, double* fill) {
  GT_LAUNCH(moist::fillq2zero_k, moist::colgrid(c.d), dim3(BX, BY), 0, c.st, c.d, nk, q, dp, fill);
  HIP_LAUNCH_CHECK();
}

int gfdl_mp_scratch_levels(int nk) { return moist::MP_NSCR * (nk + 1); }

void gfdl_1m(const Ctx& c, const Gfdl1mArgs& g) {
  if (!g.scr) throw std::runtime_error("gfdl_1m: scratch planes required");
  if (g.nk < 3) throw std::runtime_error("gfdl_1m: nk >= 3 required");
  const double mp_time = 150.0;
  const int ntimes = std::max(1, (int)std::ceil(g.dt / mp_time - 1.0e-9));
  const double dts = g.dt / ntimes;
  moist::MpArgs a{c.d, g.nk, g.qsub > 0 ? g.qsub : g.nk, ntimes, dts, moist::device_tables(), moist::mp_const(dts),
                  g.T, g.qv, g.ql, g.qr, g.qi, g.qs, g.qg, g.dp, g.dz, g.scr, g.pr, g.ps, g.pg, g.pi};
  // the level-block form where a shape holds the column with its last two levels in one block
  // (NB M >= nk, nk mod M != 1); else (or variant 1) the column driver
  const int nk = g.nk, ncol = c.d.nx * c.d.ny;
  auto blk = [&](auto Mc, auto NBc) {
    constexpr int M = decltype(Mc)::value, NB = decltype(NBc)::value;
    if (g.variant == 1 || NB * M < nk || (NB - 1) * M >= nk + M || nk % M == 1) return false;
    const dim3 grid(cdiv(cdiv(ncol, 64 / NB), moist::MB_WAVES), 1, c.d.nsub);
    GT_LAUNCH((moist::mpdrv_blk_k<M, NB>), grid, dim3(64 * moist::MB_WAVES), 0, c.st, a);
    return true;
  };
  using std::integral_constant;
  const bool done = blk(integral_constant<int, 2>{}, integral_constant<int, 8>{}) ||
                    blk(integral_constant<int, 2>{}, integral_constant<int, 16>{}) ||
                    blk(integral_constant<int, 3>{}, integral_constant<int, 16>{}) ||
                    blk(integral_constant<int, 4>{}, integral_constant<int, 16>{}) ||
                    blk(integral_constant<int, 5>{}, integral_constant<int, 16>{});
  if (!done) GT_LAUNCH(moist::mpdrv_k, moist::colgrid(c.d), dim3(BX, BY), 0, c.st, a);
  HIP_LAUNCH_CHECK();
  // algorithmic bytes: T + 6 species read and written, dp dz read (L each), 4 surface fields
  ktimer_bytes(8.0 * c.d.nx * c.d.ny * c.d.nsub * (16.0 * g.nk + 4.0));
}

void evap_subl_pdf(const Ctx& c, const EvapSublArgs& g) {
  const double e_frz = 1.0 - std::exp(-g.dt / 450.0), e_mlt = 1.0 - std::exp(-g.dt / 450.0);
  moist::EspArgs a{c.d, g.nk, g.dt, e_frz, e_mlt, moist::device_tables(), g.T, g.qv, g.qlls, g.qils, g.qlcn, g.qicn,
                   g.clls, g.clcn, g.qv_sub > 0 ? g.qv_sub : g.nk, g.ql_sub > 0 ? g.ql_sub : g.nk,
                   g.qi_sub > 0 ? g.qi_sub : g.nk, g.pl, g.nactl, g.nacti};
  GT_LAUNCH(moist::evap_subl_pdf_k, moist::ptgrid(c.d, g.nk), dim3(BX, BY), 0, c.st, a);
  HIP_LAUNCH_CHECK();
  // T qv qlls qils qlcn qicn clls clcn read and written, pl nactl read
  ktimer_bytes(8.0 * c.d.nx * c.d.ny * c.d.nsub * g.nk * 18.0);
}

void radcouple(const Ctx& c, const RadcoupleArgs& g) {
  auto sub = [&](long v) { return v > 0 ? v : (long)g.nk; };
  moist::RadArgs a{c.d, g.nk, sub(g.qv_sub), sub(g.ql_sub), sub(g.qi_sub), sub(g.qr_sub), sub(g.qs_sub), sub(g.qg_sub),
                   g.T, g.pl, g.cf, g.af, g.qv, g.qlls, g.qils, g.qlcn, g.qicn, g.qr, g.qs, g.qg, g.nl,
                   g.rqv, g.rql, g.rqi, g.rqr, g.rqs, g.rqg, g.rcf, g.rrl, g.rri};
  GT_LAUNCH(moist::radcouple_k, moist::ptgrid(c.d, g.nk), dim3(BX, BY), 0, c.st, a);
  HIP_LAUNCH_CHECK();
  ktimer_bytes(8.0 * c.d.nx * c.d.ny * c.d.nsub * g.nk * 22.0);
}

void aer_activation(const Ctx& c, int nk, long qv_sub, const double* pl, const double* t, const double* qv,
                    const double* zm, const double* w, double* nactl, double* nacti, double* smax) {
  moist::AerArgs a{c.d, nk, qv_sub > 0 ? qv_sub : nk, moist::device_tables(), pl, t, qv, zm, w, nactl, nacti, smax, {}};
  for (int m = 0; m < 3; ++m) {
    const moist::AerMode& md = moist::kAerModes[m];
    const double ls = std::log(md.sg);
    a.mode[m] = {md.n0, md.h, 3.0 * md.rd, 2.0 / std::sqrt(md.kap), ls, 0.5 * std::exp(2.5 * ls * ls), 1.0 + 0.25 * ls};
  }
  GT_LAUNCH(moist::aer_activation_k, moist::ptgrid(c.d, nk), dim3(BX, BY), 0, c.st, a);
  HIP_LAUNCH_CHECK();
  ktimer_bytes(8.0 * c.d.nx * c.d.ny * c.d.nsub * nk * 8.0);
}

int gf_scratch_levels(int nk) { return moist::GF_NSCR * nk; }

void cup_gf_sh(const Ctx& c, const GfShArgs& g) {
  if (!g.scr) throw std::runtime_error("cup_gf_sh: scratch planes required");
  if (g.nk < 3) throw std::runtime_error("cup_gf_sh: nk >= 3 required");
  moist::GfArgs a{c.d, g.nk, g.qv_sub > 0 ? g.qv_sub : g.nk, g.dt, moist::device_tables(), g.T, g.qv, g.pl, g.zm, g.dp,
                  g.kpbl, g.hfx, g.qlcn, g.qicn, g.cf, g.mb, g.k22, g.kbcon, g.ktop, g.scr};
  GT_LAUNCH(moist::cup_gf_sh_k, moist::colgrid(c.d), dim3(BX, BY), 0, c.st, a);
  HIP_LAUNCH_CHECK();
  // T qv read and written, pl zm dp read, cf written (L each); qlcn qicn at one level
  ktimer_bytes(8.0 * c.d.nx * c.d.ny * c.d.nsub * (8.0 * g.nk + 9.0));
}

void moist_prep(const Ctx& c, int nk, const double* pe, const double* dz, double* pl, double* zm, double* kpbl) {
  GT_LAUNCH(moist::moist_prep_k, moist::colgrid(c.d), dim3(BX, BY), 0, c.st, c.d, nk, pe, dz, pl, zm, kpbl);
  HIP_LAUNCH_CHECK();
  ktimer_bytes(8.0 * c.d.nx * c.d.ny * c.d.nsub * (4.0 * nk + 1.0));
}

void buoyancy(const Ctx& c, int nk, const double* t, const double* qv, const double* pm, const double* zm,
              double* by, double* cape, double* cin, double* klcl) {
  GT_LAUNCH(moist::buoyancy_k, moist::colgrid(c.d), dim3(BX, BY), 0, c.st, c.d, nk, moist::device_tables(), t, qv,
            pm, zm, by, cape, cin, klcl);
  HIP_LAUNCH_CHECK();
}

}  // namespace gtfv3
