// moist.hip — moist column physics for gfx950.
//
// The GEOS moist schemes the Aquaplanet configuration runs (GFDL 1M driver chain,
// buoyancy, fillq2zero: geos_documentation/moist/GFDL_1M.drawio:70-618,
// experiments.yaml:42-110) live outside the reference; these kernels restate the
// published algorithms (Lin et al. 1983, Chen & Lin 2013, Kessler 1969, Klemp &
// Wilhelmson 1978; GFDL MP qs_table / implicit_fall) — oracle/moist.py holds the same
// expressions in numpy, parity unpinned by reference data.
//
// Decomposition: the K axis is never split; one lane per column,
// i-fastest, so every level access of a wavefront is one coalesced 64-wide row.  The
// whole GFDL-style step is ONE top-down pass per column: the implicit sedimentation of
// each species at level k depends only on the levels above (a carried flux), and every
// other process is pointwise in the column, so level k is final once it is reached —
// each field is read once and written once (no column scratch, unlike the dycore's
// tridiagonal sweeps).  Saturation vapour pressure comes from 0.1 K tables built on the
// host with the C library's exp/log (bit-identical to the oracle's tables) and read
// with linear interpolation (GFDL wqs1 / iqs1 style).
#include <cmath>
#include <map>
#include <mutex>
#include <vector>

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
constexpr double RHO_SFC = 1.2;
constexpr double VR_MIN = 1.0e-3, VR_MAX = 12.0, VS_MAX = 2.0, VG_MAX = 12.0, VI_MAX = 1.0;
constexpr double QMIN_FALL = 1.0e-8;
// process constants
constexpr double C_AUT = 1.0e-3, QL_CRIT = 5.0e-4;  // Kessler autoconversion
constexpr double C_ACC = 2.2;                       // Kessler accretion
constexpr double T_HOM = T_ICE - 40.0;              // homogeneous freezing
constexpr double TAU_DEP = 600.0, TAU_MLT = 600.0;  // deposition / melting relaxation (s)

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

// ---- GFDL-1M-style column step (one top-down pass) ----
struct Fall {  // implicit_fall carry: dd(k-1) * qm(k-1)
  double carry = 0.0;
  // new mixing ratio at level k, given the level's mass, fall distance and thickness
  __device__ __forceinline__ double step(double q, double dp, double dz, double dd) {
    const double m = q * dp / GRAV;
    const double qm = (m + carry) / (dz + dd);
    carry = dd * qm;
    return qm * dz * GRAV / dp;
  }
};

struct M1Args {
  Dims d;
  int nk, qsub;  // levels; levels per sub-domain of the species arrays (nk, or nq*nk in q)
  double dt;
  Tables tb;
  double *T, *qv, *ql, *qr, *qi, *qs, *qg;
  const double *dp, *dz, *pm, *pe;  // pm null: layer pressure from the interfaces pe (L+1)
  double *pr, *ps, *pg, *pi;
};

__global__ void __launch_bounds__(256) gfdl_1m_k(M1Args a) {
  int s;
  long o;
  if (!col_point(a.d, s, o)) return;
  const Col3 c{a.d, s, a.nk, o};
  const double dt = a.dt;
  const double lcp = HLV / CP_AIR, icp = HLF / CP_AIR, scp = HLS / CP_AIR;
  const double fdep = 1.0 - exp(-dt / TAU_DEP), fmlt = 1.0 - exp(-dt / TAU_MLT);
  Fall fi, fs, fg, fr;
  for (int k = 0; k < a.nk; ++k) {
    const long x = c.at(k);
    const long y = ((long)s * a.qsub + k) * a.d.plane + o;  // species
    double T = a.T[x], qv = a.qv[y], ql = a.ql[y], qr = a.qr[y], qi = a.qi[y], qs = a.qs[y], qg = a.qg[y];
    double pm;
    if (a.pm) {
      pm = a.pm[x];
    } else {
      const long e = ((long)s * (a.nk + 1) + k) * a.d.plane + o;
      pm = 0.5 * (a.pe[e] + a.pe[e + a.d.plane]);
    }
    const double dp = a.dp[x], thick = -a.dz[x];
    // 1. neg_adj
    {
      double n;
      n = fmin(ql, 0.0); qv += n; T -= n * lcp; ql -= n;
      n = fmin(qr, 0.0); qv += n; T -= n * lcp; qr -= n;
      n = fmin(qi, 0.0); qv += n; T -= n * scp; qi -= n;
      n = fmin(qs, 0.0); qv += n; T -= n * scp; qs -= n;
      n = fmin(qg, 0.0); qv += n; T -= n * scp; qg -= n;
    }
    // 2-3. fall speeds, implicit sedimentation (carried from the level above)
    const double den = dp / (GRAV * thick);
    const double rhof = sqrt(fmin(10.0, RHO_SFC / den));
    const double vr = qr > QMIN_FALL
                          ? fmin(VR_MAX, fmax(VR_MIN, VCONR * rhof * exp(0.2 * log(fmax(qr, QMIN_FALL) * den / NORMR))))
                          : VR_MIN;
    const double vs =
        qs > QMIN_FALL ? fmin(VS_MAX, VCONS * rhof * exp(0.0625 * log(fmax(qs, QMIN_FALL) * den / NORMS))) : 0.0;
    const double vg =
        qg > QMIN_FALL ? fmin(VG_MAX, VCONG * rhof * sqrt(sqrt(sqrt(fmax(qg, QMIN_FALL) * den / NORMG)))) : 0.0;
    const double vi = qi > QMIN_FALL ? fmin(VI_MAX, 3.29 * exp(0.16 * log(fmax(qi, QMIN_FALL) * den))) : 0.0;
    qi = fi.step(qi, dp, thick, dt * vi);
    qs = fs.step(qs, dp, thick, dt * vs);
    qg = fg.step(qg, dp, thick, dt * vg);
    qr = fr.step(qr, dp, thick, dt * vr);
    // 4. warm rain
    const double aut = fmin(ql, dt * C_AUT * fmax(ql - QL_CRIT, 0.0));
    ql = ql - aut;
    qr = qr + aut;
    const double acc = qr > 0.0 ? fmin(ql, dt * C_ACC * ql * exp(0.875 * log(fmax(qr, 1.0e-30)))) : 0.0;
    ql = ql - acc;
    qr = qr + acc;
    double qsw, dqsw;
    qsat(a.tb, false, T, pm, qsw, dqsw);
    {
      const double rq = den * qr;
      const double cvent = 1.6 + 124.9 * exp(0.2046 * log(fmax(rq, 1.0e-30)));
      const double erate =
          (1.0 - qv / qsw) * cvent * exp(0.525 * log(fmax(rq, 1.0e-30))) / (den * (5.4e5 + 2.55e8 / (pm * qsw)));
      const double evap =
          (qv < qsw && qr > 0.0) ? fmin(fmin(qr, dt * erate), (qsw - qv) / (1.0 + lcp * dqsw)) : 0.0;
      qr = qr - evap;
      qv = qv + evap;
      T = T - evap * lcp;
    }
    // 5. saturation adjustment of cloud water
    qsat(a.tb, false, T, pm, qsw, dqsw);
    {
      double dq = (qv - qsw) / (1.0 + lcp * dqsw);
      dq = dq > 0.0 ? dq : fmax(dq, -ql);
      qv = qv - dq;
      ql = ql + dq;
      T = T + dq * lcp;
    }
    // 6. homogeneous freezing
    {
      const double frz = T < T_HOM ? ql : 0.0;
      ql = ql - frz;
      qi = qi + frz;
      T = T + frz * icp;
    }
    // 7. ice deposition / sublimation
    {
      double qsi, dqsi;
      qsat(a.tb, true, T, pm, qsi, dqsi);
      double ddep = fdep * (qv - qsi) / (1.0 + scp * dqsi);
      ddep = T < T_ICE ? (ddep > 0.0 ? ddep : fmax(ddep, -qi)) : 0.0;
      qv = qv - ddep;
      qi = qi + ddep;
      T = T + ddep * scp;
    }
    // 8. melting: ice -> cloud water, snow and graupel -> rain
    {
      double cap = fmax(T - T_ICE, 0.0) / icp;
      double mlt = T > T_ICE ? fmin(fmlt * qi, cap) : 0.0;
      qi -= mlt; ql = ql + mlt; T = T - mlt * icp;
      cap = fmax(T - T_ICE, 0.0) / icp;
      mlt = T > T_ICE ? fmin(fmlt * qs, cap) : 0.0;
      qs -= mlt; qr = qr + mlt; T = T - mlt * icp;
      cap = fmax(T - T_ICE, 0.0) / icp;
      mlt = T > T_ICE ? fmin(fmlt * qg, cap) : 0.0;
      qg -= mlt; qr = qr + mlt; T = T - mlt * icp;
    }
    a.T[x] = T; a.qv[y] = qv; a.ql[y] = ql; a.qr[y] = qr; a.qi[y] = qi; a.qs[y] = qs; a.qg[y] = qg;
  }
  const long p2 = (long)s * a.d.plane + o;
  a.pr[p2] = fr.carry;
  a.ps[p2] = fs.carry;
  a.pg[p2] = fg.carry;
  a.pi[p2] = fi.carry;
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

void gfdl_1m(const Ctx& c, const Gfdl1mArgs& g) {
  if (!g.pm && !g.pe) throw std::runtime_error("gfdl_1m: layer pressure (pm) or interfaces (pe) required");
  moist::M1Args a{c.d, g.nk, g.qsub > 0 ? g.qsub : g.nk, g.dt, moist::device_tables(), g.T, g.qv, g.ql, g.qr,
                  g.qi, g.qs, g.qg, g.dp, g.dz, g.pm, g.pe, g.pr, g.ps, g.pg, g.pi};
  GT_LAUNCH(moist::gfdl_1m_k, moist::colgrid(c.d), dim3(BX, BY), 0, c.st, a);
  HIP_LAUNCH_CHECK();
  // algorithmic bytes: T + 6 species read and written, dp dz pm read (L each), 4 surface fields
  ktimer_bytes(8.0 * c.d.nx * c.d.ny * c.d.nsub * (17.0 * g.nk + 4.0));
}

void buoyancy(const Ctx& c, int nk, const double* t, const double* qv, const double* pm, const double* zm,
              double* by, double* cape, double* cin, double* klcl) {
  GT_LAUNCH(moist::buoyancy_k, moist::colgrid(c.d), dim3(BX, BY), 0, c.st, c.d, nk, moist::device_tables(), t, qv,
            pm, zm, by, cape, cin, klcl);
  HIP_LAUNCH_CHECK();
}

}  // namespace gtfv3
