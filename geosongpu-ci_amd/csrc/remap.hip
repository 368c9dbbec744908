// remap.hip — Lagrangian_to_Eulerian (FV3 fv_mapz) on gfx950: cs_profile (PPM,
// kord = 9, cs_limiters), map1_ppm (two-pointer exact integration), fillz, and
// the per-column state conversion; one column per lane (lanes = consecutive i,
// every k-plane access coalesced), per-column work arrays in scratch planes.
#include "kernels_nh.hpp"
#include "stencil_common.hpp"

namespace gtfv3 {
namespace {

constexpr double GRAV = Constants::grav;
constexpr double RDGAS = Constants::rdgas;
constexpr double KAPPA = Constants::kappa;
constexpr double R3 = 1.0 / 3.0, R23 = 2.0 / 3.0, R12 = 1.0 / 12.0;

struct Col {
  double* p;
  long st;
  __device__ __forceinline__ double& operator[](int k) const { return p[(long)k * st]; }
};
__device__ __forceinline__ Col col(double* f, const Dims& d, int s, int nk, long o) {
  return Col{f + (long)s * nk * d.plane + o, d.plane};
}

struct Prof {
  Col AL, AR, A6, Q, G;  // Q: edges (km+1), G: gam / gradient scratch (km+1)
};

__device__ __forceinline__ void lim(double a, double& AL, double& AR, double& A6, bool extm, int iv) {
  if (iv == 0) {
    if (a <= 0.0) {
      AL = a; AR = a; A6 = 0.0;
      return;
    }
    if (fabs(AR - AL) < -A6) {
      if ((a + 0.25 * ((AR - AL) * (AR - AL)) / A6 + A6 * R12) < 0.0) {
        if (a < AR && a < AL) {
          AR = a; AL = a; A6 = 0.0;
        } else if (AR > AL) {
          A6 = 3.0 * (AL - a);
          AR = AL - A6;
        } else {
          A6 = 3.0 * (AR - a);
          AL = AR - A6;
        }
      }
    }
    return;
  }
  bool flat = iv == 1 ? (a - AL) * (a - AR) >= 0.0 : extm;
  if (flat) {
    AL = a; AR = a; A6 = 0.0;
    return;
  }
  double da1 = AR - AL;
  double da2 = da1 * da1;
  double a6da = A6 * da1;
  if (a6da < -da2) {
    A6 = 3.0 * (AL - a);
    AR = AL - A6;
  } else if (a6da > da2) {
    A6 = 3.0 * (AR - a);
    AL = AR - A6;
  }
}

// cs_profile (kord = 9) of layer means A with thicknesses DP
__device__ void cs_profile(const Col& A, const Col& DP, int km, int iv, double qs, const Prof& P) {
  const Col& q = P.Q;
  const Col& gam = P.G;
  if (iv == -2) {
    gam[1] = 0.5;
    q[0] = 1.5 * A[0];
    for (int e = 1; e < km - 1; ++e) {
      double grat = DP[e - 1] / DP[e];
      double bet = 2.0 + grat + grat - gam[e];
      q[e] = (3.0 * (A[e - 1] + A[e]) - q[e - 1]) / bet;
      gam[e + 1] = grat / bet;
    }
    double grat = DP[km - 2] / DP[km - 1];
    q[km - 1] = (3.0 * (A[km - 2] + A[km - 1]) - grat * qs - q[km - 2]) / (2.0 + grat + grat - gam[km - 1]);
    q[km] = qs;
    for (int e = km - 2; e >= 0; --e) q[e] = q[e] - gam[e + 1] * q[e + 1];
  } else {
    double grat = DP[1] / DP[0];
    double bet = grat * (grat + 0.5);
    q[0] = ((grat + grat) * (grat + 1.0) * A[0] + A[1]) / bet;
    gam[0] = (1.0 + grat * (grat + 1.5)) / bet;
    double d4 = grat;
    for (int e = 1; e < km; ++e) {
      d4 = DP[e - 1] / DP[e];
      bet = 2.0 + d4 + d4 - gam[e - 1];
      q[e] = (3.0 * (A[e - 1] + d4 * A[e]) - q[e - 1]) / bet;
      gam[e] = d4 / bet;
    }
    double a_bot = 1.0 + d4 * (d4 + 1.5);
    q[km] = (2.0 * d4 * (d4 + 1.0) * A[km - 1] + A[km - 2] - a_bot * q[km - 1]) / (d4 * (d4 + 0.5) - a_bot * gam[km - 1]);
    for (int e = km - 1; e >= 0; --e) q[e] = q[e] - gam[e] * q[e + 1];
  }
  // large-scale constraints (gam now reused as g[e] = A[e] - A[e-1])
  q[1] = fmin(q[1], fmax(A[0], A[1]));
  q[1] = fmax(q[1], fmin(A[0], A[1]));
  for (int e = 1; e < km; ++e) gam[e] = A[e] - A[e - 1];
  for (int e = 2; e < km - 1; ++e) {
    double qe = q[e];
    if (gam[e - 1] * gam[e + 1] > 0.0) {
      qe = fmin(qe, fmax(A[e - 1], A[e]));
      qe = fmax(qe, fmin(A[e - 1], A[e]));
    } else if (gam[e - 1] > 0.0) {
      qe = fmax(qe, fmin(A[e - 1], A[e]));
    } else {
      qe = fmin(qe, fmax(A[e - 1], A[e]));
      if (iv == 0) qe = fmax(0.0, qe);
    }
    q[e] = qe;
  }
  q[km - 1] = fmin(q[km - 1], fmax(A[km - 2], A[km - 1]));
  q[km - 1] = fmax(q[km - 1], fmin(A[km - 2], A[km - 1]));
  for (int l = 0; l < km; ++l) {
    P.AL[l] = q[l];
    P.AR[l] = q[l + 1];
  }
  auto extm = [&](int l) { return gam[l] * gam[l + 1] < 0.0; };  // interior layers only
  // top layer
  {
    double a = A[0], AL = P.AL[0], AR = P.AR[0], A6;
    if (iv == 0) AL = fmax(0.0, AL);
    else if (iv == -1 && AL * a <= 0.0) AL = 0.0;
    A6 = 3.0 * (2.0 * a - (AL + AR));
    lim(a, AL, AR, A6, false, 1);
    P.AL[0] = AL; P.AR[0] = AR; P.A6[0] = A6;
  }
  {
    double a = A[1], AL = P.AL[1], AR = P.AR[1];
    double A6 = 3.0 * (2.0 * a - (AL + AR));
    lim(a, AL, AR, A6, extm(1), 2);
    P.AL[1] = AL; P.AR[1] = AR; P.A6[1] = A6;
  }
  for (int l = 2; l < km - 2; ++l) {
    double a = A[l], AL = P.AL[l], AR = P.AR[l], A6;
    bool el = extm(l);
    if ((el && extm(l - 1)) || (el && extm(l + 1))) {
      AL = a; AR = a; A6 = 0.0;
    } else {
      A6 = 6.0 * a - 3.0 * (AL + AR);
      if (fabs(A6) > fabs(AL - AR)) {
        double pmp_1 = a - 2.0 * gam[l + 1];
        double lac_1 = pmp_1 + 1.5 * gam[l + 2];
        AL = fmin(fmax(AL, fmin(fmin(a, pmp_1), lac_1)), fmax(fmax(a, pmp_1), lac_1));
        double pmp_2 = a + 2.0 * gam[l];
        double lac_2 = pmp_2 - 1.5 * gam[l - 1];
        AR = fmin(fmax(AR, fmin(fmin(a, pmp_2), lac_2)), fmax(fmax(a, pmp_2), lac_2));
        A6 = 6.0 * a - 3.0 * (AL + AR);
      }
    }
    if (iv == 0) lim(a, AL, AR, A6, el, 0);
    P.AL[l] = AL; P.AR[l] = AR; P.A6[l] = A6;
  }
  {
    int l = km - 1;
    double AR = P.AR[l];
    if (iv == 0) AR = fmax(0.0, AR);
    else if (iv == -1 && AR * A[l] <= 0.0) AR = 0.0;
    P.AR[l] = AR;
  }
  for (int l = km - 2; l < km; ++l) {
    double a = A[l], AL = P.AL[l], AR = P.AR[l];
    double A6 = 3.0 * (2.0 * a - (AL + AR));
    lim(a, AL, AR, A6, l == km - 2 ? extm(l) : false, l == km - 2 ? 2 : 1);
    P.AL[l] = AL; P.AR[l] = AR; P.A6[l] = A6;
  }
}

// map1_ppm: A (layer means, km) on source edges PE1 -> OUT (kn layers) on target edges PE2
__device__ void map1(const Col& PE1, const Col& A, const Col& PE2, const Col& OUT, int km, int kn, int iv, double qs,
                     const Prof& P, const Col& DP1) {
  for (int l = 0; l < km; ++l) DP1[l] = PE1[l + 1] - PE1[l];
  cs_profile(A, DP1, km, iv, qs, P);
  int k0 = 0;
  for (int k = 0; k < kn; ++k) {
    const double top = PE2[k], bot = PE2[k + 1];
    for (int l = k0; l < km; ++l) {
      if (top >= PE1[l] && top <= PE1[l + 1]) {
        const double dpl = DP1[l];
        const double pl = (top - PE1[l]) / dpl;
        const double AL = P.AL[l], AR = P.AR[l], A6 = P.A6[l];
        if (bot <= PE1[l + 1]) {
          const double pr = (bot - PE1[l]) / dpl;
          OUT[k] = AL + 0.5 * (A6 + AR - AL) * (pr + pl) - A6 * R3 * (pr * (pr + pl) + pl * pl);
          k0 = l;
        } else {
          double qsum = (PE1[l + 1] - top) * (AL + 0.5 * (A6 + AR - AL) * (1.0 + pl) - A6 * (R3 * (1.0 + pl * (1.0 + pl))));
          for (int m = l + 1; m < km; ++m) {
            if (bot > PE1[m + 1]) {
              qsum = qsum + DP1[m] * A[m];
            } else {
              const double dp = bot - PE1[m];
              const double esl = dp / DP1[m];
              qsum = qsum + dp * (P.AL[m] + 0.5 * esl * (P.AR[m] - P.AL[m] + P.A6[m] * (1.0 - R23 * esl)));
              k0 = m;
              break;
            }
          }
          OUT[k] = qsum / (bot - top);
        }
        break;
      }
    }
  }
}

__device__ void fillz_col(const Col& q, const Col& dp, int km) {
  if (q[0] < 0.0) {
    q[1] = q[1] + q[0] * dp[0] / dp[1];
    q[0] = 0.0;
  }
  bool zfix = false;
  for (int k = 1; k < km - 1; ++k) {
    if (q[k] < 0.0) {
      zfix = true;
      if (q[k - 1] > 0.0) {
        double dq = fmin(q[k - 1] * dp[k - 1], -q[k] * dp[k]);
        q[k - 1] = q[k - 1] - dq / dp[k - 1];
        q[k] = q[k] + dq / dp[k];
      }
      if (q[k] < 0.0 && q[k + 1] > 0.0) {
        double dq = fmin(q[k + 1] * dp[k + 1], -q[k] * dp[k]);
        q[k + 1] = q[k + 1] - dq / dp[k + 1];
        q[k] = q[k] + dq / dp[k];
      }
    }
  }
  const int k = km - 1;
  if (q[k] < 0.0 && q[k - 1] > 0.0) {
    zfix = true;
    double qup = q[k - 1] * dp[k - 1];
    double qly = -q[k] * dp[k];
    double dup = fmin(qly, qup);
    q[k - 1] = q[k - 1] - dup / dp[k - 1];
    q[k] = q[k] + dup / dp[k];
  }
  if (zfix) {
    double sum0 = 0.0, sum1 = 0.0;
    for (int kk = 1; kk < km; ++kk) sum0 = sum0 + q[kk] * dp[kk];
    if (sum0 > 0.0) {
      for (int kk = 1; kk < km; ++kk) sum1 = sum1 + fmax(0.0, q[kk] * dp[kk]);
      double fac = sum0 / sum1;
      for (int kk = 1; kk < km; ++kk) {
        double dm = q[kk] * dp[kk];
        q[kk] = fmax(0.0, fac * dm / dp[kk]);
      }
    }
  }
}

__device__ __forceinline__ Prof prof_cols(const RemapScratch& r, const Dims& d, int s, int k1, long o) {
  Prof P;
  P.AL = col(r.s[0], d, s, k1, o);
  P.AR = col(r.s[1], d, s, k1, o);
  P.A6 = col(r.s[2], d, s, k1, o);
  P.Q = col(r.s[3], d, s, k1, o);
  P.G = col(r.s[4], d, s, k1, o);
  return P;
}

__global__ void __launch_bounds__(256) remap_scalar_k(Dims d, int npz, int nq, double ptop, int fill,
                                                      const double* __restrict__ ak, const double* __restrict__ bk,
                                                      RemapState S, RemapScratch R) {
  Launch2D L{0, 0, d.nx, d.ny};
  int i, j;
  if (!thread_point(L, i, j)) return;
  const int s = blockIdx.z;
  const long o = pidx(d, i, j);
  const int km = npz, k1 = npz + 1;
  const double rrg = -RDGAS / GRAV;
  const double k1k = KAPPA / (1.0 - KAPPA);
  Col PE1 = col(S.pe, d, s, k1, o), PELN = col(S.peln, d, s, k1, o), PK = col(S.pk, d, s, k1, o);
  Col DELP = col(S.delp, d, s, km, o), DELZ = col(S.delz, d, s, km, o), PT = col(S.pt, d, s, km, o);
  Col W = col(S.w, d, s, km, o), PKZ = col(S.pkz, d, s, km, o);
  Col PE2 = col(R.s[5], d, s, k1, o), PN2 = col(R.s[6], d, s, k1, o), A = col(R.s[7], d, s, k1, o),
      DP1 = col(R.s[8], d, s, k1, o), DP2 = col(R.s[9], d, s, k1, o), DZS = col(R.s[10], d, s, k1, o);
  Prof P = prof_cols(R, d, s, k1, o);
  // theta_v -> T_v (kord_tm < 0 remaps T_v in log p), delz -> specific volume / g
  for (int k = 0; k < km; ++k) {
    double pt = PT[k];
    A[k] = pt * exp(k1k * log(rrg * DELP[k] / DELZ[k] * pt));
    DZS[k] = -DELZ[k] / DELP[k];
  }
  const double psurf = PE1[km];
  S.ps[(long)s * d.plane + o] = psurf;
  PE2[0] = ptop;
  PE2[km] = psurf;
  for (int k = 1; k < km; ++k) PE2[k] = ak[k] + bk[k] * psurf;
  for (int k = 0; k < km; ++k) DP2[k] = PE2[k + 1] - PE2[k];
  PN2[0] = PELN[0];
  PN2[km] = PELN[km];
  for (int k = 1; k < km; ++k) PN2[k] = log(PE2[k]);
  // T_v in log(p)
  map1(PELN, A, PN2, PT, km, km, 1, 0.0, P, DP1);
  // tracers
  for (int iq = 0; iq < nq; ++iq) {
    Col Q = col(S.q + (long)iq * km * d.plane, d, s, nq * km, o);
    for (int k = 0; k < km; ++k) A[k] = Q[k];
    map1(PE1, A, PE2, Q, km, km, 0, 0.0, P, DP1);
    if (fill) fillz_col(Q, DP2, km);
  }
  // w (iv = -2 with the surface w as lower boundary value)
  const double ws = S.ws[(long)s * d.plane + o];
  for (int k = 0; k < km; ++k) A[k] = W[k];
  map1(PE1, A, PE2, W, km, km, -2, ws, P, DP1);
  // delz
  for (int k = 0; k < km; ++k) A[k] = DZS[k];
  map1(PE1, A, PE2, DELZ, km, km, 1, 0.0, P, DP1);
  for (int k = 0; k < km; ++k) {
    DELZ[k] = -DELZ[k] * DP2[k];
    DELP[k] = DP2[k];
  }
  for (int k = 0; k <= km; ++k) {
    PK[k] = exp(KAPPA * PN2[k]);
    PELN[k] = PN2[k];
  }
  for (int k = 0; k < km; ++k) PKZ[k] = exp(KAPPA * log(rrg * DELP[k] / DELZ[k] * PT[k]));
}

// staggered winds: u on x-edges (rows 0..ny, cols 0..nx-1), v on y-edges (cols 0..nx, rows 0..ny-1)
__global__ void __launch_bounds__(256) remap_wind_k(Dims d, int npz, const double* __restrict__ ak,
                                                    const double* __restrict__ bk, const double* __restrict__ pe,
                                                    double* __restrict__ u, double* __restrict__ v, RemapScratch R) {
  Launch2D L{0, 0, d.nx + 1, d.ny + 1};
  int i, j;
  if (!thread_point(L, i, j)) return;
  const int s = blockIdx.z;
  const long o = pidx(d, i, j);
  const int km = npz, k1 = npz + 1;
  Prof P = prof_cols(R, d, s, k1, o);
  Col PE0 = col(R.s[5], d, s, k1, o), PE3 = col(R.s[6], d, s, k1, o), A = col(R.s[7], d, s, k1, o),
      DP1 = col(R.s[8], d, s, k1, o);
  Col PE = col(const_cast<double*>(pe), d, s, k1, o);
  if (i < d.nx) {
    // x-edge (i,j) between cells (i,j-1) and (i,j)
    const long w = -d.pitch;
    PE0[0] = PE[0];
    for (int k = 1; k <= km; ++k) PE0[k] = 0.5 * (PE.p[(long)k * d.plane + w] + PE[k]);
    const double pb = PE.p[(long)km * d.plane + w] + PE[km];
    for (int k = 0; k <= km; ++k) {
      double bkh = 0.5 * bk[k];
      PE3[k] = ak[k] + bkh * pb;
    }
    Col U = col(u, d, s, km, o);
    for (int k = 0; k < km; ++k) A[k] = U[k];
    map1(PE0, A, PE3, U, km, km, -1, 0.0, P, DP1);
  }
  if (j < d.ny) {
    const long w = -1;
    PE0[0] = PE[0];
    PE3[0] = ak[0];
    const double pb = PE.p[(long)km * d.plane + w] + PE[km];
    for (int k = 1; k <= km; ++k) {
      double bkh = 0.5 * bk[k];
      PE0[k] = 0.5 * (PE.p[(long)k * d.plane + w] + PE[k]);
      PE3[k] = ak[k] + bkh * pb;
    }
    Col V = col(v, d, s, km, o);
    for (int k = 0; k < km; ++k) A[k] = V[k];
    map1(PE0, A, PE3, V, km, km, -1, 0.0, P, DP1);
  }
}

__global__ void __launch_bounds__(256) pe_eulerian_k(Dims d, int npz, const double* __restrict__ ak,
                                                     const double* __restrict__ bk, double* __restrict__ pe) {
  Launch2D L{0, 0, d.nx, d.ny};
  int i, j;
  if (!thread_point(L, i, j)) return;
  const int s = blockIdx.z;
  const long o = pidx(d, i, j);
  Col PE = col(pe, d, s, npz + 1, o);
  const double ps = PE[npz];
  for (int k = 1; k < npz; ++k) PE[k] = ak[k] + bk[k] * ps;
}

}  // namespace

void lagrangian_to_eulerian(const Ctx& c, int npz, int nq, double ptop, bool fill, const double* ak_dev,
                            const double* bk_dev, const RemapState& S, const RemapScratch& R) {
  const Dims& d = c.d;
  dim3 g(cdiv(d.nx, BX), cdiv(d.ny, BY), d.nsub);
  GT_LAUNCH(remap_scalar_k, g, dim3(BX, BY), 0, c.st, d, npz, nq, ptop, fill ? 1 : 0, ak_dev, bk_dev, S, R);
  HIP_LAUNCH_CHECK();
  dim3 g1(cdiv(d.nx + 1, BX), cdiv(d.ny + 1, BY), d.nsub);
  GT_LAUNCH(remap_wind_k, g1, dim3(BX, BY), 0, c.st, d, npz, ak_dev, bk_dev, S.pe, S.u, S.v, R);
  HIP_LAUNCH_CHECK();
  GT_LAUNCH(pe_eulerian_k, g, dim3(BX, BY), 0, c.st, d, npz, ak_dev, bk_dev, S.pe);
  HIP_LAUNCH_CHECK();
}

}  // namespace gtfv3
