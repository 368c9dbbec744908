// remap.hip — Lagrangian_to_Eulerian (FV3 fv_mapz) on gfx950: cs_profile (PPM,
// kord = 9, cs_limiters), map1_ppm (two-pointer exact integration), fillz, and the
// per-column state conversion.
//
// Work decomposition: one lane per (column, field) JOB — T_v (in log p), delz, w,
// u, v and the nq tracers are independent remaps of the same column, so the launch
// has (nq + 5) x columns lanes instead of one lane doing every field in series.
// Lanes are consecutive i, so every k-plane access of a wave is coalesced.
//
// Per job only two work columns live in HBM scratch: the constrained PPM edge values
// q (L+1) and the tridiagonal gam (L+1), plus a copy of the source layer means (the
// output is written in place).  The per-layer coefficients (AL, AR, A6) of the
// kord = 9 profile are recomputed on the fly from q and the source means inside the
// integration walk, with the same expressions as oracle/fv_mapz.py (bit-identical to
// the stored-coefficient formulation).
#include "kernels_nh.hpp"
#include "stencil_common.hpp"

namespace gtfv3 {
namespace {

constexpr double GRAV = Constants::grav;
constexpr double RDGAS = Constants::rdgas;
constexpr double KAPPA = Constants::kappa;
constexpr double R3 = 1.0 / 3.0, R23 = 2.0 / 3.0, R12 = 1.0 / 12.0;
constexpr int BLOCK = 256;

// job ids
enum { J_PT = 0, J_DZ = 1, J_W = 2, J_U = 3, J_V = 4, J_Q0 = 5 };

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

// strided column access
struct Col {
  double* p;
  long st;
  __device__ __forceinline__ double& operator[](int k) const { return p[(long)k * st]; }
};

// Source interface pressures of one job (one column, or the average of two for winds)
struct Edges {
  int kind;
  const double* a;  // own column (stride P)
  const double* b;  // neighbour column (kind 1)
  long P;
  __device__ __forceinline__ double operator()(int k) const {
    if (kind == 0) return a[k * P];
    return k == 0 ? a[0] : 0.5 * (b[k * P] + a[k * P]);
  }
};
// Target (Eulerian) interfaces: 0: ak + bk ps (top ptop, bottom ps); 1: log of that
// (top / bottom from peln); 2: winds, ak + bk/2 (ps_left + ps_right)
struct Targets {
  int kind;
  const double *ak, *bk;
  double ptop, ps, lntop, lnbot, pb;
  int km;
  __device__ __forceinline__ double operator()(int k) const {
    if (kind == 0) return k == 0 ? ptop : (k == km ? ps : ak[k] + bk[k] * ps);
    if (kind == 1) return k == 0 ? lntop : (k == km ? lnbot : log(ak[k] + bk[k] * ps));
    return ak[k] + 0.5 * bk[k] * pb;
  }
};

// PPM coefficients of source layer l (kord = 9 cs_profile + cs_limiters), from the
// constrained edge values q and the layer means A.
__device__ __forceinline__ void layer_coef(int l, int km, int iv, const Col& q, const Col& A, double& AL, double& AR,
                                           double& A6) {
  auto gm = [&](int e) { return A[e] - A[e - 1]; };
  auto extm = [&](int e) { return gm(e) * gm(e + 1) < 0.0; };
  const double a = A[l];
  AL = q[l];
  AR = q[l + 1];
  if (l == 0) {
    if (iv == 0) AL = fmax(0.0, AL);
    else if (iv == -1 && AL * a <= 0.0) AL = 0.0;
    A6 = 3.0 * (2.0 * a - (AL + AR));
    lim(a, AL, AR, A6, false, 1);
  } else if (l == 1) {
    A6 = 3.0 * (2.0 * a - (AL + AR));
    lim(a, AL, AR, A6, extm(1), 2);
  } else if (l < km - 2) {
    const bool el = extm(l);
    if ((el && extm(l - 1)) || (el && extm(l + 1))) {
      AL = a; AR = a; A6 = 0.0;
    } else {
      A6 = 6.0 * a - 3.0 * (AL + AR);
      if (fabs(A6) > fabs(AL - AR)) {
        double pmp_1 = a - 2.0 * gm(l + 1);
        double lac_1 = pmp_1 + 1.5 * gm(l + 2);
        AL = fmin(fmax(AL, fmin(fmin(a, pmp_1), lac_1)), fmax(fmax(a, pmp_1), lac_1));
        double pmp_2 = a + 2.0 * gm(l);
        double lac_2 = pmp_2 - 1.5 * gm(l - 1);
        AR = fmin(fmax(AR, fmin(fmin(a, pmp_2), lac_2)), fmax(fmax(a, pmp_2), lac_2));
        A6 = 6.0 * a - 3.0 * (AL + AR);
      }
    }
    if (iv == 0) lim(a, AL, AR, A6, el, 0);
  } else if (l == km - 2) {
    A6 = 3.0 * (2.0 * a - (AL + AR));
    lim(a, AL, AR, A6, extm(l), 2);
  } else {
    if (iv == 0) AR = fmax(0.0, AR);
    else if (iv == -1 && AR * a <= 0.0) AR = 0.0;
    A6 = 3.0 * (2.0 * a - (AL + AR));
    lim(a, AL, AR, A6, false, 1);
  }
}

// constrained edge values q of the kord = 9 profile (gam: scratch column); the large-
// scale constraint of each edge is applied as the back substitution finalises it
__device__ void cs_edges(const Col& A, const Edges& E, int km, int iv, double qs, const Col& q, const Col& gam) {
  auto DP = [&](int l) { return E(l + 1) - E(l); };
  auto constrain = [&](int e, double v) {
    if (e == 1 || e == km - 1) {
      v = fmin(v, fmax(A[e - 1], A[e]));
      return fmax(v, fmin(A[e - 1], A[e]));
    }
    if (e >= 2 && e <= km - 2) {
      const double g0 = A[e - 1] - A[e - 2], g1 = A[e + 1] - A[e];
      if (g0 * g1 > 0.0) {
        v = fmin(v, fmax(A[e - 1], A[e]));
        v = fmax(v, fmin(A[e - 1], A[e]));
      } else if (g0 > 0.0) {
        v = fmax(v, fmin(A[e - 1], A[e]));
      } else {
        v = fmin(v, fmax(A[e - 1], A[e]));
        if (iv == 0) v = fmax(0.0, v);
      }
    }
    return v;
  };
  if (iv == -2) {
    gam[1] = 0.5;
    double qp = 1.5 * A[0];
    q[0] = qp;
    double dprev = DP(0);
    for (int e = 1; e < km - 1; ++e) {
      const double dcur = DP(e);
      const double grat = dprev / dcur;
      const double bet = 2.0 + grat + grat - gam[e];
      qp = (3.0 * (A[e - 1] + A[e]) - qp) / bet;
      q[e] = qp;
      gam[e + 1] = grat / bet;
      dprev = dcur;
    }
    const double grat = DP(km - 2) / DP(km - 1);
    double x = (3.0 * (A[km - 2] + A[km - 1]) - grat * qs - qp) / (2.0 + grat + grat - gam[km - 1]);
    q[km] = qs;
    q[km - 1] = constrain(km - 1, x);
    for (int e = km - 2; e >= 0; --e) {
      x = q[e] - gam[e + 1] * x;
      q[e] = constrain(e, x);
    }
  } else {
    double dprev = DP(0), dcur = DP(1);
    const double grat = dcur / dprev;
    double bet = grat * (grat + 0.5);
    double qp = ((grat + grat) * (grat + 1.0) * A[0] + A[1]) / bet;
    q[0] = qp;
    double gp = (1.0 + grat * (grat + 1.5)) / bet;
    gam[0] = gp;
    double d4 = grat;
    for (int e = 1; e < km; ++e) {
      dcur = DP(e);
      d4 = dprev / dcur;
      bet = 2.0 + d4 + d4 - gp;
      qp = (3.0 * (A[e - 1] + d4 * A[e]) - qp) / bet;
      q[e] = qp;
      gp = d4 / bet;
      gam[e] = gp;
      dprev = dcur;
    }
    const double a_bot = 1.0 + d4 * (d4 + 1.5);
    double x = (2.0 * d4 * (d4 + 1.0) * A[km - 1] + A[km - 2] - a_bot * qp) / (d4 * (d4 + 0.5) - a_bot * gp);
    q[km] = x;
    for (int e = km - 1; e >= 0; --e) {
      x = q[e] - gam[e] * x;
      q[e] = constrain(e, x);
    }
  }
}

// map1_ppm: source means A on edges E -> OUT on target edges T (same layer count)
__device__ void map1(const Edges& E, const Col& A, const Targets& T, const Col& OUT, int km, int iv, const Col& q) {
  int k0 = 0;
  int lc = -1;  // layer whose coefficients are cached
  double cAL = 0.0, cAR = 0.0, cA6 = 0.0;
  for (int k = 0; k < km; ++k) {
    const double top = T(k), bot = T(k + 1);
    for (int l = k0; l < km; ++l) {
      const double e0 = E(l), e1 = E(l + 1);
      if (top >= e0 && top <= e1) {
        const double dpl = e1 - e0;
        const double pl = (top - e0) / dpl;
        if (lc != l) {
          layer_coef(l, km, iv, q, A, cAL, cAR, cA6);
          lc = l;
        }
        const double AL = cAL, AR = cAR, A6 = cA6;
        if (bot <= e1) {
          const double pr = (bot - e0) / dpl;
          OUT[k] = AL + 0.5 * (A6 + AR - AL) * (pr + pl) - A6 * R3 * (pr * (pr + pl) + pl * pl);
          k0 = l;
        } else {
          double qsum = (e1 - top) * (AL + 0.5 * (A6 + AR - AL) * (1.0 + pl) - A6 * (R3 * (1.0 + pl * (1.0 + pl))));
          double em = e1;
          for (int m = l + 1; m < km; ++m) {
            const double em1 = E(m + 1);
            const double dpm = em1 - em;
            if (bot > em1) {
              qsum = qsum + dpm * A[m];
            } else {
              const double dp = bot - em;
              const double esl = dp / dpm;
              layer_coef(m, km, iv, q, A, cAL, cAR, cA6);
              lc = m;
              qsum = qsum + dp * (cAL + 0.5 * esl * (cAR - cAL + cA6 * (1.0 - R23 * esl)));
              k0 = m;
              break;
            }
            em = em1;
          }
          OUT[k] = qsum / (bot - top);
        }
        break;
      }
    }
  }
}

template <typename DPF>
__device__ void fillz_col(const Col& q, const DPF& dp, int km) {
  if (q[0] < 0.0) {
    q[1] = q[1] + q[0] * dp(0) / dp(1);
    q[0] = 0.0;
  }
  bool zfix = false;
  for (int k = 1; k < km - 1; ++k) {
    if (q[k] < 0.0) {
      zfix = true;
      if (q[k - 1] > 0.0) {
        double dq = fmin(q[k - 1] * dp(k - 1), -q[k] * dp(k));
        q[k - 1] = q[k - 1] - dq / dp(k - 1);
        q[k] = q[k] + dq / dp(k);
      }
      if (q[k] < 0.0 && q[k + 1] > 0.0) {
        double dq = fmin(q[k + 1] * dp(k + 1), -q[k] * dp(k));
        q[k + 1] = q[k + 1] - dq / dp(k + 1);
        q[k] = q[k] + dq / dp(k);
      }
    }
  }
  const int k = km - 1;
  if (q[k] < 0.0 && q[k - 1] > 0.0) {
    zfix = true;
    double qup = q[k - 1] * dp(k - 1);
    double qly = -q[k] * dp(k);
    double dup = fmin(qly, qup);
    q[k - 1] = q[k - 1] - dup / dp(k - 1);
    q[k] = q[k] + dup / dp(k);
  }
  if (zfix) {
    double sum0 = 0.0, sum1 = 0.0;
    for (int kk = 1; kk < km; ++kk) sum0 = sum0 + q[kk] * dp(kk);
    if (sum0 > 0.0) {
      for (int kk = 1; kk < km; ++kk) sum1 = sum1 + fmax(0.0, q[kk] * dp(kk));
      double fac = sum0 / sum1;
      for (int kk = 1; kk < km; ++kk) {
        double dm = q[kk] * dp(kk);
        q[kk] = fmax(0.0, fac * dm / dp(kk));
      }
    }
  }
}

struct RemapArgs {
  Dims d;
  int npz, nq, fill, njob;
  double ptop;
  const double *ak, *bk;
  RemapState S;
  double *qs, *gs, *src;  // scratch: njob * (npz+1) levels each
};

// theta_v -> T_v (kord_tm < 0 remaps T_v in log p) and delz -> -delz/delp, into the
// source slots of the T and delz jobs, before any job overwrites delz / pt
__global__ void __launch_bounds__(BLOCK) remap_prep_k(RemapArgs a) {
  const Dims& d = a.d;
  const int km = a.npz, k1 = km + 1;
  const int c = blockIdx.x * BLOCK + threadIdx.x;
  const int s = blockIdx.y;
  if (c >= d.nx * d.ny) return;
  const int i = c % d.nx, j = c / d.nx;
  const long P = d.plane, o = pidx(d, i, j);
  const double rrg = -RDGAS / GRAV;
  const double k1k = KAPPA / (1.0 - KAPPA);
  const double* DELP = a.S.delp + (long)s * km * P + o;
  const double* DELZ = a.S.delz + (long)s * km * P + o;
  const double* PT = a.S.pt + (long)s * km * P + o;
  double* TV = a.src + ((long)s * a.njob + J_PT) * k1 * P + o;
  double* DZ = a.src + ((long)s * a.njob + J_DZ) * k1 * P + o;
  for (int k = 0; k < km; ++k) {
    const double pt = PT[k * P];
    TV[k * P] = pt * exp(k1k * log(rrg * DELP[k * P] / DELZ[k * P] * pt));
    DZ[k * P] = -DELZ[k * P] / DELP[k * P];
  }
}

__global__ void __launch_bounds__(BLOCK) remap_job_k(RemapArgs a) {
  const Dims& d = a.d;
  const int km = a.npz, k1 = km + 1;
  const int job = blockIdx.y;
  const int s = blockIdx.z;
  const int nxe = d.nx + 1;
  const int c = blockIdx.x * BLOCK + threadIdx.x;
  if (c >= nxe * (d.ny + 1)) return;
  const int i = c % nxe, j = c / nxe;
  if (job == J_U) {
    if (i >= d.nx) return;
  } else if (job == J_V) {
    if (j >= d.ny) return;
  } else if (i >= d.nx || j >= d.ny) {
    return;
  }
  const long P = d.plane, o = pidx(d, i, j);
  const long b1 = (long)s * k1 * P + o, bk = (long)s * km * P + o;
  const long slot = ((long)s * a.njob + job) * k1 * P + o;
  Col q{a.qs + slot, P}, gam{a.gs + slot, P}, A{a.src + slot, P};
  const double* pe = a.S.pe + b1;
  Edges E{0, pe, nullptr, P};
  Targets T{0, a.ak, a.bk, a.ptop, pe[km * P], 0.0, 0.0, 0.0, km};
  Col OUT{nullptr, P};
  int iv = 1;
  double qs = 0.0;
  if (job == J_PT) {
    const double* peln = a.S.peln + b1;
    E.a = peln;
    T.kind = 1;
    T.lntop = peln[0];
    T.lnbot = peln[km * P];
    OUT.p = a.S.pt + bk;
  } else if (job == J_DZ) {
    OUT.p = a.S.delz + bk;
  } else {
    double* f;
    if (job == J_W) {
      f = a.S.w + bk;
      iv = -2;
      qs = a.S.ws[(long)s * P + o];
    } else if (job == J_U || job == J_V) {
      f = (job == J_U ? a.S.u : a.S.v) + bk;
      iv = -1;
      const long w = job == J_U ? -d.pitch : -1;
      E.kind = 1;
      E.b = pe + w;
      T.kind = 2;
      T.pb = pe[km * P + w] + pe[km * P];
    } else {
      f = a.S.q + ((long)s * a.nq + (job - J_Q0)) * km * P + o;
      iv = 0;
    }
    for (int k = 0; k < km; ++k) A[k] = f[k * P];
    OUT.p = f;
  }
  cs_edges(A, E, km, iv, qs, q, gam);
  map1(E, A, T, OUT, km, iv, q);
  if (job >= J_Q0 && a.fill) fillz_col(OUT, [&](int k) { return T(k + 1) - T(k); }, km);
}

// Eulerian state from the remapped fields
__global__ void __launch_bounds__(BLOCK) remap_finish_k(RemapArgs a) {
  const Dims& d = a.d;
  const int km = a.npz, k1 = km + 1;
  const int c = blockIdx.x * BLOCK + threadIdx.x;
  const int s = blockIdx.y;
  if (c >= d.nx * d.ny) return;
  const int i = c % d.nx, j = c / d.nx;
  const long P = d.plane, o = pidx(d, i, j);
  const long b1 = (long)s * k1 * P + o, bk = (long)s * km * P + o;
  const double rrg = -RDGAS / GRAV;
  double* PE = a.S.pe + b1;
  double* PELN = a.S.peln + b1;
  double* PK = a.S.pk + b1;
  double* DELP = a.S.delp + bk;
  double* DELZ = a.S.delz + bk;
  double* PT = a.S.pt + bk;
  double* PKZ = a.S.pkz + bk;
  const double psurf = PE[km * P];
  a.S.ps[(long)s * P + o] = psurf;
  double pe_t = a.ptop, pn_t = PELN[0];
  for (int k = 0; k < km; ++k) {
    const double pe_b = k + 1 == km ? psurf : a.ak[k + 1] + a.bk[k + 1] * psurf;
    const double pn_b = k + 1 == km ? PELN[km * P] : log(pe_b);
    const double dp2 = pe_b - pe_t;
    const double dz = -DELZ[k * P] * dp2;
    DELZ[k * P] = dz;
    DELP[k * P] = dp2;
    PK[k * P] = exp(KAPPA * pn_t);
    PELN[k * P] = pn_t;
    PKZ[k * P] = exp(KAPPA * log(rrg * dp2 / dz * PT[k * P]));
    if (k >= 1) PE[k * P] = pe_t;
    pe_t = pe_b;
    pn_t = pn_b;
  }
  PK[km * P] = exp(KAPPA * pn_t);
  PELN[km * P] = pn_t;
}

}  // namespace

int remap_jobs(int nq) { return nq + J_Q0; }

void lagrangian_to_eulerian(const Ctx& c, int npz, int nq, double ptop, bool fill, const double* ak_dev,
                            const double* bk_dev, const RemapState& S, const RemapScratch& R) {
  if (npz < 6) throw std::runtime_error("remap: npz >= 6 required");
  const Dims& d = c.d;
  RemapArgs a{};
  a.d = d;
  a.npz = npz;
  a.nq = nq;
  a.fill = fill ? 1 : 0;
  a.njob = remap_jobs(nq);
  a.ptop = ptop;
  a.ak = ak_dev;
  a.bk = bk_dev;
  a.S = S;
  a.qs = R.s[0];
  a.gs = R.s[1];
  a.src = R.s[2];
  const int nc = d.nx * d.ny, nce = (d.nx + 1) * (d.ny + 1);
  GT_LAUNCH(remap_prep_k, dim3(cdiv(nc, BLOCK), d.nsub), dim3(BLOCK), 0, c.st, a);
  HIP_LAUNCH_CHECK();
  GT_LAUNCH(remap_job_k, dim3(cdiv(nce, BLOCK), a.njob, d.nsub), dim3(BLOCK), 0, c.st, a);
  HIP_LAUNCH_CHECK();
  // algorithmic bytes per column: every job reads its field and writes it back (L each),
  // pe (+ peln for T) read once, ws
  ktimer_bytes(8.0 * nc * d.nsub * (2.0 * npz * a.njob + 2.0 * (npz + 1) + 1));
  GT_LAUNCH(remap_finish_k, dim3(cdiv(nc, BLOCK), d.nsub), dim3(BLOCK), 0, c.st, a);
  HIP_LAUNCH_CHECK();
}

}  // namespace gtfv3
