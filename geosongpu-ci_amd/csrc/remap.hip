// remap.hip — Lagrangian_to_Eulerian (FV3 fv_mapz) on gfx950: cs_profile (PPM,
// kord = 9, cs_limiters), map1_ppm (two-pointer exact integration), fillz, and the
// per-column state conversion.
//
// Work decomposition: one lane per (column, field) JOB — T_v (in log p), delz, w,
// u, v and the nq tracers are independent remaps of the same column, so a launch has
// columns x jobs lanes instead of one lane doing every field in series.  Lanes are
// consecutive i, so every k-plane access of a wave is coalesced.
//
// Two forms, bit-identical, both with the expressions of oracle/fv_mapz.py: the level-block
// form (remap_blk_k / remap_blkq_k, default where a block shape covers the level count,
// see below) and remap_job_k (the generic form for any level count: per job the edge values
// q, the tridiagonal gam and a copy of the source means live in HBM scratch columns; the
// per-layer coefficients are recomputed on the fly in the integration walk).
#include <cstdlib>
#include <type_traits>
#include <utility>

#include "blockscan.hpp"
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

// f(integral_constant<int, 0>) ... f(integral_constant<int, N-1>) in order: a loop body
// instantiated once per index, so every array index inside it is a compile-time constant
template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

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
// scale constraint of each edge is applied as the back substitution finalises it.  The
// columns are __restrict__ parameters and the values a level shares with the next (the
// edge pressure, the mean, the factor just formed) are carried in registers, so the
// forward and backward sweeps issue their loads ahead instead of waiting out a store ->
// load round trip per level; same operations in the same order as before.
__device__ __forceinline__ void cs_edges_r(int km, int iv, double qs, long P, int ekind,
                                           const double* __restrict__ A, const double* __restrict__ Ea,
                                           const double* __restrict__ Eb, double* __restrict__ q,
                                           double* __restrict__ gam) {
  auto E = [&](int l) -> double {
    if (ekind == 0) return Ea[(long)l * P];
    return l == 0 ? Ea[0] : 0.5 * (Eb[(long)l * P] + Ea[(long)l * P]);
  };
  auto Ak = [&](int k) { return A[(long)k * P]; };
  auto constrain = [&](int e, double v, double am2, double am1, double a0, double ap1) {
    // am2 .. ap1 = A[e-2] .. A[e+1] (only those in range are used)
    if (e == 1 || e == km - 1) {
      v = fmin(v, fmax(am1, a0));
      return fmax(v, fmin(am1, a0));
    }
    if (e >= 2 && e <= km - 2) {
      const double g0 = am1 - am2, g1 = ap1 - a0;
      if (g0 * g1 > 0.0) {
        v = fmin(v, fmax(am1, a0));
        v = fmax(v, fmin(am1, a0));
      } else if (g0 > 0.0) {
        v = fmax(v, fmin(am1, a0));
      } else {
        v = fmin(v, fmax(am1, a0));
        if (iv == 0) v = fmax(0.0, v);
      }
    }
    return v;
  };
  // back substitution from edge `top` down to 0 with the A window carried downwards
  auto back = [&](int top, double x, int gofs) {
    // window: A[e-2], A[e-1], A[e], A[e+1] for e = top
    double a0 = top <= km - 1 ? Ak(top) : 0.0;
    double ap1 = top + 1 <= km - 1 ? Ak(top + 1) : 0.0;
    double am1 = top >= 1 ? Ak(top - 1) : 0.0;
    double am2 = top >= 2 ? Ak(top - 2) : 0.0;
    for (int e = top; e >= 0; --e) {
      x = q[(long)e * P] - gam[(long)(e + gofs) * P] * x;
      q[(long)e * P] = constrain(e, x, am2, am1, a0, ap1);
      ap1 = a0;
      a0 = am1;
      am1 = am2;
      am2 = e >= 3 ? Ak(e - 3) : 0.0;
    }
  };
  if (iv == -2) {
    double gp = 0.5;
    gam[P] = gp;
    double qp = 1.5 * Ak(0);
    q[0] = qp;
    double el = E(1);
    double dprev = el - E(0);
    double aprev = Ak(0);
    for (int e = 1; e < km - 1; ++e) {
      const double en = E(e + 1);
      const double dcur = en - el;
      const double ae = Ak(e);
      const double grat = dprev / dcur;
      const double bet = 2.0 + grat + grat - gp;
      qp = (3.0 * (aprev + ae) - qp) / bet;
      q[(long)e * P] = qp;
      gp = grat / bet;
      gam[(long)(e + 1) * P] = gp;
      dprev = dcur;
      el = en;
      aprev = ae;
    }
    const double grat = (E(km - 1) - E(km - 2)) / (E(km) - E(km - 1));
    double x = (3.0 * (Ak(km - 2) + Ak(km - 1)) - grat * qs - qp) / (2.0 + grat + grat - gp);
    q[(long)km * P] = qs;
    const double a_km1 = Ak(km - 1), a_km2 = Ak(km - 2), a_km3 = km >= 3 ? Ak(km - 3) : 0.0;
    q[(long)(km - 1) * P] = constrain(km - 1, x, a_km3, a_km2, a_km1, 0.0);
    back(km - 2, x, 1);
  } else {
    double e0 = E(0), e1 = E(1);
    double dprev = e1 - e0, dcur = E(2) - e1;
    const double grat = dcur / dprev;
    double bet = grat * (grat + 0.5);
    double qp = ((grat + grat) * (grat + 1.0) * Ak(0) + Ak(1)) / bet;
    q[0] = qp;
    double gp = (1.0 + grat * (grat + 1.5)) / bet;
    gam[0] = gp;
    double d4 = grat;
    double el = e1;
    double aprev = Ak(0);
    for (int e = 1; e < km; ++e) {
      const double en = E(e + 1);
      dcur = en - el;
      const double ae = Ak(e);
      d4 = dprev / dcur;
      bet = 2.0 + d4 + d4 - gp;
      qp = (3.0 * (aprev + d4 * ae) - qp) / bet;
      q[(long)e * P] = qp;
      gp = d4 / bet;
      gam[(long)e * P] = gp;
      dprev = dcur;
      el = en;
      aprev = ae;
    }
    const double a_bot = 1.0 + d4 * (d4 + 1.5);
    double x = (2.0 * d4 * (d4 + 1.0) * Ak(km - 1) + Ak(km - 2) - a_bot * qp) / (d4 * (d4 + 0.5) - a_bot * gp);
    q[(long)km * P] = x;
    back(km - 1, x, 0);
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

// map1_ppm as ONE streaming sweep over the source layers with the target pointer dynamic
// (remap_job_k's walk): per source layer the PPM coefficients from
// a sliding window of means A[l-2 .. l+2] and edges q[l], q[l+1], then every target piece
// inside the layer.  The loads of a layer are issued two layers ahead, independent of the
// data-dependent walk, instead of the two-pointer search's chain of dependent HBM round
// trips.  Same terms in the same order as map1 (bit-identical).  Returns whether a value < 0
// was written (fillz has work only then).
__device__ __forceinline__ bool map1_stream(int km, int iv, long P, int ekind, const double* __restrict__ Ea,
                                            const double* __restrict__ Eb, const double* __restrict__ A,
                                            const double* __restrict__ q, double* __restrict__ out,
                                            const Targets& T) {
  auto E = [&](int l) -> double {
    if (ekind == 0) return Ea[(long)l * P];
    return l == 0 ? Ea[0] : 0.5 * (Eb[(long)l * P] + Ea[(long)l * P]);
  };
  auto Ak = [&](int k) { return k < km ? A[(long)k * P] : 0.0; };
  auto Qk = [&](int e) { return e <= km ? q[(long)e * P] : 0.0; };
  auto Ek = [&](int e) { return e <= km ? E(e) : 0.0; };
  double am2 = 0.0, am1 = 0.0, a0 = Ak(0), ap1 = Ak(1), ap2 = Ak(2), ap3 = Ak(3);
  double qL = Qk(0), qR = Qk(1), qn1 = Qk(2);
  double e0 = E(0), e1 = Ek(1), en1 = Ek(2);
  int k = 0;
  bool open = false, neg = false;
  double qsum = 0.0, topk = 0.0, bot = 0.0;
  double topv = T(0);
  double tb1 = T(1);
  for (int l = 0; l < km; ++l) {
    const double ap4 = Ak(l + 4), qn2 = Qk(l + 3), en2 = Ek(l + 3);
    // PPM coefficients of layer l (layer_coef's expressions on the window)
    double AL = qL, AR = qR, A6;
    {
      const double av = a0;
      const double g_m1 = am1 - am2, g_0 = a0 - am1, g_p1 = ap1 - a0, g_p2 = ap2 - ap1;  // gm(l-1 .. l+2)
      if (l == 0) {
        if (iv == 0) AL = fmax(0.0, AL);
        else if (iv == -1 && AL * av <= 0.0) AL = 0.0;
        A6 = 3.0 * (2.0 * av - (AL + AR));
        lim(av, AL, AR, A6, false, 1);
      } else if (l == 1) {
        A6 = 3.0 * (2.0 * av - (AL + AR));
        lim(av, AL, AR, A6, g_0 * g_p1 < 0.0, 2);
      } else if (l < km - 2) {
        const bool el = g_0 * g_p1 < 0.0;
        if ((el && g_m1 * g_0 < 0.0) || (el && g_p1 * g_p2 < 0.0)) {
          AL = av; AR = av; A6 = 0.0;
        } else {
          A6 = 6.0 * av - 3.0 * (AL + AR);
          if (fabs(A6) > fabs(AL - AR)) {
            double pmp_1 = av - 2.0 * g_p1;
            double lac_1 = pmp_1 + 1.5 * g_p2;
            AL = fmin(fmax(AL, fmin(fmin(av, pmp_1), lac_1)), fmax(fmax(av, pmp_1), lac_1));
            double pmp_2 = av + 2.0 * g_0;
            double lac_2 = pmp_2 - 1.5 * g_m1;
            AR = fmin(fmax(AR, fmin(fmin(av, pmp_2), lac_2)), fmax(fmax(av, pmp_2), lac_2));
            A6 = 6.0 * av - 3.0 * (AL + AR);
          }
        }
        if (iv == 0) lim(av, AL, AR, A6, el, 0);
      } else if (l == km - 2) {
        A6 = 3.0 * (2.0 * av - (AL + AR));
        lim(av, AL, AR, A6, g_0 * g_p1 < 0.0, 2);
      } else {
        if (iv == 0) AR = fmax(0.0, AR);
        else if (iv == -1 && AR * av <= 0.0) AR = 0.0;
        A6 = 3.0 * (2.0 * av - (AL + AR));
        lim(av, AL, AR, A6, false, 1);
      }
    }
    const double dpl = e1 - e0;
    while (k < km) {
      if (open) {
        if (bot > e1) {  // whole layer
          qsum = qsum + dpl * a0;
          break;
        }
        const double dp = bot - e0;  // last (partial) piece
        const double esl = dp / dpl;
        qsum = qsum + dp * (AL + 0.5 * esl * (AR - AL + A6 * (1.0 - R23 * esl)));
        const double v = qsum / (bot - topk);
        out[(long)k * P] = v;
        neg = neg || v < 0.0;
        ++k;
        tb1 = T(k + 1 <= km ? k + 1 : km);
        open = false;
        topv = bot;
        continue;
      }
      if (!(topv >= e0 && topv <= e1)) break;
      bot = tb1;
      const double pl = (topv - e0) / dpl;
      if (bot <= e1) {  // target inside this layer
        const double pr = (bot - e0) / dpl;
        const double v = AL + 0.5 * (A6 + AR - AL) * (pr + pl) - A6 * R3 * (pr * (pr + pl) + pl * pl);
        out[(long)k * P] = v;
        neg = neg || v < 0.0;
        ++k;
        tb1 = T(k + 1 <= km ? k + 1 : km);
        topv = bot;
        continue;
      }
      // first (partial) piece; the target continues below
      qsum = (e1 - topv) * (AL + 0.5 * (A6 + AR - AL) * (1.0 + pl) - A6 * (R3 * (1.0 + pl * (1.0 + pl))));
      topk = topv;
      open = true;
      break;
    }
    am2 = am1; am1 = a0; a0 = ap1; ap1 = ap2; ap2 = ap3; ap3 = ap4;
    qL = qR; qR = qn1; qn1 = qn2;
    e0 = e1; e1 = en1; en1 = en2;
  }
  if (open) {  // bottom beyond the last source edge (the walk ran out of layers)
    const double v = qsum / (bot - topk);
    out[(long)k * P] = v;
    neg = neg || v < 0.0;
  }
  return neg;
}

template <typename DPF>
__device__ __forceinline__ void fillz_col(const Col& q, const DPF& dp, int km) {
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
  int job0, nslot;  // scratch slots per sub-domain: jobs job0 .. job0+nslot-1 of a launch
  double ptop;
  const double *ak, *bk;
  RemapState S;
  double *qs, *gs, *src;  // scratch: njob * (npz+1) levels each
};

// theta_v -> T_v (kord_tm < 0 remaps T_v in log p) and delz -> -delz/delp, into the
// source slots of the T and delz jobs, before any job overwrites delz / pt; one lane per
// (column, level) (pointwise: the levels run in parallel)
__global__ void __launch_bounds__(BLOCK) remap_prep_k(RemapArgs a) {
  const Dims& d = a.d;
  const int km = a.npz, k1 = km + 1;
  const int c = blockIdx.x * BLOCK + threadIdx.x;
  const int s = blockIdx.y / km, k = blockIdx.y % km;
  if (c >= d.nx * d.ny) return;
  const int i = c % d.nx, j = c / d.nx;
  const long P = d.plane, o = pidx(d, i, j);
  const double rrg = -RDGAS / GRAV;
  const double k1k = KAPPA / (1.0 - KAPPA);
  const long x = ((long)s * km + k) * P + o;
  double* TV = a.src + ((long)s * a.nslot + J_PT) * k1 * P + o;
  double* DZ = a.src + ((long)s * a.nslot + J_DZ) * k1 * P + o;
  const double pt = a.S.pt[x], dp = a.S.delp[x], dz = a.S.delz[x];
  TV[k * P] = pt * exp(k1k * log(rrg * dp / dz * pt));
  DZ[k * P] = -dz / dp;
}

__global__ void __launch_bounds__(BLOCK) remap_job_k(RemapArgs a) {
  const Dims& d = a.d;
  const int km = a.npz, k1 = km + 1;
  const int job = a.job0 + blockIdx.y;
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
  const long slot = ((long)s * a.nslot + job - a.job0) * k1 * P + o;
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
  cs_edges_r(km, iv, qs, P, E.kind, A.p, E.a, E.b, q.p, gam.p);
  const bool neg = map1_stream(km, iv, P, E.kind, E.a, E.b, A.p, q.p, OUT.p, T);
  if (job >= J_Q0 && a.fill && neg) fillz_col(OUT, [&](int k) { return T(k + 1) - T(k); }, km);
}

// job kinds of the level-block form: one kernel instantiation per kind, so no branch on the
// kind is left in the body (a single kernel for all kinds was unswitched by the compiler into
// one copy of the column code per kind: 90-170 KB of code)
enum { JK_PT = 0, JK_DZ = 1, JK_W = 2, JK_UV = 3, JK_Q = 4 };

// ---------------- level-block form (default where instantiated) ----------------
//
// A job's column split into NB level blocks on NB consecutive lanes of one 16-lane DPP row
// (lane = NB * column + b; block b: source layers / edges b M .. b M + M - 1), as the SIM1
// solver's scan form (riem.hip, blockscan.hpp).  Every stage runs on all lanes:
//   * the kord = 9 edge values: cs_profile's tridiagonal system (the bottom edge eliminated
//     into the last real row, so the km unknowns fill the blocks), solved by tri_solve with
//     Möbius-scan pivots (strongly diagonally dominant rows [1, 2 + 2 d4, d4]), then the
//     large-scale constraints pointwise -- the neighbouring blocks' means by DPP;
//   * the PPM coefficients of each layer (cs_limiters) pointwise;
//   * map1_ppm through the mass function Q(p) = integral of the profile from the top to p:
//     each block forms its layers' running mass, a scan of the block totals gives each block
//     its offset, each block evaluates Q at the target interfaces inside its source range
//     (the profile's partial integral in the layer holding the interface) into LDS, and each
//     target layer's mean is (Q(bottom) - Q(top)) / dp -- taken from block-local values when
//     both interfaces lie in one block, so the column's mass above does not cancel there.
// The same expressions as cs_profile / map1_ppm, associated differently (sums through the
// scan, a target's pieces as a difference of running integrals): agreement with the oracle and
// the column forms to rounding (tests/test_gpu_remap.py), not bit for bit.  No scratch planes;
// each job's source column and output field move once, the source edges once per job.
constexpr int RB_WAVES = 4;
constexpr int RB_NT = 4;  // tracers per wave of remap_blkq_k at nq <= 4 (more above: the launcher)
typedef unsigned int RbU2 __attribute__((ext_vector_type(2)));
template <int M, int NB, bool PART, int JK>
__global__ void __launch_bounds__(64 * RB_WAVES) remap_blk_k(RemapArgs a) {
  constexpr int NC = 64 / NB, KX = NB * M;  // KX: the largest level count of this shape
  __shared__ double lab[2 * (KX + 1)];                 // ak | bk
  __shared__ double lq[RB_WAVES][NC][KX + 1];          // block-local Q at target interface k
  __shared__ double lt[RB_WAVES][NC][KX + 1];          // target interface k
  __shared__ int lown[RB_WAVES][NC][KX + 1];           // the block holding target interface k
  __shared__ double loff[RB_WAVES][NC][NB];            // Q at each block's top edge
  const int km = a.npz;  // launcher: (NB - 1) M < km <= NB M
  for (int k = threadIdx.x; k <= km; k += 64 * RB_WAVES) {
    lab[k] = a.ak[k];
    lab[KX + 1 + k] = a.bk[k];
  }
  __syncthreads();
  const Dims d = a.d;
  const double ptop = a.ptop;
  const int fill = a.fill;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int b = lane & (NB - 1), cl = lane / NB;
  const bool last = b == NB - 1;
  const int nv = PART && last ? km - (NB - 1) * M : M;  // real layers of this block
  auto real = [&](int m) { return !PART || m < nv; };
  const int job = JK == JK_PT ? J_PT : JK == JK_DZ ? J_DZ : JK == JK_W ? J_W
                : JK == JK_UV ? J_U + (int)blockIdx.y : J_Q0 + (int)blockIdx.y;
  const int s = blockIdx.z;
  // the job's columns: cells nx x ny, u edges nx x (ny + 1), v edges (nx + 1) x ny
  const int ni = job == J_V ? d.nx + 1 : d.nx, nj = job == J_U ? d.ny + 1 : d.ny;
  const int ncol = ni * nj;
  const int c0 = ((int)xcd_block() * RB_WAVES + wv) * NC;  // XCD-aware order, as riem_scan_k
  if (c0 >= ncol) return;  // whole wavefront (no barrier follows)
  int c = c0 + cl;
  const bool valid = c < ncol;
  if (!valid) c = ncol - 1;
  const int i = c % ni, j = c / ni;
  const long P = d.plane, o = pidx(d, i, j);
  const uint32_t PB = (uint32_t)P * 8u, vo = (uint32_t)o * 8u;
  const uint32_t vb = vo + (uint32_t)(b * M) * PB;  // the block's first level
  auto rsrc = [&](const double* base, int nk) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, (int)(nk * PB), 0x00020000);
  };
  auto ld = [&](__amdgpu_buffer_rsrc_t r, uint32_t v, int lev) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, v + (uint32_t)lev * PB, 0, 0));
  };
  const double* pe_s = a.S.pe + (long)s * (km + 1) * P;
  const auto rPE = rsrc(pe_s, km + 1);
  auto rEA = rPE;
  uint32_t vob = vo;
  constexpr bool ewind = JK == JK_UV;
  constexpr int tkind = JK == JK_PT ? 1 : (JK == JK_UV ? 2 : 0);
  constexpr int iv = JK == JK_W ? -2 : (JK == JK_UV ? -1 : (JK == JK_Q ? 0 : 1));
  const double ps = ld(rPE, vo, km);
  double lntop = 0.0, lnbot = 0.0, pb = 0.0, qs = 0.0;
  const double* src;
  double* out;
  const long slot = ((long)s * a.nslot + job) * (km + 1) * P;
  if (JK == JK_PT) {
    rEA = rsrc(a.S.peln + (long)s * (km + 1) * P, km + 1);
    lntop = ld(rEA, vo, 0);
    lnbot = ld(rEA, vo, km);
    src = a.src + slot;
    out = a.S.pt + (long)s * km * P;
  } else if (JK == JK_DZ) {
    src = a.src + slot;
    out = a.S.delz + (long)s * km * P;
  } else {
    double* f;
    if (JK == JK_W) {
      f = a.S.w + (long)s * km * P;
      qs = a.S.ws[(long)s * P + o];
    } else if (JK == JK_UV) {
      f = (job == J_U ? a.S.u : a.S.v) + (long)s * km * P;
      const long w = job == J_U ? -d.pitch : -1;
      vob = (uint32_t)(o + w) * 8u;
      pb = ld(rPE, vob, km) + ps;
    } else {
      f = a.S.q + ((long)s * a.nq + (job - J_Q0)) * km * P;
    }
    src = f;
    out = f;
  }
  const auto rSRC = rsrc(src, km), rOUT = rsrc(out, km);
  // source edge of the block's local interface m (levels past the bottom read 0 -> replaced)
  auto Eloc = [&](int m) -> double {
    const int lev = b * M + m;
    if (!ewind) return ld(rEA, vb, m);
    const double x0 = ld(rEA, vb, m);
    const double x1 = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rEA, vob + (uint32_t)(b * M + m) * PB, 0, 0));
    return lev == 0 ? x0 : 0.5 * (x1 + x0);
  };
  auto T = [&](int k) -> double {
    if (tkind == 0) return k == 0 ? ptop : (k == km ? ps : lab[k] + lab[KX + 1 + k] * ps);
    if (tkind == 1) return k == 0 ? lntop : (k == km ? lnbot : fm_log(lab[k] + lab[KX + 1 + k] * ps));
    return lab[k] + 0.5 * lab[KX + 1 + k] * pb;
  };

  // ---- loads: means and edges of the block (a partial block's virtual layers: A = 0, edges
  // held at its bottom edge, so their thickness is 0)
  double A[M], Ev[M + 1];
#pragma unroll
  for (int m = 0; m < M; ++m) A[m] = ld(rSRC, vb, m);
#pragma unroll
  for (int m = 0; m <= M; ++m) Ev[m] = Eloc(m);
  if constexpr (PART) {
    double eb = Ev[M];
#pragma unroll
    for (int m = 0; m <= M; ++m)
      if (m == nv) eb = Ev[m];
#pragma unroll
    for (int m = 0; m <= M; ++m) Ev[m] = m > nv ? eb : Ev[m];
  }
  double dp[M];
#pragma unroll
  for (int m = 0; m < M; ++m) dp[m] = Ev[m + 1] - Ev[m];
  // neighbouring blocks' means and thicknesses (shifted outside any select; blockscan.hpp)
  const double am1_ = blk_prev(A[M - 1]), am2_ = blk_prev(A[M - 2 >= 0 ? M - 2 : 0]), dpm1_ = blk_prev(dp[M - 1]);
  const double ap1_ = blk_next(A[0]), ap2_ = blk_next(A[M > 1 ? 1 : 0]);
  const double am1 = b == 0 ? 0.0 : am1_, am2 = b == 0 ? 0.0 : am2_, dpm1 = b == 0 ? 1.0 : dpm1_;
  const double ap1 = last ? 0.0 : ap1_, ap2 = last ? 0.0 : ap2_;
  // mean of local layer m in [-2, M + 1]
  auto Aw = [&](int m) -> double {
    return m == -2 ? am2 : m == -1 ? am1 : m == M ? ap1 : m == M + 1 ? ap2 : A[m < 0 ? 0 : (m > M - 1 ? M - 1 : m)];
  };
  auto dpw = [&](int m) -> double { return m < 0 ? dpm1 : dp[m]; };
  auto glob = [&](int m) { return b * M + m; };

  // ---- edge values: rows e = 0 .. km - 1 (cs_profile's system with q[km] eliminated from the
  // last row; iv = -2: q[km] = qs given)
  double abot = 0.0, dbot = 1.0, rbot = 0.0;  // the bottom edge's row (iv != -2), last block
  if constexpr (iv != -2) {
    double d4b = 0.0, a1 = 0.0, a2 = 0.0;
#pragma unroll
    for (int m = 0; m < M; ++m)
      if (m == nv - 1) {  // the column's last layer (last block)
        d4b = dpw(m - 1) / dp[m];
        a1 = A[m];
        a2 = Aw(m - 1);
      }
    abot = 1.0 + d4b * (d4b + 1.5);
    dbot = d4b * (d4b + 0.5);
    rbot = 2.0 * d4b * (d4b + 1.0) * a1 + a2;
  }
  auto row = [&](int m, double& am, double& dg, double& cm) {
    const int e = glob(m);
    const bool bt = last && m == nv - 1;  // row km - 1
    if (!real(m)) {
      am = 0.0; dg = 1.0; cm = 0.0;
      return;
    }
    if (e == 0) {
      am = 0.0;
      if (iv == -2) {
        dg = 1.0; cm = 0.5;
      } else {
        const double grat = dp[1 < M ? 1 : 0] / dp[0];
        dg = grat * (grat + 0.5);
        cm = 1.0 + grat * (grat + 1.5);
      }
      return;
    }
    const double d4 = dpw(m - 1) / dp[m];
    am = 1.0;
    dg = 2.0 + d4 + d4;
    cm = d4;
    if (bt) {
      if (iv == -2) cm = 0.0;
      else {
        dg = dg - cm * abot / dbot;
        cm = 0.0;
      }
    }
  };
  auto rhs = [&](int m) -> double {
    const int e = glob(m);
    const bool bt = last && m == nv - 1;
    if (!real(m)) return 0.0;
    if (e == 0) {
      if (iv == -2) return 1.5 * A[0];
      const double grat = dp[1 < M ? 1 : 0] / dp[0];
      return (grat + grat) * (grat + 1.0) * A[0] + A[1 < M ? 1 : 0];
    }
    const double d4 = dpw(m - 1) / dp[m];
    double r = iv == -2 ? 3.0 * (Aw(m - 1) + A[m]) : 3.0 * (Aw(m - 1) + d4 * A[m]);
    if (bt) r = iv == -2 ? r - d4 * qs : r - d4 * rbot / dbot;
    return r;
  };
  double qe[M];
  tri_solve<M, NB, true>(row, rhs, qe, b, last);
  // the bottom edge q[km] (last block)
  double qlast = qe[M - 1];
#pragma unroll
  for (int m = 0; m < M; ++m)
    if (m == nv - 1) qlast = qe[m];
  const double qbot = iv == -2 ? qs : (rbot - abot * qlast) / dbot;
  // large-scale constraints of edges 1 .. km - 1
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const int e = glob(m);
    double v = qe[m];
    const double a0 = Aw(m - 1), a1 = A[m];
    if (e == 1 || e == km - 1) {
      v = fmin(v, fmax(a0, a1));
      v = fmax(v, fmin(a0, a1));
    } else if (e >= 2 && e <= km - 2) {
      const double g0 = a0 - Aw(m - 2), g1 = Aw(m + 1) - a1;
      if (g0 * g1 > 0.0) {
        v = fmin(v, fmax(a0, a1));
        v = fmax(v, fmin(a0, a1));
      } else if (g0 > 0.0) {
        v = fmax(v, fmin(a0, a1));
      } else {
        v = fmin(v, fmax(a0, a1));
        if (iv == 0) v = fmax(0.0, v);
      }
    }
    qe[m] = real(m) ? v : 0.0;
  }
  const double qn_ = blk_next(qe[0]);
  // edge at local interface m + 1 of layer m
  auto qr = [&](int m) -> double {
    if (m + 1 < M) return (last && m == nv - 1) ? qbot : qe[m + 1 < M ? m + 1 : 0];
    return last ? qbot : qn_;
  };

  // ---- running mass of the block, block offsets
  double C[M + 1];
  C[0] = 0.0;
#pragma unroll
  for (int m = 0; m < M; ++m) C[m + 1] = C[m] + A[m] * dp[m];
  const double offx = blk_prev(scan_sum<NB, true>(C[M], b));
  const double off = b == 0 ? 0.0 : offx;
  loff[wv][cl][b] = off;
  // the target interfaces in the block's source range [Ev[0], Ev[M]) (the last block's
  // last real layer takes every remaining one, k = km included)
  int k = b * M < km ? b * M : km;
  if (b == 0) {
    k = 0;
  } else {
    while (k > 0 && T(k - 1) >= Ev[0]) --k;
    while (k <= km && T(k) < Ev[0]) ++k;
  }
#pragma unroll
  for (int m = 0; m < M; ++m) {
    if (!real(m)) continue;
    // PPM coefficients of layer l (kord = 9 cs_profile + cs_limiters)
    const int l = glob(m);
    auto gm = [&](int mm) { return Aw(mm) - Aw(mm - 1); };
    auto extm = [&](int mm) { return gm(mm) * gm(mm + 1) < 0.0; };
    const double av = A[m];
    double AL = qe[m], AR = qr(m), A6;
    if (l == 0) {
      if (iv == 0) AL = fmax(0.0, AL);
      else if (iv == -1 && AL * av <= 0.0) AL = 0.0;
      A6 = 3.0 * (2.0 * av - (AL + AR));
      lim(av, AL, AR, A6, false, 1);
    } else if (l == 1) {
      A6 = 3.0 * (2.0 * av - (AL + AR));
      lim(av, AL, AR, A6, extm(m), 2);
    } else if (l < km - 2) {
      const bool el = extm(m);
      if ((el && extm(m - 1)) || (el && extm(m + 1))) {
        AL = av; AR = av; A6 = 0.0;
      } else {
        A6 = 6.0 * av - 3.0 * (AL + AR);
        if (fabs(A6) > fabs(AL - AR)) {
          double pmp_1 = av - 2.0 * gm(m + 1);
          double lac_1 = pmp_1 + 1.5 * gm(m + 2);
          AL = fmin(fmax(AL, fmin(fmin(av, pmp_1), lac_1)), fmax(fmax(av, pmp_1), lac_1));
          double pmp_2 = av + 2.0 * gm(m);
          double lac_2 = pmp_2 - 1.5 * gm(m - 1);
          AR = fmin(fmax(AR, fmin(fmin(av, pmp_2), lac_2)), fmax(fmax(av, pmp_2), lac_2));
          A6 = 6.0 * av - 3.0 * (AL + AR);
        }
      }
      if (iv == 0) lim(av, AL, AR, A6, el, 0);
    } else if (l == km - 2) {
      A6 = 3.0 * (2.0 * av - (AL + AR));
      lim(av, AL, AR, A6, extm(m), 2);
    } else {
      if (iv == 0) AR = fmax(0.0, AR);
      else if (iv == -1 && AR * av <= 0.0) AR = 0.0;
      A6 = 3.0 * (2.0 * av - (AL + AR));
      lim(av, AL, AR, A6, false, 1);
    }
    // Q at the target interfaces inside layer l: C + the profile's integral from its top
    const bool lastlayer = last && m == nv - 1;
    const double e0 = Ev[m], e1 = Ev[m + 1], rdp = 1.0 / dp[m];
    while (k <= km) {
      const double t = T(k);
      if (!lastlayer && t >= e1) break;
      const double y = t - e0, x = y * rdp;
      lq[wv][cl][k] = C[m] + y * (AL + 0.5 * x * (AR - AL + A6 * (1.0 - R23 * x)));
      lt[wv][cl][k] = t;
      lown[wv][cl][k] = b;
      ++k;
    }
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
  // ---- target layer means for levels b M .. b M + M - 1
  bool neg = false;
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const int kk = glob(m);
    if (kk >= km) break;
    const int o0 = lown[wv][cl][kk], o1 = lown[wv][cl][kk + 1];
    const double q0 = lq[wv][cl][kk], q1 = lq[wv][cl][kk + 1];
    const double num = o0 == o1 ? q1 - q0 : (loff[wv][cl][o1] - loff[wv][cl][o0]) + (q1 - q0);
    const double v = num / (lt[wv][cl][kk + 1] - lt[wv][cl][kk]);
    if (valid)
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(RbU2, v), rOUT, vb + (uint32_t)m * PB, 0, 0);
    neg = neg || v < 0.0;
  }
  if constexpr (JK == JK_Q) {
    // fillz: one lane of a column with a negative value walks the column (rare)
    const unsigned long long any = __ballot(neg);
    const bool col_neg = ((any >> (cl * NB)) & ((NB == 64 ? ~0ull : (1ull << NB) - 1))) != 0;
    if (fill && col_neg && b == 0 && valid) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      fillz_col(Col{out + o, P}, [&](int k2) { return lt[wv][cl][k2 + 1] - lt[wv][cl][k2]; }, km);
    }
  }
}

// The tracer jobs of the level-block form, NT tracers per wave: everything that depends on
// the pressures only -- the layer thicknesses, the cs_profile pivots (tri_factor, the Moebius
// scan: the row coefficients [1, 2 + 2 d4, d4] and the eliminated bottom row involve dp
// alone), the target interfaces and which block / layer holds each -- is formed once per
// column and shared by the NT tracers; per tracer only the right-hand side, tri_apply, the
// constraints, the PPM coefficients and the mass-function pieces run.  Same expressions per
// tracer as remap_blk_k<.., JK_Q> (bit-identical to it).
template <int M, int NB, bool PART, int NT>
__global__ void __launch_bounds__(64 * RB_WAVES, 2) remap_blkq_k(RemapArgs a) {
  constexpr int NC = 64 / NB, KX = NB * M;
  __shared__ double lab[2 * (KX + 1)];
  __shared__ double lq[RB_WAVES][NC][KX + 1];
  // per target interface k, formed once from the pressures: its offset y from the top edge of
  // the source layer holding it and y / dp of that layer (the source edges and 1 / dp then
  // hold no registers across the tracers; the target thicknesses are T(k + 1) - T(k))
  __shared__ double ly[RB_WAVES][NC][KX + 1];
  __shared__ double lx[RB_WAVES][NC][KX + 1];
  __shared__ int lown[RB_WAVES][NC][KX + 1];
  __shared__ double loff[RB_WAVES][NC][NB];
  const int km = a.npz;
  for (int k = threadIdx.x; k <= km; k += 64 * RB_WAVES) {
    lab[k] = a.ak[k];
    lab[KX + 1 + k] = a.bk[k];
  }
  __syncthreads();
  const Dims d = a.d;
  const double ptop = a.ptop;
  const int fill = a.fill;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int b = lane & (NB - 1), cl = lane / NB;
  const bool last = b == NB - 1;
  const int nv = PART && last ? km - (NB - 1) * M : M;
  auto real = [&](int m) { return !PART || m < nv; };
  const int s = blockIdx.z;
  const int ncol = d.nx * d.ny;
  const int c0 = ((int)xcd_block() * RB_WAVES + wv) * NC;  // XCD-aware order, as riem_scan_k
  if (c0 >= ncol) return;  // whole wavefront (no barrier follows)
  int c = c0 + cl;
  const bool valid = c < ncol;
  if (!valid) c = ncol - 1;
  const long P = d.plane, o = pidx(d, c % d.nx, c / d.nx);
  const uint32_t PB = (uint32_t)P * 8u, vo = (uint32_t)o * 8u;
  const uint32_t vb = vo + (uint32_t)(b * M) * PB;
  auto rsrc = [&](const double* base, int nk) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, (int)(nk * PB), 0x00020000);
  };
  // the level in the scalar offset (no VGPRs: the vector-offset form, or a per-level select of
  // an out-of-range vector offset, runs this kernel out of them).  The scalar offset is outside
  // the descriptor's range check, so a partial block's loads past the bottom read the planes
  // that follow (the next sub-domain's, or the field allocation's tail pad of kFieldTailPlanes
  // planes, Dycore::field): values replaced below (virtual layers), never a fault; its stores
  // are guarded by the level (kk < km).
  auto ld = [&](__amdgpu_buffer_rsrc_t r, uint32_t v, int lev) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, v, (uint32_t)lev * PB, 0));
  };
  const auto rPE = rsrc(a.S.pe + (long)s * (km + 1) * P, km + 1);
  const double ps = ld(rPE, vo, km);
  auto T = [&](int k) -> double { return k == 0 ? ptop : (k == km ? ps : lab[k] + lab[KX + 1 + k] * ps); };
  auto glob = [&](int m) { return b * M + m; };

  // ---- the pressure part, once: edges, thicknesses, pivots, target ownership
  double Ev[M + 1];
#pragma unroll
  for (int m = 0; m <= M; ++m) Ev[m] = ld(rPE, vb, m);
  if constexpr (PART) {
    double eb = Ev[M];
#pragma unroll
    for (int m = 0; m <= M; ++m)
      if (m == nv) eb = Ev[m];
#pragma unroll
    for (int m = 0; m <= M; ++m) Ev[m] = m > nv ? eb : Ev[m];
  }
  double dp[M];
#pragma unroll
  for (int m = 0; m < M; ++m) dp[m] = Ev[m + 1] - Ev[m];
  const double dpm1_ = blk_prev(dp[M - 1]);
  const double dpm1 = b == 0 ? 1.0 : dpm1_;
  auto dpw = [&](int m) -> double { return m < 0 ? dpm1 : dp[m]; };
  double abot = 0.0, dbot = 1.0, d4b = 0.0;
#pragma unroll
  for (int m = 0; m < M; ++m)
    if (m == nv - 1) {
      d4b = dpw(m - 1) / dp[m];
    }
  abot = 1.0 + d4b * (d4b + 1.5);
  dbot = d4b * (d4b + 0.5);
  auto row = [&](int m, double& am, double& dg, double& cm) {
    const int e = glob(m);
    const bool bt = last && m == nv - 1;
    if (!real(m)) {
      am = 0.0; dg = 1.0; cm = 0.0;
      return;
    }
    if (e == 0) {
      const double grat = dp[1 < M ? 1 : 0] / dp[0];
      am = 0.0;
      dg = grat * (grat + 0.5);
      cm = 1.0 + grat * (grat + 1.5);
      return;
    }
    const double d4 = dpw(m - 1) / dp[m];
    am = 1.0;
    dg = 2.0 + d4 + d4;
    cm = d4;
    if (bt) {
      dg = dg - cm * abot / dbot;
      cm = 0.0;
    }
  };
  double gam[M], rbs[M];
  tri_factor<M, NB, true>(row, gam, rbs, b);
  // target interfaces of each source layer: kb[m] .. kb[m + 1] - 1
  int kb[M + 1];
  {
    int k = b * M < km ? b * M : km;
    if (b == 0) {
      k = 0;
    } else {
      while (k > 0 && T(k - 1) >= Ev[0]) --k;
      while (k <= km && T(k) < Ev[0]) ++k;
    }
#pragma unroll
    for (int m = 0; m < M; ++m) {
      kb[m] = k;
      if (!real(m)) continue;
      const bool lastlayer = last && m == nv - 1;
      const double e0 = Ev[m], rdp = 1.0 / dp[m];
      while (k <= km) {
        const double t = T(k);
        if (!lastlayer && t >= Ev[m + 1]) break;
        const double y = t - e0;
        ly[wv][cl][k] = y;
        lx[wv][cl][k] = y * rdp;
        lown[wv][cl][k] = b;
        ++k;
      }
    }
    kb[M] = k;
  }

  // ---- per tracer
  const int q0 = blockIdx.y * NT;
#pragma unroll 1
  for (int tq = 0; tq < NT; ++tq) {
    const int iq = q0 + tq;
    if (iq >= a.nq) break;  // (wave-uniform)
    asm volatile("" ::: "memory");
    double* const out = a.S.q + ((long)s * a.nq + iq) * km * P;
    const auto rQ = rsrc(out, km);
    double A[M];
#pragma unroll
    for (int m = 0; m < M; ++m) A[m] = ld(rQ, vb, m);
    const double am1_ = blk_prev(A[M - 1]), am2_ = blk_prev(A[M - 2 >= 0 ? M - 2 : 0]);
    const double ap1_ = blk_next(A[0]), ap2_ = blk_next(A[M > 1 ? 1 : 0]);
    const double am1 = b == 0 ? 0.0 : am1_, am2 = b == 0 ? 0.0 : am2_;
    const double ap1 = last ? 0.0 : ap1_, ap2 = last ? 0.0 : ap2_;
    auto Aw = [&](int m) -> double {
      return m == -2 ? am2 : m == -1 ? am1 : m == M ? ap1 : m == M + 1 ? ap2 : A[m < 0 ? 0 : (m > M - 1 ? M - 1 : m)];
    };
    double rbot = 0.0;
    {
      double a1 = 0.0, a2 = 0.0;
#pragma unroll
      for (int m = 0; m < M; ++m)
        if (m == nv - 1) {
          a1 = A[m];
          a2 = Aw(m - 1);
        }
      rbot = 2.0 * d4b * (d4b + 1.0) * a1 + a2;
    }
    auto rhs = [&](int m) -> double {
      const int e = glob(m);
      const bool bt = last && m == nv - 1;
      if (!real(m)) return 0.0;
      if (e == 0) {
        const double grat = dp[1 < M ? 1 : 0] / dp[0];
        return (grat + grat) * (grat + 1.0) * A[0] + A[1 < M ? 1 : 0];
      }
      const double d4 = dpw(m - 1) / dp[m];
      double r = 3.0 * (Aw(m - 1) + d4 * A[m]);
      if (bt) r = r - d4 * rbot / dbot;
      return r;
    };
    double qe[M];
    tri_apply<M, NB>(row, rhs, gam, rbs, qe, b, last);
    double qlast = qe[M - 1];
#pragma unroll
    for (int m = 0; m < M; ++m)
      if (m == nv - 1) qlast = qe[m];
    const double qbot = (rbot - abot * qlast) / dbot;
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const int e = glob(m);
      double v = qe[m];
      const double a0 = Aw(m - 1), a1 = A[m];
      if (e == 1 || e == km - 1) {
        v = fmin(v, fmax(a0, a1));
        v = fmax(v, fmin(a0, a1));
      } else if (e >= 2 && e <= km - 2) {
        const double g0 = a0 - Aw(m - 2), g1 = Aw(m + 1) - a1;
        if (g0 * g1 > 0.0) {
          v = fmin(v, fmax(a0, a1));
          v = fmax(v, fmin(a0, a1));
        } else if (g0 > 0.0) {
          v = fmax(v, fmin(a0, a1));
        } else {
          v = fmin(v, fmax(a0, a1));
          v = fmax(0.0, v);
        }
      }
      qe[m] = real(m) ? v : 0.0;
    }
    const double qn_ = blk_next(qe[0]);
    auto qr = [&](int m) -> double {
      if (m + 1 < M) return (last && m == nv - 1) ? qbot : qe[m + 1 < M ? m + 1 : 0];
      return last ? qbot : qn_;
    };
    double C[M + 1];
    C[0] = 0.0;
#pragma unroll
    for (int m = 0; m < M; ++m) C[m + 1] = C[m] + A[m] * dp[m];
    const double offx = blk_prev(scan_sum<NB, true>(C[M], b));
    loff[wv][cl][b] = b == 0 ? 0.0 : offx;
#pragma unroll
    for (int m = 0; m < M; ++m) {
      if (!real(m)) continue;
      const int l = glob(m);
      auto gm = [&](int mm) { return Aw(mm) - Aw(mm - 1); };
      auto extm = [&](int mm) { return gm(mm) * gm(mm + 1) < 0.0; };
      const double av = A[m];
      double AL = qe[m], AR = qr(m), A6;
      if (l == 0) {
        AL = fmax(0.0, AL);
        A6 = 3.0 * (2.0 * av - (AL + AR));
        lim(av, AL, AR, A6, false, 1);
      } else if (l == 1) {
        A6 = 3.0 * (2.0 * av - (AL + AR));
        lim(av, AL, AR, A6, extm(m), 2);
      } else if (l < km - 2) {
        const bool el = extm(m);
        if ((el && extm(m - 1)) || (el && extm(m + 1))) {
          AL = av; AR = av; A6 = 0.0;
        } else {
          A6 = 6.0 * av - 3.0 * (AL + AR);
          if (fabs(A6) > fabs(AL - AR)) {
            double pmp_1 = av - 2.0 * gm(m + 1);
            double lac_1 = pmp_1 + 1.5 * gm(m + 2);
            AL = fmin(fmax(AL, fmin(fmin(av, pmp_1), lac_1)), fmax(fmax(av, pmp_1), lac_1));
            double pmp_2 = av + 2.0 * gm(m);
            double lac_2 = pmp_2 - 1.5 * gm(m - 1);
            AR = fmin(fmax(AR, fmin(fmin(av, pmp_2), lac_2)), fmax(fmax(av, pmp_2), lac_2));
            A6 = 6.0 * av - 3.0 * (AL + AR);
          }
        }
        lim(av, AL, AR, A6, el, 0);
      } else if (l == km - 2) {
        A6 = 3.0 * (2.0 * av - (AL + AR));
        lim(av, AL, AR, A6, extm(m), 2);
      } else {
        AR = fmax(0.0, AR);
        A6 = 3.0 * (2.0 * av - (AL + AR));
        lim(av, AL, AR, A6, false, 1);
      }
      for (int k = kb[m]; k < kb[m + 1]; ++k) {
        const double y = ly[wv][cl][k], x = lx[wv][cl][k];
        lq[wv][cl][k] = C[m] + y * (AL + 0.5 * x * (AR - AL + A6 * (1.0 - R23 * x)));
      }
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    bool neg = false;
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const int kk = glob(m);
      if (kk < km) {
        const int o0 = lown[wv][cl][kk], o1 = lown[wv][cl][kk + 1];
        const double q0v = lq[wv][cl][kk], q1v = lq[wv][cl][kk + 1];
        const double num = o0 == o1 ? q1v - q0v : (loff[wv][cl][o1] - loff[wv][cl][o0]) + (q1v - q0v);
        const double v = num / (T(kk + 1) - T(kk));
        if (valid)
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(RbU2, v), rQ, vb, (uint32_t)m * PB, 0);
        neg = neg || v < 0.0;
      }
    }
    const unsigned long long any = __ballot(neg);
    const bool col_neg = ((any >> (cl * NB)) & ((NB == 64 ? ~0ull : (1ull << NB) - 1))) != 0;
    if (fill && col_neg && b == 0 && valid) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      fillz_col(Col{out + o, P}, [&](int k2) { return T(k2 + 1) - T(k2); }, km);
    }
    // the next tracer rewrites lq / loff: this one's reads (and fillz's) come first
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  }
}

// Eulerian state from the remapped fields, one lane per (column, interface k = 0 .. km): the
// top interface of layer k is ptop (k = 0) or ak + bk ps, its log the stored peln (k = 0, km)
// or the log of that -- the same values a top-down walk carries from layer to layer
__global__ void __launch_bounds__(BLOCK) remap_finish_k(RemapArgs a) {
  const Dims& d = a.d;
  const int km = a.npz, k1 = km + 1;
  const int c = blockIdx.x * BLOCK + threadIdx.x;
  const int s = blockIdx.y / k1, k = blockIdx.y % k1;
  if (c >= d.nx * d.ny) return;
  const int i = c % d.nx, j = c / d.nx;
  const long P = d.plane, o = pidx(d, i, j);
  const long b1 = (long)s * k1 * P + o, bk = (long)s * km * P + o;
  const double rrg = -RDGAS / GRAV;
  double* PE = a.S.pe + b1;
  double* PELN = a.S.peln + b1;
  double* PK = a.S.pk + b1;
  const double psurf = PE[km * P];
  if (k == km) {  // bottom interface: peln kept, pk from it
    const double pn = PELN[km * P];
    PK[km * P] = exp(KAPPA * pn);
    PELN[km * P] = pn;
    return;
  }
  if (k == 0) a.S.ps[(long)s * P + o] = psurf;
  double* DELP = a.S.delp + bk;
  double* DELZ = a.S.delz + bk;
  double* PT = a.S.pt + bk;
  double* PKZ = a.S.pkz + bk;
  const double pe_t = k == 0 ? a.ptop : a.ak[k] + a.bk[k] * psurf;
  const double pn_t = k == 0 ? PELN[0] : log(pe_t);
  const double pe_b = k + 1 == km ? psurf : a.ak[k + 1] + a.bk[k + 1] * psurf;
  const double dp2 = pe_b - pe_t;
  const double dz = -DELZ[k * P] * dp2;
  DELZ[k * P] = dz;
  DELP[k * P] = dp2;
  PK[k * P] = exp(KAPPA * pn_t);
  PELN[k * P] = pn_t;
  PKZ[k * P] = exp(KAPPA * log(rrg * dp2 / dz * PT[k * P]));
  if (k >= 1) PE[k * P] = pe_t;
}

}  // namespace

int remap_jobs(int nq) { return nq + J_Q0; }

// the step's remap form: GTFV3_REMAP (0 the level-block form, 1 the scratch-column jobs, 3 the
// level-block form one tracer per wave; see lagrangian_to_eulerian)
int remap_variant() {
  static const int env = [] {
    const char* e = std::getenv("GTFV3_REMAP");
    return e ? std::atoi(e) : 0;
  }();
  return env;
}

// The column-job form keeps three scratch columns (edge values, factors, source copy) per
// job: at most RM_CHUNK jobs share one set of scratch planes (jobs launched in chunks), so
// L137 with 54 tracers needs 3 x 8 x 138 planes per sub-domain, not 3 x 59 x 138.
constexpr int RM_CHUNK = 8;
int remap_scratch_slots(int nq) { return std::min(remap_jobs(nq), RM_CHUNK); }

void lagrangian_to_eulerian(const Ctx& c, int npz, int nq, double ptop, bool fill, const double* ak_dev,
                            const double* bk_dev, const RemapState& S, const RemapScratch& R, int variant,
                            int phase) {
  if (npz < 6) throw std::runtime_error("remap: npz >= 6 required");
  // phase 1: prep and the T_v / delz / w / wind jobs; phase 2: the tracer jobs and the
  // finish (so the tracer transport can run beside phase 1); 0: both
  const bool p1 = phase != 2, p2 = phase != 1;
  const Dims& d = c.d;
  RemapArgs a{};
  a.d = d;
  a.npz = npz;
  a.nq = nq;
  a.fill = fill ? 1 : 0;
  a.njob = remap_jobs(nq);
  a.nslot = remap_scratch_slots(nq);
  a.job0 = 0;
  a.ptop = ptop;
  a.ak = ak_dev;
  a.bk = bk_dev;
  a.S = S;
  a.qs = R.s[0];
  a.gs = R.s[1];
  a.src = R.s[2];
  const int nc = d.nx * d.ny, nce = (d.nx + 1) * (d.ny + 1);
  const Ext e = ext(d);
  const double L = npz, L1 = npz + 1;
  if (p1) {
    GT_LAUNCH(remap_prep_k, dim3(cdiv(nc, BLOCK), d.nsub * npz), dim3(BLOCK), 0, c.st, a);
    HIP_LAUNCH_CHECK();
    gt_bytes(L * 5 * e.C);  // delp delz pt read, T_v and -delz/delp source columns written
  }
  // variant 0: the level-block form where a shape is instantiated ((NB - 1) M < npz <= NB M),
  // tracers RB_NT per wave (remap_blkq_k); 3: the same with one tracer per wave (remap_blk_k,
  // the bit-identity reference of the shared-pivot form); 1 (or a level count no block shape
  // covers: 6, 9, 13-15, 21-63, 73-90, 97-135, > 144): the scratch-column jobs, the generic form
  auto fits = [&](int m, int nb) { return (nb - 1) * m < npz && npz <= nb * m; };
  auto blk = [&](auto Mc, auto NBc, auto PARTc) {
    constexpr int M = decltype(Mc)::value, NB = decltype(NBc)::value;
    constexpr bool PART = decltype(PARTc)::value;
    const unsigned gx = xcd_pad(cdiv(cdiv(nce, 64 / NB), RB_WAVES));
    const dim3 tb(64 * RB_WAVES);
    if (p1) {
      GT_LAUNCH((remap_blk_k<M, NB, PART, JK_PT>), dim3(gx, 1, d.nsub), tb, 0, c.st, a);
      gt_bytes(L * 2 * e.C + L1 * 2 * e.C);
      GT_LAUNCH((remap_blk_k<M, NB, PART, JK_DZ>), dim3(gx, 1, d.nsub), tb, 0, c.st, a);
      gt_bytes(L * 2 * e.C + L1 * e.C);
      GT_LAUNCH((remap_blk_k<M, NB, PART, JK_W>), dim3(gx, 1, d.nsub), tb, 0, c.st, a);
      gt_bytes(L * 2 * e.C + L1 * e.C + e.C);
      GT_LAUNCH((remap_blk_k<M, NB, PART, JK_UV>), dim3(gx, 2, d.nsub), tb, 0, c.st, a);
      gt_bytes(L * 2 * (e.X + e.Y) + L1 * e.C);
    }
    if (p2 && nq > 0) {
      // tracers: RB_NT per wave sharing the pressure part (remap_blkq_k), or one per wave
      if (variant == 3) {
        GT_LAUNCH((remap_blk_k<M, NB, PART, JK_Q>), dim3(gx, nq, d.nsub), tb, 0, c.st, a);
      } else {
        // tracers per wave: the pressure part is formed once per wave and shared, so more
        // tracers per wave cost less per tracer -- C360 L137 x 54: 76.1 / 69.8 / 66.8 / 65.6 ms
        // per step for 4 / 8 / 16 / 32 (`profiles/r05n_*`).  Default 32 above 16 tracers, 16
        // above 8, 8 above 4; GTFV3_REMAP_NT (4, 8, 16, 32) overrides
        static const int nt_env = [] {
          const char* e = std::getenv("GTFV3_REMAP_NT");
          return e ? std::atoi(e) : 0;
        }();
        const int nt = nt_env > 0 ? nt_env : (nq > 16 ? 32 : (nq > 8 ? 16 : (nq > 4 ? 8 : RB_NT)));
        if (nt >= 32 && nq > 16)
          GT_LAUNCH((remap_blkq_k<M, NB, PART, 32>), dim3(gx, cdiv(nq, 32), d.nsub), tb, 0, c.st, a);
        else if (nt >= 16 && nq > 8)
          GT_LAUNCH((remap_blkq_k<M, NB, PART, 16>), dim3(gx, cdiv(nq, 16), d.nsub), tb, 0, c.st, a);
        else if (nt >= 8 && nq > RB_NT)
          GT_LAUNCH((remap_blkq_k<M, NB, PART, 8>), dim3(gx, cdiv(nq, 8), d.nsub), tb, 0, c.st, a);
        else
          GT_LAUNCH((remap_blkq_k<M, NB, PART, RB_NT>), dim3(gx, cdiv(nq, RB_NT), d.nsub), tb, 0, c.st, a);
      }
      gt_bytes(nq * L * 2 * e.C + L1 * e.C);
    }
  };
  using std::integral_constant;
  const bool b0 = variant == 0 || variant == 3;
  if (b0 && npz == 72) {
    blk(integral_constant<int, 9>{}, integral_constant<int, 8>{}, std::false_type{});
  } else if (b0 && fits(9, 8)) {
    blk(integral_constant<int, 9>{}, integral_constant<int, 8>{}, std::true_type{});
  } else if (b0 && fits(9, 16)) {
    blk(integral_constant<int, 9>{}, integral_constant<int, 16>{}, std::true_type{});
  } else if (b0 && fits(6, 16)) {
    blk(integral_constant<int, 6>{}, integral_constant<int, 16>{}, std::true_type{});
  } else if (b0 && fits(5, 4)) {
    blk(integral_constant<int, 5>{}, integral_constant<int, 4>{}, std::true_type{});
  } else if (b0 && fits(3, 4)) {
    blk(integral_constant<int, 3>{}, integral_constant<int, 4>{}, std::true_type{});
  } else if (b0 && fits(2, 4)) {
    blk(integral_constant<int, 2>{}, integral_constant<int, 4>{}, std::true_type{});
  } else {
    // every job reads its source column and writes its field (L each), pe + peln once, ws;
    // each chunk registers its jobs' share
    const double all = L * 2 * ((a.njob - 2) * e.C + e.X + e.Y) + L1 * 2 * e.C + e.C;
    // phase 1 the first J_Q0 jobs (T_v, delz, w, u, v: their source slots from the prep),
    // phase 2 the tracers; within a phase, chunks of nslot jobs share the scratch
    const int jlo = p1 ? 0 : J_Q0, jhi = p2 ? a.njob : J_Q0;
    for (int j0 = jlo; j0 < jhi; j0 += a.nslot) {
      a.job0 = j0;
      const int nj = std::min(a.nslot, jhi - j0);
      GT_LAUNCH(remap_job_k, dim3(cdiv(nce, BLOCK), nj, d.nsub), dim3(BLOCK), 0, c.st, a);
      gt_bytes(all * nj / a.njob);
    }
  }
  HIP_LAUNCH_CHECK();
  if (!p2) return;
  GT_LAUNCH(remap_finish_k, dim3(cdiv(nc, BLOCK), d.nsub * (npz + 1)), dim3(BLOCK), 0, c.st, a);
  HIP_LAUNCH_CHECK();
  // reads delz pt (L) pe peln (L+1); writes delz delp pkz (L) pk peln pe (L+1) ps
  gt_bytes(L * 5 * e.C + L1 * 5 * e.C + e.C);
}

}  // namespace gtfv3
