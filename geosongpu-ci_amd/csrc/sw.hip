// sw.hip — FV3 C-D grid shallow-water core on gfx950: c_sw (with d2a2c_vect)
// and d_sw (nord = 0, no vorticity / w damping, d_con = 0).  Each routine is a
// short chain of plane-parallel kernels over (i, j) x (sub, level); fv_tp_2d is
// the shared transport operator (tp.hip).  Index conventions: stencil_common.hpp.
// Fortran index f (1-based, npx = N+1) appears here as tile-global g = f-1.
#include <cmath>
#include <cstdlib>

#include "kernels_damp.hpp"
#include "kernels_sw.hpp"
#include "stencil_common.hpp"

namespace gtfv3 {
namespace {

constexpr double A1 = 0.5625, A2 = -0.0625;
constexpr double BIG = 1.0e8;

#define KSETUP(nk_)                                                  \
  int i, j, z;                                                       \
  if (!thread_point_lv(L, (long)d.nsub * (nk_), i, j, z)) return;    \
  const int s = z / (nk_);                                           \
  const SubInfo sub = subs[s];                                       \
  const int N = sub.N;                                               \
  const int I = i + sub.ioff, J = j + sub.joff;                      \
  const long zo = (long)z * d.plane;                                 \
  const long o = pidx(d, i, j);                                      \
  (void)I; (void)J; (void)N; (void)zo;
#define MT(name) met(M, d, name, s)
#define AT(arr, di, dj) arr[zo + o + (long)(dj) * d.pitch + (di)]
#define MA(arr, di, dj) arr[o + (long)(dj) * d.pitch + (di)]

__device__ __forceinline__ double ei4(double u0, double u1, double u2, double u3, double d0, double d1, double d2,
                                      double d3) {
  double t1 = d0 + d1;
  double t2 = d2 + d3;
  return 0.5 * (((t1 + d1) * u1 - d1 * u0) / t1 + ((t2 + d2) * u2 - d2 * u3) / t2);
}

// d_sw's advective Courant number and area flux of one face (ds_courant's expressions and order):
// x faces from ut with rdxa(i-1) / rdxa(i), dy and sin_sg3(i-1) / sin_sg1(i) by the upwind side;
// y faces from vt with rdya(j-1) / rdya(j), dx and sin_sg4(j-1) / sin_sg2(j)
__device__ __forceinline__ void courant_face(double dt, double w, double r_up, double r_dn, double len, double s_up,
                                             double s_dn, double& c, double& f) {
  const double xf = dt * w;
  if (xf > 0.0) {
    c = xf * r_up;
    f = len * xf * s_up;
  } else {
    c = xf * r_dn;
    f = len * xf * s_dn;
  }
}

// ---------------- c_sw ----------------

// d2a2c_vect part 1's interpolation form at tile-global (I, J): second order within three
// cells of a tile edge (on the sub-domain's data range), fourth order elsewhere
__device__ __forceinline__ bool cs_two(const Dims& d, const SubInfo& sub, int I, int J) {
  const int N = sub.N, io = sub.ioff, jo = sub.joff;
  const int jsd = jo - NG, jed = jo + d.ny + NG - 1, isd = io - NG, ied = io + d.nx + NG - 1;
  const bool mid = J >= max(3, jsd) && J <= min(N - 4, jed);
  bool two = false;
  if (J >= jsd && J <= 2) two = true;
  if (J >= N - 3 && J <= jed) two = true;
  if (mid && I >= isd && I <= 2) two = true;
  if (mid && I >= N - 3 && I <= ied) two = true;
  return two;
}

// d2a2c_vect part 1 at one point (local i, j of sub-domain s, level plane zo): the 4th-order
// interpolated ut, vt (2nd order next to the tile edges, BIG outside the range) and the A-grid
// winds ua, va from them; u0 u1 v0 v1 are u(j), u(j+1), v(i), v(i+1) for the vorticity
struct CsTmpPt {
  double ut, vt, a, b, u0, u1, v0, v1;
  bool inr;
};

__device__ __forceinline__ CsTmpPt cs_tmp_pt(const Dims& d, const SubInfo& sub, const double* __restrict__ M, int s,
                                             const double* __restrict__ u, const double* __restrict__ v, long zo,
                                             int i, int j) {
  const int N = sub.N, io = sub.ioff, jo = sub.joff, nx = d.nx, ny = d.ny;
  const int I = i + io, J = j + jo;
  const long o = pidx(d, i, j);
  const long p = d.pitch;
  CsTmpPt r;
  r.inr = i <= nx + NG - 1 && j <= ny + NG - 1;
  const bool rows = r.inr && J >= max(3, jo - 1) && J <= min(N - 4, jo + ny);
  const bool cols = r.inr && I >= max(3, io - 1) && I <= min(N - 4, io + nx);
  const double* U = u + zo + o;
  const double* V = v + zo + o;
  const long u1o = r.inr ? p : 0, umo = rows ? -p : 0, u2o = rows ? 2 * p : 0;
  const long v1o = r.inr ? 1 : 0, vmo = cols ? -1 : 0, v2o = cols ? 2 : 0;
  r.u0 = U[0];
  r.u1 = U[u1o];
  r.v0 = V[0];
  r.v1 = V[v1o];
  const double um = U[umo], u2 = U[u2o];
  const double vm = V[vmo], v2 = V[v2o];
  const double cs = MA(MT(M_COSA_S), 0, 0), r2 = MA(MT(M_RSIN2), 0, 0);
  double ut = BIG, vt = BIG;
  if (r.inr) {
    if (rows) ut = A2 * (um + u2) + A1 * (r.u0 + r.u1);
    if (cols) vt = A2 * (vm + v2) + A1 * (r.v0 + r.v1);
    if (cs_two(d, sub, I, J)) {
      ut = 0.5 * (r.u0 + r.u1);
      vt = 0.5 * (r.v0 + r.v1);
    }
  }
  r.ut = ut;
  r.vt = vt;
  r.a = 0.0;
  r.b = 0.0;
  if (i >= -2 && i <= nx + 1 && j >= -2 && j <= ny + 1) {
    r.a = (ut - vt * cs) * r2;
    r.b = (vt - ut * cs) * r2;
  }
  return r;
}

// d2a2c_vect's cube-corner fills, as targets: the tile-global source point (SI, SJ) and sign of
// a target of utmp (f 0), vtmp (1), ua (2) or va (3) at (I, J) of an owned corner, false if
// (I, J) is not one.  utmp / vtmp take the source's vtmp / utmp, ua / va its va / ua; sources
// are never targets, so a target point computes its source's own values
__device__ __forceinline__ bool cs_corner_src(int f, int I, int J, int N, bool own_sw, bool own_se, bool own_ne,
                                              bool own_nw, int& SI, int& SJ, double& sg) {
  if (f == 0) {
    if (own_sw && J == -1 && I >= -3 && I <= -1) { SI = -1; SJ = -I - 1; sg = -1.0; return true; }
    if (own_se && J == -1 && I >= N && I <= N + 2) { SI = N; SJ = I - N; sg = 1.0; return true; }
    if (own_ne && J == N && I >= N && I <= N + 2) { SI = N; SJ = 2 * N - 1 - I; sg = -1.0; return true; }
    if (own_nw && J == N && I >= -3 && I <= -1) { SI = -1; SJ = N + I; sg = 1.0; return true; }
  } else if (f == 1) {
    if (own_sw && I == -1 && J >= -3 && J <= -1) { SI = -J - 1; SJ = -1; sg = -1.0; return true; }
    if (own_se && I == N && J >= -3 && J <= -1) { SI = N + J; SJ = -1; sg = 1.0; return true; }
    if (own_ne && I == N && J >= N && J <= N + 2) { SI = 2 * N - 1 - J; SJ = N; sg = -1.0; return true; }
    if (own_nw && I == -1 && J >= N && J <= N + 2) { SI = J - N; SJ = N; sg = 1.0; return true; }
  } else if (f == 2) {
    if (own_sw && J == -1 && (I == -2 || I == -1)) { SI = -1; SJ = -1 - I; sg = -1.0; return true; }
    if (own_se && J == -1 && (I == N || I == N + 1)) { SI = N; SJ = I - N; sg = 1.0; return true; }
    if (own_ne && J == N && (I == N || I == N + 1)) { SI = N; SJ = 2 * N - 1 - I; sg = -1.0; return true; }
    if (own_nw && J == N && (I == -2 || I == -1)) { SI = -1; SJ = N + I; sg = 1.0; return true; }
  } else {
    if (own_sw && I == -1 && (J == -2 || J == -1)) { SI = -1 - J; SJ = -1; sg = -1.0; return true; }
    if (own_se && I == N && (J == -1 || J == -2)) { SI = N + J; SJ = -1; sg = 1.0; return true; }
    if (own_ne && I == N && (J == N || J == N + 1)) { SI = 2 * N - 1 - J; SJ = N; sg = -1.0; return true; }
    if (own_nw && I == -1 && (J == N || J == N + 1)) { SI = J - N; SJ = N; sg = 1.0; return true; }
  }
  return false;
}

// d2a2c_vect part 2 (uc, ut | vc, vt) + the dt2*area scaling of ut, vt done by c_sw
__global__ void __launch_bounds__(256) cs_cgrid(Dims d, const SubInfo* __restrict__ subs, const double* __restrict__ M,
                                                int npz, double dt2, const double* __restrict__ u,
                                                const double* __restrict__ v, const double* __restrict__ utmp,
                                                const double* __restrict__ vtmp, const double* __restrict__ ua,
                                                const double* __restrict__ va, double* __restrict__ uc,
                                                double* __restrict__ vc, double* __restrict__ ut,
                                                double* __restrict__ vt) {
  Launch2D L{-NG, -NG, d.nx + 2 * NG + 1, d.ny + 2 * NG + 1};
  KSETUP(npz)
  const int nx = d.nx, ny = d.ny;
  // x: y-edges, local i in [-1, nx+1], j in [-1, ny]
  double ucv = 0.0, utv = 0.0;
  if (i >= -1 && i <= nx + 1 && j >= -1 && j <= ny) {
    if (I == 0 || I == N) {
      const double* dxa = MT(M_DXA);
      double e = ei4(AT(ua, -2, 0), AT(ua, -1, 0), AT(ua, 0, 0), AT(ua, 1, 0), MA(dxa, -2, 0), MA(dxa, -1, 0),
                     MA(dxa, 0, 0), MA(dxa, 1, 0));
      ucv = e * (e > 0.0 ? MA(MT(M_SIN3), -1, 0) : MA(MT(M_SIN1), 0, 0));
      utv = e;
    } else {
      if (I == -1 || I == N - 1) ucv = C1 * AT(utmp, -2, 0) + C2 * AT(utmp, -1, 0) + C3 * AT(utmp, 0, 0);
      else if (I == 1) ucv = C1 * AT(utmp, 1, 0) + C2 * AT(utmp, 0, 0) + C3 * AT(utmp, -1, 0);
      else if (I == N + 1) ucv = C3 * AT(utmp, -1, 0) + C2 * AT(utmp, 0, 0) + C1 * AT(utmp, 1, 0);
      else ucv = A2 * (AT(utmp, -2, 0) + AT(utmp, 1, 0)) + A1 * (AT(utmp, -1, 0) + AT(utmp, 0, 0));
      utv = (ucv - AT(v, 0, 0) * MA(MT(M_COSA_U), 0, 0)) * MA(MT(M_RSIN_U), 0, 0);
    }
    // c_sw: ut -> dt2 * ut * dy * sin_sg (upwind side)
    const double dy = MA(MT(M_DY), 0, 0);
    utv = utv > 0.0 ? dt2 * utv * dy * MA(MT(M_SIN3), -1, 0) : dt2 * utv * dy * MA(MT(M_SIN1), 0, 0);
  }
  AT(uc, 0, 0) = ucv;
  AT(ut, 0, 0) = utv;
  double vcv = 0.0, vtv = 0.0;
  if (i >= -1 && i <= nx && j >= -1 && j <= ny + 1) {
    if (J == 0 || J == N) {
      const double* dya = MT(M_DYA);
      double e = ei4(AT(va, 0, -2), AT(va, 0, -1), AT(va, 0, 0), AT(va, 0, 1), MA(dya, 0, -2), MA(dya, 0, -1),
                     MA(dya, 0, 0), MA(dya, 0, 1));
      vcv = e * (e > 0.0 ? MA(MT(M_SIN4), 0, -1) : MA(MT(M_SIN2), 0, 0));
      vtv = e;
    } else {
      if (J == -1 || J == N - 1) vcv = C1 * AT(vtmp, 0, -2) + C2 * AT(vtmp, 0, -1) + C3 * AT(vtmp, 0, 0);
      else if (J == 1 || J == N + 1) vcv = C1 * AT(vtmp, 0, 1) + C2 * AT(vtmp, 0, 0) + C3 * AT(vtmp, 0, -1);
      else vcv = A2 * (AT(vtmp, 0, -2) + AT(vtmp, 0, 1)) + A1 * (AT(vtmp, 0, -1) + AT(vtmp, 0, 0));
      vtv = (vcv - AT(u, 0, 0) * MA(MT(M_COSA_V), 0, 0)) * MA(MT(M_RSIN_V), 0, 0);
    }
    const double dx = MA(MT(M_DX), 0, 0);
    vtv = vtv > 0.0 ? dt2 * vtv * dx * MA(MT(M_SIN4), 0, -1) : dt2 * vtv * dx * MA(MT(M_SIN2), 0, 0);
  }
  AT(vc, 0, 0) = vcv;
  AT(vt, 0, 0) = vtv;
}

// level-loop form of cs_cgrid (stencil_common.hpp kloop_levels): the point's metric terms --
// which of them it needs is fixed by its position -- loaded once for its block of levels, so
// the upwind sin_sg pick is a select instead of a dependent load per level; per level the same
// expressions as cs_cgrid
__global__ void __launch_bounds__(256) cs_cgrid_kl(Dims d, const SubInfo* __restrict__ subs,
                                                   const double* __restrict__ M, int npz, int nkb, int klb,
                                                   double dt2, const double* __restrict__ u,
                                                   const double* __restrict__ v, const double* __restrict__ utmp,
                                                   const double* __restrict__ vtmp, const double* __restrict__ ua,
                                                   const double* __restrict__ va, double* __restrict__ uc,
                                                   double* __restrict__ vc, double* __restrict__ ut,
                                                   double* __restrict__ vt) {
  Launch2D L{-NG, -NG, d.nx + 2 * NG + 1, d.ny + 2 * NG + 1};
  KLSETUP(npz)
  const SubInfo sub = subs[s];
  const int N = sub.N, I = i + sub.ioff, J = j + sub.joff, nx = d.nx, ny = d.ny;
  const long pt = d.pitch;
  // x: y-edges, local i in [-1, nx+1], j in [-1, ny]; y: x-edges, i in [-1, nx], j in [-1, ny+1]
  const bool xr = i >= -1 && i <= nx + 1 && j >= -1 && j <= ny;
  const bool yr = i >= -1 && i <= nx && j >= -1 && j <= ny + 1;
  const bool xl = I == 0 || I == N, yl = J == 0 || J == N;
  double dxa[4] = {0, 0, 0, 0}, dya[4] = {0, 0, 0, 0};
  double cau = 0, rsu = 0, dyp = 0, s3m = 0, s10 = 0, cav = 0, rsv = 0, dxp = 0, s4m = 0, s20 = 0;
  if (xr) {
    if (xl) {
      const double* m = met(M, d, M_DXA, s) + o;
#pragma unroll
      for (int q = 0; q < 4; ++q) dxa[q] = m[q - 2];
    } else {
      cau = met(M, d, M_COSA_U, s)[o];
      rsu = met(M, d, M_RSIN_U, s)[o];
    }
    dyp = met(M, d, M_DY, s)[o];
    s3m = met(M, d, M_SIN3, s)[o - 1];
    s10 = met(M, d, M_SIN1, s)[o];
  }
  if (yr) {
    if (yl) {
      const double* m = met(M, d, M_DYA, s) + o;
#pragma unroll
      for (int q = 0; q < 4; ++q) dya[q] = m[(q - 2) * pt];
    } else {
      cav = met(M, d, M_COSA_V, s)[o];
      rsv = met(M, d, M_RSIN_V, s)[o];
    }
    dxp = met(M, d, M_DX, s)[o];
    s4m = met(M, d, M_SIN4, s)[o - pt];
    s20 = met(M, d, M_SIN2, s)[o];
  }
  // the x stencil's four inputs along i (ua on the tile-edge lines, utmp elsewhere), the y
  // stencil's along j
  const double* XS = (xl ? ua : utmp) + o;
  const double* YS = (yl ? va : vtmp) + o;
  for (int k = k0; k < k1; ++k) {
    const long zo = ((long)s * npz + k) * P;
    double ucv = 0.0, utv = 0.0, vcv = 0.0, vtv = 0.0;
    double xs[4] = {0, 0, 0, 0}, ys[4] = {0, 0, 0, 0};
    double v0 = 0.0, u0 = 0.0;
    if (xr) {
#pragma unroll
      for (int q = 0; q < 4; ++q) xs[q] = XS[zo + q - 2];
      v0 = v[zo + o];
    }
    if (yr) {
#pragma unroll
      for (int q = 0; q < 4; ++q) ys[q] = YS[zo + (q - 2) * pt];
      u0 = u[zo + o];
    }
    if (xr) {
      if (xl) {
        const double e = ei4(xs[0], xs[1], xs[2], xs[3], dxa[0], dxa[1], dxa[2], dxa[3]);
        ucv = e * (e > 0.0 ? s3m : s10);
        utv = e;
      } else {
        if (I == -1 || I == N - 1) ucv = C1 * xs[0] + C2 * xs[1] + C3 * xs[2];
        else if (I == 1) ucv = C1 * xs[3] + C2 * xs[2] + C3 * xs[1];
        else if (I == N + 1) ucv = C3 * xs[1] + C2 * xs[2] + C1 * xs[3];
        else ucv = A2 * (xs[0] + xs[3]) + A1 * (xs[1] + xs[2]);
        utv = (ucv - v0 * cau) * rsu;
      }
      utv = utv > 0.0 ? dt2 * utv * dyp * s3m : dt2 * utv * dyp * s10;
    }
    if (yr) {
      if (yl) {
        const double e = ei4(ys[0], ys[1], ys[2], ys[3], dya[0], dya[1], dya[2], dya[3]);
        vcv = e * (e > 0.0 ? s4m : s20);
        vtv = e;
      } else {
        if (J == -1 || J == N - 1) vcv = C1 * ys[0] + C2 * ys[1] + C3 * ys[2];
        else if (J == 1 || J == N + 1) vcv = C1 * ys[3] + C2 * ys[2] + C3 * ys[1];
        else vcv = A2 * (ys[0] + ys[3]) + A1 * (ys[1] + ys[2]);
        vtv = (vcv - u0 * cav) * rsv;
      }
      vtv = vtv > 0.0 ? dt2 * vtv * dxp * s4m : dt2 * vtv * dxp * s20;
    }
    uc[zo + o] = ucv;
    ut[zo + o] = utv;
    vc[zo + o] = vcv;
    vt[zo + o] = vtv;
  }
}

// ---- loads-first forms: every input a point needs is loaded before any arithmetic --
// addresses of the points outside the kernel's ranges clamped to an interior point, tile-edge
// inputs loaded only by the waves holding tile-edge lines, both upwind candidates of a
// data-dependent pick loaded and selected afterwards -- so a wave keeps its loads in flight
// together instead of waiting out a chain of dependent round trips through the branches
// (the branch-ordered forms, bit-identical and deleted in round 4, had 11-15
// vmcnt(0) waits per wave; rocprof SQ counters 63-65 % of wave cycles waiting).  The same form
// of cs_cgrid and ds_courant measured slower (1.84 -> 1.87 and 1.33 -> 1.47 ms per step):
// loading both upwind choices of their metric terms costs more than the round trips it saves.

// c_sw: upwind transport of delp/pt/w -> delpc/ptc/wc and the cell kinetic energy ke.  The
// Courant numbers, the cell's own values and the kinetic-energy inputs in one group, then
// the four upwind sources the signs select
__global__ void __launch_bounds__(256) cs_transport_ke_ld(
    Dims d, const SubInfo* __restrict__ subs, const double* __restrict__ M, int npz, double dt2,
    const double* __restrict__ delp, const double* __restrict__ pt, const double* __restrict__ w,
    const double* __restrict__ u, const double* __restrict__ v, const double* __restrict__ uc,
    const double* __restrict__ vc, const double* __restrict__ ua, const double* __restrict__ va,
    const double* __restrict__ ut, const double* __restrict__ vt, double* __restrict__ delpc,
    double* __restrict__ ptc, double* __restrict__ wc, double* __restrict__ ke, double* __restrict__ vort) {
  Launch2D L{-1, -1, d.nx + 2, d.ny + 2};
  KSETUP(npz)
  const long p = d.pitch;
  const double* dp = delp + zo;
  const double* pp = pt + zo;
  const double* ww = w + zo;
  const double c0 = ut[zo + o], c1 = ut[zo + o + 1], e0 = vt[zo + o], e1 = vt[zo + o + p];
  const double uav = ua[zo + o], vav = va[zo + o];
  const double uc0 = uc[zo + o], uc1 = uc[zo + o + 1], vc0 = vc[zo + o], vc1 = vc[zo + o + p];
  const long oc = cc_off(d, sub, i, j, 2);
  const double dpo = dp[oc], ppo = pp[oc], wwo = ww[oc];
  const double ra = MA(MT(M_RAREA), 0, 0);
  const bool xe = I == 0 || I == N || I == -1 || I == N - 1, ye = J == 0 || J == N || J == -1 || J == N - 1;
  double v00 = 0, v10 = 0, s1 = 0, k1 = 0, s3 = 0, k3 = 0, u00 = 0, u01 = 0, s2 = 0, k2 = 0, s4 = 0, k4 = 0;
  if (xe) {
    v00 = v[zo + o]; v10 = v[zo + o + 1];
    s1 = MT(M_SIN1)[o]; k1 = MT(M_COS1)[o]; s3 = MT(M_SIN3)[o]; k3 = MT(M_COS3)[o];
  }
  if (ye) {
    u00 = u[zo + o]; u01 = u[zo + o + p];
    s2 = MT(M_SIN2)[o]; k2 = MT(M_COS2)[o]; s4 = MT(M_SIN4)[o]; k4 = MT(M_COS4)[o];
  }
  const long sx0 = c0 > 0.0 ? cc_off(d, sub, i - 1, j, 1) : cc_off(d, sub, i, j, 1);
  const long sx1 = c1 > 0.0 ? cc_off(d, sub, i, j, 1) : cc_off(d, sub, i + 1, j, 1);
  const long sy0 = e0 > 0.0 ? cc_off(d, sub, i, j - 1, 2) : cc_off(d, sub, i, j, 2);
  const long sy1 = e1 > 0.0 ? cc_off(d, sub, i, j, 2) : cc_off(d, sub, i, j + 1, 2);
  const double dx0 = dp[sx0], px0 = pp[sx0], wx0 = ww[sx0], dx1 = dp[sx1], px1 = pp[sx1], wx1 = ww[sx1];
  const double dy0 = dp[sy0], py0 = pp[sy0], wy0 = ww[sy0], dy1 = dp[sy1], py1 = pp[sy1], wy1 = ww[sy1];
  double fx1[2], fx[2], fx2[2], fy1[2], fy[2], fy2[2];
  fx1[0] = c0 * dx0; fx[0] = fx1[0] * px0; fx2[0] = fx1[0] * wx0;
  fy1[0] = e0 * dy0; fy[0] = fy1[0] * py0; fy2[0] = fy1[0] * wy0;
  fx1[1] = c1 * dx1; fx[1] = fx1[1] * px1; fx2[1] = fx1[1] * wx1;
  fy1[1] = e1 * dy1; fy[1] = fy1[1] * py1; fy2[1] = fy1[1] * wy1;
  const double dpc = dpo + (fx1[0] - fx1[1] + fy1[0] - fy1[1]) * ra;
  AT(delpc, 0, 0) = dpc;
  AT(ptc, 0, 0) = (ppo * dpo + (fx[0] - fx[1] + fy[0] - fy[1]) * ra) / dpc;
  AT(wc, 0, 0) = (wwo * dpo + (fx2[0] - fx2[1] + fy2[0] - fy2[1]) * ra) / dpc;
  double kk, vv;
  if (uav > 0.0) {
    if (I == 0 || I == N) kk = uc0 * s1 + v00 * k1;
    else kk = uc0;
  } else {
    if (I == -1 || I == N - 1) kk = uc1 * s3 + v10 * k3;
    else kk = uc1;
  }
  if (vav > 0.0) {
    if (J == 0 || J == N) vv = vc0 * s2 + u00 * k2;
    else vv = vc0;
  } else {
    if (J == -1 || J == N - 1) vv = vc1 * s4 + u01 * k4;
    else vv = vc1;
  }
  const double dt4 = 0.5 * dt2;
  AT(ke, 0, 0) = dt4 * (uav * kk + vav * vv);
  // c_sw's absolute vorticity at the cell corners [0, nx] x [0, ny] (cs_vort's expressions and
  // order): uc, vc here are final, and the point's own uc0 / vc0 are already loaded
  if (i >= 0 && j >= 0) {
    const double* dxc = MT(M_DXC);
    const double* dyc = MT(M_DYC);
    const double fxs = AT(uc, 0, -1) * MA(dxc, 0, -1);
    const double fx0 = uc0 * MA(dxc, 0, 0);
    const double fyw = AT(vc, -1, 0) * MA(dyc, -1, 0);
    const double fy0 = vc0 * MA(dyc, 0, 0);
    double cv = fxs - fx0 - fyw + fy0;
    if ((I == 0 && J == 0) || (I == 0 && J == N)) cv = cv + fyw;
    if ((I == N && J == 0) || (I == N && J == N)) cv = cv - fy0;
    AT(vort, 0, 0) = MA(MT(M_FC), 0, 0) + MA(MT(M_RAREA_C), 0, 0) * cv;
  }
}

// d2a2c_vect part 1: utmp, vtmp (4th order interior / 2nd order near tile edges) and generic
// ua, va (cs_tmp_pt: the four u rows and four v columns of the 4th-order forms and the two
// metric terms in one group, the 4th-order / tile-edge / BIG choice made afterwards), the
// cube-corner fills included (formerly a cs_corner_fix launch after this one: a target thread
// forms its source point's values itself, same expressions, so the same bits)
// (L: the whole plane or its interior, H: a hole of L left to another launch -- the interior /
// boundary split of the u, v exchange, Dycore::step)
__global__ void __launch_bounds__(256) cs_tmp_ld(Dims d, Launch2D L, Launch2D H, const SubInfo* __restrict__ subs,
                                                 const double* __restrict__ M, int npz,
                                                 const double* __restrict__ u, const double* __restrict__ v,
                                                 double* __restrict__ utmp, double* __restrict__ vtmp,
                                                 double* __restrict__ ua, double* __restrict__ va,
                                                 double* __restrict__ dvort) {
  KSETUP(npz)
  if (i >= H.i0 && i < H.i0 + H.ni && j >= H.j0 && j < H.j0 + H.nj) return;
  const CsTmpPt t = cs_tmp_pt(d, sub, M, s, u, v, zo, i, j);
  double out[4] = {t.ut, t.vt, t.a, t.b};
  // cube-corner halo points (at most 10 per owned corner of a level): rare, so divergent
  const int io = sub.ioff, jo = sub.joff;
  // (every target lies west or east of the tile: I < 0 or I >= N)
  if (I < 0 || I >= N) {
    auto own = [&](int CI, int CJ) { return CI >= io && CI <= io + d.nx && CJ >= jo && CJ <= jo + d.ny; };
    const bool osw = own(0, 0), ose = own(N, 0), one = own(N, N), onw = own(0, N);
    for (int f = 0; f < 4; ++f) {
      int SI, SJ;
      double sg;
      if (!cs_corner_src(f, I, J, N, osw, ose, one, onw, SI, SJ, sg)) continue;
      const CsTmpPt q = cs_tmp_pt(d, sub, M, s, u, v, zo, SI - io, SJ - jo);
      const double src = f == 0 ? q.vt : f == 1 ? q.ut : f == 2 ? q.b : q.a;
      out[f] = sg < 0.0 ? -src : src;
    }
  }
  AT(utmp, 0, 0) = out[0];
  AT(vtmp, 0, 0) = out[1];
  AT(ua, 0, 0) = out[2];
  AT(va, 0, 0) = out[3];
  // d_sw's cell vorticity + Coriolis on [-NG, nx+NG-1] x [-NG, ny+NG-1] (ds_vort's expressions
  // and order) from the u(j+1), v(i+1) loaded above
  if (dvort && t.inr) {
    const double* dx = MT(M_DX);
    const double* dy = MT(M_DY);
    const double udx0 = t.u0 * MA(dx, 0, 0), udx1 = t.u1 * MA(dx, 0, 1);
    const double vdy0 = t.v0 * MA(dy, 0, 0), vdy1 = t.v1 * MA(dy, 1, 0);
    const double wk = MA(MT(M_RAREA), 0, 0) * (udx0 - udx1 + vdy1 - vdy0);
    AT(dvort, 0, 0) = wk + MA(MT(M_F0), 0, 0);
  }
}

// c_sw: time-centred C-grid winds (vorticity flux + KE gradient).  Both upwind vorticity
// values are loaded (the neighbour's are the same cache lines) and selected afterwards
__global__ void __launch_bounds__(256) cs_update_ld(Dims d, const SubInfo* __restrict__ subs,
                                                    const double* __restrict__ M, int npz, double dt2,
                                                    const double* __restrict__ u, const double* __restrict__ v,
                                                    const double* __restrict__ vort, const double* __restrict__ ke,
                                                    double* __restrict__ uc, double* __restrict__ vc) {
  Launch2D L{0, 0, d.nx + 1, d.ny + 1};
  KSETUP(npz)
  const long p = d.pitch;
  const double v0 = AT(v, 0, 0), u0 = AT(u, 0, 0), uc0 = AT(uc, 0, 0), vc0 = AT(vc, 0, 0);
  const double w00 = AT(vort, 0, 0), w01 = AT(vort, 0, 1), w10 = AT(vort, 1, 0);
  const double k00 = AT(ke, 0, 0), km0 = AT(ke, -1, 0), k0m = AT(ke, 0, -1);
  const double cau = MT(M_COSA_U)[o], sau = MT(M_SINA_U)[o], rdxc = MT(M_RDXC)[o];
  const double cav = MT(M_COSA_V)[o], sav = MT(M_SINA_V)[o], rdyc = MT(M_RDYC)[o];
  (void)p;
  if (j < d.ny) {
    double fy1 = (I == 0 || I == N) ? dt2 * v0 : dt2 * (v0 - uc0 * cau) / sau;
    double fy = fy1 > 0.0 ? w00 : w01;
    AT(uc, 0, 0) = uc0 + fy1 * fy + rdxc * (km0 - k00);
  }
  if (i < d.nx) {
    double fx1 = (J == 0 || J == N) ? dt2 * u0 : dt2 * (u0 - vc0 * cav) / sav;
    double fx = fx1 > 0.0 ? w00 : w10;
    AT(vc, 0, 0) = vc0 - fx1 * fx + rdyc * (k0m - k00);
  }
}

// ---------------- d_sw ----------------

// contravariant ut, vt: generic + direct tile-edge values
__global__ void __launch_bounds__(256) ds_utvt1(Dims d, const SubInfo* __restrict__ subs, const double* __restrict__ M,
                                                int npz, double dt, const double* __restrict__ uc,
                                                const double* __restrict__ vc, double* __restrict__ ut,
                                                double* __restrict__ vt) {
  Launch2D L{-NG, -NG, d.nx + 2 * NG + 1, d.ny + 2 * NG + 1};
  KSETUP(npz)
  const int nx = d.nx, ny = d.ny;
  double a = 0.0, b = 0.0;
  if (j <= ny + NG - 1) {
    if ((I == 0 || I == N) && i >= -1 && i <= nx + 1) {
      double c = AT(uc, 0, 0);
      a = c * dt > 0.0 ? c / MA(MT(M_SIN3), -1, 0) : c / MA(MT(M_SIN1), 0, 0);
    } else if (i >= -1 && i <= nx + 1 && J != -1 && J != 0 && J != N - 1 && J != N) {
      a = (AT(uc, 0, 0) - 0.25 * MA(MT(M_COSA_U), 0, 0) * (AT(vc, -1, 0) + AT(vc, 0, 0) + AT(vc, -1, 1) + AT(vc, 0, 1))) *
          MA(MT(M_RSIN_U), 0, 0);
    }
  }
  if (i <= nx + NG - 1) {
    if ((J == 0 || J == N)) {
      double c = AT(vc, 0, 0);
      b = c * dt > 0.0 ? c / MA(MT(M_SIN4), 0, -1) : c / MA(MT(M_SIN2), 0, 0);
    } else if (j >= -1 && j <= ny + 1) {
      b = (AT(vc, 0, 0) - 0.25 * MA(MT(M_COSA_V), 0, 0) * (AT(uc, 0, -1) + AT(uc, 1, -1) + AT(uc, 0, 0) + AT(uc, 1, 0))) *
          MA(MT(M_RSIN_V), 0, 0);
    }
  }
  AT(ut, 0, 0) = a;
  AT(vt, 0, 0) = b;
}

struct CornerMap {
  int N, fx, fy;
  __device__ int L0(int l) const { return fx == 1 ? l : N - l; }
  __device__ int L1(int l) const { return fy == 1 ? l : N - l; }
  __device__ int C0(int c) const { return fx == 1 ? c : N - 1 - c; }
  __device__ int C1(int c) const { return fy == 1 ? c : N - 1 - c; }
};

// ut, vt edge-adjacent cross terms and the cube-corner 2x2 solves (in place; sources never targets)
// (crx non-null: the Courant numbers of the lane's point re-formed from the final ut / vt, and
// the flux capacitor's sums on the lines ds_utvt1_kl leaves to this kernel -- see there)
__global__ void __launch_bounds__(256) ds_utvt2(Dims d, const SubInfo* __restrict__ subs, const double* __restrict__ M,
                                                int npz, const double* __restrict__ uc, const double* __restrict__ vc,
                                                double* __restrict__ ut, double* __restrict__ vt, double dt,
                                                double* __restrict__ crx, double* __restrict__ cry,
                                                double* __restrict__ xfx, double* __restrict__ yfx,
                                                double* __restrict__ cx, double* __restrict__ cy) {
  // all targets lie on the tile-edge lines: one lane per line point
  const int z = blockIdx.z, s = z / npz;
  const SubInfo sub = subs[s];
  int i, j;
  if (!edge_line_point(blockIdx.x * blockDim.x + threadIdx.x, sub, -NG, d.nx + NG, -NG, d.ny + NG, i, j)) return;
  const int N = sub.N;
  const int I = i + sub.ioff, J = j + sub.joff;
  const long zo = (long)z * d.plane;
  const long o = pidx(d, i, j);
  const int io = sub.ioff, jo = sub.joff, nx = d.nx, ny = d.ny;
  // cross terms
  bool has_vt = false, has_ut = false;
  double nvt = 0.0, nut = 0.0;
  if ((I == -1 || I == 0 || I == N - 1 || I == N) && J >= max(2, jo) && J <= min(N - 2, jo + ny)) {
    nvt = AT(vc, 0, 0) - 0.25 * MA(MT(M_COSA_V), 0, 0) * (AT(ut, 0, -1) + AT(ut, 1, -1) + AT(ut, 0, 0) + AT(ut, 1, 0));
    has_vt = true;
  }
  if ((J == -1 || J == 0 || J == N - 1 || J == N) && I >= max(2, io) && I <= min(N - 2, io + nx)) {
    nut = AT(uc, 0, 0) - 0.25 * MA(MT(M_COSA_U), 0, 0) * (AT(vt, -1, 0) + AT(vt, 0, 0) + AT(vt, -1, 1) + AT(vt, 0, 1));
    has_ut = true;
  }
  // cube-corner solves: each target point of each owned corner
  const int cc[4][2] = {{0, 0}, {N, 0}, {N, N}, {0, N}};
  for (int q = 0; q < 4; ++q) {
    const int cxg = cc[q][0], cyg = cc[q][1];
    if (!(cxg >= io && cxg <= io + nx && cyg >= jo && cyg <= jo + ny)) continue;
    CornerMap cm{N, cxg == N ? -1 : 1, cyg == N ? -1 : 1};
    auto g = [&](const double* a, int Ig, int Jg) { return a[zo + pidx(d, Ig - io, Jg - jo)]; };
    auto gm = [&](int metric, int Ig, int Jg) { return met(M, d, metric, s)[pidx(d, Ig - io, Jg - jo)]; };
    auto UT = [&](int a, int b) { return g(ut, cm.L0(a), cm.C1(b)); };
    auto VT = [&](int a, int b) { return g(vt, cm.C0(a), cm.L1(b)); };
    auto UC = [&](int a, int b) { return g(uc, cm.L0(a), cm.C1(b)); };
    auto VC = [&](int a, int b) { return g(vc, cm.C0(a), cm.L1(b)); };
    auto CU = [&](int a, int b) { return gm(M_COSA_U, cm.L0(a), cm.C1(b)); };
    auto CV = [&](int a, int b) { return gm(M_COSA_V, cm.C0(a), cm.L1(b)); };
    if (I == cm.L0(1) && J == cm.C1(-1)) {
      double d1 = 1.0 / (1.0 - 0.0625 * CU(1, -1) * CV(0, -1));
      nut = (UC(1, -1) - 0.25 * CU(1, -1) *
                             (VT(0, 0) + VT(1, 0) + VT(1, -1) + VC(0, -1) -
                              0.25 * CV(0, -1) * (UT(0, -1) + UT(0, -2) + UT(1, -2)))) * d1;
      has_ut = true;
    }
    if (I == cm.L0(1) && J == cm.C1(0)) {
      double d3 = 1.0 / (1.0 - 0.0625 * CU(1, 0) * CV(0, 1));
      nut = (UC(1, 0) - 0.25 * CU(1, 0) *
                            (VT(0, 0) + VT(1, 0) + VT(1, 1) + VC(0, 1) -
                             0.25 * CV(0, 1) * (UT(0, 0) + UT(0, 1) + UT(1, 1)))) * d3;
      has_ut = true;
    }
    if (I == cm.C0(-1) && J == cm.L1(1)) {
      double d2 = 1.0 / (1.0 - 0.0625 * CU(-1, 0) * CV(-1, 1));
      nvt = (VC(-1, 1) - 0.25 * CV(-1, 1) *
                             (UT(0, 0) + UT(0, 1) + UT(-1, 1) + UC(-1, 0) -
                              0.25 * CU(-1, 0) * (VT(-1, 0) + VT(-2, 0) + VT(-2, 1)))) * d2;
      has_vt = true;
    }
    if (I == cm.C0(0) && J == cm.L1(1)) {
      double d3 = 1.0 / (1.0 - 0.0625 * CU(1, 0) * CV(0, 1));
      nvt = (VC(0, 1) - 0.25 * CV(0, 1) *
                            (UT(0, 0) + UT(0, 1) + UT(1, 1) + UC(1, 0) -
                             0.25 * CU(1, 0) * (VT(0, 0) + VT(1, 0) + VT(1, 1)))) * d3;
      has_vt = true;
    }
  }
  // targets and sources are disjoint point sets, so no barrier is needed
  if (has_ut) AT(ut, 0, 0) = nut;
  if (has_vt) AT(vt, 0, 0) = nvt;
  if (crx) {
    const long pt = d.pitch;
    // x faces on the y-lines (ut's targets), y faces on the x-lines (vt's): one lane per point
    // (re-formed where this kernel changed ut / vt; elsewhere ds_utvt1_kl's values stand and
    // only the sum is taken)
    if ((J == -1 || J == 0 || J == N - 1 || J == N) && i >= 0 && i <= nx && j <= ny + NG - 1) {
      double c, f;
      if (has_ut) {
        courant_face(dt, nut, met(M, d, M_RDXA, s)[o - 1], met(M, d, M_RDXA, s)[o], met(M, d, M_DY, s)[o],
                     met(M, d, M_SIN3, s)[o - 1], met(M, d, M_SIN1, s)[o], c, f);
        AT(crx, 0, 0) = c;
        AT(xfx, 0, 0) = f;
      } else {
        c = AT(crx, 0, 0);
      }
      if (cx) AT(cx, 0, 0) += c;
    }
    if ((I == -1 || I == 0 || I == N - 1 || I == N) && j >= 0 && j <= ny && i <= nx + NG - 1) {
      double c, f;
      if (has_vt) {
        courant_face(dt, nvt, met(M, d, M_RDYA, s)[o - pt], met(M, d, M_RDYA, s)[o], met(M, d, M_DX, s)[o],
                     met(M, d, M_SIN4, s)[o - pt], met(M, d, M_SIN2, s)[o], c, f);
        AT(cry, 0, 0) = c;
        AT(yfx, 0, 0) = f;
      } else {
        c = AT(cry, 0, 0);
      }
      if (cy) AT(cy, 0, 0) += c;
    }
  }
}

// advective Courant numbers and area fluxes (saved per level for update_dz_d) + ra_x, ra_y
__global__ void __launch_bounds__(256) ds_courant(Dims d, const SubInfo* __restrict__ subs,
                                                  const double* __restrict__ M, int npz, double dt,
                                                  const double* __restrict__ ut, const double* __restrict__ vt,
                                                  double* __restrict__ crx, double* __restrict__ cry,
                                                  double* __restrict__ xfx, double* __restrict__ yfx,
                                                  double* __restrict__ cx, double* __restrict__ cy) {
  Launch2D L{-NG, -NG, d.nx + 2 * NG + 1, d.ny + 2 * NG + 1};
  KSETUP(npz)
  const int nx = d.nx, ny = d.ny;
  double a = 0.0, b = 0.0, c = 0.0, e = 0.0;
  if (i >= 0 && i <= nx && j <= ny + NG - 1) {
    double xf = dt * AT(ut, 0, 0);
    if (xf > 0.0) {
      a = xf * MA(MT(M_RDXA), -1, 0);
      b = MA(MT(M_DY), 0, 0) * xf * MA(MT(M_SIN3), -1, 0);
    } else {
      a = xf * MA(MT(M_RDXA), 0, 0);
      b = MA(MT(M_DY), 0, 0) * xf * MA(MT(M_SIN1), 0, 0);
    }
  }
  if (j >= 0 && j <= ny && i <= nx + NG - 1) {
    double yf = dt * AT(vt, 0, 0);
    if (yf > 0.0) {
      c = yf * MA(MT(M_RDYA), 0, -1);
      e = MA(MT(M_DX), 0, 0) * yf * MA(MT(M_SIN4), 0, -1);
    } else {
      c = yf * MA(MT(M_RDYA), 0, 0);
      e = MA(MT(M_DX), 0, 0) * yf * MA(MT(M_SIN2), 0, 0);
    }
  }
  AT(crx, 0, 0) = a;
  AT(xfx, 0, 0) = b;
  AT(cry, 0, 0) = c;
  AT(yfx, 0, 0) = e;
  // Courant accumulation of the flux capacitor (ds_accum's cx / cy part, same ranges), here
  // when the thermo march accumulates the mass fluxes itself
  if (cx) {
    if (i >= 0 && i <= nx && j <= ny + NG - 1) AT(cx, 0, 0) += a;
    if (j >= 0 && j <= ny && i <= nx + NG - 1) AT(cy, 0, 0) += c;
  }
}

// ---- level-loop form of ds_utvt1 (stencil_common.hpp kloop_levels): the metric terms of
// the point are loaded once for its block of levels (which of them a point needs is fixed by
// its position), then the same expressions per level as above.  (The same form of
// ds_courant and ds_ke measured slower: 1.56 -> 1.68 and 2.65 -> 3.37 ms per step)
// (L: the whole plane or its interior, H: a hole of L left to another launch -- the interior /
// boundary split of the uc, vc exchange)
// With crx non-null the Courant numbers and area fluxes of ds_courant are formed here too from
// the ut / vt just computed (ds_utvt2 re-forms them on the tile-edge lines where it corrects ut /
// vt), and with cx / cy non-null the flux capacitor's Courant sums take them -- except on the
// lines ds_utvt2 owns (x faces on J = -1, 0, N-1, N; y faces on I = -1, 0, N-1, N), which it sums.
__global__ void __launch_bounds__(256) ds_utvt1_kl(Dims d, Launch2D L, Launch2D H, const SubInfo* __restrict__ subs,
                                                   const double* __restrict__ M, int npz, int nkb, int klb,
                                                   double dt, const double* __restrict__ uc,
                                                   const double* __restrict__ vc, double* __restrict__ ut,
                                                   double* __restrict__ vt, double* __restrict__ crx,
                                                   double* __restrict__ cry, double* __restrict__ xfx,
                                                   double* __restrict__ yfx, double* __restrict__ cx,
                                                   double* __restrict__ cy) {
  KLSETUP(npz)
  if (i >= H.i0 && i < H.i0 + H.ni && j >= H.j0 && j < H.j0 + H.nj) return;
  const SubInfo sub = subs[s];
  const int N = sub.N, I = i + sub.ioff, J = j + sub.joff, nx = d.nx, ny = d.ny;
  const long pt = d.pitch;
  // ds_courant's regions and metric terms of the point (once for its block of levels)
  const bool xr = crx && i >= 0 && i <= nx && j <= ny + NG - 1, yr = crx && j >= 0 && j <= ny && i <= nx + NG - 1;
  double rxm = 0.0, rx0 = 0.0, dyp = 0.0, s3m = 0.0, s10 = 0.0, rym = 0.0, ry0 = 0.0, dxp = 0.0, s4m = 0.0, s20 = 0.0;
  if (xr) {
    rxm = met(M, d, M_RDXA, s)[o - 1]; rx0 = met(M, d, M_RDXA, s)[o]; dyp = met(M, d, M_DY, s)[o];
    s3m = met(M, d, M_SIN3, s)[o - 1]; s10 = met(M, d, M_SIN1, s)[o];
  }
  if (yr) {
    rym = met(M, d, M_RDYA, s)[o - pt]; ry0 = met(M, d, M_RDYA, s)[o]; dxp = met(M, d, M_DX, s)[o];
    s4m = met(M, d, M_SIN4, s)[o - pt]; s20 = met(M, d, M_SIN2, s)[o];
  }
  const bool xsum = xr && cx && !(J == -1 || J == 0 || J == N - 1 || J == N);
  const bool ysum = yr && cy && !(I == -1 || I == 0 || I == N - 1 || I == N);
  // x: 0 none, 1 tile-edge division, 2 generic; y likewise
  int mx = 0, my = 0;
  double ax = 0.0, bx = 0.0, ay = 0.0, by = 0.0;
  if (j <= ny + NG - 1) {
    if ((I == 0 || I == N) && i >= -1 && i <= nx + 1) {
      mx = 1; ax = met(M, d, M_SIN3, s)[o - 1]; bx = met(M, d, M_SIN1, s)[o];
    } else if (i >= -1 && i <= nx + 1 && J != -1 && J != 0 && J != N - 1 && J != N) {
      mx = 2; ax = met(M, d, M_COSA_U, s)[o]; bx = met(M, d, M_RSIN_U, s)[o];
    }
  }
  if (i <= nx + NG - 1) {
    if (J == 0 || J == N) {
      my = 1; ay = met(M, d, M_SIN4, s)[o - pt]; by = met(M, d, M_SIN2, s)[o];
    } else if (j >= -1 && j <= ny + 1) {
      my = 2; ay = met(M, d, M_COSA_V, s)[o]; by = met(M, d, M_RSIN_V, s)[o];
    }
  }
  // loads first: the point's uc / vc and the four neighbours of each generic form in one
  // group per level (offset 0 where the form is not taken)
  const long xw = mx == 2 ? -1 : 0, xn = mx == 2 ? pt : 0;
  const long ys = my == 2 ? -pt : 0, ye = my == 2 ? 1 : 0;
  // with the Courant numbers formed here, ut / vt are read afterwards only within three points
  // of a tile edge (ds_utvt2's lines and cube-corner solves, ds_ke's tile-edge lines): stored
  // there only
  // (A/B in one box: 31.53-31.85 -> 31.21-31.62 ms per step)
  const bool wut = !crx || I <= 3 || I >= N - 3 || J <= 3 || J >= N - 3;
  for (int k = k0; k < k1; ++k) {
    const long lk = ((long)s * npz + k) * P + o;
    const double u0 = uc[lk], v0 = vc[lk];
    const double vw = vc[lk + xw], vwn = vc[lk + xw + xn], vn = vc[lk + xn];
    const double us = uc[lk + ys], use = uc[lk + ye + ys], ue = uc[lk + ye];
    double a = 0.0, b = 0.0;
    if (mx == 1) a = u0 * dt > 0.0 ? u0 / ax : u0 / bx;
    else if (mx == 2) a = (u0 - 0.25 * ax * (vw + v0 + vwn + vn)) * bx;
    if (my == 1) b = v0 * dt > 0.0 ? v0 / ay : v0 / by;
    else if (my == 2) b = (v0 - 0.25 * ay * (us + use + u0 + ue)) * by;
    if (wut) {
      ut[lk] = a;
      vt[lk] = b;
    }
    if (crx) {
      double ca = 0.0, fa = 0.0, cb = 0.0, fb = 0.0;
      if (xr) courant_face(dt, a, rxm, rx0, dyp, s3m, s10, ca, fa);
      if (yr) courant_face(dt, b, rym, ry0, dxp, s4m, s20, cb, fb);
      crx[lk] = ca;
      xfx[lk] = fa;
      cry[lk] = cb;
      yfx[lk] = fb;
      if (xsum) cx[lk] += ca;
      if (ysum) cy[lk] += cb;
    }
  }
}

// Courant / mass-flux accumulation for tracer transport ("flux capacitor")
__global__ void __launch_bounds__(256) ds_accum(Dims d, const SubInfo* __restrict__ subs, int npz,
                                                const double* __restrict__ crx, const double* __restrict__ cry,
                                                const double* __restrict__ fx, const double* __restrict__ fy,
                                                double* __restrict__ cx, double* __restrict__ cy,
                                                double* __restrict__ mfx, double* __restrict__ mfy) {
  Launch2D L{-NG, -NG, d.nx + 2 * NG + 1, d.ny + 2 * NG + 1};
  KSETUP(npz)
  const int nx = d.nx, ny = d.ny;
  if (i >= 0 && i <= nx && j <= ny + NG - 1) AT(cx, 0, 0) += AT(crx, 0, 0);
  if (i >= 0 && i <= nx && j >= 0 && j < ny) AT(mfx, 0, 0) += AT(fx, 0, 0);
  if (j >= 0 && j <= ny && i <= nx + NG - 1) AT(cy, 0, 0) += AT(cry, 0, 0);
  if (j >= 0 && j <= ny && i >= 0 && i < nx) AT(mfy, 0, 0) += AT(fy, 0, 0);
}

// delp, pt, w update from the transported fluxes (compute cells)
__global__ void __launch_bounds__(256) ds_thermo(Dims d, const SubInfo* __restrict__ subs, const double* __restrict__ M,
                                                 int npz, const double* __restrict__ fx, const double* __restrict__ fy,
                                                 const double* __restrict__ gwx, const double* __restrict__ gwy,
                                                 const double* __restrict__ gtx, const double* __restrict__ gty,
                                                 double* __restrict__ delp, double* __restrict__ pt,
                                                 double* __restrict__ w) {
  Launch2D L{0, 0, d.nx, d.ny};
  KSETUP(npz)
  const double ra = MA(MT(M_RAREA), 0, 0);
  const double dp = AT(delp, 0, 0);
  double wn = dp * AT(w, 0, 0) + (AT(gwx, 0, 0) - AT(gwx, 1, 0) + AT(gwy, 0, 0) - AT(gwy, 0, 1)) * ra;
  double ptn = AT(pt, 0, 0) * dp + (AT(gtx, 0, 0) - AT(gtx, 1, 0) + AT(gty, 0, 0) - AT(gty, 0, 1)) * ra;
  double dpn = dp + (AT(fx, 0, 0) - AT(fx, 1, 0) + AT(fy, 0, 0) - AT(fy, 0, 1)) * ra;
  AT(pt, 0, 0) = ptn / dpn;
  AT(delp, 0, 0) = dpn;
  AT(w, 0, 0) = wn / dpn;
}

// kinetic energy at cell corners: B-grid contravariant winds, upwind PPM of v (ytp_v) and u
// (xtp_u), cube-corner values, plus nord = 0 divergence damping added to ke.  Every value an
// interior corner needs -- the B-grid wind inputs, both
// six-point PPM stencils, the Courant metric and the divergence-damping terms -- is loaded
// unconditionally before any arithmetic, so a wave has ~45 loads in flight at once instead of
// ~15 dependent round trips through branches (rocprof SQ counters: ds_ke waited 63 % of its
// wave cycles).  Tile-edge inputs (vt / ut stencils, dx / dy for the edge PPM forms, sin1-4)
// are loaded only by the waves holding such points.  hord_mt and "some level has nord = 0"
// are template constants; the level's own parameters (nord, d2_divg: the sponge layers') come
// from the column table lv, one value per wave.
template <int ORD, bool DAMP>
__global__ void __launch_bounds__(256) ds_ke_ld(Dims d, const SubInfo* __restrict__ subs,
                                                const double* __restrict__ M, int npz, double dt, double dddmp,
                                                const LevelDamp* __restrict__ lv, double da_min_c,
                                                const double* __restrict__ u,
                                                const double* __restrict__ v, const double* __restrict__ uc,
                                                const double* __restrict__ vc, const double* __restrict__ ua,
                                                const double* __restrict__ va, const double* __restrict__ ut,
                                                const double* __restrict__ vt, double* __restrict__ ke,
                                                double* __restrict__ vd) {
  Launch2D L{0, 0, d.nx + 1, d.ny + 1};
  KSETUP(npz)
  const int io = sub.ioff, jo = sub.joff, nx = d.nx, ny = d.ny;
  const long p = d.pitch;
  const double dt5 = 0.5 * dt, dt4 = 0.25 * dt;
  const int kl = z - s * npz;
  const bool dmp = DAMP && lv[kl].nord == 0;  // nord = 0 divergence damping at this level
  const int Ilo = max(1, io), Ihi = min(N - 1, io + nx), Jlo = max(1, jo), Jhi = min(N - 1, jo + ny);
  const bool inner = I >= Ilo && I <= Ihi && J >= Jlo && J <= Jhi;
  const bool xe = !(I - 1 >= 2 && I + 1 <= N - 2), ye = !(J - 1 >= 2 && J + 1 <= N - 2);
  const bool xl = I == 0 || I == N, yl = J == 0 || J == N;
  const double *U = u + zo + o, *V = v + zo + o, *UC = uc + zo + o, *VC = vc + zo + o;
  // ---- every interior input, issued together
  const double vcm = VC[-1], vc0 = VC[0], ucm = UC[-p], uc0 = UC[0];
  const double cosa = MT(M_COSA)[o], rsina = MT(M_RSINA)[o];
  double qv[6], qu[6];
#pragma unroll
  for (int m = 0; m < 6; ++m) {
    qv[m] = V[(long)(m - 3) * p];
    qu[m] = U[m - 3];
  }
  const double* rdy = MT(M_RDY) + o;
  const double* rdx = MT(M_RDX) + o;
  const double rdym = rdy[-p], rdy0 = rdy[0], rdxm = rdx[-1], rdx0 = rdx[0];
  double dycm = 0, dyc0 = 0, vamm = 0, vam0 = 0, va0m = 0, va00 = 0, cvm = 0, cv0 = 0, svm = 0, sv0 = 0;
  double dxcm = 0, dxc0 = 0, uamm = 0, ua0m = 0, uam0 = 0, ua00 = 0, cum = 0, cu0 = 0, sum_ = 0, su0 = 0, rac = 0;
  if (dmp) {
    const double* dyc = MT(M_DYC) + o;
    const double* dxc = MT(M_DXC) + o;
    const double* cav = MT(M_COSA_V) + o;
    const double* sav = MT(M_SINA_V) + o;
    const double* cau = MT(M_COSA_U) + o;
    const double* sau = MT(M_SINA_U) + o;
    const double *VA = va + zo + o, *UA = ua + zo + o;
    dycm = dyc[-1]; dyc0 = dyc[0];
    vamm = VA[-1 - p]; vam0 = VA[-1]; va0m = VA[-p]; va00 = VA[0];
    cvm = cav[-1]; cv0 = cav[0]; svm = sav[-1]; sv0 = sav[0];
    dxcm = dxc[-p]; dxc0 = dxc[0];
    uamm = UA[-1 - p]; ua0m = UA[-p]; uam0 = UA[-1]; ua00 = UA[0];
    cum = cau[-p]; cu0 = cau[0]; sum_ = sau[-p]; su0 = sau[0];
    rac = MT(M_RAREA_C)[o];
  }
  // ---- tile-edge inputs (waves with an edge point only)
  double vts[4] = {0, 0, 0, 0}, uts[4] = {0, 0, 0, 0}, spy[6] = {0, 0, 0, 0, 0, 0}, spx[6] = {0, 0, 0, 0, 0, 0};
  double s4m = 0, s40 = 0, s2m = 0, s20 = 0, s3m = 0, s30 = 0, s1m = 0, s10 = 0;
  if (xe || ye) {
    const double *VT = vt + zo + o, *UT = ut + zo + o;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      vts[m] = VT[m - 2];
      uts[m] = UT[(long)(m - 2) * p];
    }
    const double* dy = MT(M_DY) + o;
    const double* dxm = MT(M_DX) + o;
#pragma unroll
    for (int m = 0; m < 6; ++m) {
      spy[m] = ye ? dy[(long)(m - 3) * p] : 0.0;
      spx[m] = xe ? dxm[m - 3] : 0.0;
    }
    if (dmp) {
      const double* s4 = MT(M_SIN4) + o;
      const double* s2 = MT(M_SIN2) + o;
      const double* s3 = MT(M_SIN3) + o;
      const double* s1 = MT(M_SIN1) + o;
      s4m = s4[-1 - p]; s40 = s4[-p]; s2m = s2[-1]; s20 = s2[0];
      s3m = s3[-1 - p]; s30 = s3[-1]; s1m = s1[-p]; s10 = s1[0];
    }
  }
  // ---- ds_ke's expressions
  double vb = 0.0, ub = 0.0;
  if (inner) vb = dt5 * (vcm + vc0 - (ucm + uc0) * cosa) * rsina;
  if (xl) vb = dt4 * (-vts[0] + 3.0 * (vts[1] + vts[2]) - vts[3]);
  else if (yl && I >= Ilo && I <= Ihi) vb = dt5 * (vts[1] + vts[2]);
  if (inner) ub = dt5 * (ucm + uc0 - (vcm + vc0) * cosa) * rsina;
  if (yl) ub = dt4 * (-uts[0] + 3.0 * (uts[1] + uts[2]) - uts[3]);
  else if (xl && J >= Jlo && J <= Jhi) ub = dt5 * (uts[1] + uts[2]);
  double cfl = vb > 0.0 ? vb * rdym : vb * rdy0;
  const double ubf = ye ? ppm_flux<ORD>(J, N, qv, spy, cfl) : ppm_flux<ORD, false>(J, N, qv, spy, cfl);
  double kk = vb * ubf;
  cfl = ub > 0.0 ? ub * rdxm : ub * rdx0;
  const double vbf = xe ? ppm_flux<ORD>(I, N, qu, spx, cfl) : ppm_flux<ORD, false>(I, N, qu, spx, cfl);
  kk = 0.5 * (kk + ub * vbf);
  // cube corners: u(0,0) = qu[3], u(-1,0) = qu[2], v(0,0) = qv[3], v(0,-1) = qv[2]
  const double dt6 = dt / 6.0;
  if (I == 0 && J == 0)
    kk = dt6 * ((uts[2] + uts[1]) * qu[3] + (vts[2] + vts[1]) * qv[3] + (uts[2] + vts[2]) * qu[2]);
  else if (I == N && J == 0)
    kk = dt6 * ((uts[2] + uts[1]) * qu[2] + (vts[2] + vts[1]) * qv[3] + (uts[2] - vts[1]) * qu[3]);
  else if (I == N && J == N)
    kk = dt6 * ((uts[2] + uts[1]) * qu[2] + (vts[2] + vts[1]) * qv[2] + (uts[1] + vts[1]) * qu[3]);
  else if (I == 0 && J == N)
    kk = dt6 * ((uts[2] + uts[1]) * qu[3] + (vts[2] + vts[1]) * qv[2] + (uts[1] - vts[2]) * qu[2]);
  if (!dmp) {
    AT(ke, 0, 0) = kk;
    return;
  }
  // divergence damping (nord = 0), ds_ke's ptc_at / vrt_at
  double ptm, pt0;
  if (yl) {
    ptm = vcm > 0.0 ? qu[2] * dycm * s4m : qu[2] * dycm * s2m;
    pt0 = vc0 > 0.0 ? qu[3] * dyc0 * s40 : qu[3] * dyc0 * s20;
  } else {
    ptm = (qu[2] - 0.5 * (vamm + vam0) * cvm) * dycm * svm;
    pt0 = (qu[3] - 0.5 * (va0m + va00) * cv0) * dyc0 * sv0;
  }
  double vS = 0.0, v0 = 0.0;
  if (xl) {
    vS = ucm > 0.0 ? qv[2] * dxcm * s3m : qv[2] * dxcm * s1m;
    v0 = uc0 > 0.0 ? qv[3] * dxc0 * s30 : qv[3] * dxc0 * s10;
  } else if (I >= Ilo && I <= Ihi) {
    vS = (qv[2] - 0.5 * (uamm + ua0m) * cum) * dxcm * sum_;
    v0 = (qv[3] - 0.5 * (uam0 + ua00) * cu0) * dxc0 * su0;
  }
  double dpc = vS - v0 + ptm - pt0;
  if ((I == 0 && J == 0) || (I == N && J == 0)) dpc = dpc - vS;
  if ((I == N && J == N) || (I == 0 && J == N)) dpc = dpc + v0;
  dpc = rac * dpc;
  double damp = da_min_c * fmax(lv[kl].d2_divg, fmin(0.20, dddmp * fabs(dpc * dt)));
  AT(ke, 0, 0) = kk + damp * dpc;
  if (vd) AT(vd, 0, 0) = damp * dpc;
}

// relative vorticity (cell mean) + Coriolis -> the field transported by fv_tp_2d
__global__ void __launch_bounds__(256) ds_vort(Dims d, const SubInfo* __restrict__ subs, const double* __restrict__ M,
                                               int npz, const double* __restrict__ u, const double* __restrict__ v,
                                               double* __restrict__ vort) {
  Launch2D L{-NG, -NG, d.nx + 2 * NG, d.ny + 2 * NG};
  KSETUP(npz)
  const double* dx = MT(M_DX);
  const double* dy = MT(M_DY);
  double udx0 = AT(u, 0, 0) * MA(dx, 0, 0), udx1 = AT(u, 0, 1) * MA(dx, 0, 1);
  double vdy0 = AT(v, 0, 0) * MA(dy, 0, 0), vdy1 = AT(v, 1, 0) * MA(dy, 1, 0);
  double wk = MA(MT(M_RAREA), 0, 0) * (udx0 - udx1 + vdy1 - vdy0);
  AT(vort, 0, 0) = wk + MA(MT(M_F0), 0, 0);
}


inline dim3 g2(const Dims& d, const Launch2D& L, int nz) {
  (void)d;
  return plane_grid_lv(L, nz);
}

}  // namespace

void c_sw(const Ctx& c, const CswArgs& a) {
  c_sw_transport(c, a, 0);
  c_sw_winds(c, a);
}

// c_sw first stage: d2a2c_vect (uc, vc, ua, va, ut, vt), the half-step transport (delpc,
// ptc, wc), the kinetic energy and the corner vorticity
// the boundary frame runs as one whole-plane launch with the interior as its hole (four
// rectangle launches cost more in launch latency at the small per-rank shares)
static const Launch2D kNoHole{0, 0, 0, 0};

bool split_fits(const Dims& d) { return d.nx >= 6 && d.ny >= 6; }

void c_sw_transport(const Ctx& c, const CswArgs& a, int part) {
  const Dims& d = c.d;
  const int nz = d.nsub * a.npz;
  Launch2D full{-NG, -NG, d.nx + 2 * NG + 1, d.ny + 2 * NG + 1};
  const Ext e = ext(d);
  const double L = a.npz;
  // cs_tmp reads u on rows j-1 .. j+2 and v on columns i-1 .. i+2 of the point: on
  // [1, nx-2] x [1, ny-2] only owned values, none an exchange writes
  const Launch2D inner{1, 1, d.nx - 2, d.ny - 2};
  auto tmp = [&](const Launch2D& r, const Launch2D& h) {
    GT_LAUNCH_N("cs_tmp", cs_tmp_ld, g2(d, r, nz), dim3(BX, BY), 0, c.st, d, r, h, c.subs, c.met, a.npz, a.u, a.v,
                a.utmp, a.vtmp, a.ua, a.va, a.dvort);
    HIP_LAUNCH_CHECK();
  };
  // (d_sw's cell vorticity when asked: one more plane written, dx dy rarea f0 read)
  const double tb = L * (e.Y + e.X + 4 * e.C) + 2 * e.C + (a.dvort ? L * e.C + 4 * e.C : 0.0);
  if (part == 1) {
    tmp(inner, kNoHole);
    gt_bytes(tb);
    return;
  }
  tmp(full, part == 2 ? inner : kNoHole);
  if (part == 0) gt_bytes(tb);
  // (the level-loop form: 32.0-32.15 -> 31.54-31.57 ms per step as an A/B pair)
  if (const int klb = kloop_levels()) {
    const int nkb = (a.npz + klb - 1) / klb;
    GT_LAUNCH_N("cs_cgrid", cs_cgrid_kl, kloop_grid(full, d.nsub, nkb), dim3(BX, BY), 0, c.st, d, c.subs, c.met,
                a.npz, nkb, klb, a.dt2, a.u, a.v, a.utmp, a.vtmp, a.ua, a.va, a.uc, a.vc, a.ut, a.vt);
  } else {
    GT_LAUNCH(cs_cgrid, g2(d, full, nz), dim3(BX, BY), 0, c.st, d, c.subs, c.met, a.npz, a.dt2, a.u, a.v,
                       a.utmp, a.vtmp, a.ua, a.va, a.uc, a.vc, a.ut, a.vt);
  }
  HIP_LAUNCH_CHECK();
  gt_bytes(L * (3 * e.X + 3 * e.Y + 4 * e.C) + 12 * e.C);
  Launch2D Lt{-1, -1, d.nx + 2, d.ny + 2};
  // the corner vorticity of the wind stage formed here too (the separate cs_vort launch
  // re-read uc, vc: 32.17-32.47 -> 31.98-32.23 ms per step)
  double* vort = a.vort;
  GT_LAUNCH_N("cs_transport_ke", cs_transport_ke_ld, g2(d, Lt, nz), dim3(BX, BY), 0, c.st, d, c.subs, c.met,
              a.npz, a.dt2, a.delp, a.pt, a.w, a.u, a.v, a.uc, a.vc, a.ua, a.va, a.ut, a.vt, a.delpc, a.ptc, a.wc, a.ke,
              vort);
  HIP_LAUNCH_CHECK();
  gt_bytes(L * (9 * e.C + 3 * e.X + 3 * e.Y + e.K) + 13 * e.C);
}

// c_sw second stage: the time-centred C-grid winds from the corner vorticity and ke of the
// first stage (touches uc, vc: independent of update_dz_c / riem_solver_c, which may run
// beside it)
void c_sw_winds(const Ctx& c, const CswArgs& a) {
  const Dims& d = c.d;
  const int nz = d.nsub * a.npz;
  const Ext e = ext(d);
  const double L = a.npz;
  Launch2D Lc{0, 0, d.nx + 1, d.ny + 1};
  GT_LAUNCH_N("cs_update", cs_update_ld, g2(d, Lc, nz), dim3(BX, BY), 0, c.st, d, c.subs, c.met, a.npz, a.dt2,
              a.u, a.v, a.vort, a.ke, a.uc, a.vc);
  HIP_LAUNCH_CHECK();
  gt_bytes(L * (e.C + e.K + 3 * e.X + 3 * e.Y) + 6 * e.C);
}

// d_sw in three stages: the contravariant winds and Courant numbers; the mass-flux and
// thermodynamic transport (delp, w, pt); the kinetic energy and vorticity transport that
// update u, v.  After the first stage the other two touch disjoint fields (the vorticity
// transport writes its own flux planes gvx, gvy), so the dycore runs them on two streams.
// d_sw's delp / w / pt transport as one register-resident march (tp.hip) when the three
// PPM orders agree and the caller provides the output planes (GTFV3_THERMO_FUSED=0: the
// separate fv_tp_2d launches, ds_accum and ds_thermo)
bool d_sw_thermo_fused(const DswArgs& a) {
  static const bool on = [] {
    const char* e = getenv("GTFV3_THERMO_FUSED");
    return !(e && e[0] == '0');
  }();
  // the march carries no del-n flux damping of delp / pt: levels with it take the separate launches
  const bool deln = a.hlv && (any_level(a.hlv, a.npz, &LevelDamp::dp4) || any_level(a.hlv, a.npz, &LevelDamp::pt4));
  return on && !deln && a.delp_o && a.w_o && a.pt_o && a.hord_dp == a.hord_vt && a.hord_vt == a.hord_tm;
}

void d_sw_courant(const Ctx& c, const DswArgs& a, hipEvent_t utvt_done, int part) {
  const Dims& d = c.d;
  const int nz = d.nsub * a.npz;
  Launch2D full{-NG, -NG, d.nx + 2 * NG + 1, d.ny + 2 * NG + 1};
  const int klb = kloop_levels(), nkb = klb ? (a.npz + klb - 1) / klb : 0;
  const Ext e = ext(d);
  const double L = a.npz;
  // ds_utvt1 reads uc at (i, j), (i+1, j-1), (i+1, j) and vc at (i, j), (i-1, j), (i-1, j+1),
  // (i, j+1): on [1, nx-1] x [1, ny-1] only owned values, none an exchange writes (the split
  // form needs the level-loop kernel, which takes its region)
  const Launch2D inner{1, 1, d.nx - 1, d.ny - 1};
  // the Courant numbers (and with the fused thermo march, the flux capacitor's Courant sums)
  // inside the level-loop ds_utvt1 and ds_utvt2: ds_courant's launch and its re-read of ut / vt
  // only with GTFV3_KLOOP=0
  const bool acc = d_sw_thermo_fused(a);
  // (A/B in one box: 32.34 -> 31.59-31.63 ms per step)
  const bool fold = klb > 0;
  double* const ccx = fold && acc ? a.cx : nullptr;
  double* const ccy = fold && acc ? a.cy : nullptr;
  const double cb = fold ? L * ((acc ? 4 : 2) * e.X + (acc ? 4 : 2) * e.Y) + 8 * e.C : 0.0;
  // uc, vc read; ut, vt written (with the fold only near the tile edges: not counted)
  const double ub = L * ((fold ? 1 : 2) * e.X + (fold ? 1 : 2) * e.Y) + 8 * e.C;
  auto utvt1 = [&](const Launch2D& r, const Launch2D& h) {
    GT_LAUNCH_N("ds_utvt1_kl", ds_utvt1_kl, kloop_grid(r, d.nsub, nkb), dim3(BX, BY), 0, c.st, d, r, h, c.subs,
                c.met, a.npz, nkb, klb, a.dt, a.uc, a.vc, a.ut, a.vt, a.crx, a.cry, a.xfx, a.yfx, ccx, ccy);
    HIP_LAUNCH_CHECK();
  };
  if (part == 1) {
    if (!klb) throw std::runtime_error("d_sw_courant: the split form needs GTFV3_KLOOP > 0");
    utvt1(inner, kNoHole);
    gt_bytes(ub + cb);
    return;
  }
  if (klb) {
    utvt1(full, part == 2 ? inner : kNoHole);
  } else {
    GT_LAUNCH(ds_utvt1, g2(d, full, nz), dim3(BX, BY), 0, c.st, d, c.subs, c.met, a.npz, a.dt, a.uc, a.vc,
                       a.ut, a.vt);
    HIP_LAUNCH_CHECK();
  }
  if (part == 0) gt_bytes((klb ? ub : L * (2 * e.X + 2 * e.Y) + 8 * e.C) + cb);
  GT_LAUNCH(ds_utvt2, dim3(cdiv(edge_line_count(-NG, d.nx + NG, -NG, d.ny + NG), 256), 1, nz), dim3(256), 0, c.st,
            d, c.subs, c.met, a.npz, a.uc, a.vc, a.ut, a.vt, a.dt, fold ? a.crx : nullptr, a.cry, a.xfx, a.yfx,
            ccx, ccy);
  HIP_LAUNCH_CHECK();
  if (utvt_done) HIP_CHECK(hipEventRecord(utvt_done, c.st));
  if (fold) return;
  GT_LAUNCH(ds_courant, g2(d, full, nz), dim3(BX, BY), 0, c.st, d, c.subs, c.met, a.npz, a.dt, a.ut, a.vt,
                     a.crx, a.cry, a.xfx, a.yfx, acc ? a.cx : nullptr, acc ? a.cy : nullptr);
  HIP_LAUNCH_CHECK();
  gt_bytes(L * ((acc ? 5 : 3) * e.X + (acc ? 5 : 3) * e.Y) + 8 * e.C);
}

static TpArgs d_sw_tp(const DswArgs& a) {
  TpArgs t{};
  t.nt = 1;
  t.nk = a.npz;
  t.crx = a.crx; t.cry = a.cry; t.xfx = a.xfx; t.yfx = a.yfx;
  return t;
}

// d_sw's w damping (non-hydrostatic, before w's transport) on the levels that have it: the
// increment dw of w's del-(2 nord_w + 2) fluxes and its heat hw.  fused0: the nord_w = 0 runs
// are left to d_sw_w_damping_add (one pass after the fused march, from the old w it leaves)
static void d_sw_w_damping(const Ctx& c, const DswArgs& a, bool fused0) {
  level_runs(a.hlv, a.npz, [](const LevelDamp& l) { return l.w4 > 0.0 ? l.nord_w : -1; },
             [&](int k0, int nk, int nord) {
               if (fused0 && nord == 0) return;
               deln_fluxes(c, a.npz, k0, nk, nord, a.lv, DL_W4, a.w, a.td2, a.tfx2, a.tfy2);
               w_damping(c, a.npz, k0, nk, a.ke_dt, a.tfx2, a.tfy2, a.w, a.dw, a.hw);
             });
}

// w = w / delp + dw (after the transport's update, into w_new)
static void d_sw_w_damping_add(const Ctx& c, const DswArgs& a, double* w_new, bool fused0) {
  level_runs(a.hlv, a.npz, [](const LevelDamp& l) { return l.w4 > 0.0 ? l.nord_w : -1; },
             [&](int k0, int nk, int nord) {
               if (fused0 && nord == 0)
                 w_damping0_fused(c, a.npz, k0, nk, a.lv, a.ke_dt, a.w, w_new, a.d_con > 1e-5 ? a.hw : nullptr);
               else
                 w_damping_add(c, a.npz, k0, nk, a.dw, w_new);
             });
}

void d_sw_thermo(const Ctx& c, const DswArgs& a) {
  const Dims& d = c.d;
  if (!a.lv || !a.hlv) throw std::runtime_error("d_sw: the column damping table is required");
  const bool fused = d_sw_thermo_fused(a);
  d_sw_w_damping(c, a, fused);
  if (fused) {
    ThermoArgs t{};
    t.npz = a.npz;
    t.ord = a.hord_dp;
    t.delp = a.delp; t.w = a.w; t.pt = a.pt;
    t.delp_o = a.delp_o; t.w_o = a.w_o; t.pt_o = a.pt_o;
    t.crx = a.crx; t.cry = a.cry; t.xfx = a.xfx; t.yfx = a.yfx;
    t.mfx = a.mfx; t.mfy = a.mfy;
    d_sw_thermo_march(c, t);
    d_sw_w_damping_add(c, a, a.w_o, true);
    return;
  }
  const int nz = d.nsub * a.npz;
  Launch2D full{-NG, -NG, d.nx + 2 * NG + 1, d.ny + 2 * NG + 1};
  TpArgs t = d_sw_tp(a);
  // mass fluxes, with delp's del-(2 nord_v + 2) diffusive fluxes where damp_vt > 1e-4
  // (fv_tp_2d(delp, ..., nord = nord_v, damp_c = damp_vt))
  t.q = a.delp; t.mfx = nullptr; t.mfy = nullptr; t.fx = a.fx; t.fy = a.fy; t.ord = a.hord_dp;
  fv_tp_2d(c, t);
  level_runs(a.hlv, a.npz, [](const LevelDamp& l) { return l.dp4 > 0.0 ? l.nord_v : -1; },
             [&](int k0, int nk, int nord) {
               deln_fluxes(c, a.npz, k0, nk, nord, a.lv, DL_DP4, a.delp, a.td2, a.tfx2, a.tfy2);
               deln_add(c, a.npz, k0, nk, a.lv, a.tfx2, a.tfy2, nullptr, a.fx, a.fy);
             });
  GT_LAUNCH(ds_accum, g2(d, full, nz), dim3(BX, BY), 0, c.st, d, c.subs, a.npz, a.crx, a.cry, a.fx, a.fy,
                     a.cx, a.cy, a.mfx, a.mfy);
  HIP_LAUNCH_CHECK();
  const Ext e = ext(d);
  const double L = a.npz;
  gt_bytes(L * (6 * e.X + 6 * e.Y));
  // w and pt with the mass fluxes: one launch for the pair when their PPM orders agree
  // (each wave carries both fields and loads the shared Courant numbers and fluxes once)
  t.mfx = a.fx; t.mfy = a.fy;
  if (a.hord_vt == a.hord_tm) {
    t.q = a.w; t.fx = a.gwx; t.fy = a.gwy;
    t.q2 = a.pt; t.fx_2 = a.gtx; t.fy_2 = a.gty; t.ord = a.hord_vt;
    fv_tp_2d(c, t);
  } else {
    t.q = a.w; t.fx = a.gwx; t.fy = a.gwy; t.ord = a.hord_vt;
    fv_tp_2d(c, t);
    t.q = a.pt; t.fx = a.gtx; t.fy = a.gty; t.ord = a.hord_tm;
    fv_tp_2d(c, t);
  }
  // pt's mass-weighted del-(2 nord_t + 2) fluxes where damp_t > 1e-4 (fv_tp_2d(pt, ..., mass =
  // delp, nord = nord_t, damp_c = damp_t))
  level_runs(a.hlv, a.npz, [](const LevelDamp& l) { return l.pt4 > 0.0 ? l.nord_t : -1; },
             [&](int k0, int nk, int nord) {
               deln_fluxes(c, a.npz, k0, nk, nord, a.lv, DL_ONE, a.pt, a.td2, a.tfx2, a.tfy2);
               deln_add(c, a.npz, k0, nk, a.lv, a.tfx2, a.tfy2, a.delp, a.gtx, a.gty);
             });
  Launch2D Li{0, 0, d.nx, d.ny};
  GT_LAUNCH(ds_thermo, g2(d, Li, nz), dim3(BX, BY), 0, c.st, d, c.subs, c.met, a.npz, a.fx, a.fy, a.gwx,
                     a.gwy, a.gtx, a.gty, a.delp, a.pt, a.w);
  HIP_LAUNCH_CHECK();
  gt_bytes(L * (6 * e.C + 3 * e.X + 3 * e.Y) + e.C);
  d_sw_w_damping_add(c, a, a.w, false);
}

void d_sw_vort(const Ctx& c, const DswArgs& a) {
  const Dims& d = c.d;
  const int nz = d.nsub * a.npz;
  Launch2D Lr{-NG, -NG, d.nx + 2 * NG, d.ny + 2 * NG};
  GT_LAUNCH(ds_vort, g2(d, Lr, nz), dim3(BX, BY), 0, c.st, d, c.subs, c.met, a.npz, a.u, a.v, a.vort);
  HIP_LAUNCH_CHECK();
  const Ext e = ext(d);
  gt_bytes((double)a.npz * (e.X + e.Y + e.C) + 4 * e.C);
}

void d_sw_winds(const Ctx& c, const DswArgs& a, bool vort_done, const hipEvent_t* march_wait, int nwait) {
  const Dims& d = c.d;
  const int nz = d.nsub * a.npz;
  if (!a.lv || !a.hlv) throw std::runtime_error("d_sw: the column damping table is required");
  // kinetic energy (+ divergence damping) at corners
  Launch2D Lc{0, 0, d.nx + 1, d.ny + 1};
  const bool dcon = a.d_con > 1e-5, vdamp = any_level(a.hlv, a.npz, &LevelDamp::vt4);
  bool nord0 = false, nordn = false;  // some level with nord = 0 / nord > 0
  for (int k = 0; k < a.npz; ++k) (a.hlv[k].nord == 0 ? nord0 : nordn) = true;
  {
    double* vdp = dcon ? a.vd : nullptr;
#define KE_LD(O, D)                                                                                          \
  GT_LAUNCH_N("ds_ke", (ds_ke_ld<O, D>), g2(d, Lc, nz), dim3(BX, BY), 0, c.st, d, c.subs, c.met, a.npz, a.dt, \
              a.dddmp, a.lv, c.da_min_c, a.u, a.v, a.uc, a.vc, a.ua, a.va, a.ut, a.vt, a.ke, vdp)
    if (a.hord_mt == 5) {
      if (nord0) KE_LD(5, true); else KE_LD(5, false);
    } else {
      if (nord0) KE_LD(6, true); else KE_LD(6, false);
    }
#undef KE_LD
  }
  HIP_LAUNCH_CHECK();
  const Ext e = ext(d);
  const double L = a.npz;
  gt_bytes(L * (2 * e.C + 3 * e.X + 3 * e.Y + e.K) + 17 * e.C);
  // damping beyond nord = 0 (damp.hip), from the old winds' cell vorticity
  if (nordn && !a.divg) throw std::runtime_error("d_sw: nord > 0 needs c_sw's corner divergence");
  if (nordn || vdamp) vorticity_wk(c, a.npz, a.u, a.v, a.wk);
  if (nordn) {
    DampArgs da{};
    da.npz = a.npz; da.nord = a.nord;
    da.dt = a.dt; da.dddmp = a.dddmp; da.d4_bg = a.d4_bg; da.lv = a.lv;
    da.divg = a.divg; da.wk = a.wk; da.ke = a.ke; da.vd = a.vd;
    da.dd = a.dd; da.vcx = a.dvcx; da.ucy = a.ducy; da.vort = a.dvort; da.qx = a.dqx; da.qy = a.dqy;
    divergence_damping(c, da);
  }
  // vorticity damping fluxes (del6_vt_flux) on the levels that have it
  level_runs(a.hlv, a.npz, [](const LevelDamp& l) { return l.vt4 > 0.0 ? l.nord_v : -1; },
             [&](int k0, int nk, int nord) { deln_fluxes(c, a.npz, k0, nk, nord, a.lv, DL_VT4, a.wk, a.d2, a.fx2, a.fy2); });
  // vorticity transport
  if (!vort_done) d_sw_vort(c, a);
  for (int n = 0; n < nwait; ++n) HIP_CHECK(hipStreamWaitEvent(c.st, march_wait[n], 0));
  TpArgs t = d_sw_tp(a);
  t.mfx = nullptr; t.mfy = nullptr;
  t.q = a.vort; t.fx = a.gvx; t.fy = a.gvy; t.ord = a.hord_vt;
  // u, v updated inside the vorticity march (tp.hip TM = 3: ds_uv's expressions on the
  // fluxes in registers, no flux planes)
  t.ke_uv = a.ke;
  t.u_uv = a.u;
  t.v_uv = a.v;
  fv_tp_2d(c, t);
}

bool d_sw_post_needed(const DswArgs& a) {
  return a.d_con > 1e-5 || (a.hlv && any_level(a.hlv, a.npz, &LevelDamp::vt4));
}

void d_sw_post(const Ctx& c, const DswArgs& a) {
  const bool vdamp = any_level(a.hlv, a.npz, &LevelDamp::vt4);
  if (a.d_con > 1e-5)
    damping_heat(c, a.npz, a.lv, a.u, a.v, a.vd, a.fx2, a.fy2,
                 any_level(a.hlv, a.npz, &LevelDamp::w4) ? a.hw : nullptr, a.delp, a.heat, a.diss);
  if (vdamp) vorticity_damping_apply(c, a.npz, a.lv, a.fx2, a.fy2, a.u, a.v);
}

void d_sw(const Ctx& c, const DswArgs& a) {
  d_sw_courant(c, a);
  d_sw_thermo(c, a);
  d_sw_winds(c, a);
}

}  // namespace gtfv3
