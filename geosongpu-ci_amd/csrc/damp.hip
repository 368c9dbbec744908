// damp.hip — d_sw's damping on gfx950 (FV3 dyn_core's per-level parameters, sw_core d_sw /
// c_sw divergence_corner / del6_vt_flux, tp_core deln_flux, del2_cubed, fv_grid_utils
// fill_corners; restated in oracle/sw_core.py with the same expressions and order):
//   * the column of d_sw parameters (column_damping): every level nord, min(0.2, d2_bg),
//     nord_v = min(2, nord), damp_vt = vtdm4 with do_vort_damp, w and pt following nord_v /
//     damp_vt; the sponge layers (n_sponge >= 0) in the top three levels: del-2 divergence
//     damping from d2_bg_k1 / d2_bg_k2, del-2 w damping, vorticity / delp del-2 damping with
//     do_vort_damp, d_con 0;
//   * nord = 1..3: del-(2 nord + 2) damping of the corner divergence (c_sw's divg_d, halo
//     exchanged as a corner field) with d4_bg, plus the del-2 Smagorinsky-type term whose
//     coefficient uses the corner vorticity (a2b_ord4 of the cell vorticity wk) when dddmp > 0;
//   * damp_vt: del-(2 nord_v + 2) diffusive fluxes of wk added to u, v, and of delp added to
//     the mass fluxes inside fv_tp_2d; damp_t: mass-weighted del-(2 nord_t + 2) fluxes of pt;
//     damp_w: w's del-(2 nord_w + 2) increment and its heat;
//   * d_con > 0: the kinetic energy the damping removes as a heat source (summed over the
//     acoustic sub-steps, smoothed by del2_cubed on the top n_con levels, added to pt there
//     with the delt_max limiter) and the dissipation estimate diss_est.
// In the Held-Suarez benchmark namelist (nord = 0, vtdm4 = 0, d_con = 0) only the sponge's
// per-level divergence damping and the top levels' w damping run.
// The cube-corner fills (B-grid XDir / YDir, the D-grid vector pair, copy_corners of the
// cell field) are not separate passes: each kernel reads a cube-corner halo point through
// the fill's source map, which leaves every other value as it was.
// Kernels on a level window [k0, k0 + nkw) of an npz-level field take (npz, k0, nkw) and a
// grid of nsub * nkw planes (WSETUP).
#include <algorithm>
#include <cmath>
#include <stdexcept>

#include "kernels_damp.hpp"
#include "kernels_nh.hpp"
#include "stencil_common.hpp"

namespace gtfv3 {
namespace {

#define DSETUP(nk_)                                                  \
  int i, j;                                                          \
  if (!thread_point(L, i, j)) return;                                \
  const int z = blockIdx.z, s = z / (nk_);                           \
  const SubInfo sub = subs[s];                                       \
  const int N = sub.N;                                               \
  const int I = i + sub.ioff, J = j + sub.joff;                      \
  const long zo = (long)z * d.plane;                                 \
  const long o = pidx(d, i, j);                                      \
  (void)I; (void)J; (void)N; (void)zo;
#define WSETUP()                                                          \
  int i, j;                                                               \
  if (!thread_point(L, i, j)) return;                                     \
  const int s = (int)blockIdx.z / nkw, k = k0 + (int)blockIdx.z % nkw;    \
  const SubInfo sub = subs[s];                                            \
  const int N = sub.N;                                                    \
  const int I = i + sub.ioff, J = j + sub.joff;                           \
  const long zo = ((long)s * npz + k) * d.plane;                          \
  const long o = pidx(d, i, j);                                           \
  (void)I; (void)J; (void)N; (void)zo; (void)k;
#define MT(name) met(M, d, name, s)
#define MA(arr, di, dj) arr[o + (long)(dj) * d.pitch + (di)]
#define AT(arr, di, dj) arr[zo + o + (long)(dj) * d.pitch + (di)]

__device__ __forceinline__ bool in_reg(int i, int j, int i0, int i1, int j0, int j1) {
  return i >= i0 && i <= i1 && j >= j0 && j <= j1;
}

// c_sw divergence_corner: rarea_c times the dual-cell divergence of the D-grid winds at the
// compute corners, zero elsewhere on the plane
__global__ void __launch_bounds__(256) dd_divg_corner_k(Dims d, const SubInfo* __restrict__ subs,
                                                        const double* __restrict__ M, int npz,
                                                        const double* __restrict__ u, const double* __restrict__ v,
                                                        const double* __restrict__ ua, const double* __restrict__ va,
                                                        double* __restrict__ divg) {
  Launch2D L{-NG, -NG, d.nx + 2 * NG + 1, d.ny + 2 * NG + 1};
  DSETUP(npz)
  if (!in_reg(i, j, 0, d.nx, 0, d.ny)) {
    AT(divg, 0, 0) = 0.0;
    return;
  }
  const double *s1 = MT(M_SIN1), *s2 = MT(M_SIN2), *s3 = MT(M_SIN3), *s4 = MT(M_SIN4);
  const double *c1 = MT(M_COS1), *c2 = MT(M_COS2), *c3 = MT(M_COS3), *c4 = MT(M_COS4);
  const double *dyc = MT(M_DYC), *dxc = MT(M_DXC);
  // uf on the x-edge (i + di, j) (u position), vf on the y-edge (i, j + dj) (v position)
  auto uf = [&](int di) {
    const double sx = MA(dyc, di, 0) * 0.5 * (MA(s4, di, -1) + MA(s2, di, 0));
    if (J == 0 || J == N) return AT(u, di, 0) * sx;
    return (AT(u, di, 0) - 0.25 * (AT(va, di, -1) + AT(va, di, 0)) * (MA(c4, di, -1) + MA(c2, di, 0))) * sx;
  };
  auto vf = [&](int dj) {
    const double sy = MA(dxc, 0, dj) * 0.5 * (MA(s3, -1, dj) + MA(s1, 0, dj));
    if (I == 0 || I == N) return AT(v, 0, dj) * sy;
    return (AT(v, 0, dj) - 0.25 * (AT(ua, -1, dj) + AT(ua, 0, dj)) * (MA(c3, -1, dj) + MA(c1, 0, dj))) * sy;
  };
  const double vS = vf(-1), v0 = vf(0);
  double dd = vS - v0 + uf(-1) - uf(0);
  if ((I == 0 && J == 0) || (I == N && J == 0)) dd = dd - vS;
  if ((I == N && J == N) || (I == 0 && J == N)) dd = dd + v0;
  AT(divg, 0, 0) = MA(MT(M_RAREA_C), 0, 0) * dd;
}

// FV3 fill_corners(q, XDir (dir 1) | YDir (dir 2), BGRID): source of a corner point (I, J)
// in a cube-corner halo region (global indices); false when (I, J) is not in one
__device__ __forceinline__ bool bfill_src(int I, int J, int N, int dir, int& Is, int& Js) {
  const bool wi = I < 0, ei = I > N, sj = J < 0, nj_ = J > N;
  if (!((wi || ei) && (sj || nj_))) return false;
  if (dir == 1) {
    if (wi && sj) { Is = J; Js = -I; }
    else if (ei && sj) { Is = N - J; Js = I - N; }
    else if (ei && nj_) { Is = J; Js = 2 * N - I; }
    else { Is = N - J; Js = N + I; }
  } else {
    if (wi && sj) { Is = -J; Js = I; }
    else if (ei && sj) { Is = N + J; Js = N - I; }
    else if (ei && nj_) { Is = 2 * N - J; Js = I; }
    else { Is = J - N; Js = N - I; }
  }
  return true;
}

// one Laplacian step's gradients of the corner field dd: vc on x-edges (the x difference,
// divg_u = sina_v dyc / dx) over i in [-1-nt, nx+nt], j in [-nt, ny+nt]; uc on y-edges
// (divg_v = sina_u dxc / dy) over i in [-nt, nx+nt], j in [-1-nt, ny+nt]; zero elsewhere.
// fill: dd read through the B-grid corner fills (XDir for vc, YDir for uc).
__global__ void __launch_bounds__(256) dd_grad_k(Dims d, const SubInfo* __restrict__ subs,
                                                 const double* __restrict__ M, int npz, int nt, int fill,
                                                 const double* __restrict__ dd, double* __restrict__ vcx,
                                                 double* __restrict__ ucy) {
  Launch2D L{-NG, -NG, d.nx + 2 * NG + 1, d.ny + 2 * NG + 1};
  DSETUP(npz)
  auto at = [&](int ii, int jj, int dir) {
    int Is, Js;
    if (fill && bfill_src(ii + sub.ioff, jj + sub.joff, N, dir, Is, Js)) {
      ii = Is - sub.ioff;
      jj = Js - sub.joff;
    }
    return dd[zo + pidx(d, ii, jj)];
  };
  double gx = 0.0, gy = 0.0;
  if (in_reg(i, j, -1 - nt, d.nx + nt, -nt, d.ny + nt))
    gx = (at(i + 1, j, 1) - at(i, j, 1)) * (MA(MT(M_SINA_V), 0, 0) * MA(MT(M_DYC), 0, 0) / MA(MT(M_DX), 0, 0));
  if (in_reg(i, j, -nt, d.nx + nt, -1 - nt, d.ny + nt))
    gy = (at(i, j + 1, 2) - at(i, j, 2)) * (MA(MT(M_SINA_U), 0, 0) * MA(MT(M_DXC), 0, 0) / MA(MT(M_DY), 0, 0));
  AT(vcx, 0, 0) = gx;
  AT(ucy, 0, 0) = gy;
}

// FV3 fill_corners(x, y, DGRID, VECTOR) read map: the value of component c (0 = x on
// x-edges, 1 = y on y-edges) at a point of its cube-corner halo region comes from the other
// component at the source point, with the vector sign at the south-west / north-east corners
__device__ __forceinline__ bool dfill_src(int c, int I, int J, int N, int& Is, int& Js, double& sg) {
  if (c == 0) {  // x-edge (I, J): I in [-3, -1] or [N, N+2], J in [-3, -1] or [N+1, N+3]
    const bool wi = I < 0, ei = I >= N, sj = J < 0, nj_ = J > N;
    if (!((wi || ei) && (sj || nj_))) return false;
    if (wi && sj) { Is = J; Js = -I - 1; sg = -1.0; }
    else if (ei && sj) { Is = N - J; Js = I - N; sg = 1.0; }
    else if (ei && nj_) { Is = J; Js = 2 * N - I - 1; sg = -1.0; }
    else { Is = N - J; Js = N + I; sg = 1.0; }
    return true;
  }
  // y-edge (I, J): I in [-3, -1] or [N+1, N+3], J in [-3, -1] or [N, N+2]
  const bool wi = I < 0, ei = I > N, sj = J < 0, nj_ = J >= N;
  if (!((wi || ei) && (sj || nj_))) return false;
  if (wi && sj) { Is = -J - 1; Js = I; sg = -1.0; }
  else if (ei && sj) { Is = N + J; Js = N - I; sg = 1.0; }
  else if (ei && nj_) { Is = 2 * N - J - 1; Js = I; sg = -1.0; }
  else { Is = J - N; Js = N - I; sg = 1.0; }
  return true;
}

// the Laplacian's divergence: dd = (uc(i,j-1) - uc(i,j) + vc(i-1,j) - vc(i,j)) (+ the
// cube-corner corrections) * rarea_c over [-nt, n+nt], zero elsewhere; in place (reads only
// vc, uc).  fill: vc / uc read through the D-grid vector corner fill.
__global__ void __launch_bounds__(256) dd_div_k(Dims d, const SubInfo* __restrict__ subs, const double* __restrict__ M,
                                                int npz, int nt, int fill, const double* __restrict__ vcx,
                                                const double* __restrict__ ucy, double* __restrict__ dd) {
  Launch2D L{-NG, -NG, d.nx + 2 * NG + 1, d.ny + 2 * NG + 1};
  DSETUP(npz)
  if (!in_reg(i, j, -nt, d.nx + nt, -nt, d.ny + nt)) {
    AT(dd, 0, 0) = 0.0;
    return;
  }
  auto get = [&](int c, int ii, int jj) {
    int Is, Js;
    double sg = 1.0;
    int cc = c;
    if (fill && dfill_src(c, ii + sub.ioff, jj + sub.joff, N, Is, Js, sg)) {
      ii = Is - sub.ioff;
      jj = Js - sub.joff;
      cc = 1 - c;
    }
    return sg * (cc == 0 ? vcx : ucy)[zo + pidx(d, ii, jj)];
  };
  const double uS = get(1, i, j - 1), u0 = get(1, i, j);
  double nw = uS - u0 + get(0, i - 1, j) - get(0, i, j);
  if ((I == 0 && J == 0) || (I == N && J == 0)) nw = nw - uS;
  if ((I == N && J == N) || (I == 0 && J == N)) nw = nw + u0;
  AT(dd, 0, 0) = nw * MA(MT(M_RAREA_C), 0, 0);
}

// the corner damping term vd = damp2 * delpc + dd8 * dd (delpc: c_sw's divergence), added
// to ke; vort: the corner vorticity (a2b_ord4 of wk) or null (dddmp = 0).  Levels whose
// column parameters say nord = 0 (the sponge layers) took ds_ke's del-2 term instead.
__global__ void __launch_bounds__(256) dd_term_k(Dims d, const SubInfo* __restrict__ subs, int npz,
                                                 const LevelDamp* __restrict__ lv, double dt, double dddmp,
                                                 double da_min_c, double dd8,
                                                 const double* __restrict__ delpc, const double* __restrict__ dd,
                                                 const double* __restrict__ vort, double* __restrict__ ke,
                                                 double* __restrict__ vd) {
  Launch2D L{0, 0, d.nx + 1, d.ny + 1};
  DSETUP(npz)
  const LevelDamp& lk = lv[z % npz];
  if (lk.nord == 0) return;
  const double dp = AT(delpc, 0, 0);
  double vc = 0.0;
  if (vort) {
    const double w = AT(vort, 0, 0);
    vc = fabs(dt) * sqrt(dp * dp + w * w);
  }
  const double damp2 = da_min_c * fmax(lk.d2_divg, fmin(0.20, dddmp * vc));
  const double t = damp2 * dp + dd8 * AT(dd, 0, 0);
  AT(ke, 0, 0) = AT(ke, 0, 0) + t;
  AT(vd, 0, 0) = t;
}

// relative vorticity wk (cell mean, halo included), the expression of ds_vort without f0
__global__ void __launch_bounds__(256) dd_wk_k(Dims d, const SubInfo* __restrict__ subs, const double* __restrict__ M,
                                               int npz, const double* __restrict__ u, const double* __restrict__ v,
                                               double* __restrict__ wk) {
  Launch2D L{-NG, -NG, d.nx + 2 * NG, d.ny + 2 * NG};
  DSETUP(npz)
  const double* dx = MT(M_DX);
  const double* dy = MT(M_DY);
  const double udx0 = AT(u, 0, 0) * MA(dx, 0, 0), udx1 = AT(u, 0, 1) * MA(dx, 0, 1);
  const double vdy0 = AT(v, 0, 0) * MA(dy, 0, 0), vdy1 = AT(v, 1, 0) * MA(dy, 1, 0);
  AT(wk, 0, 0) = MA(MT(M_RAREA), 0, 0) * (udx0 - udx1 + vdy1 - vdy0);
}

// ---- tp_core deln_flux / del6_vt_flux on a level window ----
// d2 = coef * q over [-1-nord, n+nord] (coef from the level's LevelDamp, DL_ONE: 1), zero
// elsewhere on the plane
__device__ __forceinline__ double deln_coef(const LevelDamp& l, int coef) {
  return coef == DL_VT4 ? l.vt4 : (coef == DL_DP4 ? l.dp4 : (coef == DL_W4 ? l.w4 : 1.0));
}
__global__ void __launch_bounds__(256) dl_init_k(Dims d, const SubInfo* __restrict__ subs, int npz, int k0, int nkw,
                                                 int nord, const LevelDamp* __restrict__ lv, int coef,
                                                 const double* __restrict__ q, double* __restrict__ d2) {
  Launch2D L{-NG, -NG, d.nx + 2 * NG + 1, d.ny + 2 * NG + 1};
  WSETUP()
  if (!in_reg(i, j, -1 - nord, d.nx + nord, -1 - nord, d.ny + nord)) {
    AT(d2, 0, 0) = 0.0;
    return;
  }
  AT(d2, 0, 0) = coef == DL_ONE ? AT(q, 0, 0) : deln_coef(lv[k], coef) * AT(q, 0, 0);
}

// fx2 on y-edges over [-r, nx+r] x [-r, ny-1+r], fy2 on x-edges over [-r, nx-1+r] x [-r, ny+r]
// (zero elsewhere) from d2 read through copy_corners (cc: XDir for fx2, YDir for fy2);
// first: (d2(i-1) - d2(i)) as deln_flux's first pass and del2_cubed, else (d2(i) - d2(i-1))
__global__ void __launch_bounds__(256) dl_flux_k(Dims d, const SubInfo* __restrict__ subs,
                                                 const double* __restrict__ M, int npz, int k0, int nkw, int r, int cc,
                                                 int first, const double* __restrict__ d2, double* __restrict__ fx2,
                                                 double* __restrict__ fy2) {
  Launch2D L{-NG, -NG, d.nx + 2 * NG + 1, d.ny + 2 * NG + 1};
  WSETUP()
  auto at = [&](int ii, int jj, int dir) { return d2[zo + (cc ? cc_off(d, sub, ii, jj, dir) : pidx(d, ii, jj))]; };
  double fx = 0.0, fy = 0.0;
  if (in_reg(i, j, -r, d.nx + r, -r, d.ny - 1 + r)) {
    const double d6v = MA(MT(M_SINA_U), 0, 0) * MA(MT(M_DY), 0, 0) / MA(MT(M_DXC), 0, 0);
    fx = first ? d6v * (at(i - 1, j, 1) - at(i, j, 1)) : d6v * (at(i, j, 1) - at(i - 1, j, 1));
  }
  if (in_reg(i, j, -r, d.nx - 1 + r, -r, d.ny + r)) {
    const double d6u = MA(MT(M_SINA_V), 0, 0) * MA(MT(M_DX), 0, 0) / MA(MT(M_DYC), 0, 0);
    fy = first ? d6u * (at(i, j - 1, 2) - at(i, j, 2)) : d6u * (at(i, j, 2) - at(i, j - 1, 2));
  }
  AT(fx2, 0, 0) = fx;
  AT(fy2, 0, 0) = fy;
}

// d2 = (fx2 - fx2(i+1) + fy2 - fy2(j+1)) * rarea over [-nt-1, n+nt], zero elsewhere
__global__ void __launch_bounds__(256) dl_div_k(Dims d, const SubInfo* __restrict__ subs, const double* __restrict__ M,
                                                int npz, int k0, int nkw, int nt, const double* __restrict__ fx2,
                                                const double* __restrict__ fy2, double* __restrict__ d2) {
  Launch2D L{-NG, -NG, d.nx + 2 * NG + 1, d.ny + 2 * NG + 1};
  WSETUP()
  AT(d2, 0, 0) = in_reg(i, j, -nt - 1, d.nx + nt, -nt - 1, d.ny + nt)
                     ? (AT(fx2, 0, 0) - AT(fx2, 1, 0) + AT(fy2, 0, 0) - AT(fy2, 0, 1)) * MA(MT(M_RAREA), 0, 0)
                     : 0.0;
}

// deln_flux's last step: the diffusive fluxes into the transport fluxes on [0, nx] x [0, ny-1]
// (fx) and [0, nx-1] x [0, ny] (fy); with mass, weighted by 0.5 pt4 (mass(i-1) + mass(i))
__global__ void __launch_bounds__(256) dl_add_k(Dims d, const SubInfo* __restrict__ subs, int npz, int k0, int nkw,
                                                const LevelDamp* __restrict__ lv, const double* __restrict__ fx2,
                                                const double* __restrict__ fy2, const double* __restrict__ mass,
                                                double* __restrict__ fx, double* __restrict__ fy) {
  Launch2D L{0, 0, d.nx + 1, d.ny + 1};
  WSETUP()
  if (mass) {
    const double damp2 = 0.5 * lv[k].pt4;
    if (j < d.ny) AT(fx, 0, 0) = AT(fx, 0, 0) + damp2 * (AT(mass, -1, 0) + AT(mass, 0, 0)) * AT(fx2, 0, 0);
    if (i < d.nx) AT(fy, 0, 0) = AT(fy, 0, 0) + damp2 * (AT(mass, 0, -1) + AT(mass, 0, 0)) * AT(fy2, 0, 0);
  } else {
    if (j < d.ny) AT(fx, 0, 0) = AT(fx, 0, 0) + AT(fx2, 0, 0);
    if (i < d.nx) AT(fy, 0, 0) = AT(fy, 0, 0) + AT(fy2, 0, 0);
  }
}

// d_sw's w damping on compute cells: dw = div(fx2, fy2) rarea, hw = ke_bg |dt| - dw (w + dw / 2)
__global__ void __launch_bounds__(256) dl_wdamp_k(Dims d, const SubInfo* __restrict__ subs,
                                                  const double* __restrict__ M, int npz, int k0, int nkw,
                                                  double ke_dt, const double* __restrict__ fx2,
                                                  const double* __restrict__ fy2, const double* __restrict__ w,
                                                  double* __restrict__ dw, double* __restrict__ hw) {
  Launch2D L{0, 0, d.nx, d.ny};
  WSETUP()
  const double x = (AT(fx2, 0, 0) - AT(fx2, 1, 0) + AT(fy2, 0, 0) - AT(fy2, 0, 1)) * MA(MT(M_RAREA), 0, 0);
  AT(dw, 0, 0) = x;
  AT(hw, 0, 0) = ke_dt - x * (AT(w, 0, 0) + 0.5 * x);
}

// update_dz_d's damping of the heights (FV3 nh_utils update_dz_d: del6_vt_flux of zh with
// (nord_v, damp_vt), zh += (fx2 - fx2(i+1) + fy2 - fy2(j+1)) rarea) on compute cells
__global__ void __launch_bounds__(256) dl_divadd_k(Dims d, const SubInfo* __restrict__ subs,
                                                   const double* __restrict__ M, int npz, int k0, int nkw,
                                                   const double* __restrict__ fx2, const double* __restrict__ fy2,
                                                   double* __restrict__ q) {
  Launch2D L{0, 0, d.nx, d.ny};
  WSETUP()
  AT(q, 0, 0) = AT(q, 0, 0) + (AT(fx2, 0, 0) - AT(fx2, 1, 0) + AT(fy2, 0, 0) - AT(fy2, 0, 1)) * MA(MT(M_RAREA), 0, 0);
}

__global__ void __launch_bounds__(256) dl_wadd_k(Dims d, const SubInfo* __restrict__ subs, int npz, int k0, int nkw,
                                                 const double* __restrict__ dw, double* __restrict__ w) {
  Launch2D L{0, 0, d.nx, d.ny};
  WSETUP()
  AT(w, 0, 0) = AT(w, 0, 0) + AT(dw, 0, 0);
}

// the nord_w = 0 w damping in one pass after the fused thermo march: the del-2 fluxes of
// d2 = w4 w from the OLD w (the march wrote the new values to w_new and left w as it was), dw
// and its heat, w_new += dw -- the expressions and order of dl_init_k / dl_flux_k /
// dl_wdamp_k / dl_wadd_k, without their planes
__global__ void __launch_bounds__(256) dl_wdamp0_k(Dims d, const SubInfo* __restrict__ subs,
                                                   const double* __restrict__ M, int npz, int k0, int nkw,
                                                   const LevelDamp* __restrict__ lv, double ke_dt,
                                                   const double* __restrict__ w, double* __restrict__ w_new,
                                                   double* __restrict__ hw) {
  Launch2D L{0, 0, d.nx, d.ny};
  WSETUP()
  const double damp = lv[k].w4;
  const double *sau = MT(M_SINA_U), *dy = MT(M_DY), *dxc = MT(M_DXC);
  const double *sav = MT(M_SINA_V), *dx = MT(M_DX), *dyc = MT(M_DYC);
  const double d2c = damp * AT(w, 0, 0), d2w = damp * AT(w, -1, 0), d2e = damp * AT(w, 1, 0);
  const double d2s = damp * AT(w, 0, -1), d2n = damp * AT(w, 0, 1);
  const double fx0 = MA(sau, 0, 0) * MA(dy, 0, 0) / MA(dxc, 0, 0) * (d2w - d2c);
  const double fx1 = MA(sau, 1, 0) * MA(dy, 1, 0) / MA(dxc, 1, 0) * (d2c - d2e);
  const double fy0 = MA(sav, 0, 0) * MA(dx, 0, 0) / MA(dyc, 0, 0) * (d2s - d2c);
  const double fy1 = MA(sav, 0, 1) * MA(dx, 0, 1) / MA(dyc, 0, 1) * (d2c - d2n);
  const double x = (fx0 - fx1 + fy0 - fy1) * MA(MT(M_RAREA), 0, 0);
  if (hw) AT(hw, 0, 0) = ke_dt - x * (AT(w, 0, 0) + 0.5 * x);
  AT(w_new, 0, 0) = AT(w_new, 0, 0) + x;
}

// d_con: the damped kinetic energy on compute cells into heat (+=) and diss (+=); u, v: the
// updated winds times dx / dy before the vorticity-damping fluxes.  Per level: the
// vorticity-damping fluxes where lv.vt4 > 0, the w damping's heat hw where lv.w4 > 0; levels
// with d_con_k <= 1e-5 (the sponge) add hw alone.
__global__ void __launch_bounds__(256) dd_heat_k(Dims d, const SubInfo* __restrict__ subs,
                                                 const double* __restrict__ M, int npz, const LevelDamp* __restrict__ lv,
                                                 const double* __restrict__ u, const double* __restrict__ v,
                                                 const double* __restrict__ vd, const double* __restrict__ fx2,
                                                 const double* __restrict__ fy2, const double* __restrict__ hw,
                                                 const double* __restrict__ delp, double* __restrict__ heat,
                                                 double* __restrict__ diss) {
  Launch2D L{0, 0, d.nx, d.ny};
  DSETUP(npz)
  const LevelDamp lk = lv[z % npz];
  const double hwv = hw && lk.w4 > 0.0 ? AT(hw, 0, 0) : 0.0;
  if (!(lk.d_con > 1e-5)) {
    AT(heat, 0, 0) = AT(heat, 0, 0) + hwv;
    AT(diss, 0, 0) = AT(diss, 0, 0) + hwv;
    return;
  }
  const bool vt = lk.vt4 > 0.0;
  const double *rdx = MT(M_RDX), *rdy = MT(M_RDY);
  auto ub = [&](int dj) {
    const double f2 = vt ? AT(fy2, 0, dj) : 0.0;
    return (AT(vd, 0, dj) - AT(vd, 1, dj) + f2) * MA(rdx, 0, dj);
  };
  auto vb = [&](int di) {
    const double f2 = vt ? AT(fx2, di, 0) : 0.0;
    return (AT(vd, di, 0) - AT(vd, di, 1) - f2) * MA(rdy, di, 0);
  };
  const double ub0 = ub(0), ub1 = ub(1), vb0 = vb(0), vb1 = vb(1);
  const double fy0 = AT(u, 0, 0) * MA(rdx, 0, 0), fy1 = AT(u, 0, 1) * MA(rdx, 0, 1);
  const double fx0 = AT(v, 0, 0) * MA(rdy, 0, 0), fx1 = AT(v, 1, 0) * MA(rdy, 1, 0);
  const double gy0 = fy0 * ub0, gy1 = fy1 * ub1, gx0 = fx0 * vb0, gx1 = fx1 * vb1;
  const double u2 = fy0 + fy1, du2 = ub0 + ub1, v2 = fx0 + fx1, dv2 = vb0 + vb1;
  const double t = (ub0 * ub0 + ub1 * ub1 + vb0 * vb0 + vb1 * vb1) + 2.0 * (gy0 + gy1 + gx0 + gx1) -
                   MA(MT(M_COSA_S), 0, 0) * (u2 * dv2 + v2 * du2 + du2 * dv2);
  const double rs2 = MA(MT(M_RSIN2), 0, 0);
  AT(heat, 0, 0) = AT(heat, 0, 0) + AT(delp, 0, 0) * (hwv - 0.25 * lk.d_con * rs2 * t);
  AT(diss, 0, 0) = AT(diss, 0, 0) + (hwv - rs2 * t);
}

// vorticity damping: u += fy2 on x-edges, v -= fx2 on y-edges, on the levels that have it
__global__ void __launch_bounds__(256) dd_vflux_k(Dims d, const SubInfo* __restrict__ subs, int npz,
                                                  const LevelDamp* __restrict__ lv, const double* __restrict__ fx2,
                                                  const double* __restrict__ fy2, double* __restrict__ u,
                                                  double* __restrict__ v) {
  Launch2D L{0, 0, d.nx + 1, d.ny + 1};
  DSETUP(npz)
  if (!(lv[z % npz].vt4 > 0.0)) return;
  if (i < d.nx) AT(u, 0, 0) = AT(u, 0, 0) + AT(fy2, 0, 0);
  if (j < d.ny) AT(v, 0, 0) = AT(v, 0, 0) - AT(fx2, 0, 0);
}

// ---- del2_cubed ----
// the cube-corner cells this sub-domain owns and their west / east and south / north halo
// neighbours set to the three's mean (one lane per plane and corner)
__global__ void __launch_bounds__(64) h2_corner_k(Dims d, const SubInfo* __restrict__ subs, int npz, int k0, int nkw,
                                                  double* __restrict__ q) {
  const int t = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (t >= d.nsub * nkw * 4) return;
  const int c = t & 3, z = t >> 2, s = z / nkw, k = k0 + z % nkw;
  const SubInfo sub = subs[s];
  const int N = sub.N;
  const bool west = sub.ioff == 0, east = sub.ioff + d.nx == N, south = sub.joff == 0, north = sub.joff + d.ny == N;
  int ci, cj, di, dj;  // corner cell (global) and the side of its halo neighbours
  if (c == 0) { if (!(west && south)) return; ci = 0; cj = 0; di = -1; dj = -1; }
  else if (c == 1) { if (!(east && south)) return; ci = N - 1; cj = 0; di = 1; dj = -1; }
  else if (c == 2) { if (!(east && north)) return; ci = N - 1; cj = N - 1; di = 1; dj = 1; }
  else { if (!(west && north)) return; ci = 0; cj = N - 1; di = -1; dj = 1; }
  double* p = q + ((long)s * npz + k) * d.plane;
  const int i = ci - sub.ioff, j = cj - sub.joff;
  const long a = pidx(d, i, j), b = pidx(d, i + di, j), e = pidx(d, i, j + dj);
  const double avg = (p[a] + p[b] + p[e]) * (1.0 / 3.0);
  p[a] = avg;
  p[b] = avg;
  p[e] = avg;
}

// q += cd rarea (fx - fx(i+1) + fy - fy(j+1)) over [-nt, n-1+nt]
__global__ void __launch_bounds__(256) h2_update_k(Dims d, const SubInfo* __restrict__ subs,
                                                   const double* __restrict__ M, int npz, int k0, int nkw, int nt,
                                                   double cd, const double* __restrict__ fx,
                                                   const double* __restrict__ fy, double* __restrict__ q) {
  Launch2D L{-nt, -nt, d.nx + 2 * nt, d.ny + 2 * nt};
  WSETUP()
  AT(q, 0, 0) = AT(q, 0, 0) + cd * MA(MT(M_RAREA), 0, 0) *
                                  (AT(fx, 0, 0) - AT(fx, 1, 0) + AT(fy, 0, 0) - AT(fy, 0, 1));
}

// after the acoustic sub-steps, levels [0, n_con): dT = heat / (cv_air delp), limited to delt
// (0.1x / 0.5x in the top two layers), added to the potential temperature through pkz of the
// current state
__global__ void __launch_bounds__(256) dd_heat_apply_k(Dims d, const SubInfo* __restrict__ subs, int npz, int k0,
                                                       int nkw, double delt, const double* __restrict__ heat,
                                                       const double* __restrict__ delp,
                                                       const double* __restrict__ delz, double* __restrict__ pt) {
  Launch2D L{0, 0, d.nx, d.ny};
  WSETUP()
  constexpr double RDG = -Constants::rdgas * (1.0 / Constants::grav);
  constexpr double K1K = Constants::kappa / (1.0 - Constants::kappa);
  constexpr double CV = Constants::rdgas / Constants::kappa - Constants::rdgas;
  const double lim = k == 0 ? 0.1 * delt : (k == 1 ? 0.5 * delt : delt);
  const double dp = AT(delp, 0, 0);
  const double pkz = exp(K1K * log(RDG * dp / AT(delz, 0, 0) * AT(pt, 0, 0)));
  const double dtmp = AT(heat, 0, 0) / (CV * dp);
  const double sg = dtmp > 0.0 ? 1.0 : (dtmp < 0.0 ? -1.0 : 0.0);
  AT(pt, 0, 0) = AT(pt, 0, 0) + sg * fmin(lim, fabs(dtmp)) / pkz;
}

inline dim3 g2(const Launch2D& L, int nz) { return plane_grid(L, nz); }

}  // namespace

void divergence_corner(const Ctx& c, int npz, const double* u, const double* v, const double* ua, const double* va,
                       double* divg) {
  const Dims& d = c.d;
  Launch2D L{-NG, -NG, d.nx + 2 * NG + 1, d.ny + 2 * NG + 1};
  GT_LAUNCH(dd_divg_corner_k, g2(L, d.nsub * npz), dim3(BX, BY), 0, c.st, d, c.subs, c.met, npz, u, v, ua, va, divg);
  HIP_LAUNCH_CHECK();
  const Ext e = ext(d);
  gt_bytes(npz * (e.X + e.Y + 2 * e.C + e.K) + 13 * e.C);
}

// the corner damping term (nord > 0): ke += vd.  s: scratch planes (npz levels each) dd, vcx,
// ucy, wk, vort (a2b), a2b work qx / qy
void divergence_damping(const Ctx& c, const DampArgs& a) {
  const Dims& d = c.d;
  const int nz = d.nsub * a.npz;
  Launch2D full{-NG, -NG, d.nx + 2 * NG + 1, d.ny + 2 * NG + 1};
  copy_levels(c, (long)nz * d.plane, a.divg, a.dd);
  bool corner_sub = false;
  for (int s = 0; s < d.nsub; ++s) {
    const SubInfo& h = c.hsubs[s];
    for (int q = 0; q < 4; ++q) {
      const int CI = q == 1 || q == 2 ? h.N : 0, CJ = q >= 2 ? h.N : 0;
      corner_sub = corner_sub || (CI >= h.ioff && CI <= h.ioff + d.nx && CJ >= h.joff && CJ <= h.joff + d.ny);
    }
  }
  for (int n = 1; n <= a.nord; ++n) {
    const int nt = a.nord - n;
    const int fill = nt != 0 && corner_sub ? 1 : 0;
    GT_LAUNCH(dd_grad_k, g2(full, nz), dim3(BX, BY), 0, c.st, d, c.subs, c.met, a.npz, nt, fill, a.dd, a.vcx, a.ucy);
    HIP_LAUNCH_CHECK();
    GT_LAUNCH(dd_div_k, g2(full, nz), dim3(BX, BY), 0, c.st, d, c.subs, c.met, a.npz, nt, fill, a.vcx, a.ucy, a.dd);
    HIP_LAUNCH_CHECK();
  }
  const double* vort = nullptr;
  if (a.dddmp >= 1e-5) {
    a2b_ord4(c, a.npz, a.wk, a.vort, a.qx, a.qy);
    vort = a.vort;
  }
  const double dd8 = std::pow(c.da_min_c * a.d4_bg, (double)(a.nord + 1));
  Launch2D Lc{0, 0, d.nx + 1, d.ny + 1};
  GT_LAUNCH(dd_term_k, g2(Lc, nz), dim3(BX, BY), 0, c.st, d, c.subs, a.npz, a.lv, a.dt, a.dddmp, c.da_min_c, dd8,
            a.divg, a.dd, vort, a.ke, a.vd);
  HIP_LAUNCH_CHECK();
}

void vorticity_wk(const Ctx& c, int npz, const double* u, const double* v, double* wk) {
  const Dims& d = c.d;
  Launch2D L{-NG, -NG, d.nx + 2 * NG, d.ny + 2 * NG};
  GT_LAUNCH(dd_wk_k, g2(L, d.nsub * npz), dim3(BX, BY), 0, c.st, d, c.subs, c.met, npz, u, v, wk);
  HIP_LAUNCH_CHECK();
}

std::vector<LevelDamp> column_damping(const Namelist& nl, double da_min, double da_min_c) {
  const int npz = nl.npz;
  struct P {
    int nord, nord_v, nord_w, nord_t;
    double d2, dvt, dw, dt, dcon;
  };
  const double dvt = nl.do_vort_damp ? nl.vtdm4 : 0.0;
  std::vector<P> p(npz, P{nl.nord, nl.nord_v, nl.nord_v, nl.nord_v, std::min(0.20, nl.d2_bg), dvt, dvt, dvt, nl.d_con});
  if (npz == 1 || nl.n_sponge < 0) {
    for (P& x : p) x.d2 = nl.d2_bg;
  } else {
    // sponge layers: del-2 damping of divergence, w and (with do_vort_damp) vorticity and delp;
    // no special damping of pt
    auto sponge = [&](P& x, double d2, bool vort) {
      x.nord = 0;
      x.d2 = d2;
      x.nord_w = 0;
      x.dw = d2;
      x.dcon = 0.0;
      if (vort && nl.do_vort_damp) {
        x.nord_v = 0;
        x.dvt = 0.5 * d2;
      }
    };
    // FV3 dyn_core: k == 1, k == max(2, n_sponge - 1), k == max(3, n_sponge) (1-based)
    const int k2 = std::max(1, nl.n_sponge - 2), k3 = std::max(2, nl.n_sponge - 1);
    sponge(p[0], std::max(std::max(0.01, nl.d2_bg), nl.d2_bg_k1), true);
    if (npz > k2 && nl.d2_bg_k2 > 0.01) sponge(p[k2], std::max(nl.d2_bg, nl.d2_bg_k2), true);
    if (npz > k3 && nl.d2_bg_k2 > 0.05) sponge(p[k3], std::max(nl.d2_bg, 0.2 * nl.d2_bg_k2), false);
  }
  std::vector<LevelDamp> out(npz);
  for (int k = 0; k < npz; ++k) {
    const P& x = p[k];
    LevelDamp& l = out[k];
    l.d2_divg = x.d2;
    l.vt4 = x.dvt > 1e-5 ? std::pow(x.dvt * da_min_c, (double)(x.nord_v + 1)) : 0.0;
    l.dp4 = x.dvt > 1e-4 ? std::pow(x.dvt * da_min, (double)(x.nord_v + 1)) : 0.0;
    l.w4 = x.dw > 1e-5 ? std::pow(x.dw * da_min_c, (double)(x.nord_w + 1)) : 0.0;
    l.pt4 = x.dt > 1e-4 ? std::pow(x.dt * da_min, (double)(x.nord_t + 1)) : 0.0;
    l.d_con = x.dcon;
    l.nord = x.nord;
    l.nord_v = x.nord_v;
    l.nord_w = x.nord_w;
    l.nord_t = x.nord_t;
  }
  return out;
}

int heat_levels(const Namelist& nl) {
  int n = 2;
  if (nl.convert_ke || nl.vtdm4 > 1e-4) n = nl.npz;
  else if (nl.d2_bg_k1 < 1e-3) n = 0;
  else if (nl.d2_bg_k2 < 1e-3) n = 1;
  return std::min(n, nl.npz);
}

bool any_level(const LevelDamp* lv, int n, double LevelDamp::*coef) {
  for (int k = 0; k < n; ++k)
    if (lv[k].*coef > 0.0) return true;
  return false;
}

void deln_fluxes(const Ctx& c, int npz, int k0, int nk, int nord, const LevelDamp* lv, int coef, const double* q,
                 double* d2, double* fx2, double* fy2) {
  const Dims& d = c.d;
  if (nord < 0 || nord > 2) throw std::runtime_error("deln_flux: nord must be 0, 1 or 2");
  if (k0 < 0 || nk < 1 || k0 + nk > npz) throw std::runtime_error("deln_flux: level window outside the field");
  const int nz = d.nsub * nk;
  Launch2D full{-NG, -NG, d.nx + 2 * NG + 1, d.ny + 2 * NG + 1};
  GT_LAUNCH(dl_init_k, g2(full, nz), dim3(BX, BY), 0, c.st, d, c.subs, npz, k0, nk, nord, lv, coef, q, d2);
  HIP_LAUNCH_CHECK();
  GT_LAUNCH(dl_flux_k, g2(full, nz), dim3(BX, BY), 0, c.st, d, c.subs, c.met, npz, k0, nk, nord, nord > 0 ? 1 : 0, 1,
            d2, fx2, fy2);
  HIP_LAUNCH_CHECK();
  for (int n = 1; n <= nord; ++n) {
    const int nt = nord - n;
    GT_LAUNCH(dl_div_k, g2(full, nz), dim3(BX, BY), 0, c.st, d, c.subs, c.met, npz, k0, nk, nt, fx2, fy2, d2);
    HIP_LAUNCH_CHECK();
    GT_LAUNCH(dl_flux_k, g2(full, nz), dim3(BX, BY), 0, c.st, d, c.subs, c.met, npz, k0, nk, nt, 1, 0, d2, fx2, fy2);
    HIP_LAUNCH_CHECK();
  }
}

void deln_add(const Ctx& c, int npz, int k0, int nk, const LevelDamp* lv, const double* fx2, const double* fy2,
              const double* mass, double* fx, double* fy) {
  const Dims& d = c.d;
  Launch2D L{0, 0, d.nx + 1, d.ny + 1};
  GT_LAUNCH(dl_add_k, g2(L, d.nsub * nk), dim3(BX, BY), 0, c.st, d, c.subs, npz, k0, nk, lv, fx2, fy2, mass, fx, fy);
  HIP_LAUNCH_CHECK();
}

void w_damping(const Ctx& c, int npz, int k0, int nk, double ke_dt, const double* fx2, const double* fy2,
               const double* w, double* dw, double* hw) {
  const Dims& d = c.d;
  Launch2D L{0, 0, d.nx, d.ny};
  GT_LAUNCH(dl_wdamp_k, g2(L, d.nsub * nk), dim3(BX, BY), 0, c.st, d, c.subs, c.met, npz, k0, nk, ke_dt, fx2, fy2, w,
            dw, hw);
  HIP_LAUNCH_CHECK();
}

void w_damping0_fused(const Ctx& c, int npz, int k0, int nk, const LevelDamp* lv, double ke_dt, const double* w,
                      double* w_new, double* hw) {
  const Dims& d = c.d;
  Launch2D L{0, 0, d.nx, d.ny};
  GT_LAUNCH(dl_wdamp0_k, g2(L, d.nsub * nk), dim3(BX, BY), 0, c.st, d, c.subs, c.met, npz, k0, nk, lv, ke_dt, w, w_new,
            hw);
  HIP_LAUNCH_CHECK();
  // w read, w_new read and written (hw written) per level; seven metric planes
  const Ext e = ext(d);
  gt_bytes(nk * (hw ? 4.0 : 3.0) * e.C + 7.0 * e.C);
}

void deln_div_add(const Ctx& c, int npz, int k0, int nk, const double* fx2, const double* fy2, double* q) {
  const Dims& d = c.d;
  Launch2D L{0, 0, d.nx, d.ny};
  GT_LAUNCH(dl_divadd_k, g2(L, d.nsub * nk), dim3(BX, BY), 0, c.st, d, c.subs, c.met, npz, k0, nk, fx2, fy2, q);
  HIP_LAUNCH_CHECK();
}

std::vector<LevelDamp> height_damping(const std::vector<LevelDamp>& col) {
  // FV3 update_dz_d: damp(km+1) = damp(km), ndif(km+1) = ndif(km)
  std::vector<LevelDamp> out(col);
  if (!out.empty()) out.push_back(out.back());
  return out;
}

void w_damping_add(const Ctx& c, int npz, int k0, int nk, const double* dw, double* w) {
  const Dims& d = c.d;
  Launch2D L{0, 0, d.nx, d.ny};
  GT_LAUNCH(dl_wadd_k, g2(L, d.nsub * nk), dim3(BX, BY), 0, c.st, d, c.subs, npz, k0, nk, dw, w);
  HIP_LAUNCH_CHECK();
}

void damping_heat(const Ctx& c, int npz, const LevelDamp* lv, const double* u, const double* v, const double* vd,
                  const double* fx2, const double* fy2, const double* hw, const double* delp, double* heat,
                  double* diss) {
  const Dims& d = c.d;
  Launch2D L{0, 0, d.nx, d.ny};
  GT_LAUNCH(dd_heat_k, g2(L, d.nsub * npz), dim3(BX, BY), 0, c.st, d, c.subs, c.met, npz, lv, u, v, vd, fx2, fy2, hw,
            delp, heat, diss);
  HIP_LAUNCH_CHECK();
}

void vorticity_damping_apply(const Ctx& c, int npz, const LevelDamp* lv, const double* fx2, const double* fy2,
                             double* u, double* v) {
  const Dims& d = c.d;
  Launch2D L{0, 0, d.nx + 1, d.ny + 1};
  GT_LAUNCH(dd_vflux_k, g2(L, d.nsub * npz), dim3(BX, BY), 0, c.st, d, c.subs, npz, lv, fx2, fy2, u, v);
  HIP_LAUNCH_CHECK();
}

void del2_cubed(const Ctx& c, int npz, int k0, int nk, int nmax, double cd, double* q, double* fx, double* fy) {
  const Dims& d = c.d;
  if (k0 < 0 || nk < 1 || k0 + nk > npz) throw std::runtime_error("del2_cubed: level window outside the field");
  const int nz = d.nsub * nk;
  const int ntimes = std::min(3, nmax);
  Launch2D full{-NG, -NG, d.nx + 2 * NG + 1, d.ny + 2 * NG + 1};
  for (int n = 1; n <= ntimes; ++n) {
    const int nt = ntimes - n;
    GT_LAUNCH(h2_corner_k, dim3((unsigned)((nz * 4 + 63) / 64)), dim3(64), 0, c.st, d, c.subs, npz, k0, nk, q);
    HIP_LAUNCH_CHECK();
    GT_LAUNCH(dl_flux_k, g2(full, nz), dim3(BX, BY), 0, c.st, d, c.subs, c.met, npz, k0, nk, nt, nt > 0 ? 1 : 0, 1, q,
              fx, fy);
    HIP_LAUNCH_CHECK();
    Launch2D Lu{-nt, -nt, d.nx + 2 * nt, d.ny + 2 * nt};
    GT_LAUNCH(h2_update_k, g2(Lu, nz), dim3(BX, BY), 0, c.st, d, c.subs, c.met, npz, k0, nk, nt, cd, fx, fy, q);
    HIP_LAUNCH_CHECK();
  }
}

void damping_heat_apply(const Ctx& c, int npz, int n_con, double delt, const double* heat, const double* delp,
                        const double* delz, double* pt) {
  const Dims& d = c.d;
  if (n_con < 1) return;
  Launch2D L{0, 0, d.nx, d.ny};
  GT_LAUNCH(dd_heat_apply_k, g2(L, d.nsub * n_con), dim3(BX, BY), 0, c.st, d, c.subs, npz, 0, n_con, delt, heat, delp,
            delz, pt);
  HIP_LAUNCH_CHECK();
}

}  // namespace gtfv3
