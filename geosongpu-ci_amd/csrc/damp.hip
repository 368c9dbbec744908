// damp.hip — d_sw's damping options beyond nord = 0 on gfx950 (FV3 sw_core d_sw / c_sw
// divergence_corner / del6_vt_flux, fv_grid_utils fill_corners; restated in
// oracle/sw_core.py with the same expressions and order):
//   * nord = 1..3: del-(2 nord + 2) damping of the corner divergence (c_sw's divg_d, halo
//     exchanged as a corner field) with d4_bg, plus the del-2 Smagorinsky-type term whose
//     coefficient uses the corner vorticity (a2b_ord4 of the cell vorticity wk) when dddmp > 0;
//   * vtdm4 > 0: del-(2 nord_v + 2) diffusive fluxes of wk added to u, v;
//   * d_con > 0: the kinetic energy both remove as a heat source (summed over the acoustic
//     sub-steps, added to pt after them with the delt_max limiter) and the dissipation
//     estimate diss_est.
// None of this runs in the Held-Suarez benchmark namelist (nord = 0, vtdm4 = 0, d_con = 0).
// The cube-corner fills (B-grid XDir / YDir, the D-grid vector pair, copy_corners of the
// cell field) are not separate passes: each kernel reads a cube-corner halo point through
// the fill's source map, which leaves every other value as it was.
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
// to ke; vort: the corner vorticity (a2b_ord4 of wk) or null (dddmp = 0)
__global__ void __launch_bounds__(256) dd_term_k(Dims d, const SubInfo* __restrict__ subs, int npz, double dt,
                                                 double dddmp, double d2_bg, double da_min_c, double dd8,
                                                 const double* __restrict__ delpc, const double* __restrict__ dd,
                                                 const double* __restrict__ vort, double* __restrict__ ke,
                                                 double* __restrict__ vd) {
  Launch2D L{0, 0, d.nx + 1, d.ny + 1};
  DSETUP(npz)
  const double dp = AT(delpc, 0, 0);
  double vc = 0.0;
  if (vort) {
    const double w = AT(vort, 0, 0);
    vc = fabs(dt) * sqrt(dp * dp + w * w);
  }
  const double damp2 = da_min_c * fmax(d2_bg, fmin(0.20, dddmp * vc));
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

// ---- del6_vt_flux ----
// d2 = damp * wk over [-nord, n-1+nord], zero elsewhere on the plane
__global__ void __launch_bounds__(256) d6_init_k(Dims d, const SubInfo* __restrict__ subs, int npz, int nord,
                                                 double damp, const double* __restrict__ wk, double* __restrict__ d2) {
  Launch2D L{-NG, -NG, d.nx + 2 * NG + 1, d.ny + 2 * NG + 1};
  DSETUP(npz)
  AT(d2, 0, 0) = in_reg(i, j, -nord, d.nx - 1 + nord, -nord, d.ny - 1 + nord) ? damp * AT(wk, 0, 0) : 0.0;
}

// fx2 on y-edges over [-r, nx+r] x [-r, ny-1+r], fy2 on x-edges over [-r, nx-1+r] x [-r, ny+r]
// (zero elsewhere) from d2 read through copy_corners (cc: XDir for fx2, YDir for fy2);
// first: (d2(i-1) - d2(i)) as del6_vt_flux's first pass, else (d2(i) - d2(i-1))
__global__ void __launch_bounds__(256) d6_flux_k(Dims d, const SubInfo* __restrict__ subs,
                                                 const double* __restrict__ M, int npz, int r, int cc, int first,
                                                 const double* __restrict__ d2, double* __restrict__ fx2,
                                                 double* __restrict__ fy2) {
  Launch2D L{-NG, -NG, d.nx + 2 * NG + 1, d.ny + 2 * NG + 1};
  DSETUP(npz)
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
__global__ void __launch_bounds__(256) d6_div_k(Dims d, const SubInfo* __restrict__ subs, const double* __restrict__ M,
                                                int npz, int nt, const double* __restrict__ fx2,
                                                const double* __restrict__ fy2, double* __restrict__ d2) {
  Launch2D L{-NG, -NG, d.nx + 2 * NG + 1, d.ny + 2 * NG + 1};
  DSETUP(npz)
  AT(d2, 0, 0) = in_reg(i, j, -nt - 1, d.nx + nt, -nt - 1, d.ny + nt)
                     ? (AT(fx2, 0, 0) - AT(fx2, 1, 0) + AT(fy2, 0, 0) - AT(fy2, 0, 1)) * MA(MT(M_RAREA), 0, 0)
                     : 0.0;
}

// d_con: the damped kinetic energy on compute cells into heat (+=) and diss (+=); u, v: the
// updated winds times dx / dy before the vorticity-damping fluxes; fx2 / fy2 may be null
__global__ void __launch_bounds__(256) dd_heat_k(Dims d, const SubInfo* __restrict__ subs,
                                                 const double* __restrict__ M, int npz, double d_con,
                                                 const double* __restrict__ u, const double* __restrict__ v,
                                                 const double* __restrict__ vd, const double* __restrict__ fx2,
                                                 const double* __restrict__ fy2, const double* __restrict__ delp,
                                                 double* __restrict__ heat, double* __restrict__ diss) {
  Launch2D L{0, 0, d.nx, d.ny};
  DSETUP(npz)
  const double *rdx = MT(M_RDX), *rdy = MT(M_RDY);
  auto ub = [&](int dj) {
    const double f2 = fy2 ? AT(fy2, 0, dj) : 0.0;
    return (AT(vd, 0, dj) - AT(vd, 1, dj) + f2) * MA(rdx, 0, dj);
  };
  auto vb = [&](int di) {
    const double f2 = fx2 ? AT(fx2, di, 0) : 0.0;
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
  AT(heat, 0, 0) = AT(heat, 0, 0) + AT(delp, 0, 0) * (0.0 - 0.25 * d_con * rs2 * t);
  AT(diss, 0, 0) = AT(diss, 0, 0) + -rs2 * t;
}

// vorticity damping: u += fy2 on x-edges, v -= fx2 on y-edges
__global__ void __launch_bounds__(256) dd_vflux_k(Dims d, const SubInfo* __restrict__ subs, int npz,
                                                  const double* __restrict__ fx2, const double* __restrict__ fy2,
                                                  double* __restrict__ u, double* __restrict__ v) {
  Launch2D L{0, 0, d.nx + 1, d.ny + 1};
  DSETUP(npz)
  if (i < d.nx) AT(u, 0, 0) = AT(u, 0, 0) + AT(fy2, 0, 0);
  if (j < d.ny) AT(v, 0, 0) = AT(v, 0, 0) - AT(fx2, 0, 0);
}

// after the acoustic sub-steps: dT = heat / (cp delp), limited to delt (0.1x / 0.5x in the top
// two layers), added to the potential temperature through pkz of the current state
__global__ void __launch_bounds__(256) dd_heat_apply_k(Dims d, const SubInfo* __restrict__ subs, int npz,
                                                       double delt, const double* __restrict__ heat,
                                                       const double* __restrict__ delp,
                                                       const double* __restrict__ delz, double* __restrict__ pt) {
  Launch2D L{0, 0, d.nx, d.ny};
  DSETUP(npz)
  const int k = z % npz;
  constexpr double RDG = -Constants::rdgas * (1.0 / Constants::grav);
  constexpr double K1K = Constants::kappa / (1.0 - Constants::kappa);
  constexpr double CP = Constants::rdgas / Constants::kappa;
  const double lim = k == 0 ? 0.1 * delt : (k == 1 ? 0.5 * delt : delt);
  const double dp = AT(delp, 0, 0);
  const double pkz = exp(K1K * log(RDG * dp / AT(delz, 0, 0) * AT(pt, 0, 0)));
  const double dtmp = AT(heat, 0, 0) / (CP * dp);
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
  GT_LAUNCH(dd_term_k, g2(Lc, nz), dim3(BX, BY), 0, c.st, d, c.subs, a.npz, a.dt, a.dddmp, a.d2_bg, c.da_min_c, dd8,
            a.divg, a.dd, vort, a.ke, a.vd);
  HIP_LAUNCH_CHECK();
}

void vorticity_wk(const Ctx& c, int npz, const double* u, const double* v, double* wk) {
  const Dims& d = c.d;
  Launch2D L{-NG, -NG, d.nx + 2 * NG, d.ny + 2 * NG};
  GT_LAUNCH(dd_wk_k, g2(L, d.nsub * npz), dim3(BX, BY), 0, c.st, d, c.subs, c.met, npz, u, v, wk);
  HIP_LAUNCH_CHECK();
}

void del6_vt_flux(const Ctx& c, int npz, int nord, double damp, const double* wk, double* d2, double* fx2,
                  double* fy2) {
  const Dims& d = c.d;
  if (nord < 0 || nord > 2) throw std::runtime_error("del6_vt_flux: nord_v must be 0, 1 or 2");
  const int nz = d.nsub * npz;
  Launch2D full{-NG, -NG, d.nx + 2 * NG + 1, d.ny + 2 * NG + 1};
  GT_LAUNCH(d6_init_k, g2(full, nz), dim3(BX, BY), 0, c.st, d, c.subs, npz, nord, damp, wk, d2);
  HIP_LAUNCH_CHECK();
  GT_LAUNCH(d6_flux_k, g2(full, nz), dim3(BX, BY), 0, c.st, d, c.subs, c.met, npz, nord, nord > 0 ? 1 : 0, 1, d2, fx2,
            fy2);
  HIP_LAUNCH_CHECK();
  for (int n = 1; n <= nord; ++n) {
    const int nt = nord - n;
    GT_LAUNCH(d6_div_k, g2(full, nz), dim3(BX, BY), 0, c.st, d, c.subs, c.met, npz, nt, fx2, fy2, d2);
    HIP_LAUNCH_CHECK();
    GT_LAUNCH(d6_flux_k, g2(full, nz), dim3(BX, BY), 0, c.st, d, c.subs, c.met, npz, nt, 1, 0, d2, fx2, fy2);
    HIP_LAUNCH_CHECK();
  }
}

void damping_heat(const Ctx& c, int npz, double d_con, const double* u, const double* v, const double* vd,
                  const double* fx2, const double* fy2, const double* delp, double* heat, double* diss) {
  const Dims& d = c.d;
  Launch2D L{0, 0, d.nx, d.ny};
  GT_LAUNCH(dd_heat_k, g2(L, d.nsub * npz), dim3(BX, BY), 0, c.st, d, c.subs, c.met, npz, d_con, u, v, vd, fx2, fy2,
            delp, heat, diss);
  HIP_LAUNCH_CHECK();
}

void vorticity_damping_apply(const Ctx& c, int npz, const double* fx2, const double* fy2, double* u, double* v) {
  const Dims& d = c.d;
  Launch2D L{0, 0, d.nx + 1, d.ny + 1};
  GT_LAUNCH(dd_vflux_k, g2(L, d.nsub * npz), dim3(BX, BY), 0, c.st, d, c.subs, npz, fx2, fy2, u, v);
  HIP_LAUNCH_CHECK();
}

void damping_heat_apply(const Ctx& c, int npz, double delt, const double* heat, const double* delp, const double* delz,
                        double* pt) {
  const Dims& d = c.d;
  Launch2D L{0, 0, d.nx, d.ny};
  GT_LAUNCH(dd_heat_apply_k, g2(L, d.nsub * npz), dim3(BX, BY), 0, c.st, d, c.subs, npz, delt, heat, delp, delz, pt);
  HIP_LAUNCH_CHECK();
}

}  // namespace gtfv3
