// stencil_common.hpp — device helpers shared by the FV3 stencil kernels.
//
// Index conventions (0-based, local to a sub-domain; global = local + ioff/joff):
//   cell (i,j)      i in [0,nx)         centre of cell i
//   x-edge (i,j)    edge from corner (i,j) to (i+1,j)   (D-grid u, C-grid vc, fy, yfx, cry)
//   y-edge (i,j)    edge from corner (i,j) to (i,j+1)   (D-grid v, C-grid uc, fx, xfx, crx)
//   corner (i,j)    grid point (i,j)
// FV3 Fortran index f (is=1) maps to global 0-based g = f-1; "npx" as an index is g = N.
#pragma once
#include <hip/hip_runtime.h>

#include "grid.hpp"
#include "hip_util.hpp"

namespace gtfv3 {

// metric plane of sub-domain s
__device__ __forceinline__ const double* met(const double* __restrict__ M, const Dims& d, int metric, int s) {
  return M + ((long)metric * d.nsub + s) * d.plane;
}

// Block shape for plane-parallel stencils: 256 threads (64 x 4).  thread_point maps the
// block's threads onto the launch region flattened row-major (i fastest), so the waves are
// full whatever the region's width (a 91-wide sub-domain row in 64-wide blocks left 29 %
// of the lanes idle) and consecutive lanes still read consecutive i.
constexpr int BX = 64, BY = 4;

struct Launch2D {
  int i0, j0;  // first point covered
  int ni, nj;  // extent
};

// XCD-aware block order.  Workgroups are dealt round-robin over the 8 XCDs (blocks b and
// b + 8 share one L2; placement is a speed matter only, never correctness).  When a plane's
// block count gridDim.x is a multiple of 8, physical block x covers logical block
// (x % 8) * (gridDim.x / 8) + x / 8: each XCD sweeps one contiguous eighth of the plane, so
// the j +- 1 rows a stencil reads were fetched by the same L2, and the next level's plane
// (blockIdx.z) puts the same eighth on the same XCD, whose L2 still holds its metric terms.
// Any other gridDim.x keeps the identity order (plane_grid pads to a multiple of 8).
__device__ __forceinline__ unsigned xcd_block() {
  const unsigned gx = gridDim.x, x = blockIdx.x;
  if (gx & 7u) return x;
  return (x & 7u) * (gx >> 3) + (x >> 3);
}

__device__ __forceinline__ bool thread_point(const Launch2D& L, int& i, int& j) {
  const int t = (int)(xcd_block() * (BX * BY) + threadIdx.y * BX + threadIdx.x);
  if (t >= L.ni * L.nj) return false;
  j = t / L.ni;
  i = L.i0 + (t - j * L.ni);
  j += L.j0;
  return true;
}
// grid for thread_point over region L and nz planes (blockIdx.z), padded to a multiple of 8
// blocks per plane (xcd_block; GTFV3_XCD=0: one block more, which keeps the identity order)
bool xcd_order_enabled();
// a 1-D workgroup count padded for xcd_block (its extra workgroups must find no work)
inline unsigned xcd_pad(long g) { return (unsigned)(xcd_order_enabled() ? (g + 7) / 8 * 8 : (g + 7) / 8 * 8 + 1); }
inline dim3 plane_grid(const Launch2D& L, long nz) {
  long gx = ((long)L.ni * L.nj + BX * BY - 1) / (BX * BY);
  gx = xcd_order_enabled() ? (gx + 7) / 8 * 8 : (gx + 7) / 8 * 8 + 1;
  return dim3((unsigned)gx, 1, (unsigned)nz);
}

// Level-interleaved blocks (plane_grid_lv / thread_point_lv): a 256-thread block covers 64
// consecutive points of BY = 4 consecutive planes (wave w: plane 4 * blockIdx.z + w) instead
// of 256 points of one plane.  The four waves read the same metric-plane addresses (the 2-D
// metric terms are shared by every level), so three of every four metric loads are served
// by the CU's vector L1 instead of the L2 / Infinity Cache.  Used from 8 planes up (a last
// group of fewer than 4 planes idles its spare waves; GTFV3_LVB=0: never); the kernel tells
// the two launch shapes apart by gridDim.z (= the plane count in the one-plane form).
bool level_blocks_enabled();
inline dim3 plane_grid_lv(const Launch2D& L, long nz) {
  if (!level_blocks_enabled() || nz < 2 * BY) return plane_grid(L, nz);
  long gx = ((long)L.ni * L.nj + BX - 1) / BX;
  gx = xcd_order_enabled() ? (gx + 7) / 8 * 8 : (gx + 7) / 8 * 8 + 1;
  return dim3((unsigned)gx, 1, (unsigned)((nz + BY - 1) / BY));
}
__device__ __forceinline__ bool thread_point_lv(const Launch2D& L, long nz, int& i, int& j, int& z) {
  if ((long)gridDim.z == nz) {
    z = blockIdx.z;
    return thread_point(L, i, j);
  }
  // the wave's plane through readfirstlane (threadIdx.y is one value per 64-lane wave):
  // the sub-domain, its SubInfo and the metric-plane bases stay in SGPRs
  z = (int)(blockIdx.z * BY + __builtin_amdgcn_readfirstlane(threadIdx.y));
  if (z >= nz) return false;
  const int t = (int)(xcd_block() * BX + threadIdx.x);
  if (t >= L.ni * L.nj) return false;
  j = t / L.ni;
  i = L.i0 + (t - j * L.ni);
  j += L.j0;
  return true;
}

// Level-loop forms (KL kernels): one thread per (point, sub-domain, block of kloop_levels()
// consecutive levels) walking its levels top-down.  Kernels whose level k reads interface
// planes k and k+1 (or layers k-1 and k) carry the shared plane in registers to the next
// level, and the metric terms are loaded once per block instead of once per level.
// GTFV3_KLOOP = levels per thread (default 8; 0: the one-level-per-thread forms).
int kloop_levels();
inline dim3 kloop_grid(const Launch2D& L, int nsub, int nkb) {
  long gx = ((long)L.ni * L.nj + BX * BY - 1) / (BX * BY);
  gx = xcd_order_enabled() ? (gx + 7) / 8 * 8 : (gx + 7) / 8 * 8 + 1;
  return dim3((unsigned)gx, 1, (unsigned)(nsub * nkb));
}
// setup of a KL kernel with parameters (..., int nkb, int klb, ...) over region L: point
// (i, j), sub-domain s, levels k0 .. k1-1 (nk_ levels in all), plane size P, plane offset o
#define KLSETUP(nk_)                                                            \
  int i, j;                                                                     \
  if (!thread_point(L, i, j)) return;                                           \
  const int s = blockIdx.z / nkb;                                               \
  const int k0 = (int)(blockIdx.z % nkb) * klb, k1 = min((nk_), k0 + klb);      \
  const long P = d.plane, o = pidx(d, i, j);

// Wavefront-wide lane shifts of a double through DPP (no LDS): lane_prev(v) in lane L is v of
// lane L-1, lane_next(v) is v of lane L+1; the lanes shifted in at the ends read 0.  Every
// lane of the wave must execute them (no lane-divergent branch around a shift).
template <int CTRL>
__device__ __forceinline__ double lane_shift(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, true);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double lane_prev(double v) { return lane_shift<0x138>(v); }  // wave_shr:1
__device__ __forceinline__ double lane_next(double v) { return lane_shift<0x130>(v); }  // wave_shl:1

// FV3 copy_corners source cell (global indices) for a cube-corner halo cell,
// dir = 1 (x sweep) or 2 (y sweep).  Restated from fv_grid_utils copy_corners;
// fill_4corners / fill2_4corners are the same map restricted to the first ring.
__device__ __forceinline__ void corner_src(int I, int J, int N, int dir, int& Is, int& Js) {
  if (dir == 1) {
    if (I < 0 && J < 0) { Is = J; Js = -I - 1; }
    else if (I >= N && J < 0) { Is = N - J - 1; Js = I - N; }
    else if (I >= N && J >= N) { Is = J; Js = 2 * N - I - 1; }
    else { Is = N - J - 1; Js = N + I; }
  } else {
    if (I < 0 && J < 0) { Is = -J - 1; Js = I; }
    else if (I >= N && J < 0) { Is = N + J; Js = N - I - 1; }
    else if (I >= N && J >= N) { Is = 2 * N - J - 1; Js = I; }
    else { Is = J - N; Js = N - I - 1; }
  }
}

// plane offset of cell (i,j) after the copy_corners remap for sweep `dir`
__device__ __forceinline__ long cc_off(const Dims& d, const SubInfo& s, int i, int j, int dir) {
  int I = i + s.ioff, J = j + s.joff, N = s.N;
  if ((I < 0 || I >= N) && (J < 0 || J >= N)) {
    int Is, Js;
    corner_src(I, J, N, dir, Is, Js);
    i = Is - s.ioff;
    j = Js - s.joff;
  }
  return pidx(d, i, j);
}

// Candidate points of the tile-edge lines I in {-1, 0, N-1, N} (any j in [jlo, jhi]) and
// J in {-1, 0, N-1, N} (any i in [ilo, ihi]) of a sub-domain, enumerated by t in
// [0, edge_line_count): kernels whose targets all lie on those lines launch this many
// lanes per plane instead of the whole plane.  Points outside the ranges and the
// duplicates of the second family return false.
__host__ __device__ inline int edge_line_count(int ilo, int ihi, int jlo, int jhi) {
  return 4 * (jhi - jlo + 1) + 4 * (ihi - ilo + 1);
}
__device__ __forceinline__ bool edge_line_point(int t, const SubInfo& sub, int ilo, int ihi, int jlo, int jhi, int& i,
                                       int& j) {
  const int N = sub.N, nj = jhi - jlo + 1, ni = ihi - ilo + 1;
  auto line = [&](int l) { return l == 0 ? -1 : (l == 1 ? 0 : (l == 2 ? N - 1 : N)); };
  if (t < 4 * nj) {
    i = line(t / nj) - sub.ioff;
    j = jlo + t % nj;
    return i >= ilo && i <= ihi;
  }
  t -= 4 * nj;
  if (t >= 4 * ni) return false;
  j = line(t / ni) - sub.joff;
  i = ilo + t % ni;
  const int I = i + sub.ioff;
  if (I == -1 || I == 0 || I == N - 1 || I == N) return false;  // already a column-line point
  return j >= jlo && j <= jhi;
}

// PPM constants (FV3 tp_core)
constexpr double P1 = 7.0 / 12.0, P2 = -1.0 / 12.0;
constexpr double C1 = -2.0 / 14.0, C2 = 11.0 / 14.0, C3 = 5.0 / 14.0;

// 4th-order interface value al at global interface g (between cells g-1, g),
// with the cubed-sphere tile-edge treatment (grid_type < 3):
//   q[0..3] = q(g-2), q(g-1), q(g), q(g+1);  dx[0..3] = dxa at the same cells.
__device__ __forceinline__ double ppm_al(int g, int N, const double* q, const double* dx) {
  if (g == -1 || g == N - 1) return C1 * q[0] + C2 * q[1] + C3 * q[2];
  if (g == 1 || g == N + 1) return C3 * q[1] + C2 * q[2] + C1 * q[3];
  if (g == 0 || g == N)
    return 0.5 * (((2.0 * dx[1] + dx[0]) * q[1] - dx[1] * q[0]) / (dx[0] + dx[1]) +
                  ((2.0 * dx[2] + dx[3]) * q[2] - dx[2] * q[3]) / (dx[2] + dx[3]));
  return P1 * (q[1] + q[2]) + P2 * (q[0] + q[3]);
}

__device__ __forceinline__ double ppm_al_in(const double* q) { return P1 * (q[1] + q[2]) + P2 * (q[0] + q[3]); }

// PPM flux through interface g for hord 5 / 6 (FV3 xppm/yppm, iord < 8 branch).
//   q[0..5] = q(g-3) .. q(g+2); dx[0..5] = dxa at those cells; c = Courant number.
// EDGE = false: the caller guarantees g-1..g+1 are away from the tile edges, so only
// the interior interface formula can apply (dx is not read).
template <int ORD, bool EDGE = true>
__device__ __forceinline__ double ppm_flux(int g, int N, const double* q, const double* dx, double c) {
  double alm = EDGE ? ppm_al(g - 1, N, q + 0, dx + 0) : ppm_al_in(q + 0);
  double al0 = EDGE ? ppm_al(g, N, q + 1, dx + 1) : ppm_al_in(q + 1);
  double alp = EDGE ? ppm_al(g + 1, N, q + 2, dx + 2) : ppm_al_in(q + 2);
  double blm = alm - q[2], brm = al0 - q[2], b0m = blm + brm;
  double bl0 = al0 - q[3], br0 = alp - q[3], b00 = bl0 + br0;
  bool sm, s0;
  if (ORD == 5) {
    sm = blm * brm < 0.0;
    s0 = bl0 * br0 < 0.0;
  } else {
    sm = 3.0 * fabs(b0m) < fabs(blm - brm);
    s0 = 3.0 * fabs(b00) < fabs(bl0 - br0);
  }
  bool smooth = sm || s0;
  if (c > 0.0) {
    double fx1 = (1.0 - c) * (brm - c * b0m);
    return q[2] + (smooth ? fx1 : 0.0);
  } else {
    double fx1 = (1.0 + c) * (bl0 + c * b00);
    return q[3] + (smooth ? fx1 : 0.0);
  }
}

template <bool EDGE>
__device__ __forceinline__ double ppm_flux_o(int ord, int g, int N, const double* q, const double* dx, double c) {
  return ord == 5 ? ppm_flux<5, EDGE>(g, N, q, dx, c) : ppm_flux<6, EDGE>(g, N, q, dx, c);
}

__device__ __forceinline__ double ppm_flux_ord(int ord, int g, int N, const double* q, const double* dx, double c) {
  return ord == 5 ? ppm_flux<5>(g, N, q, dx, c) : ppm_flux<6>(g, N, q, dx, c);
}

}  // namespace gtfv3
