// tp.hip — fv_tp_2d (Lin & Rood 1996 two-dimensional flux-form PPM transport,
// FV3 tp_core) and the tracer_2d_1l pieces (FV3 fv_tracer2d), HIP for gfx950.
//
// fv_tp_2d (HBM-bound, no MFMA) is one fused LDS-tiled kernel computing, per tile:
//   fx2 = xppm(q, crx) [x-corner-filled q]   fy2 = yppm(q, cry) [y-corner-filled q]
//   q_i = (q*area + yfx*fy2|j - yfx*fy2|j+1)/ra_y    q_j = (q*area + xfx*fx2|i - ...)/ra_x
//   fx = 0.5*(xppm(q_i) + fx2)*mfx     fy = 0.5*(yppm(q_j) + fy2)*mfy
// Operation order inside each expression follows the Fortran so the fp64
// numpy oracle (oracle/fv3.py) matches to the last bits.
#include "kernels.hpp"
#include "stencil_common.hpp"

namespace gtfv3 {
namespace {

constexpr int ZMAX = 65535;

inline dim3 grid_for(const Launch2D& L, long nz) {
  return dim3(cdiv(L.ni, BX), cdiv(L.nj, BY), (unsigned)(nz < ZMAX ? nz : ZMAX));
}

// Fused fv_tp_2d: one workgroup = one TX x TY tile of one (sub-domain, level); the
// corner-filled q tiles, the inner fluxes fx2 / fy2 and the advective updates
// q_i / q_j all stay in LDS, so HBM sees q, the Courant numbers and area fluxes once
// and the two output fluxes once (the unfused form round-tripped four scratch
// fields).  Regions and expressions are exactly those of the three-pass form.
constexpr int TX = 64, TY = 8, TBLOCK = 256;
constexpr int QX_C = TX + 6, QX_R = TY + 5;   // q (x corner fill): cols i0-3..i0+TX+2, rows j0-3..j0+TY+1
constexpr int QY_C = TX + 5, QY_R = TY + 6;   // q (y corner fill): cols i0-3..i0+TX+1, rows j0-3..j0+TY+2
constexpr int FX_C = TX + 1, FX_R = TY + 5;   // fx2: edges i0..i0+TX, rows j0-3..j0+TY+1
constexpr int FY_C = TX + 5, FY_R = TY + 1;   // fy2: cols i0-3..i0+TX+1, edges j0..j0+TY
constexpr int QI_C = TX + 5, QI_R = TY;       // q_i: cols i0-3..i0+TX+1, rows j0..j0+TY-1
constexpr int QJ_C = TX, QJ_R = TY + 5;       // q_j: cols i0..i0+TX-1, rows j0-3..j0+TY+1

__global__ void __launch_bounds__(TBLOCK) tp_fused(Dims d, const SubInfo* __restrict__ subs,
                                                   const double* __restrict__ M, const double* __restrict__ q, int nt,
                                                   int nk, const double* __restrict__ crx,
                                                   const double* __restrict__ cry, const double* __restrict__ xfx,
                                                   const double* __restrict__ yfx, const double* __restrict__ ra_x,
                                                   const double* __restrict__ ra_y, const double* __restrict__ mx,
                                                   const double* __restrict__ my, double* __restrict__ fx,
                                                   double* __restrict__ fy, int ord, int nz) {
  __shared__ double QX[QX_R][QX_C];
  __shared__ double QY[QY_R][QY_C];
  __shared__ double FX2[FX_R][FX_C];
  __shared__ double FY2[FY_R][FY_C];
  __shared__ double QI[QI_R][QI_C];
  __shared__ double QJ[QJ_R][QJ_C];
  const int i0 = blockIdx.x * TX, j0 = blockIdx.y * TY;
  const int tid = threadIdx.x;
  const int nx = d.nx, ny = d.ny;
  // cell halo only (not the +1 staggered row/column): copy_corners sources of points
  // beyond it would leave the plane
  auto inplane = [&](int i, int j) { return i >= -NG && i < nx + NG && j >= -NG && j < ny + NG; };
  for (int z = blockIdx.z; z < nz; z += gridDim.z) {
    const int k = z % nk, s = z / nk / nt;
    const SubInfo sub = subs[s];
    const double* qq = q + (long)z * d.plane;
    const long fo = ((long)s * nk + k) * d.plane;
    const long zo = (long)z * d.plane;
    const double* dxa = met(M, d, M_DXA, s);
    const double* dya = met(M, d, M_DYA, s);
    const double* area = met(M, d, M_AREA, s);
    __syncthreads();  // previous level's readers are done with the tiles
    for (int p = tid; p < QX_R * QX_C; p += TBLOCK) {
      const int r = p / QX_C, c = p % QX_C;
      const int i = i0 - 3 + c, j = j0 - 3 + r;
      QX[r][c] = inplane(i, j) ? qq[cc_off(d, sub, i, j, 1)] : 0.0;
    }
    for (int p = tid; p < QY_R * QY_C; p += TBLOCK) {
      const int r = p / QY_C, c = p % QY_C;
      const int i = i0 - 3 + c, j = j0 - 3 + r;
      QY[r][c] = inplane(i, j) ? qq[cc_off(d, sub, i, j, 2)] : 0.0;
    }
    __syncthreads();
    // inner fluxes: fx2 on x-edges i in [0, nx], rows [-3, ny+2]; fy2 on y-edges j in [0, ny], cols [-3, nx+2]
    for (int p = tid; p < FX_R * FX_C; p += TBLOCK) {
      const int r = p / FX_C, c = p % FX_C;
      const int i = i0 + c, j = j0 - 3 + r;
      double v = 0.0;
      if (i >= 0 && i <= nx && j >= -NG && j <= ny + NG - 1) {
        double qv[6], dx[6];
#pragma unroll
        for (int m = 0; m < 6; ++m) {
          qv[m] = QX[r][c + m];
          dx[m] = dxa[pidx(d, i - 3 + m, j)];
        }
        v = ppm_flux_ord(ord, i + sub.ioff, sub.N, qv, dx, crx[fo + pidx(d, i, j)]);
      }
      FX2[r][c] = v;
    }
    for (int p = tid; p < FY_R * FY_C; p += TBLOCK) {
      const int r = p / FY_C, c = p % FY_C;
      const int i = i0 - 3 + c, j = j0 + r;
      double v = 0.0;
      if (j >= 0 && j <= ny && i >= -NG && i <= nx + NG - 1) {
        double qv[6], dy[6];
#pragma unroll
        for (int m = 0; m < 6; ++m) {
          qv[m] = QY[r + m][c];
          dy[m] = dya[pidx(d, i, j - 3 + m)];
        }
        v = ppm_flux_ord(ord, j + sub.joff, sub.N, qv, dy, cry[fo + pidx(d, i, j)]);
      }
      FY2[r][c] = v;
    }
    __syncthreads();
    // advective updates q_i (rows [0, ny)) and q_j (cols [0, nx))
    for (int p = tid; p < QI_R * QI_C; p += TBLOCK) {
      const int r = p / QI_C, c = p % QI_C;
      const int i = i0 - 3 + c, j = j0 + r;
      double v = 0.0;
      if (j >= 0 && j < ny && i >= -NG && i < nx + NG) {
        const long o = pidx(d, i, j), on = pidx(d, i, j + 1);
        const double fyy0 = yfx[fo + o] * FY2[r][c];
        const double fyy1 = yfx[fo + on] * FY2[r + 1][c];
        v = (QY[r + 3][c] * area[o] + fyy0 - fyy1) / ra_y[fo + o];
      }
      QI[r][c] = v;
    }
    for (int p = tid; p < QJ_R * QJ_C; p += TBLOCK) {
      const int r = p / QJ_C, c = p % QJ_C;
      const int i = i0 + c, j = j0 - 3 + r;
      double v = 0.0;
      if (i >= 0 && i < nx && j >= -NG && j < ny + NG) {
        const long o = pidx(d, i, j), oe = pidx(d, i + 1, j);
        const double fxx0 = xfx[fo + o] * FX2[r][c];
        const double fxx1 = xfx[fo + oe] * FX2[r][c + 1];
        v = (QX[r][c + 3] * area[o] + fxx0 - fxx1) / ra_x[fo + o];
      }
      QJ[r][c] = v;
    }
    __syncthreads();
    // outer fluxes
    for (int p = tid; p < TX * TY; p += TBLOCK) {
      const int r = p / TX, c = p % TX;
      const int i = i0 + c, j = j0 + r;
      const long o = pidx(d, i, j);
      if (j < ny && i <= nx) {
        double qv[6], dx[6];
#pragma unroll
        for (int m = 0; m < 6; ++m) {
          qv[m] = QI[r][c + m];
          dx[m] = dxa[pidx(d, i - 3 + m, j)];
        }
        const double f = ppm_flux_ord(ord, i + sub.ioff, sub.N, qv, dx, crx[fo + o]);
        fx[zo + o] = 0.5 * (f + FX2[r + 3][c]) * mx[fo + o];
      }
      if (i < nx && j <= ny) {
        double qv[6], dy[6];
#pragma unroll
        for (int m = 0; m < 6; ++m) {
          qv[m] = QJ[r + m][c];
          dy[m] = dya[pidx(d, i, j - 3 + m)];
        }
        const double f = ppm_flux_ord(ord, j + sub.joff, sub.N, qv, dy, cry[fo + o]);
        fy[zo + o] = 0.5 * (f + FY2[r][c + 3]) * my[fo + o];
      }
    }
  }
}

// ---------------- tracer_2d_1l ----------------

__device__ __forceinline__ void atomic_max_pos(double* addr, double v) {
  // non-negative doubles order like their bit patterns
  atomicMax(reinterpret_cast<unsigned long long*>(addr), (unsigned long long)__double_as_longlong(v));
}

__global__ void __launch_bounds__(256) tracer_prep_k(Dims d, const double* __restrict__ M, int npz,
                                                     const double* __restrict__ cx, const double* __restrict__ cy,
                                                     double* __restrict__ xfx, double* __restrict__ yfx,
                                                     double* __restrict__ cmax) {
  Launch2D L{-NG, -NG, d.nx + 2 * NG + 1, d.ny + 2 * NG + 1};
  int i, j;
  bool act = thread_point(L, i, j);
  const int z = blockIdx.z, k = z % npz, s = z / npz;
  const long fo = (long)z * d.plane;
  double cm = 0.0;
  if (act) {
    const long o = pidx(d, i, j);
    if (i >= 0 && i <= d.nx && j >= -NG && j <= d.ny + NG - 1) {
      double c = cx[fo + o];
      double v;
      if (c > 0.0)
        v = c * met(M, d, M_DXA, s)[pidx(d, i - 1, j)] * met(M, d, M_DY, s)[o] * met(M, d, M_SIN3, s)[pidx(d, i - 1, j)];
      else
        v = c * met(M, d, M_DXA, s)[o] * met(M, d, M_DY, s)[o] * met(M, d, M_SIN1, s)[o];
      xfx[fo + o] = v;
    }
    if (j >= 0 && j <= d.ny && i >= -NG && i <= d.nx + NG - 1) {
      double c = cy[fo + o];
      double v;
      if (c > 0.0)
        v = c * met(M, d, M_DYA, s)[pidx(d, i, j - 1)] * met(M, d, M_DX, s)[o] * met(M, d, M_SIN4, s)[pidx(d, i, j - 1)];
      else
        v = c * met(M, d, M_DYA, s)[o] * met(M, d, M_DX, s)[o] * met(M, d, M_SIN2, s)[o];
      yfx[fo + o] = v;
    }
    if (i >= 0 && i < d.nx && j >= 0 && j < d.ny) {
      double a = fmax(fabs(cx[fo + o]), fabs(cy[fo + o]));
      if (!(k + 1 < npz / 6)) a = a + 1.0 - met(M, d, M_SIN5, s)[o];
      cm = a;
    }
  }
  // wave reduction then one atomic per wave
  for (int off = 32; off > 0; off >>= 1) cm = fmax(cm, __shfl_xor(cm, off));
  if ((threadIdx.x & 63) == 0) atomic_max_pos(&cmax[k], cm);
}

__global__ void __launch_bounds__(256) tracer_split_k(Dims d, const double* __restrict__ M, int npz,
                                                      const int* __restrict__ nsplt, double* __restrict__ cx,
                                                      double* __restrict__ cy, double* __restrict__ xfx,
                                                      double* __restrict__ yfx, double* __restrict__ mfx,
                                                      double* __restrict__ mfy, double* __restrict__ ra_x,
                                                      double* __restrict__ ra_y) {
  Launch2D L{-NG, -NG, d.nx + 2 * NG + 1, d.ny + 2 * NG + 1};
  int i, j;
  if (!thread_point(L, i, j)) return;
  const int z = blockIdx.z, k = z % npz;
  const long fo = (long)z * d.plane;
  const long o = pidx(d, i, j);
  const int ns = nsplt[k];
  if (ns > 1) {
    const double frac = 1.0 / (double)ns;
    if (i >= 0 && i <= d.nx && j >= -NG && j <= d.ny + NG - 1) {
      cx[fo + o] *= frac;
      xfx[fo + o] *= frac;
      if (j >= 0 && j < d.ny) mfx[fo + o] *= frac;
    }
    if (j >= 0 && j <= d.ny && i >= -NG && i <= d.nx + NG - 1) {
      cy[fo + o] *= frac;
      yfx[fo + o] *= frac;
      if (i >= 0 && i < d.nx) mfy[fo + o] *= frac;
    }
  }
}

__global__ void __launch_bounds__(256) tracer_ra_k(Dims d, const double* __restrict__ M, int npz,
                                                   const double* __restrict__ xfx, const double* __restrict__ yfx,
                                                   double* __restrict__ ra_x, double* __restrict__ ra_y) {
  Launch2D L{-NG, -NG, d.nx + 2 * NG, d.ny + 2 * NG};
  int i, j;
  if (!thread_point(L, i, j)) return;
  const int z = blockIdx.z, s = z / npz;
  const long fo = (long)z * d.plane;
  const long o = pidx(d, i, j);
  const double area = met(M, d, M_AREA, s)[o];
  if (i >= 0 && i < d.nx) ra_x[fo + o] = area + xfx[fo + o] - xfx[fo + pidx(d, i + 1, j)];
  if (j >= 0 && j < d.ny) ra_y[fo + o] = area + yfx[fo + o] - yfx[fo + pidx(d, i, j + 1)];
}

__global__ void __launch_bounds__(256) tracer_dp2_k(Dims d, const double* __restrict__ M, int npz,
                                                    const double* __restrict__ dp1, const double* __restrict__ mfx,
                                                    const double* __restrict__ mfy, double* __restrict__ dp2) {
  Launch2D L{0, 0, d.nx, d.ny};
  int i, j;
  if (!thread_point(L, i, j)) return;
  const int z = blockIdx.z, s = z / npz;
  const long fo = (long)z * d.plane, o = pidx(d, i, j);
  dp2[fo + o] = dp1[fo + o] + (mfx[fo + o] - mfx[fo + pidx(d, i + 1, j)] + mfy[fo + o] - mfy[fo + pidx(d, i, j + 1)]) *
                                  met(M, d, M_RAREA, s)[o];
}

__global__ void __launch_bounds__(256) tracer_update_k(Dims d, const double* __restrict__ M, int npz, int nq,
                                                       double* __restrict__ q, const double* __restrict__ dp1,
                                                       const double* __restrict__ dp2, const double* __restrict__ fx,
                                                       const double* __restrict__ fy, const int* __restrict__ nsplt,
                                                       int it, int nz) {
  Launch2D L{0, 0, d.nx, d.ny};
  int i, j;
  if (!thread_point(L, i, j)) return;
  for (int z = blockIdx.z; z < nz; z += gridDim.z) {
    const int k = z % npz, s = z / npz / nq;
    if (it >= nsplt[k]) continue;
    const long zo = (long)z * d.plane, fo = ((long)s * npz + k) * d.plane, o = pidx(d, i, j);
    const double ra = met(M, d, M_RAREA, s)[o];
    q[zo + o] = (q[zo + o] * dp1[fo + o] +
                 (fx[zo + o] - fx[zo + pidx(d, i + 1, j)] + fy[zo + o] - fy[zo + pidx(d, i, j + 1)]) * ra) /
                dp2[fo + o];
  }
}

__global__ void copy_k(long n, const double* __restrict__ a, double* __restrict__ b) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long stride = (long)gridDim.x * blockDim.x;
  for (; i < n; i += stride) b[i] = a[i];
}

}  // namespace

void fv_tp_2d(const Ctx& c, const TpArgs& a) {
  const Dims& d = c.d;
  long nz = (long)d.nsub * a.nt * a.nk;
  dim3 g(cdiv(d.nx + 1, TX), cdiv(d.ny + 1, TY), (unsigned)(nz < ZMAX ? nz : ZMAX));
  GT_LAUNCH(tp_fused, g, dim3(TBLOCK), 0, c.st, d, c.subs, c.met, a.q, a.nt, a.nk, a.crx, a.cry, a.xfx, a.yfx,
            a.ra_x, a.ra_y, a.mfx ? a.mfx : a.xfx, a.mfy ? a.mfy : a.yfx, a.fx, a.fy, a.ord, (int)nz);
  HIP_LAUNCH_CHECK();
}

void tracer_prep(const Ctx& c, int npz, const double* cx, const double* cy, double* xfx, double* yfx, double* ra_x,
                 double* ra_y, double* cmax_dev) {
  const Dims& d = c.d;
  (void)ra_x; (void)ra_y;
  HIP_CHECK(hipMemsetAsync(cmax_dev, 0, sizeof(double) * npz, c.st));
  Launch2D L{-NG, -NG, d.nx + 2 * NG + 1, d.ny + 2 * NG + 1};
  GT_LAUNCH(tracer_prep_k, dim3(cdiv(L.ni, BX), cdiv(L.nj, BY), d.nsub * npz), dim3(BX, BY), 0, c.st, d,
                     c.met, npz, cx, cy, xfx, yfx, cmax_dev);
  HIP_LAUNCH_CHECK();
}

void tracer_split(const Ctx& c, int npz, const int* nsplt_dev, double* cx, double* cy, double* xfx, double* yfx,
                  double* mfx, double* mfy, double* ra_x, double* ra_y) {
  const Dims& d = c.d;
  Launch2D L{-NG, -NG, d.nx + 2 * NG + 1, d.ny + 2 * NG + 1};
  GT_LAUNCH(tracer_split_k, dim3(cdiv(L.ni, BX), cdiv(L.nj, BY), d.nsub * npz), dim3(BX, BY), 0, c.st, d,
                     c.met, npz, nsplt_dev, cx, cy, xfx, yfx, mfx, mfy, ra_x, ra_y);
  HIP_LAUNCH_CHECK();
  Launch2D L2{-NG, -NG, d.nx + 2 * NG, d.ny + 2 * NG};
  GT_LAUNCH(tracer_ra_k, dim3(cdiv(L2.ni, BX), cdiv(L2.nj, BY), d.nsub * npz), dim3(BX, BY), 0, c.st, d,
                     c.met, npz, xfx, yfx, ra_x, ra_y);
  HIP_LAUNCH_CHECK();
}

void tracer_dp2(const Ctx& c, int npz, const double* dp1, const double* mfx, const double* mfy, double* dp2) {
  const Dims& d = c.d;
  GT_LAUNCH(tracer_dp2_k, dim3(cdiv(d.nx, BX), cdiv(d.ny, BY), d.nsub * npz), dim3(BX, BY), 0, c.st, d,
                     c.met, npz, dp1, mfx, mfy, dp2);
  HIP_LAUNCH_CHECK();
}

void tracer_update(const Ctx& c, int npz, int nq, double* q, const double* qn, const double* dp1, const double* dp2,
                   const double* fx, const double* fy, const int* nsplt_dev, int it) {
  (void)qn;
  const Dims& d = c.d;
  long nz = (long)d.nsub * nq * npz;
  GT_LAUNCH(tracer_update_k, dim3(cdiv(d.nx, BX), cdiv(d.ny, BY), (unsigned)(nz < ZMAX ? nz : ZMAX)),
                     dim3(BX, BY), 0, c.st, d, c.met, npz, nq, q, dp1, dp2, fx, fy, nsplt_dev, it, (int)nz);
  HIP_LAUNCH_CHECK();
}

void copy_levels(const Ctx& c, long n, const double* src, double* dst) {
  GT_LAUNCH(copy_k, dim3(cdiv(n, 256) < 8192 ? cdiv(n, 256) : 8192), dim3(256), 0, c.st, n, src, dst);
  HIP_LAUNCH_CHECK();
}

}  // namespace gtfv3
