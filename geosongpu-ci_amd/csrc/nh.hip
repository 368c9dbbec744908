// nh.hip — non-hydrostatic pieces of dyn_core on gfx950: update_dz_c,
// riem_solver_c / riem_solver3 (SIM1 semi-implicit vertical acoustic solve),
// p_grad_c, edge_profile + update_dz_d, pk3_halo / pe_halo, a2b_ord4, nh_p_grad.
// Column kernels put one (i,j) column per lane: a wavefront covers 64 consecutive
// i, so every k-plane access is coalesced; per-column work arrays are planes of
// scratch fields (same [sub][k][plane] layout).
#include <cstdlib>
#include <algorithm>
#include <climits>

#include "fastmath.hpp"
#include "kernels_damp.hpp"
#include "kernels_nh.hpp"
#include "stencil_common.hpp"

namespace gtfv3 {
namespace {

constexpr double KAPPA = Constants::kappa;
constexpr double R3 = 1.0 / 3.0;

#define KSETUP2(nk_)                                                 \
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

// strided column view
struct Col {
  double* p;
  long st;
  __device__ __forceinline__ double& operator[](int k) const { return p[(long)k * st]; }
};
__device__ __forceinline__ Col col(double* f, const Dims& d, int s, int nk, long o) {
  return Col{f + (long)s * nk * d.plane + o, d.plane};
}
__device__ __forceinline__ Col ccol(const double* f, const Dims& d, int s, int nk, long o) {
  return Col{const_cast<double*>(f) + (long)s * nk * d.plane + o, d.plane};
}

// ---------------- update_dz_c (per interface level, out of place) ----------------
__global__ void __launch_bounds__(256) udzc_k(Dims d, const SubInfo* __restrict__ subs, const double* __restrict__ M,
                                              int npz, const double* __restrict__ dp0, const double* __restrict__ ut,
                                              const double* __restrict__ vt, const double* __restrict__ gz,
                                              double* __restrict__ gzo) {
  Launch2D L{-1, -1, d.nx + 2, d.ny + 2};
  KSETUP2(npz + 1)
  const int k = z % (npz + 1);
  const int km = npz;
  // xfx / yfx at faces (0: own, 1: +1 neighbour)
  auto flux_lvl = [&](const double* a, long off) -> double {
    const long b = (long)s * npz * d.plane + off;
    if (k == 0) {
      double top_ratio = dp0[0] / (dp0[1] + dp0[0]);
      return a[b] + (a[b] - a[b + d.plane]) * top_ratio;
    } else if (k == km) {
      double bot_ratio = dp0[km - 1] / (dp0[km - 2] + dp0[km - 1]);
      const double* c = a + (long)(km - 1) * d.plane;
      return c[b] + (c[b] - c[b - d.plane]) * bot_ratio;
    } else {
      double int_ratio = 1.0 / (dp0[k - 1] + dp0[k]);
      const double* c = a + (long)k * d.plane;
      return (dp0[k] * c[b - d.plane] + dp0[k - 1] * c[b]) * int_ratio;
    }
  };
  const double* g = gz + zo;
  double xf0 = flux_lvl(ut, o), xf1 = flux_lvl(ut, o + 1);
  double yf0 = flux_lvl(vt, o), yf1 = flux_lvl(vt, o + d.pitch);
  double fx0 = xf0 * (xf0 > 0.0 ? g[cc_off(d, sub, i - 1, j, 1)] : g[cc_off(d, sub, i, j, 1)]);
  double fx1 = xf1 * (xf1 > 0.0 ? g[cc_off(d, sub, i, j, 1)] : g[cc_off(d, sub, i + 1, j, 1)]);
  double fy0 = yf0 * (yf0 > 0.0 ? g[cc_off(d, sub, i, j - 1, 2)] : g[cc_off(d, sub, i, j, 2)]);
  double fy1 = yf1 * (yf1 > 0.0 ? g[cc_off(d, sub, i, j, 2)] : g[cc_off(d, sub, i, j + 1, 2)]);
  const double area = MA(MT(M_AREA), 0, 0);
  const double gc = g[cc_off(d, sub, i, j, 2)];
  gzo[zo + o] = (gc * area + fx0 - fx1 + fy0 - fy1) / (area + xf0 - xf1 + yf0 - yf1);
}

// C-grid pressure gradient (non-hydrostatic: wk = delpc)
__global__ void __launch_bounds__(256) pgradc_k(Dims d, const SubInfo* __restrict__ subs, const double* __restrict__ M,
                                                int npz, double dt2, const double* __restrict__ delpc,
                                                const double* __restrict__ pkc, const double* __restrict__ gz,
                                                double* __restrict__ uc, double* __restrict__ vc) {
  Launch2D L{0, 0, d.nx + 1, d.ny + 1};
  KSETUP2(npz)
  const int k = z % npz;
  const long p0 = ((long)s * (npz + 1) + k) * d.plane + o;  // interface k
  const long p1 = p0 + d.plane;                             // interface k+1
  if (j < d.ny) {
    const long w = -1;
    double wsum = AT(delpc, -1, 0) + AT(delpc, 0, 0);
    AT(uc, 0, 0) = AT(uc, 0, 0) + dt2 * MA(MT(M_RDXC), 0, 0) / wsum *
                                      ((gz[p1 + w] - gz[p0]) * (pkc[p1] - pkc[p0 + w]) +
                                       (gz[p0 + w] - gz[p1]) * (pkc[p1 + w] - pkc[p0]));
  }
  if (i < d.nx) {
    const long w = -d.pitch;
    double wsum = AT(delpc, 0, -1) + AT(delpc, 0, 0);
    AT(vc, 0, 0) = AT(vc, 0, 0) + dt2 * MA(MT(M_RDYC), 0, 0) / wsum *
                                      ((gz[p1 + w] - gz[p0]) * (pkc[p1] - pkc[p0 + w]) +
                                       (gz[p0 + w] - gz[p1]) * (pkc[p1 + w] - pkc[p0]));
  }
}

// edge_profile of (crx, xfx) on x-face columns and (cry, yfx) on y-face columns.
// The tridiagonal coefficients depend only on the reference thicknesses dp0, so the
// ratios gk, the pivots bet and the elimination factors gam are computed once per
// workgroup into LDS (same expressions as the per-column form).  Each lane then runs
// its four columns together (four independent recurrences in flight) and reads the
// levels in blocks of EP_B, all loads of a block issued before the first use, so a
// sweep waits for one memory latency per block instead of one per level.
constexpr int EP_KMAX = 256, EP_B = 8;

__global__ void __launch_bounds__(256) edge_prof_k(Dims d, int npz, const double* __restrict__ dp0,
                                                   const double* __restrict__ crx, const double* __restrict__ xfx,
                                                   const double* __restrict__ cry, const double* __restrict__ yfx,
                                                   double* __restrict__ crx_e, double* __restrict__ xfx_e,
                                                   double* __restrict__ cry_e, double* __restrict__ yfx_e) {
  __shared__ double gam[EP_KMAX], gks[EP_KMAX], bets[EP_KMAX];
  const int km = npz, k1 = npz + 1;
  const int tid = threadIdx.y * blockDim.x + threadIdx.x;
  for (int k = 1 + tid; k < km; k += blockDim.x * blockDim.y) gks[k] = dp0[k - 1] / dp0[k];
  __syncthreads();
  const double g0 = dp0[1] / dp0[0];
  const double bet0 = g0 * (g0 + 0.5);
  if (tid == 0) {
    gam[0] = (1.0 + g0 * (g0 + 1.5)) / bet0;
    for (int k = 1; k < km; ++k) {
      const double bet = 2.0 + 2.0 * gks[k] - gam[k - 1];
      bets[k] = bet;
      gam[k] = gks[k] / bet;
    }
  }
  __syncthreads();
  Launch2D L{-NG, -NG, d.nx + 2 * NG + 1, d.ny + 2 * NG + 1};
  int i, j;
  if (!thread_point(L, i, j)) return;
  const int s = blockIdx.z;
  const long P = d.plane;
  const long o = pidx(d, i, j);
  const bool xface = i >= 0 && i <= d.nx && j <= d.ny + NG - 1;
  const bool yface = j >= 0 && j <= d.ny && i <= d.nx + NG - 1;
  if (!xface && !yface) return;
  const long bq = (long)s * km * P + o, be = (long)s * k1 * P + o;
  const double* __restrict__ Q[4] = {crx + bq, xfx + bq, cry + bq, yfx + bq};
  double* __restrict__ E[4] = {crx_e + be, xfx_e + be, cry_e + be, yfx_e + be};
  const bool ok[4] = {xface, xface, yface, yface};
  // forward elimination
  const double xt1_0 = 2.0 * g0 * (g0 + 1.0);
  double qp[4], qprev[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const double q0 = Q[c][0], q1 = Q[c][P];
    qp[c] = (xt1_0 * q0 + q1) / bet0;
    if (ok[c]) E[c][0] = qp[c];
    qprev[c] = q0;
  }
  for (int kb = 1; kb < km; kb += EP_B) {
    double qv[EP_B][4];
#pragma unroll
    for (int u = 0; u < EP_B; ++u) {
      const int k = kb + u < km ? kb + u : km - 1;
#pragma unroll
      for (int c = 0; c < 4; ++c) qv[u][c] = Q[c][k * P];
    }
#pragma unroll
    for (int u = 0; u < EP_B; ++u) {
      const int k = kb + u;
      if (k >= km) break;
      const double gk = gks[k], bet = bets[k];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        qp[c] = (3.0 * (qprev[c] + gk * qv[u][c]) - qp[c]) / bet;
        if (ok[c]) E[c][k * P] = qp[c];
        qprev[c] = qv[u][c];
      }
    }
  }
  // bottom edge and back substitution
  const double gk = km > 1 ? gks[km - 1] : g0;
  const double a_bot = 1.0 + gk * (gk + 1.5);
  const double xt1 = 2.0 * gk * (gk + 1.0);
  const double xt2 = gk * (gk + 0.5) - a_bot * gam[km - 1];
  double x[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    x[c] = (xt1 * qprev[c] + Q[c][(km - 2) * P] - a_bot * qp[c]) / xt2;
    if (ok[c]) E[c][km * P] = x[c];
  }
  for (int kb = km - 1; kb >= 0; kb -= EP_B) {
    double ev[EP_B][4];
#pragma unroll
    for (int u = 0; u < EP_B; ++u) {
      const int k = kb - u >= 0 ? kb - u : 0;
#pragma unroll
      for (int c = 0; c < 4; ++c) ev[u][c] = E[c][k * P];
    }
#pragma unroll
    for (int u = 0; u < EP_B; ++u) {
      const int k = kb - u;
      if (k < 0) break;
      const double gm = gam[k];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        x[c] = ev[u][c] - gm * x[c];
        if (ok[c]) E[c][k * P] = x[c];
      }
    }
  }
}

// Register-resident edge_profile: one lane per (face column, field), the column's KMAX
// levels held in VGPRs.  The forward pivots overwrite the inputs in place and the back
// substitution reads them from registers, so each field is read once and its result
// written once (8 field passes instead of the 16 of edge_prof_k, whose forward values
// round-trip through the output).  Same expressions in the same order as edge_prof_k:
// bit-identical results.  Loops are unrolled over KMAX with uniform guards k < km.
template <int KMAX>
__global__ void __launch_bounds__(256) edge_prof_reg_k(Dims d, int npz, const double* __restrict__ dp0,
                                                       const double* __restrict__ crx, const double* __restrict__ xfx,
                                                       const double* __restrict__ cry, const double* __restrict__ yfx,
                                                       double* __restrict__ crx_e, double* __restrict__ xfx_e,
                                                       double* __restrict__ cry_e, double* __restrict__ yfx_e) {
  __shared__ double gam[KMAX], gks[KMAX], bets[KMAX];
  const int km = npz, k1 = npz + 1;
  const int tid = threadIdx.y * blockDim.x + threadIdx.x;
  for (int k = 1 + tid; k < km; k += blockDim.x * blockDim.y) gks[k] = dp0[k - 1] / dp0[k];
  __syncthreads();
  const double g0 = dp0[1] / dp0[0];
  const double bet0 = g0 * (g0 + 0.5);
  if (tid == 0) {
    gam[0] = (1.0 + g0 * (g0 + 1.5)) / bet0;
    for (int k = 1; k < km; ++k) {
      const double bet = 2.0 + 2.0 * gks[k] - gam[k - 1];
      bets[k] = bet;
      gam[k] = gks[k] / bet;
    }
  }
  __syncthreads();
  Launch2D L{-NG, -NG, d.nx + 2 * NG + 1, d.ny + 2 * NG + 1};
  int i, j;
  if (!thread_point(L, i, j)) return;
  const int s = blockIdx.z >> 2, c = blockIdx.z & 3;
  const long P = d.plane;
  const long o = pidx(d, i, j);
  const bool ok = c < 2 ? (i >= 0 && i <= d.nx && j <= d.ny + NG - 1) : (j >= 0 && j <= d.ny && i <= d.nx + NG - 1);
  if (!ok) return;
  const double* __restrict__ Q = (c == 0 ? crx : c == 1 ? xfx : c == 2 ? cry : yfx) + (long)s * km * P + o;
  double* __restrict__ E = (c == 0 ? crx_e : c == 1 ? xfx_e : c == 2 ? cry_e : yfx_e) + (long)s * k1 * P + o;
  double q[KMAX];
#pragma unroll
  for (int k = 0; k < KMAX; ++k)
    if (k < km) q[k] = Q[k * P];
  // forward elimination, pivots in place of the inputs
  const double xt1_0 = 2.0 * g0 * (g0 + 1.0);
  double qprev = q[0], qkm2 = q[0];
  q[0] = (xt1_0 * q[0] + q[1]) / bet0;
#pragma unroll
  for (int k = 1; k < KMAX; ++k) {
    if (k < km) {
      const double qk = q[k];
      if (k == km - 2) qkm2 = qk;
      q[k] = (3.0 * (qprev + gks[k] * qk) - q[k - 1]) / bets[k];
      qprev = qk;
    }
  }
  double qlast = q[0];
#pragma unroll
  for (int k = 1; k < KMAX; ++k)
    if (k == km - 1) qlast = q[k];
  // bottom edge and back substitution
  const double gk = gks[km - 1];
  const double a_bot = 1.0 + gk * (gk + 1.5);
  const double xt1 = 2.0 * gk * (gk + 1.0);
  const double xt2 = gk * (gk + 0.5) - a_bot * gam[km - 1];
  double x = (xt1 * qprev + qkm2 - a_bot * qlast) / xt2;
  E[km * P] = x;
#pragma unroll
  for (int k = KMAX - 1; k >= 0; --k) {
    if (k < km) {
      x = q[k] - gam[k] * x;
      E[k * P] = x;
    }
  }
}

// pk3 on the 2-wide halo ring and pe on the 1-wide ring (from the halo-updated delp):
// one lane per (ring column, level); each lane sums delp from the top in the same order
// as the sequential column loop, so the values are identical
__device__ __forceinline__ bool ring2_point(int t, int nx, int ny, int& i, int& j) {
  const int w = nx + 4;
  if (t < 2 * w) { i = t % w - 2; j = t / w - 2; return true; }            // rows -2, -1
  t -= 2 * w;
  if (t < 2 * w) { i = t % w - 2; j = ny + t / w; return true; }           // rows ny, ny+1
  t -= 2 * w;
  if (t < 2 * ny) { i = t % 2 - 2; j = t / 2; return true; }               // cols -2, -1
  t -= 2 * ny;
  if (t < 2 * ny) { i = nx + t % 2; j = t / 2; return true; }              // cols nx, nx+1
  return false;
}

// One lane per (ring column, block of PK_B levels): the interface pressure of level k+1
// is the running sum ptop + delp[0] + ... + delp[k], which each lane forms from the top
// with the same additions in the same order (bit-identical to one sequential walk, and to
// the interior columns' values); pk3 = exp(kappa log pe).  The blocks give the ring's few
// columns (a band of 180 x 45: ~900 per sub-domain) nine lanes each, so the transcendentals
// of a column's levels run in parallel instead of one after another.
constexpr int PK_B = 8;
__global__ void __launch_bounds__(64) pk3_pe_halo_k(Dims d, int npz, double ptop, int do_pe,
                                                    const double* __restrict__ delp, double* __restrict__ pk3,
                                                    double* __restrict__ pe) {
  const int nb = (npz + PK_B - 1) / PK_B;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = t % nb;
  int i, j;
  if (!ring2_point(t / nb, d.nx, d.ny, i, j)) return;
  const int s = blockIdx.y;
  const long o = pidx(d, i, j);
  const int km = npz, k1 = npz + 1;
  const long P = d.plane;
  const double* DP = delp + (long)s * km * P + o;
  const bool ring1 = i >= -1 && i <= d.nx && j >= -1 && j <= d.ny;
  const long b1 = (long)s * k1 * P + o;
  const int k0 = b * PK_B, k1e = k0 + PK_B < km ? k0 + PK_B : km;
  if (do_pe && ring1 && b == 0) pe[b1] = ptop;
  double pei = ptop;
  // the sum in blocks of PK_B loads issued together (one memory latency per block)
  for (int m0 = 0; m0 < k0; m0 += PK_B) {
    double v[PK_B];
#pragma unroll
    for (int u = 0; u < PK_B; ++u) v[u] = DP[(long)(m0 + u) * P];
#pragma unroll
    for (int u = 0; u < PK_B; ++u) pei = pei + v[u];
  }
  double v[PK_B];
#pragma unroll
  for (int u = 0; u < PK_B; ++u) v[u] = k0 + u < k1e ? DP[(long)(k0 + u) * P] : 0.0;
#pragma unroll
  for (int u = 0; u < PK_B; ++u) {
    if (k0 + u < k1e) {
      pei = pei + v[u];
      const long x = b1 + (long)(k0 + u + 1) * P;
      pk3[x] = fm_exp(KAPPA * fm_log(pei));  // as riem_scan_k forms pk3 in the compute domain
      if (do_pe && ring1) pe[x] = pei;
    }
  }
}

// ---------------- a2b_ord4 (3 passes) ----------------
constexpr double B1 = 7.0 / 12.0, B2 = -1.0 / 12.0;
constexpr double AA1 = 0.5625, AA2 = -0.0625;
constexpr double AC1 = 2.0 / 3.0, AC2 = -1.0 / 6.0;

// x- and y-interpolated values of a2b_ord4 at one point (the former qx / qy planes),
// evaluated on the fly by the corner-value kernels so those planes never touch HBM.
// Zero where the 3-pass form left them unset.
struct A2bPoint {
  // held by value: a reference to the kernel's Dims argument would need its address and
  // put the struct in scratch memory
  Dims d;
  SubInfo sub;
  const double* q;   // plane of the level
  const double* dxa;
  const double* dya;
  double sc;         // the field's scale, applied as it is loaded (sc * q, 1 for most fields)
  __device__ __forceinline__ double Q(int i, int j) const { return sc * q[pidx(d, i, j)]; }
  __device__ __forceinline__ double qx(int i, int j) const {
    const int N = sub.N, io = sub.ioff, jo = sub.joff, nx = d.nx, ny = d.ny;
    const int I = i + io, J = j + jo;
    if (!(J >= max(0, jo - 2) && J <= min(N - 1, jo + ny + 1))) return 0.0;
    auto gen = [&](int di) { return B2 * (Q(i + di - 2, j) + Q(i + di + 1, j)) + B1 * (Q(i + di - 1, j) + Q(i + di, j)); };
    auto DX = [&](int di) { return dxa[pidx(d, i + di, j)]; };
    if (I == 0) {
      double gr = DX(1) / DX(0);
      return 0.5 * ((2.0 + gr) * (Q(i - 1, j) + Q(i, j)) - (Q(i - 2, j) + Q(i + 1, j))) / (1.0 + gr);
    } else if (I == N) {
      double gr = DX(-2) / DX(-1);
      return 0.5 * ((2.0 + gr) * (Q(i - 1, j) + Q(i, j)) - (Q(i - 2, j) + Q(i + 1, j))) / (1.0 + gr);
    } else if (I == 1) {
      double g1 = DX(0) / DX(-1);
      double gw = DX(0) / DX(-1);  // ratio at the edge I = 0: dxa(1)/dxa(0)
      double qx0 = 0.5 * ((2.0 + gw) * (Q(i - 2, j) + Q(i - 1, j)) - (Q(i - 3, j) + Q(i, j))) / (1.0 + gw);
      return (3.0 * (g1 * Q(i - 1, j) + Q(i, j)) - (g1 * qx0 + gen(1))) / (2.0 + 2.0 * g1);
    } else if (I == N - 1) {
      double g1 = DX(-1) / DX(0);
      double ge = DX(-1) / DX(0);  // ratio at the edge I = N: dxa(N-2)/dxa(N-1)
      double qxN = 0.5 * ((2.0 + ge) * (Q(i, j) + Q(i + 1, j)) - (Q(i - 1, j) + Q(i + 2, j))) / (1.0 + ge);
      return (3.0 * (Q(i - 1, j) + g1 * Q(i, j)) - (g1 * qxN + gen(-1))) / (2.0 + 2.0 * g1);
    } else if (I >= max(2, io) && I <= min(N - 2, io + nx)) {
      return gen(0);
    }
    return 0.0;
  }
  __device__ __forceinline__ double qy(int i, int j) const {
    const int N = sub.N, io = sub.ioff, jo = sub.joff, nx = d.nx, ny = d.ny;
    const int I = i + io, J = j + jo;
    if (!(I >= max(0, io - 2) && I <= min(N - 1, io + nx + 1))) return 0.0;
    auto gen = [&](int dj) { return B2 * (Q(i, j + dj - 2) + Q(i, j + dj + 1)) + B1 * (Q(i, j + dj - 1) + Q(i, j + dj)); };
    auto DY = [&](int dj) { return dya[pidx(d, i, j + dj)]; };
    if (J == 0) {
      double gr = DY(1) / DY(0);
      return 0.5 * ((2.0 + gr) * (Q(i, j - 1) + Q(i, j)) - (Q(i, j - 2) + Q(i, j + 1))) / (1.0 + gr);
    } else if (J == N) {
      double gr = DY(-2) / DY(-1);
      return 0.5 * ((2.0 + gr) * (Q(i, j - 1) + Q(i, j)) - (Q(i, j - 2) + Q(i, j + 1))) / (1.0 + gr);
    } else if (J == 1) {
      double g1 = DY(0) / DY(-1);
      double gs = DY(0) / DY(-1);
      double qy0 = 0.5 * ((2.0 + gs) * (Q(i, j - 2) + Q(i, j - 1)) - (Q(i, j - 3) + Q(i, j))) / (1.0 + gs);
      return (3.0 * (g1 * Q(i, j - 1) + Q(i, j)) - (g1 * qy0 + gen(1))) / (2.0 + 2.0 * g1);
    } else if (J == N - 1) {
      double g1 = DY(-1) / DY(0);
      double gn = DY(-1) / DY(0);
      double qyN = 0.5 * ((2.0 + gn) * (Q(i, j) + Q(i, j + 1)) - (Q(i, j - 1) + Q(i, j + 2))) / (1.0 + gn);
      return (3.0 * (Q(i, j - 1) + g1 * Q(i, j)) - (g1 * qyN + gen(-1))) / (2.0 + 2.0 * g1);
    } else if (J >= max(2, jo) && J <= min(N - 2, jo + ny)) {
      return gen(0);
    }
    return 0.0;
  }
};

// Cube-corner extrapolation points of a2b_edge (FV3 a2b_ord4 corner treatment): for
// corner c = 0 (0,0), 1 (N,0), 2 (N,N), 3 (0,N) and face r, the pair of cells
// (i1, j1, i2, j2), each coordinate A * N + B (tile-global).
__constant__ int kCornerA[4][3][4] = {{{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}},
                                      {{1, 0, 1, 0}, {1, 0, 1, 0}, {1, 0, 1, 0}},
                                      {{1, 1, 1, 1}, {1, 1, 1, 1}, {1, 1, 1, 1}},
                                      {{0, 1, 0, 1}, {0, 1, 0, 1}, {0, 1, 0, 1}}};
__constant__ int kCornerB[4][3][4] = {{{0, 0, 1, 1}, {-1, 0, -2, 1}, {0, -1, 1, -2}},
                                      {{-1, 0, -2, 1}, {-1, -1, -2, -2}, {0, 0, 1, 1}},
                                      {{-1, -1, -2, -2}, {0, -1, 1, -2}, {-1, 0, -2, 1}},
                                      {{0, -1, 1, -2}, {-1, -1, -2, -2}, {0, 0, 1, 1}}};

// The tile-edge / cube-corner forms of a2b_ord4 as force-inlined members (no lambdas
// and no references to kernel arguments: either left a stack object in scratch memory,
// and scratch-using kernels launched from several host threads on concurrent streams
// faulted in the multi-rank loopback runs).
struct A2bEdge {
  A2bPoint P;
  const double* q;   // plane of the level
  const double* cw;  // corner weights of the sub-domain [4][3]
  int N, io, jo;
  __device__ __forceinline__ double gqx(int Ig, int Jg) const { return P.qx(Ig - io, Jg - jo); }
  __device__ __forceinline__ double gqy(int Ig, int Jg) const { return P.qy(Ig - io, Jg - jo); }
  __device__ __forceinline__ double colv(int Ig, int Jg) const {  // W/E edge generic
    return AA2 * (gqx(Ig, Jg - 2) + gqx(Ig, Jg + 1)) + AA1 * (gqx(Ig, Jg - 1) + gqx(Ig, Jg));
  }
  __device__ __forceinline__ double rowv(int Ig, int Jg) const {
    return AA2 * (gqy(Ig - 2, Jg) + gqy(Ig + 1, Jg)) + AA1 * (gqy(Ig - 1, Jg) + gqy(Ig, Jg));
  }
  // cube corner value (extrapolation from the three faces), points from constant memory
  __device__ __forceinline__ double corner_val(int c) const {
    double acc = 0.0;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const double q1 = P.sc * q[pidx(P.d, kCornerA[c][r][0] * N + kCornerB[c][r][0] - io,
                                      kCornerA[c][r][1] * N + kCornerB[c][r][1] - jo)];
      const double q2 = P.sc * q[pidx(P.d, kCornerA[c][r][2] * N + kCornerB[c][r][2] - io,
                                      kCornerA[c][r][3] * N + kCornerB[c][r][3] - jo)];
      const double e = q1 + cw[c * 3 + r] * (q1 - q2);
      acc = r == 0 ? e : acc + e;
    }
    return acc * R3;
  }
  // value of qout at a tile-edge point (recursion-free)
  __device__ __forceinline__ double edge_or_corner(int Ig, int Jg) const {
    if (Ig == 0 && Jg == 0) return corner_val(0);
    if (Ig == N && Jg == 0) return corner_val(1);
    if (Ig == N && Jg == N) return corner_val(2);
    if (Ig == 0 && Jg == N) return corner_val(3);
    if (Ig == 0 || Ig == N) return colv(Ig, Jg);
    return rowv(Ig, Jg);
  }
};

// Up to four independent a2b_ord4 fields in one launch (nh_p_grad interpolates pp, pk3,
// gz and delp): plane index z runs over the fields' planes back to back, zb[f] is the
// first plane of field f (unused entries: INT_MAX).  More waves per launch overlap the
// march kernels' row-latency chains of the four fields.
constexpr int A2B_MAXF = 4;
// sc[f]: a scale applied to field f as it is loaded -- nh_p_grad interpolates gz = grav * zh
// straight from zh (the same product, so the same bits as a scaled copy, without the pass)
struct A2bF {
  const double* q[A2B_MAXF];
  double* qo[A2B_MAXF];
  int nk[A2B_MAXF];
  int zb[A2B_MAXF + 1];
  double sc[A2B_MAXF];
};
struct A2bSel {
  const double* q;
  double* qo;
  int nk, z;  // z: plane within the field
  double sc;
};
__device__ __forceinline__ A2bSel a2b_select(const A2bF& F, int z) {
  const int f = (z >= F.zb[1]) + (z >= F.zb[2]) + (z >= F.zb[3]);
  A2bSel r;
  r.q = f == 0 ? F.q[0] : (f == 1 ? F.q[1] : (f == 2 ? F.q[2] : F.q[3]));
  r.qo = f == 0 ? F.qo[0] : (f == 1 ? F.qo[1] : (f == 2 ? F.qo[2] : F.qo[3]));
  r.nk = f == 0 ? F.nk[0] : (f == 1 ? F.nk[1] : (f == 2 ? F.nk[2] : F.nk[3]));
  r.z = z - (f == 0 ? F.zb[0] : (f == 1 ? F.zb[1] : (f == 2 ? F.zb[2] : F.zb[3])));
  r.sc = f == 0 ? F.sc[0] : (f == 1 ? F.sc[1] : (f == 2 ? F.sc[2] : F.sc[3]));
  return r;
}

// qout on cube corners and tile-edge lines
__global__ void __launch_bounds__(256) a2b_edge_k(Dims d, const SubInfo* __restrict__ subs,
                                                  const double* __restrict__ M, A2bF F, const double* __restrict__ cw) {
  // all targets lie on the tile-edge lines: one lane per line point
  const int zg = blockIdx.z;
  const int f = (zg >= F.zb[1]) + (zg >= F.zb[2]) + (zg >= F.zb[3]);
  const int nk = f == 0 ? F.nk[0] : (f == 1 ? F.nk[1] : (f == 2 ? F.nk[2] : F.nk[3]));
  const int z = zg - (f == 0 ? F.zb[0] : (f == 1 ? F.zb[1] : (f == 2 ? F.zb[2] : F.zb[3]))), s = z / nk;
  const double* __restrict__ q = f == 0 ? F.q[0] : (f == 1 ? F.q[1] : (f == 2 ? F.q[2] : F.q[3]));
  double* __restrict__ qout = f == 0 ? F.qo[0] : (f == 1 ? F.qo[1] : (f == 2 ? F.qo[2] : F.qo[3]));
  const double sc = f == 0 ? F.sc[0] : (f == 1 ? F.sc[1] : (f == 2 ? F.sc[2] : F.sc[3]));
  const SubInfo sub = subs[s];
  int i, j;
  if (!edge_line_point(blockIdx.x * blockDim.x + threadIdx.x, sub, 0, d.nx, 0, d.ny, i, j)) return;
  const int N = sub.N;
  const int I = i + sub.ioff, J = j + sub.joff;
  const long zo = (long)z * d.plane;
  const long o = pidx(d, i, j);
  const int io = sub.ioff, jo = sub.joff, nx = d.nx, ny = d.ny;
  (void)cw;
  double val;
  bool set = true;
  const A2bEdge E{A2bPoint{d, sub, q + zo, met(M, d, M_DXA, s), met(M, d, M_DYA, s), sc}, q + zo, cw + (long)s * 12, N, io,
                  jo};
  if ((I == 0 || I == N) && (J == 0 || J == N)) val = E.edge_or_corner(I, J);
  else if ((I == 0 && io == 0) || (I == N && io + nx == N)) {
    if (J == 1 && jo == 0) val = AC1 * (E.gqx(I, 0) + E.gqx(I, 1)) + AC2 * (E.edge_or_corner(I, 0) + E.colv(I, 2));
    else if (J == N - 1 && jo + ny == N)
      val = AC1 * (E.gqx(I, N - 2) + E.gqx(I, N - 1)) + AC2 * (E.colv(I, N - 2) + E.edge_or_corner(I, N));
    else if (J >= max(2, jo) && J <= min(N - 2, jo + ny)) val = E.colv(I, J);
    else set = false;
  } else if ((J == 0 && jo == 0) || (J == N && jo + ny == N)) {
    if (I == 1 && io == 0) val = AC1 * (E.gqy(0, J) + E.gqy(1, J)) + AC2 * (E.edge_or_corner(0, J) + E.rowv(2, J));
    else if (I == N - 1 && io + nx == N)
      val = AC1 * (E.gqy(N - 2, J) + E.gqy(N - 1, J)) + AC2 * (E.rowv(N - 2, J) + E.edge_or_corner(N, J));
    else if (I >= max(2, io) && I <= min(N - 2, io + nx)) val = E.rowv(I, J);
    else set = false;
  } else {
    set = false;
  }
  if (set) AT(qout, 0, 0) = val;
}

// The same values as a2b_edge_k, one workgroup per 256 points of one tile-edge line of one
// plane: the line's x- (or y-) interpolants at its points and two beyond either end are formed
// once into LDS (each an edge-form PPM value: four q loads, two dxa loads, one division) and
// every point's colv / rowv reads its four from there -- a2b_edge_k formed all four per point
// (78 us per launch of nh_p_grad's four fields at C180, a quarter of a2b_march_k's time).
// blockIdx.y: 0 the west line I = 0, 1 east I = N, 2 south J = 0, 3 north J = N (lines the
// sub-domain does not have, and the y-line points an x line holds, write nothing).
constexpr int AE_T = 256;
__global__ void __launch_bounds__(AE_T) a2b_edge2_k(Dims d, const SubInfo* __restrict__ subs,
                                                    const double* __restrict__ M, A2bF F, const double* __restrict__ cw) {
  // the field of this plane by a uniform compare chain (a2b_edge_k's: a reference to the
  // kernel argument, as a2b_select takes it, put the table in scratch memory here)
  const int zg = blockIdx.z;
  const int f = (zg >= F.zb[1]) + (zg >= F.zb[2]) + (zg >= F.zb[3]);
  A2bSel fs;
  fs.nk = f == 0 ? F.nk[0] : (f == 1 ? F.nk[1] : (f == 2 ? F.nk[2] : F.nk[3]));
  fs.z = zg - (f == 0 ? F.zb[0] : (f == 1 ? F.zb[1] : (f == 2 ? F.zb[2] : F.zb[3])));
  fs.q = f == 0 ? F.q[0] : (f == 1 ? F.q[1] : (f == 2 ? F.q[2] : F.q[3]));
  fs.qo = f == 0 ? F.qo[0] : (f == 1 ? F.qo[1] : (f == 2 ? F.qo[2] : F.qo[3]));
  fs.sc = f == 0 ? F.sc[0] : (f == 1 ? F.sc[1] : (f == 2 ? F.sc[2] : F.sc[3]));
  const int s = fs.z / fs.nk;
  const SubInfo sub = subs[s];
  const int N = sub.N, io = sub.ioff, jo = sub.joff, nx = d.nx, ny = d.ny;
  const int line = blockIdx.y;
  const bool xl = line < 2;
  if (line == 0 && io != 0) return;
  if (line == 1 && io + nx != N) return;
  if (line == 2 && jo != 0) return;
  if (line == 3 && jo + ny != N) return;
  const int len = xl ? ny + 1 : nx + 1;
  const int p0 = blockIdx.x * AE_T;
  if (p0 >= len) return;
  const long zo = (long)fs.z * d.plane;
  const A2bEdge E{A2bPoint{d, sub, fs.q + zo, met(M, d, M_DXA, s), met(M, d, M_DYA, s), fs.sc}, fs.q + zo,
                  cw + (long)s * 12, N, io, jo};
  // this line's fixed local index; the interpolant along it (j on an x line, i on a y line)
  // at positions p0 - 2 .. p0 + AE_T + 1 into LDS
  const int fix = line == 0 ? 0 : (line == 1 ? nx : (line == 2 ? 0 : ny));
  __shared__ double sq[AE_T + 4];
  const int t = threadIdx.x;
  {
    const int pa = p0 - 2 + t, pb = p0 - 2 + AE_T + (t & 3);
    sq[t] = xl ? E.P.qx(fix, pa) : E.P.qy(pa, fix);
    const double vb = xl ? E.P.qx(fix, pb) : E.P.qy(pb, fix);
    if (t < 4) sq[AE_T + t] = vb;
  }
  __syncthreads();
  const int p = p0 + t;
  if (p >= len) return;
  // S(pp) = sq[pp - p0 + 2]; colv / rowv at position pp from LDS (pp - 2 .. pp + 1 lie in this
  // block's range for every pp a point of the block reads: its own, or 2 / N-2 for the
  // positions next to the ends)
  const int b = 2 - p0;
  const int i = xl ? fix : p, j = xl ? p : fix;
  const int I = i + io, J = j + jo;
  double val;
  bool set = true;
  if ((I == 0 || I == N) && (J == 0 || J == N)) {
    if (!xl && ((I == 0 && io == 0) || (I == N && io + nx == N))) return;  // the x line's point
    val = E.edge_or_corner(I, J);
  } else {
    if (!xl && ((I == 0 && io == 0) || (I == N && io + nx == N))) return;  // the x line's point
    // the position along the line and its offset in the tile (J on an x line, I on a y line)
    const int P_ = xl ? J : I, off = xl ? jo : io, lim = xl ? ny : nx;
    const int q2 = 2 - off + b, qn = N - 2 - off + b, qp = p + b;
    if (P_ == 1 && off == 0) {
      const double lv = AA2 * (sq[q2 - 2] + sq[q2 + 1]) + AA1 * (sq[q2 - 1] + sq[q2]);
      val = AC1 * (sq[b] + sq[1 + b]) + AC2 * ((xl ? E.edge_or_corner(I, 0) : E.edge_or_corner(0, J)) + lv);
    } else if (P_ == N - 1 && off + lim == N) {
      const double lv = AA2 * (sq[qn - 2] + sq[qn + 1]) + AA1 * (sq[qn - 1] + sq[qn]);
      val = AC1 * (sq[qn] + sq[qn + 1]) + AC2 * (lv + (xl ? E.edge_or_corner(I, N) : E.edge_or_corner(N, J)));
    } else if (P_ >= max(2, off) && P_ <= min(N - 2, off + lim)) {
      val = AA2 * (sq[qp - 2] + sq[qp + 1]) + AA1 * (sq[qp - 1] + sq[qp]);
    } else {
      set = false;
    }
  }
  if (set) fs.qo[zo + pidx(d, i, j)] = val;
}

// ---- a2b_ord4 interior, column-marching form (default) ----
// One wavefront owns 64 columns c = a-2 .. a+61 of one (sub-domain, level) and marches up
// a segment of corner rows; corners a .. a+60 are its outputs.  Per cell row r it loads
// q once, forms the x-interpolant qx at the lane's corner column (x neighbours by DPP)
// and keeps q and qx of rows r-5..r in registers; the corner row j = r-2 then needs the
// y-interpolant qy of its own column (from the q window) and of the neighbour columns
// (DPP again).  Same expressions as A2bPoint and oracle/nh_core.py a2b_ord4.  (It
// replaced an LDS-tiled kernel whose 8-row qx tile missed the row j-3 that the
// J = N-1 form reads, wrong whenever N-1 was the first row of a tile.)
constexpr int AM_W = 64, AM_OUT = 61, AM_WAVES = 4, AM_B = 2;

__device__ __forceinline__ double dpp_prev_d(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), 0x138, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), 0x138, 0xF, 0xF, true);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double dpp_next_d(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), 0x130, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), 0x130, 0xF, 0xF, true);
  return __hiloint2double(hi, lo);
}

struct A2bM {
  Dims d;
  const SubInfo* subs;
  const double* M;
  A2bF F;
  int nz, nstrip, nseg, seg;  // nz: planes of all fields
};

template <bool EX>
__device__ void a2b_march_strip(const A2bM& a, const double* qf, double* qof, int nk, int z, int a0, int a1, int j0,
                                int j1, double sc) {
  const Dims& d = a.d;
  const int lane = threadIdx.x & (AM_W - 1);
  const int s = z / nk;
  const SubInfo sub = a.subs[s];
  const int N = sub.N, io = sub.ioff, jo = sub.joff, nx = d.nx, ny = d.ny;
  const int c = a0 - 2 + lane;  // this lane's column (cell column for qy, corner column for qx)
  const int I = c + io;
  const long pitch = d.pitch;
  const long zo = (long)z * d.plane;
  const double* qq = qf + zo;
  const double* dxa = met(a.M, d, M_DXA, s);
  const double* dya = met(a.M, d, M_DYA, s);
  const int cc = c > nx + NG ? nx + NG : c;  // addressable
  const long xo = cc + NG;
  const bool out_lane = lane >= 2 && lane < 2 + AM_OUT && c < a1;  // corners [a0, a1)
  const bool icols = I >= max(1, io) && I <= min(N - 1, io + nx) && c <= nx;
  const bool qy_col = I >= max(0, io - 2) && I <= min(N - 1, io + nx + 1);
  const bool qx_gen = I >= max(2, io) && I <= min(N - 2, io + nx);

  double Qw[6], QXw[6];  // q and qx of rows r-5 .. r
#pragma unroll
  for (int m = 0; m < 6; ++m) Qw[m] = QXw[m] = 0.0;
  // rows are loaded in blocks of AM_B, one block ahead (double buffered, addresses
  // clamped to the plane, no conditional loads): a wave then waits for memory once per
  // block instead of once per row
  const int rlast = j1 + 1;
  auto row_of = [&](int r) { return (long)((r < rlast ? r : rlast) + NG) * pitch + xo; };
  // The tile-edge forms at I = 1, N-1 / J = 1, N-1 read qout on the neighbouring edge
  // line (written by a2b_edge_k); those loads ride in the same prefetch (a load waited
  // for in the row it is used in would drain every prefetched block: vmcnt is in order).
  const long dxs = I == 1 ? -1 : (I == N - 1 ? 1 : 0);
  const bool xs = dxs != 0;
  const double* qo = qof + zo;
  double qb[AM_B], db[AM_B], xb[AM_B], yb[AM_B], qn[AM_B], dn[AM_B], xn[AM_B], yn[AM_B];
  auto fetch = [&](int r, double& q_, double& d_, double& x_, double& y_) {
    const long o = row_of(r);
    q_ = sc * qq[o];
    d_ = EX ? dxa[o] : 0.0;
    const int j = r - 2;  // corner row of this step
    const long oj = (long)((j > -NG ? (j < rlast ? j : rlast) : -NG) + NG) * pitch + xo;
    x_ = 0.0;
    if (xs) x_ = qo[oj + dxs];
    const int J = j + jo;
    y_ = 0.0;
    // only rows that produce output: a prefetch row below j0 with J == 1 would read
    // the row before the plane (before the allocation for the first plane)
    if (j >= j0 && j < j1) {
      if (J == 1) y_ = qo[oj - pitch];
      else if (J == N - 1) y_ = qo[oj + pitch];
    }
  };
#pragma unroll
  for (int u = 0; u < AM_B; ++u) fetch(j0 - NG + u, qb[u], db[u], xb[u], yb[u]);
  for (int r0 = j0 - NG; r0 <= rlast; r0 += AM_B) {
#pragma unroll
    for (int u = 0; u < AM_B; ++u) fetch(r0 + AM_B + u, qn[u], dn[u], xn[u], yn[u]);
#pragma unroll
    for (int u = 0; u < AM_B; ++u) {
    const int r = r0 + u;
    if (r > rlast) break;
    const long o = (long)(r + NG) * pitch + xo;
    const double qv = qb[u];
    // ---- qx at (corner column c, cell row r)
    const double qm1 = dpp_prev_d(qv), qm2 = dpp_prev_d(qm1), qp1 = dpp_next_d(qv);
    double qx = 0.0;
    const int Jr = r + jo;
    if (Jr >= max(0, jo - 2) && Jr <= min(N - 1, jo + ny + 1)) {
      if (EX) {
        const double qm3 = dpp_prev_d(qm2), qp2 = dpp_next_d(qp1);
        const double dx0 = db[u], dxm1 = dpp_prev_d(dx0), dxm2 = dpp_prev_d(dxm1), dxp1 = dpp_next_d(dx0);
        if (I == 0) {
          const double gr = dxp1 / dx0;
          qx = 0.5 * ((2.0 + gr) * (qm1 + qv) - (qm2 + qp1)) / (1.0 + gr);
        } else if (I == N) {
          const double gr = dxm2 / dxm1;
          qx = 0.5 * ((2.0 + gr) * (qm1 + qv) - (qm2 + qp1)) / (1.0 + gr);
        } else if (I == 1) {
          const double g1 = dx0 / dxm1;
          const double gw = dx0 / dxm1;
          const double qx0 = 0.5 * ((2.0 + gw) * (qm2 + qm1) - (qm3 + qv)) / (1.0 + gw);
          const double gen1 = B2 * (qm1 + qp2) + B1 * (qv + qp1);
          qx = (3.0 * (g1 * qm1 + qv) - (g1 * qx0 + gen1)) / (2.0 + 2.0 * g1);
        } else if (I == N - 1) {
          const double g1 = dxm1 / dx0;
          const double ge = dxm1 / dx0;
          const double qxN = 0.5 * ((2.0 + ge) * (qv + qp1) - (qm1 + qp2)) / (1.0 + ge);
          const double genm = B2 * (qm3 + qv) + B1 * (qm2 + qm1);
          qx = (3.0 * (qm1 + g1 * qv) - (g1 * qxN + genm)) / (2.0 + 2.0 * g1);
        } else if (qx_gen) {
          qx = B2 * (qm2 + qp1) + B1 * (qm1 + qv);
        }
      } else if (qx_gen) {
        qx = B2 * (qm2 + qp1) + B1 * (qm1 + qv);
      }
    }
#pragma unroll
    for (int m = 0; m < 5; ++m) {
      Qw[m] = Qw[m + 1];
      QXw[m] = QXw[m + 1];
    }
    Qw[5] = qv;
    QXw[5] = qx;
    // ---- corner row j = r-2: qy of this column, qyy / qxx, output
    const int j = r - 2;
    if (j < j0) continue;
    const int J = j + jo;
    // Qw[m] = q(c, j-3+m)
    double qy = 0.0;
    if (qy_col) {
      auto gen = [&](int dj) { return B2 * (Qw[dj + 1] + Qw[dj + 4]) + B1 * (Qw[dj + 2] + Qw[dj + 3]); };
      const long oj = o - 2 * pitch;
      auto DY = [&](int dj) { return dya[oj + dj * pitch]; };
      if (J == 0) {
        const double gr = DY(1) / DY(0);
        qy = 0.5 * ((2.0 + gr) * (Qw[2] + Qw[3]) - (Qw[1] + Qw[4])) / (1.0 + gr);
      } else if (J == N) {
        const double gr = DY(-2) / DY(-1);
        qy = 0.5 * ((2.0 + gr) * (Qw[2] + Qw[3]) - (Qw[1] + Qw[4])) / (1.0 + gr);
      } else if (J == 1) {
        const double g1 = DY(0) / DY(-1);
        const double gs = DY(0) / DY(-1);
        const double qy0 = 0.5 * ((2.0 + gs) * (Qw[1] + Qw[2]) - (Qw[0] + Qw[3])) / (1.0 + gs);
        qy = (3.0 * (g1 * Qw[2] + Qw[3]) - (g1 * qy0 + gen(1))) / (2.0 + 2.0 * g1);
      } else if (J == N - 1) {
        const double g1 = DY(-1) / DY(0);
        const double gn = DY(-1) / DY(0);
        const double qyN = 0.5 * ((2.0 + gn) * (Qw[3] + Qw[4]) - (Qw[2] + Qw[5])) / (1.0 + gn);
        qy = (3.0 * (Qw[2] + g1 * Qw[3]) - (g1 * qyN + gen(-1))) / (2.0 + 2.0 * g1);
      } else if (J >= max(2, jo) && J <= min(N - 2, jo + ny)) {
        qy = gen(0);
      }
    }
    // neighbour columns' qy (DPP outside any lane-divergent branch)
    const double qy_m1 = dpp_prev_d(qy), qy_m2 = dpp_prev_d(qy_m1), qy_m3 = dpp_prev_d(qy_m2);
    const double qy_p1 = dpp_next_d(qy), qy_p2 = dpp_next_d(qy_p1);
    const bool jrows = J >= max(1, jo) && J <= min(N - 1, jo + ny) && j <= ny;
    if (!(out_lane && icols && jrows && j < j1)) continue;
    const long oj = o - 2 * pitch;
    // QX(dj) = qx(c, j+dj) = QXw[dj + 3]
    auto qxx_gen = [&](int dj) { return AA2 * (QXw[dj + 1] + QXw[dj + 4]) + AA1 * (QXw[dj + 2] + QXw[dj + 3]); };
    const double QY[6] = {qy_m3, qy_m2, qy_m1, qy, qy_p1, qy_p2};  // QY(di) = QY[di + 3]
    auto qyy_gen = [&](int di) { return AA2 * (QY[di + 1] + QY[di + 4]) + AA1 * (QY[di + 2] + QY[di + 3]); };
    double qxx, qyy;
    if (J == 1) qxx = AC1 * (QXw[2] + QXw[3]) + AC2 * (yb[u] + qxx_gen(1));
    else if (J == N - 1) qxx = AC1 * (QXw[2] + QXw[3]) + AC2 * (yb[u] + qxx_gen(-1));
    else qxx = qxx_gen(0);
    if (I == 1) qyy = AC1 * (QY[2] + QY[3]) + AC2 * (xb[u] + qyy_gen(1));
    else if (I == N - 1) qyy = AC1 * (QY[2] + QY[3]) + AC2 * (xb[u] + qyy_gen(-1));
    else qyy = qyy_gen(0);
    qof[zo + oj] = 0.5 * (qxx + qyy);
    }
#pragma unroll
    for (int u = 0; u < AM_B; ++u) {
      qb[u] = qn[u];
      db[u] = dn[u];
      xb[u] = xn[u];
      yb[u] = yn[u];
    }
  }
}

__global__ void __launch_bounds__(AM_W * AM_WAVES) a2b_march_k(A2bM a) {
  // wave index through readfirstlane: the plane, strip, segment and the pointers derived
  // from them stay in SGPRs (114 -> 78 VGPRs, 4 -> 6 waves per SIMD: C180 2.57 -> 1.96 ms
  // per step; prefetch blocks of 4 rows instead of 2 measured 2.22 ms)
  // XCD-aware order (xcd_block): neighbouring segments, which re-read each other's halo rows,
  // behind one L2
  const long w = (long)xcd_block() * AM_WAVES + __builtin_amdgcn_readfirstlane(threadIdx.x / AM_W);
  const int strip = (int)(w % a.nstrip);
  const long t = w / a.nstrip;
  const int seg = (int)(t % a.nseg);
  const long z = t / a.nseg;
  if (z >= a.nz) return;  // whole wavefront leaves; no workgroup barrier follows
  const A2bSel fs = a2b_select(a.F, (int)z);
  const int s = fs.z / fs.nk;
  const SubInfo& sub = a.subs[s];
  const int nx = a.d.nx;
  // strips of 61 corners; the last one is shifted left to end at corner nx (so a corner
  // next to the east tile edge is never a strip's last output: its stencil reaches c+2),
  // and each strip writes only the corners before the next strip's first one
  const int last0 = nx + 1 - AM_OUT > 0 ? nx + 1 - AM_OUT : 0;
  const int a0 = strip * AM_OUT < last0 ? strip * AM_OUT : last0;
  const int a1 = strip + 1 < a.nstrip ? ((strip + 1) * AM_OUT < last0 ? (strip + 1) * AM_OUT : last0) : nx + 1;
  const int j0 = seg * a.seg;
  const int j1 = j0 + a.seg < a.d.ny + 1 ? j0 + a.seg : a.d.ny + 1;
  const int A = a0 + sub.ioff;
  // x-interpolant edge forms are needed only where a lane's column reaches I <= 1 or I >= N-1
  const bool ex = !(A - 2 >= 2 && A + AM_OUT + 1 <= sub.N - 2);
  if (ex) a2b_march_strip<true>(a, fs.q, fs.qo, fs.nk, fs.z, a0, a1, j0, j1, fs.sc);
  else a2b_march_strip<false>(a, fs.q, fs.qo, fs.nk, fs.z, a0, a1, j0, j1, fs.sc);
}

// non-hydrostatic pressure gradient on the D-grid winds (u, v arrive x dx, dy)
__global__ void __launch_bounds__(256) nhpgrad_k(Dims d, const SubInfo* __restrict__ subs,
                                                 const double* __restrict__ M, int npz, double dt, double ptk,
                                                 const double* __restrict__ ppb, const double* __restrict__ gzb,
                                                 const double* __restrict__ pkb, const double* __restrict__ wk1,
                                                 double* __restrict__ u, double* __restrict__ v) {
  Launch2D L{0, 0, d.nx + 1, d.ny + 1};
  KSETUP2(npz)
  const int k = z % npz;
  const long p0 = ((long)s * (npz + 1) + k) * d.plane + o;
  const long p1 = p0 + d.plane;
  // level-0 interface values are the model-top constants (pp = 0, pk = ptop**kappa)
  const double pk0 = k == 0 ? ptk : pkb[p0];
  const double pp0 = k == 0 ? 0.0 : ppb[p0];
  if (i < d.nx) {
    const long e = 1;
    const double pk0e = k == 0 ? ptk : pkb[p0 + e];
    const double pp0e = k == 0 ? 0.0 : ppb[p0 + e];
    double wk0 = pkb[p1] - pk0, wke = pkb[p1 + e] - pk0e;
    double du1 = dt / (wk0 + wke) *
                 ((gzb[p1] - gzb[p0 + e]) * (pkb[p1 + e] - pk0) + (gzb[p0] - gzb[p1 + e]) * (pkb[p1] - pk0e));
    AT(u, 0, 0) = (AT(u, 0, 0) + du1 +
                   dt / (AT(wk1, 0, 0) + AT(wk1, 1, 0)) *
                       ((gzb[p1] - gzb[p0 + e]) * (ppb[p1 + e] - pp0) + (gzb[p0] - gzb[p1 + e]) * (ppb[p1] - pp0e))) *
                  MA(MT(M_RDX), 0, 0);
  }
  if (j < d.ny) {
    const long e = d.pitch;
    const double pk0e = k == 0 ? ptk : pkb[p0 + e];
    const double pp0e = k == 0 ? 0.0 : ppb[p0 + e];
    double wk0 = pkb[p1] - pk0, wke = pkb[p1 + e] - pk0e;
    double dv1 = dt / (wk0 + wke) *
                 ((gzb[p1] - gzb[p0 + e]) * (pkb[p1 + e] - pk0) + (gzb[p0] - gzb[p1 + e]) * (pkb[p1] - pk0e));
    AT(v, 0, 0) = (AT(v, 0, 0) + dv1 +
                   dt / (AT(wk1, 0, 0) + AT(wk1, 0, 1)) *
                       ((gzb[p1] - gzb[p0 + e]) * (ppb[p1 + e] - pp0) + (gzb[p0] - gzb[p1 + e]) * (ppb[p1] - pp0e))) *
                  MA(MT(M_RDY), 0, 0);
  }
}

// ---- level-loop forms (stencil_common.hpp kloop_levels): same expressions in the same
// order as udzc_k / pgradc_k / nhpgrad_k above, so the outputs are bit-identical.  The
// thread of point (i, j) walks levels k0 .. k1-1 of one sub-domain; the interface values a
// level shares with the next and the metric terms stay in registers.
// Loads first: the six gz points both upwind picks choose among are loaded with the level's
// ut / vt, before the fluxes whose signs select them (the branch-ordered twin, each pick's
// load waiting for its flux, was bit-identical and is deleted in round 4)
__global__ void __launch_bounds__(256) udzc_kl(Dims d, const SubInfo* __restrict__ subs, const double* __restrict__ M,
                                               int npz, int nkb, int klb, const double* __restrict__ dp0,
                                               const double* __restrict__ ut, const double* __restrict__ vt,
                                               const double* __restrict__ gz, double* __restrict__ gzo) {
  Launch2D L{-1, -1, d.nx + 2, d.ny + 2};
  KLSETUP(npz + 1)
  const SubInfo sub = subs[s];
  const int km = npz;
  const double* UT = ut + (long)s * npz * P + o;  // layer l of this column: UT[l * P]
  const double* VT = vt + (long)s * npz * P + o;
  const long N1 = d.pitch;
  const double area = met(M, d, M_AREA, s)[o];
  // cc_off source offsets of the five gz points (plane-relative, level independent)
  const long gw = cc_off(d, sub, i - 1, j, 1), gcx = cc_off(d, sub, i, j, 1), ge = cc_off(d, sub, i + 1, j, 1);
  const long gs = cc_off(d, sub, i, j - 1, 2), gcy = cc_off(d, sub, i, j, 2), gn = cc_off(d, sub, i, j + 1, 2);
  // layer k-1 values (ut at o, o+1; vt at o, o+pitch) carried from the previous interface
  double p0 = 0.0, p1 = 0.0, p2 = 0.0, p3 = 0.0;
  bool have = false;
  for (int k = k0; k < k1; ++k) {
    double xf0, xf1, yf0, yf1;
    const double* g = gz + ((long)s * (npz + 1) + k) * P;
    const double gW = g[gw], gCX = g[gcx], gE = g[ge], gS = g[gs], gCY = g[gcy], gN = g[gn];
    if (k == 0) {
      const double top_ratio = dp0[0] / (dp0[1] + dp0[0]);
      const double a0 = UT[0], a1 = UT[1], b0 = VT[0], b1 = VT[N1];
      xf0 = a0 + (a0 - UT[P]) * top_ratio;
      xf1 = a1 + (a1 - UT[P + 1]) * top_ratio;
      yf0 = b0 + (b0 - VT[P]) * top_ratio;
      yf1 = b1 + (b1 - VT[P + N1]) * top_ratio;
      p0 = a0; p1 = a1; p2 = b0; p3 = b1;
      have = true;
    } else if (k == km) {
      const double bot_ratio = dp0[km - 1] / (dp0[km - 2] + dp0[km - 1]);
      const long c = (long)(km - 1) * P;
      const double a0 = have ? p0 : UT[c], a1 = have ? p1 : UT[c + 1];
      const double b0 = have ? p2 : VT[c], b1 = have ? p3 : VT[c + N1];
      xf0 = a0 + (a0 - UT[c - P]) * bot_ratio;
      xf1 = a1 + (a1 - UT[c - P + 1]) * bot_ratio;
      yf0 = b0 + (b0 - VT[c - P]) * bot_ratio;
      yf1 = b1 + (b1 - VT[c - P + N1]) * bot_ratio;
    } else {
      const double int_ratio = 1.0 / (dp0[k - 1] + dp0[k]);
      const long c = (long)k * P;
      if (!have) {
        p0 = UT[c - P]; p1 = UT[c - P + 1]; p2 = VT[c - P]; p3 = VT[c - P + N1];
      }
      const double a0 = UT[c], a1 = UT[c + 1], b0 = VT[c], b1 = VT[c + N1];
      xf0 = (dp0[k] * p0 + dp0[k - 1] * a0) * int_ratio;
      xf1 = (dp0[k] * p1 + dp0[k - 1] * a1) * int_ratio;
      yf0 = (dp0[k] * p2 + dp0[k - 1] * b0) * int_ratio;
      yf1 = (dp0[k] * p3 + dp0[k - 1] * b1) * int_ratio;
      p0 = a0; p1 = a1; p2 = b0; p3 = b1;
      have = true;
    }
    const double fx0 = xf0 * (xf0 > 0.0 ? gW : gCX);
    const double fx1 = xf1 * (xf1 > 0.0 ? gCX : gE);
    const double fy0 = yf0 * (yf0 > 0.0 ? gS : gCY);
    const double fy1 = yf1 * (yf1 > 0.0 ? gCY : gN);
    const double gc = gCY;
    gzo[((long)s * (npz + 1) + k) * P + o] = (gc * area + fx0 - fx1 + fy0 - fy1) / (area + xf0 - xf1 + yf0 - yf1);
  }
}

__global__ void __launch_bounds__(256) pgradc_kl(Dims d, const SubInfo* __restrict__ subs, const double* __restrict__ M,
                                                 int npz, int nkb, int klb, double dt2, const double* __restrict__ delpc,
                                                 const double* __restrict__ pkc, const double* __restrict__ gz,
                                                 double* __restrict__ uc, double* __restrict__ vc) {
  Launch2D L{0, 0, d.nx + 1, d.ny + 1};
  KLSETUP(npz)
  (void)subs;
  const bool du = j < d.ny, dv = i < d.nx;
  const long W = -1, S = -d.pitch;
  const double rdxc = du ? met(M, d, M_RDXC, s)[o] : 0.0, rdyc = dv ? met(M, d, M_RDYC, s)[o] : 0.0;
  const double* PK = pkc + (long)s * (npz + 1) * P + o;  // interface k: PK[k * P]
  const double* GZ = gz + (long)s * (npz + 1) * P + o;
  // interface k values at o, o-1 (w) and o-pitch (s)
  long l0 = (long)k0 * P;
  double pk0 = PK[l0], gz0 = GZ[l0];
  double pk0w = du ? PK[l0 + W] : 0.0, gz0w = du ? GZ[l0 + W] : 0.0;
  double pk0s = dv ? PK[l0 + S] : 0.0, gz0s = dv ? GZ[l0 + S] : 0.0;
  // loads first: both directions' inputs of a level in one group (the west / south offsets 0
  // on the row / column that takes no update)
  const long Wd = du ? W : 0, Sd = dv ? S : 0;
  for (int k = k0; k < k1; ++k) {
    const long l1 = (long)(k + 1) * P, lk = ((long)s * npz + k) * P + o;
    const double pk1 = PK[l1], gz1 = GZ[l1];
    const double pk1w = PK[l1 + Wd], gz1w = GZ[l1 + Wd], pk1s = PK[l1 + Sd], gz1s = GZ[l1 + Sd];
    const double dcw = delpc[lk + Wd], dc = delpc[lk], dcs = delpc[lk + Sd], u0 = uc[lk], v0 = vc[lk];
    if (du) {
      const double wsum = dcw + dc;
      uc[lk] = u0 + dt2 * rdxc / wsum * ((gz1w - gz0) * (pk1 - pk0w) + (gz0w - gz1) * (pk1w - pk0));
    }
    if (dv) {
      const double wsum = dcs + dc;
      vc[lk] = v0 + dt2 * rdyc / wsum * ((gz1s - gz0) * (pk1 - pk0s) + (gz0s - gz1) * (pk1s - pk0));
    }
    pk0 = pk1; gz0 = gz1; pk0w = pk1w; gz0w = gz1w; pk0s = pk1s; gz0s = gz1s;
  }
}

__global__ void __launch_bounds__(256) nhpgrad_kl(Dims d, const SubInfo* __restrict__ subs, const double* __restrict__ M,
                                                  int npz, int nkb, int klb, double dt, double ptk,
                                                  const double* __restrict__ ppb, const double* __restrict__ gzb,
                                                  const double* __restrict__ pkb, const double* __restrict__ wk1,
                                                  double* __restrict__ u, double* __restrict__ v) {
  Launch2D L{0, 0, d.nx + 1, d.ny + 1};
  KLSETUP(npz)
  (void)subs;
  const bool du = i < d.nx, dv = j < d.ny;
  const long E = 1, Nn = d.pitch;
  const double rdx = du ? met(M, d, M_RDX, s)[o] : 0.0, rdy = dv ? met(M, d, M_RDY, s)[o] : 0.0;
  const double* PP = ppb + (long)s * (npz + 1) * P + o;
  const double* GZ = gzb + (long)s * (npz + 1) * P + o;
  const double* PK = pkb + (long)s * (npz + 1) * P + o;
  // interface k values at o, o+1 (e) and o+pitch (n); level-0 pp / pk are the model-top constants
  const long l0 = (long)k0 * P;
  const bool top = k0 == 0;
  double pk0 = top ? ptk : PK[l0], pp0 = top ? 0.0 : PP[l0], gz0 = GZ[l0];
  double pk0e = 0.0, pp0e = 0.0, gz0e = 0.0, pk0n = 0.0, pp0n = 0.0, gz0n = 0.0;
  if (du) {
    pk0e = top ? ptk : PK[l0 + E];
    pp0e = top ? 0.0 : PP[l0 + E];
    gz0e = GZ[l0 + E];
  }
  if (dv) {
    pk0n = top ? ptk : PK[l0 + Nn];
    pp0n = top ? 0.0 : PP[l0 + Nn];
    gz0n = GZ[l0 + Nn];
  }
  // loads first: both directions' inputs of a level in one group (the east / north offsets 0
  // on the column / row that takes no update)
  const long Ed = du ? E : 0, Nd = dv ? Nn : 0;
  for (int k = k0; k < k1; ++k) {
    const long l1 = (long)(k + 1) * P, lk = ((long)s * npz + k) * P + o;
    const double pk1 = PK[l1], pp1 = PP[l1], gz1 = GZ[l1];
    const double pk1e = PK[l1 + Ed], pp1e = PP[l1 + Ed], gz1e = GZ[l1 + Ed];
    const double pk1n = PK[l1 + Nd], pp1n = PP[l1 + Nd], gz1n = GZ[l1 + Nd];
    const double u0 = u[lk], v0 = v[lk], w0 = wk1[lk], we = wk1[lk + Ed], wn = wk1[lk + Nd];
    if (du) {
      const double wk0 = pk1 - pk0, wke = pk1e - pk0e;
      const double du1 = dt / (wk0 + wke) * ((gz1 - gz0e) * (pk1e - pk0) + (gz0 - gz1e) * (pk1 - pk0e));
      u[lk] = (u0 + du1 + dt / (w0 + we) * ((gz1 - gz0e) * (pp1e - pp0) + (gz0 - gz1e) * (pp1 - pp0e))) * rdx;
    }
    if (dv) {
      const double wk0 = pk1 - pk0, wke = pk1n - pk0n;
      const double dv1 = dt / (wk0 + wke) * ((gz1 - gz0n) * (pk1n - pk0) + (gz0 - gz1n) * (pk1 - pk0n));
      v[lk] = (v0 + dv1 + dt / (w0 + wn) * ((gz1 - gz0n) * (pp1n - pp0) + (gz0 - gz1n) * (pp1 - pp0n))) * rdy;
    }
    pk0 = pk1; pp0 = pp1; gz0 = gz1;
    pk0e = pk1e; pp0e = pp1e; gz0e = gz1e;
    pk0n = pk1n; pp0n = pp1n; gz0n = gz1n;
  }
}

__global__ void scale_k(long n, double a, const double* __restrict__ x, double* __restrict__ y) {
  long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long stride = (long)gridDim.x * blockDim.x;
  for (; t < n; t += stride) y[t] = a * x[t];
}

inline dim3 g2(const Dims& d, const Launch2D& L, int nz) {
  (void)d;
  return plane_grid(L, nz);
}
// launch grid of a kernel whose setup is KSETUP2 (level-interleaved blocks)
inline dim3 g2lv(const Launch2D& L, int nz) { return plane_grid_lv(L, nz); }

}  // namespace

void update_dz_c(const Ctx& c, int npz, const double* dp0, const double* ut, const double* vt, const double* gz,
                 double* gz_out) {
  const Dims& d = c.d;
  Launch2D L{-1, -1, d.nx + 2, d.ny + 2};
  if (const int klb = kloop_levels()) {
    const int nkb = (npz + 1 + klb - 1) / klb;
    GT_LAUNCH_N("udzc_kl", udzc_kl, kloop_grid(L, d.nsub, nkb), dim3(BX, BY), 0, c.st, d, c.subs, c.met, npz,
                  nkb, klb, dp0, ut, vt, gz, gz_out);
  } else {
    GT_LAUNCH(udzc_k, g2lv(L, d.nsub * (npz + 1)), dim3(BX, BY), 0, c.st, d, c.subs, c.met, npz, dp0, ut, vt,
                       gz, gz_out);
  }
  HIP_LAUNCH_CHECK();
  const Ext e = ext(d);
  gt_bytes(npz * (e.X + e.Y) + (npz + 1) * 2 * e.C + 3 * e.C);
}

void p_grad_c(const Ctx& c, int npz, double dt2, const double* delpc, const double* pkc, const double* gz, double* uc,
              double* vc) {
  const Dims& d = c.d;
  Launch2D L{0, 0, d.nx + 1, d.ny + 1};
  if (const int klb = kloop_levels()) {
    const int nkb = (npz + klb - 1) / klb;
    GT_LAUNCH_N("pgradc_kl", pgradc_kl, kloop_grid(L, d.nsub, nkb), dim3(BX, BY), 0, c.st, d, c.subs, c.met,
                  npz, nkb, klb, dt2, delpc, pkc, gz, uc, vc);
  } else {
    GT_LAUNCH(pgradc_k, g2lv(L, d.nsub * npz), dim3(BX, BY), 0, c.st, d, c.subs, c.met, npz, dt2, delpc, pkc,
                       gz, uc, vc);
  }
  HIP_LAUNCH_CHECK();
  const Ext e = ext(d);
  gt_bytes(npz * (e.C + 2 * e.X + 2 * e.Y) + (npz + 1) * 2 * e.C + 2 * e.C);
}

void edge_profile(const Ctx& c, int npz, const double* dp0, const double* crx, const double* xfx, const double* cry,
                  const double* yfx, double* crx_e, double* xfx_e, double* cry_e, double* yfx_e, int variant) {
  const Dims& d = c.d;
  Launch2D Lf{-NG, -NG, d.nx + 2 * NG + 1, d.ny + 2 * NG + 1};
  if (npz > EP_KMAX || npz < 2) throw std::runtime_error("edge_profile: 2 <= npz <= 256 required");
  if (variant != 1 && npz >= 3 && npz <= 32)
    GT_LAUNCH(edge_prof_reg_k<32>, g2(d, Lf, 4 * d.nsub), dim3(BX, BY), 0, c.st, d, npz, dp0, crx, xfx, cry, yfx,
              crx_e, xfx_e, cry_e, yfx_e);
  else if (variant != 1 && npz >= 3 && npz <= 80)
    GT_LAUNCH(edge_prof_reg_k<80>, g2(d, Lf, 4 * d.nsub), dim3(BX, BY), 0, c.st, d, npz, dp0, crx, xfx, cry, yfx,
              crx_e, xfx_e, cry_e, yfx_e);
  else if (variant != 1 && npz >= 3 && npz <= 144)
    GT_LAUNCH(edge_prof_reg_k<144>, g2(d, Lf, 4 * d.nsub), dim3(BX, BY), 0, c.st, d, npz, dp0, crx, xfx, cry, yfx,
              crx_e, xfx_e, cry_e, yfx_e);
  else
    GT_LAUNCH(edge_prof_k, g2(d, Lf, d.nsub), dim3(BX, BY), 0, c.st, d, npz, dp0, crx, xfx, cry, yfx, crx_e,
              xfx_e, cry_e, yfx_e);
  HIP_LAUNCH_CHECK();
  const Ext e = ext(d);
  gt_bytes((2.0 * npz + 1) * (2 * e.X + 2 * e.Y));
}

void update_dz_d(const Ctx& c, const UdzdArgs& a) {
  const Dims& d = c.d;
  const int k1 = a.npz + 1;
  edge_profile(c, a.npz, a.dp0, a.crx, a.xfx, a.cry, a.yfx, a.crx_e, a.xfx_e, a.cry_e, a.yfx_e, 0);
  TpArgs t{};
  t.q = a.zh; t.nt = 1; t.nk = k1;
  t.crx = a.crx_e; t.cry = a.cry_e; t.xfx = a.xfx_e; t.yfx = a.yfx_e;
  t.mfx = nullptr; t.mfy = nullptr; t.ord = a.hord;
  // the flux-form height update inside the march (tp.hip TM = 4, zh_update's expressions and
  // order): no flux planes; the new heights go to zh_out
  t.zh_out = a.zh_out;
  fv_tp_2d(c, t);
  (void)d;
  if (!a.hlv) return;
  // the heights' del-n damping from the old heights (their halo filled), added to the new ones
  // before riem_solver3's dz_min clamp (FV3 update_dz_d: one expression, transport + damping)
  level_runs(a.hlv, k1, [](const LevelDamp& l) { return l.vt4 > 0.0 ? l.nord_v : -1; },
             [&](int k0, int nk, int nord) {
               deln_fluxes(c, k1, k0, nk, nord, a.lv, DL_VT4, a.zh, a.d2, a.fx2, a.fy2);
               deln_div_add(c, k1, k0, nk, a.fx2, a.fy2, a.zh_out);
             });
}

void pk3_pe_halo(const Ctx& c, int npz, double ptop, bool do_pe, const double* delp, double* pk3, double* pe) {
  const Dims& d = c.d;
  const int nring = 4 * (d.nx + 4) + 4 * d.ny;
  const int nb = (npz + PK_B - 1) / PK_B;
  GT_LAUNCH(pk3_pe_halo_k, dim3(cdiv(nring * nb, 64), d.nsub), dim3(64), 0, c.st, d, npz, ptop, do_pe ? 1 : 0, delp,
            pk3, pe);
  HIP_LAUNCH_CHECK();
  gt_bytes((double)d.nsub * npz * (4.0 * (d.nx + 2) + 4.0 * d.ny) * (do_pe ? 3 : 2));  // halo ring only
}

void a2b_ord4_multi(const Ctx& c, int nf, const int* nk, const double* const* q, double* const* qout,
                    const double* scale) {
  const Dims& d = c.d;
  if (nf < 1 || nf > A2B_MAXF) throw std::runtime_error("a2b_ord4: 1..4 fields per launch");
  A2bF F{};
  long nz = 0, lev = 0;
  for (int f = 0; f < A2B_MAXF; ++f) {
    F.zb[f] = f < nf ? (int)nz : INT_MAX;
    if (f < nf) {
      if (nk[f] < 1 || !q[f] || !qout[f]) throw std::runtime_error("a2b_ord4: bad field");
      F.q[f] = q[f];
      F.qo[f] = qout[f];
      F.nk[f] = nk[f];
      F.sc[f] = scale ? scale[f] : 1.0;
      nz += (long)d.nsub * nk[f];
      lev += nk[f];
    } else {
      F.q[f] = q[0];
      F.qo[f] = qout[0];
      F.nk[f] = 1;
      F.sc[f] = 1.0;
    }
  }
  F.zb[A2B_MAXF] = INT_MAX;
  if (nz >= 65536) throw std::runtime_error("a2b_ord4: too many planes for one launch");
  // corner / tile-edge values first: the interior points next to the tile edges use them
  // (GTFV3_A2B_EDGE=0: the one-point-per-lane form, read per call)
  const char* ee = std::getenv("GTFV3_A2B_EDGE");
  // (the position next to a line's far end reads two positions back: not across a block start)
  auto end_ok = [](int len) { return len - 2 < AE_T || (len - 2) % AE_T >= 2; };
  if ((ee && ee[0] == '0') || !end_ok(d.nx + 1) || !end_ok(d.ny + 1)) {
    GT_LAUNCH(a2b_edge_k, dim3(cdiv(edge_line_count(0, d.nx, 0, d.ny), 256), 1, (unsigned)nz), dim3(256), 0, c.st,
              d, c.subs, c.met, F, c.cornerw);
  } else {
    GT_LAUNCH_N("a2b_edge_k", a2b_edge2_k, dim3(cdiv(std::max(d.nx, d.ny) + 1, AE_T), 4, (unsigned)nz), dim3(AE_T), 0,
                c.st, d, c.subs, c.met, F, c.cornerw);
  }
  HIP_LAUNCH_CHECK();
  // interior corners: column-marching kernel (balanced segments of at most 46 corner
  // rows: C180 has 181 corner rows -> 4 x 46, not 4 x 45 + 1)
  // (more, shorter segments, down to 15 rows, when the launch would have fewer than ~6900
  // waves: small sub-domains on 4-8 GPUs)
  A2bM m{d, c.subs, c.met, F, (int)nz, (int)cdiv(d.nx + 1, AM_OUT), 0, 0};
  {
    const long want = cdiv(6912, nz * m.nstrip);
    m.nseg = (int)std::max<long>(cdiv(d.ny + 1, 46), std::min<long>(cdiv(d.ny + 1, 15), want));
  }
  m.seg = (int)cdiv(d.ny + 1, m.nseg);
  const long waves = (long)m.nz * m.nstrip * m.nseg;
  GT_LAUNCH(a2b_march_k, dim3(xcd_pad(cdiv(waves, AM_WAVES))), dim3(AM_W * AM_WAVES), 0, c.st, m);
  HIP_LAUNCH_CHECK();
  const Ext e = ext(d);
  gt_bytes(lev * (e.C + e.K));  // q (cells) read, qout (corners) written
}

void a2b_ord4(const Ctx& c, int nk, const double* q, double* qout, double* qx, double* qy) {
  (void)qx;
  (void)qy;
  a2b_ord4_multi(c, 1, &nk, &q, &qout);
}

void nh_p_grad(const Ctx& c, const NhPgArgs& a) {
  const Dims& d = c.d;
  const int k1 = a.npz + 1;
  {
    const int nk[4] = {k1, k1, k1, a.npz};
    const double* q[4] = {a.pp, a.pk3, a.gz, a.delp};
    double* qo[4] = {a.ppb, a.pkb, a.gzb, a.wk1};
    const double sc[4] = {1.0, 1.0, a.gz_scale, 1.0};
    a2b_ord4_multi(c, 4, nk, q, qo, sc);
  }
  const double ptk = exp(Constants::kappa * log(a.ptop));
  Launch2D L{0, 0, d.nx + 1, d.ny + 1};
  if (const int klb = kloop_levels()) {
    const int nkb = (a.npz + klb - 1) / klb;
    GT_LAUNCH_N("nhpgrad_kl", nhpgrad_kl, kloop_grid(L, d.nsub, nkb), dim3(BX, BY), 0, c.st, d, c.subs,
                  c.met, a.npz, nkb, klb, a.dt, ptk, a.ppb, a.gzb, a.pkb, a.wk1, a.u, a.v);
  } else {
    GT_LAUNCH(nhpgrad_k, g2lv(L, d.nsub * a.npz), dim3(BX, BY), 0, c.st, d, c.subs, c.met, a.npz, a.dt, ptk,
                       a.ppb, a.gzb, a.pkb, a.wk1, a.u, a.v);
  }
  HIP_LAUNCH_CHECK();
  const Ext e = ext(d);
  gt_bytes(k1 * 3 * e.K + a.npz * (e.K + 2 * e.X + 2 * e.Y) + 2 * e.C);
}

void scale_field(const Ctx& c, long n, double a, const double* x, double* y) {
  GT_LAUNCH(scale_k, dim3(cdiv(n, 256) < 8192 ? cdiv(n, 256) : 8192), dim3(256), 0, c.st, n, a, x, y);
  HIP_LAUNCH_CHECK();
  gt_bytes(2.0 * n);
}

}  // namespace gtfv3
