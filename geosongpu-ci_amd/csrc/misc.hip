// misc.hip — pointwise pieces of fv_dynamics on gfx950: entry conversion to
// virtual potential temperature + pkz, zh from delz, exit conversion (T, omega),
// cubed_to_latlon (c2l_ord4) and the Held & Suarez (1994) forcing of GEOShs.
#include <algorithm>
#include <cstdlib>

#include "kernels_misc.hpp"
#include "stencil_common.hpp"

namespace gtfv3 {
namespace {

constexpr double GRAV = Constants::grav;
constexpr double RDGAS = Constants::rdgas;
constexpr double KAPPA = Constants::kappa;

#define KSETUP3(nk_)                                                 \
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

// fv_dynamics entry: pkz from the non-hydrostatic state, pt -> virtual potential temperature
__global__ void __launch_bounds__(256) prep_k(Dims d, const SubInfo* __restrict__ subs, int npz, int nq, double zvir,
                                              const double* __restrict__ delp, const double* __restrict__ delz,
                                              const double* __restrict__ q, double* __restrict__ pt,
                                              double* __restrict__ pkz) {
  Launch2D L{0, 0, d.nx, d.ny};
  KSETUP3(npz)
  const int k = z % npz;
  const double rdg = -RDGAS * (1.0 / GRAV);
  const double qv = q[((long)s * nq * npz + k) * d.plane + o];  // tracer 0 = specific humidity
  const double dp1 = zvir * qv;
  double pk = exp(KAPPA * log(rdg * AT(delp, 0, 0) * AT(pt, 0, 0) * (1.0 + dp1) / AT(delz, 0, 0)));
  AT(pkz, 0, 0) = pk;
  AT(pt, 0, 0) = AT(pt, 0, 0) * (1.0 + dp1) / pk;
}

// zh (interface heights) from delz and the surface height
__global__ void __launch_bounds__(256) zh_init_k(Dims d, int npz, const double* __restrict__ phis,
                                                 const double* __restrict__ delz, double* __restrict__ zh) {
  Launch2D L{0, 0, d.nx, d.ny};
  int i, j;
  if (!thread_point(L, i, j)) return;
  const int s = blockIdx.z;
  const long o = pidx(d, i, j);
  double* Z = zh + (long)s * (npz + 1) * d.plane + o;
  const double* DZ = delz + (long)s * npz * d.plane + o;
  double zc = phis[(long)s * d.plane + o] * (1.0 / GRAV);
  Z[(long)npz * d.plane] = zc;
  for (int k = npz - 1; k >= 0; --k) {
    zc = zc - DZ[(long)k * d.plane];
    Z[(long)k * d.plane] = zc;
  }
}

// fv_dynamics exit: T_v -> T and omega from w
__global__ void __launch_bounds__(256) wrapup_k(Dims d, const SubInfo* __restrict__ subs, int npz, int nq, double zvir,
                                                const double* __restrict__ q, const double* __restrict__ delp,
                                                const double* __restrict__ delz, const double* __restrict__ w,
                                                double* __restrict__ pt, double* __restrict__ omga) {
  Launch2D L{0, 0, d.nx, d.ny};
  KSETUP3(npz)
  const int k = z % npz;
  const double qv = q[((long)s * nq * npz + k) * d.plane + o];
  AT(pt, 0, 0) = AT(pt, 0, 0) / (1.0 + zvir * qv);
  AT(omga, 0, 0) = AT(delp, 0, 0) / AT(delz, 0, 0) * AT(w, 0, 0);
}

// cubed_to_latlon: c2l_ord4 (4-point Lagrange in the interior, 2nd order at tile edges)
__global__ void __launch_bounds__(256) c2l_k(Dims d, const SubInfo* __restrict__ subs, const double* __restrict__ M,
                                             int npz, const double* __restrict__ u, const double* __restrict__ v,
                                             double* __restrict__ ua, double* __restrict__ va) {
  Launch2D L{0, 0, d.nx, d.ny};
  KSETUP3(npz)
  const double C1 = 1.125, C2 = -0.125;
  const double* dx = MT(M_DX);
  const double* dy = MT(M_DY);
  double ut = C2 * (AT(u, 0, -1) + AT(u, 0, 2)) + C1 * (AT(u, 0, 0) + AT(u, 0, 1));
  double vt = C2 * (AT(v, -1, 0) + AT(v, 2, 0)) + C1 * (AT(v, 0, 0) + AT(v, 1, 0));
  if (J == 0 || J == N - 1) {
    vt = 2.0 * (AT(v, 0, 0) * MA(dy, 0, 0) + AT(v, 1, 0) * MA(dy, 1, 0)) / (MA(dy, 0, 0) + MA(dy, 1, 0));
    ut = 2.0 * (AT(u, 0, 0) * MA(dx, 0, 0) + AT(u, 0, 1) * MA(dx, 0, 1)) / (MA(dx, 0, 0) + MA(dx, 0, 1));
  }
  if (I == 0 || I == N - 1) {
    ut = 2.0 * (AT(u, 0, 0) * MA(dx, 0, 0) + AT(u, 0, 1) * MA(dx, 0, 1)) / (MA(dx, 0, 0) + MA(dx, 0, 1));
    vt = 2.0 * (AT(v, 0, 0) * MA(dy, 0, 0) + AT(v, 1, 0) * MA(dy, 1, 0)) / (MA(dy, 0, 0) + MA(dy, 1, 0));
  }
  AT(ua, 0, 0) = MA(MT(M_A11), 0, 0) * ut + MA(MT(M_A12), 0, 0) * vt;
  AT(va, 0, 0) = MA(MT(M_A21), 0, 0) * ut + MA(MT(M_A22), 0, 0) * vt;
}

// Held & Suarez (1994) forcing, implicit in time: Newtonian cooling of T towards
// T_eq(lat, p) and Rayleigh friction of the D-grid winds in the boundary layer.
__global__ void __launch_bounds__(256) hs_k(Dims d, const SubInfo* __restrict__ subs, const double* __restrict__ M,
                                            int npz, double dt, const double* __restrict__ pe,
                                            double* __restrict__ pt, double* __restrict__ u, double* __restrict__ v) {
  Launch2D L{0, 0, d.nx + 1, d.ny + 1};
  KSETUP3(npz)
  const int k = z % npz;
  const double p0 = 1.0e5, sigb = 0.7;
  const double ka = 1.0 / (40.0 * 86400.0), ks = 1.0 / (4.0 * 86400.0), kf = 1.0 / 86400.0;
  const double dty = 60.0, dthz = 10.0;
  const long e0 = ((long)s * (npz + 1) + k) * d.plane;
  const long e1 = e0 + d.plane;
  const long es = ((long)s * (npz + 1) + npz) * d.plane;
  auto sigma = [&](long off) { return 0.5 * (pe[e0 + off] + pe[e1 + off]) / pe[es + off]; };
  if (i < d.nx && j < d.ny) {
    const double lat = MA(MT(M_LAT), 0, 0);
    const double sl = sin(lat), cl = cos(lat);
    const double pm = 0.5 * (pe[e0 + o] + pe[e1 + o]);
    const double sg = pm / pe[es + o];
    const double teq = fmax(200.0, (315.0 - dty * sl * sl - dthz * log(pm / p0) * cl * cl) * exp(KAPPA * log(pm / p0)));
    const double kt = ka + (ks - ka) * fmax(0.0, (sg - sigb) / (1.0 - sigb)) * cl * cl * cl * cl;
    AT(pt, 0, 0) = (AT(pt, 0, 0) + dt * kt * teq) / (1.0 + dt * kt);
  }
  if (i < d.nx) {  // u on x-edges: sigma averaged over the two adjacent cells
    const double sg = 0.5 * (sigma(o) + sigma(o - d.pitch));
    const double kv = kf * fmax(0.0, (sg - sigb) / (1.0 - sigb));
    AT(u, 0, 0) = AT(u, 0, 0) / (1.0 + dt * kv);
  }
  if (j < d.ny) {
    const double sg = 0.5 * (sigma(o) + sigma(o - 1));
    const double kv = kf * fmax(0.0, (sg - sigb) / (1.0 - sigb));
    AT(v, 0, 0) = AT(v, 0, 0) / (1.0 + dt * kv);
  }
}

__global__ void fill_k(long n, double a, double* __restrict__ x) {
  long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long stride = (long)gridDim.x * blockDim.x;
  for (; t < n; t += stride) x[t] = a;
}

__global__ void max_k(long n, const double* __restrict__ x, double* __restrict__ y) {
  long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long stride = (long)gridDim.x * blockDim.x;
  for (; t < n; t += stride) y[t] = fmax(y[t], x[t]);
}

// the halo ring [-NG, n+NG) x [-NG, n+NG) minus the compute domain, src -> dst, per plane: one
// lane per ring point (the NG rows above, the NG rows below, then the 2 NG side points of each
// compute row), planes strided over grid y -- a launch over whole planes would schedule ~30x
// the lanes for the 3 % of each plane that the ring is
__global__ void __launch_bounds__(256) copy_ring_k(Dims d, long nplanes, const double* __restrict__ src,
                                                   double* __restrict__ dst) {
  const int W = d.nx + 2 * NG;
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= 2 * NG * W + 2 * NG * d.ny) return;
  int i, j;
  if (t < 2 * NG * W) {
    const int r = t / W;
    i = t - r * W - NG;
    j = r < NG ? r - NG : d.ny + r - NG;
  } else {
    const int s = t - 2 * NG * W, c = s % (2 * NG);
    j = s / (2 * NG);
    i = c < NG ? c - NG : d.nx + c - NG;
  }
  const long o = pidx(d, i, j);
  for (long p = blockIdx.y; p < nplanes; p += gridDim.y) dst[p * d.plane + o] = src[p * d.plane + o];
}

// global tracer diagnostics (FV3 fv_diagnostics prt_mass / g_sum): one block per (sub-domain,
// tracer, level) plane reduces sum(q * delp * area), min q, max q and the count of non-finite
// q over the compute domain into part[(iq * nsub + s) * npz + k][4]
__global__ void __launch_bounds__(256) tracer_stats_k(Dims d, const double* __restrict__ M, int npz, int nq,
                                                      const double* __restrict__ q, const double* __restrict__ delp,
                                                      double* __restrict__ part) {
  __shared__ double red[4][256];
  const int z = blockIdx.x;
  const int s = z / (nq * npz), r = z - s * nq * npz, iq = r / npz, k = r - iq * npz;
  const double* Q = q + (long)z * d.plane;
  const double* DP = delp + ((long)s * npz + k) * d.plane;
  const double* A = met(M, d, M_AREA, s);
  double sm = 0.0, mn = 1.0e300, mx = -1.0e300, bad = 0.0;
  for (int t = threadIdx.x; t < d.nx * d.ny; t += 256) {
    const int j = t / d.nx, i = t - j * d.nx;
    const long o = pidx(d, i, j);
    const double v = Q[o];
    if (!isfinite(v)) {
      bad += 1.0;
      continue;
    }
    sm += v * DP[o] * A[o];
    mn = fmin(mn, v);
    mx = fmax(mx, v);
  }
  red[0][threadIdx.x] = sm;
  red[1][threadIdx.x] = mn;
  red[2][threadIdx.x] = mx;
  red[3][threadIdx.x] = bad;
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h) {
      red[0][threadIdx.x] += red[0][threadIdx.x + h];
      red[1][threadIdx.x] = fmin(red[1][threadIdx.x], red[1][threadIdx.x + h]);
      red[2][threadIdx.x] = fmax(red[2][threadIdx.x], red[2][threadIdx.x + h]);
      red[3][threadIdx.x] += red[3][threadIdx.x + h];
    }
    __syncthreads();
  }
  if (threadIdx.x < 4) {
    const int nsub = gridDim.x / (nq * npz);
    part[(((long)iq * nsub + s) * npz + k) * 4 + threadIdx.x] = red[threadIdx.x][0];
  }
}

// per tracer, in a fixed order over the (sub-domain, level) partials: out[iq][4]
__global__ void tracer_stats_fin_k(int nq, int nper, const double* __restrict__ part, double* __restrict__ out) {
  const int iq = blockIdx.x * blockDim.x + threadIdx.x;
  if (iq >= nq) return;
  const double* P = part + (long)iq * nper * 4;
  double sm = 0.0, mn = 1.0e300, mx = -1.0e300, bad = 0.0;
  for (int n = 0; n < nper; ++n) {
    sm += P[4 * n];
    mn = fmin(mn, P[4 * n + 1]);
    mx = fmax(mx, P[4 * n + 2]);
    bad += P[4 * n + 3];
  }
  out[4 * iq] = sm;
  out[4 * iq + 1] = mn;
  out[4 * iq + 2] = mx;
  out[4 * iq + 3] = bad;
}

inline dim3 g2(const Dims& d, const Launch2D& L, int nz) {
  (void)d;
  return plane_grid(L, nz);
}
// launch grid of a kernel whose setup is KSETUP3 (level-interleaved blocks)
inline dim3 g2lv(const Launch2D& L, int nz) { return plane_grid_lv(L, nz); }

}  // namespace

bool level_blocks_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("GTFV3_LVB");
    return !(e && e[0] == '0');
  }();
  return on;
}

// levels per thread of the level-loop forms (read per launch: tests switch it within one
// process).  Default 8: C180 L72 on one MI355X, ms per step one level / 8 / 18 per thread:
// udzc 1.10 / 0.70 / 0.70, p_grad_c 1.30 / 1.02 / 1.07, nh_p_grad 1.61 / 1.32 / 1.30, ds_utvt1
// 0.95 / 0.88 / 0.95 (profiles/r03e_*)
int kloop_levels() {
  const char* e = std::getenv("GTFV3_KLOOP");
  return e ? std::max(0, atoi(e)) : 8;
}

bool xcd_order_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("GTFV3_XCD");
    return !(e && e[0] == '0');
  }();
  return on;
}

void fv_prep(const Ctx& c, int npz, int nq, double zvir, const double* delp, const double* delz, const double* q, double* pt,
             double* pkz) {
  const Dims& d = c.d;
  Launch2D L{0, 0, d.nx, d.ny};
  GT_LAUNCH(prep_k, g2lv(L, d.nsub * npz), dim3(BX, BY), 0, c.st, d, c.subs, npz, nq, zvir, delp, delz, q,
                     pt, pkz);
  HIP_LAUNCH_CHECK();
  gt_bytes(npz * 6 * ext(d).C);
}

void zh_init(const Ctx& c, int npz, const double* phis, const double* delz, double* zh) {
  const Dims& d = c.d;
  Launch2D L{0, 0, d.nx, d.ny};
  GT_LAUNCH(zh_init_k, g2(d, L, d.nsub), dim3(BX, BY), 0, c.st, d, npz, phis, delz, zh);
  HIP_LAUNCH_CHECK();
  gt_bytes((2.0 * npz + 2) * ext(d).C);
}

void fv_wrapup(const Ctx& c, int npz, int nq, double zvir, const double* q, const double* delp, const double* delz,
               const double* w, double* pt, double* omga) {
  const Dims& d = c.d;
  Launch2D L{0, 0, d.nx, d.ny};
  GT_LAUNCH(wrapup_k, g2lv(L, d.nsub * npz), dim3(BX, BY), 0, c.st, d, c.subs, npz, nq, zvir, q, delp, delz,
                     w, pt, omga);
  HIP_LAUNCH_CHECK();
  gt_bytes(npz * 7 * ext(d).C);
}

void c2l_ord4(const Ctx& c, int npz, const double* u, const double* v, double* ua, double* va) {
  const Dims& d = c.d;
  Launch2D L{0, 0, d.nx, d.ny};
  GT_LAUNCH(c2l_k, g2lv(L, d.nsub * npz), dim3(BX, BY), 0, c.st, d, c.subs, c.met, npz, u, v, ua, va);
  HIP_LAUNCH_CHECK();
  const Ext e = ext(d);
  gt_bytes(npz * (e.X + e.Y + 2 * e.C) + 8 * e.C);
}

void held_suarez(const Ctx& c, int npz, double dt, const double* pe, double* pt, double* u, double* v) {
  const Dims& d = c.d;
  Launch2D L{0, 0, d.nx + 1, d.ny + 1};
  GT_LAUNCH(hs_k, g2lv(L, d.nsub * npz), dim3(BX, BY), 0, c.st, d, c.subs, c.met, npz, dt, pe, pt, u, v);
  HIP_LAUNCH_CHECK();
  const Ext e = ext(d);
  gt_bytes((npz + 1) * e.C + npz * (2 * e.C + 2 * e.X + 2 * e.Y) + 2 * e.C);
}

void copy_halo_ring(const Ctx& c, int nplanes, const double* src, double* dst) {
  const Dims& d = c.d;
  if (nplanes <= 0) return;
  const int ring = 2 * NG * (d.nx + 2 * NG) + 2 * NG * d.ny;
  const dim3 grid((unsigned)cdiv(ring, 256), (unsigned)std::min(nplanes, 32768));
  GT_LAUNCH(copy_ring_k, grid, dim3(256), 0, c.st, d, (long)nplanes, src, dst);
  HIP_LAUNCH_CHECK();
  gt_bytes(2.0 * nplanes * ((d.nx + 2.0 * NG) * (d.ny + 2.0 * NG) - (double)d.nx * d.ny));
}

void tracer_stats(const Ctx& c, int npz, int nq, const double* q, const double* delp, double* part, double* out) {
  const Dims& d = c.d;
  GT_LAUNCH(tracer_stats_k, dim3((unsigned)(d.nsub * nq * npz)), dim3(256), 0, c.st, d, c.met, npz, nq, q, delp, part);
  HIP_LAUNCH_CHECK();
  gt_bytes((nq + 1.0) * npz * ext(d).C + ext(d).C);
  GT_LAUNCH(tracer_stats_fin_k, dim3(cdiv(nq, 64)), dim3(64), 0, c.st, nq, d.nsub * npz, part, out);
  HIP_LAUNCH_CHECK();
}

void fill_field(const Ctx& c, long n, double a, double* x) {
  GT_LAUNCH(fill_k, dim3(cdiv(n, 256) < 8192 ? cdiv(n, 256) : 8192), dim3(256), 0, c.st, n, a, x);
  HIP_LAUNCH_CHECK();
  gt_bytes((double)n);
}

void max_field(const Ctx& c, long n, const double* x, double* y) {
  GT_LAUNCH(max_k, dim3(cdiv(n, 256) < 8192 ? cdiv(n, 256) : 8192), dim3(256), 0, c.st, n, x, y);
  HIP_LAUNCH_CHECK();
  gt_bytes(3.0 * n);
}

}  // namespace gtfv3
