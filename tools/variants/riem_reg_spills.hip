// riem.hip — riem_solver_c / riem_solver3 (FV3 nh_utils SIM1 semi-implicit vertical
// acoustic solve, a_imp = 1) for gfx950.
//
// The column recurrences (tridiagonal eliminations, prefix sums) are cheap arithmetic;
// the expensive part is the fp64 log/exp of every level (log p at interfaces, the
// pressure of the gas law pl = (-dm/dz R pt)^gamma, p^kappa), which does NOT depend on
// the recurrences.  Inside a column sweep those transcendentals sat on a long serial
// chain with ~3 columns per SIMD to hide it, so the solve is split into
//   riem_pre_k   column   : dz_min clamp of the heights (bottom-up), surface w, the
//                           Lagrangian interface pressure pem (prefix sum of delp)
//   riem_pt_k    pointwise: one lane per (column, level): log pem, p^kappa, pm, pl
//                           (every transcendental of the elimination sweep; a full-chip
//                           launch whose latency thousands of waves hide)
//   riem_col_k   column   : the SIM1 eliminations and back substitutions for pp and w,
//                           the pressure perturbation, and the new heights (one exp/log
//                           per level left, in the bottom-up height sweep)
// Same expressions as the single-sweep form (and as oracle/nh_core.py sim1_solver), so
// results are bit-identical to it.  Column lanes are i-fastest: every k-plane access of
// a wavefront is a coalesced row read.
//   scratch: pp / pe (L+1), w2 (L+1), gam (L+1), pl (L), pm (L)
//   the Lagrangian interface pressure pem is parked in the output array (pef for the
//   C-grid solve, ppe for the D-grid one) and overwritten last.
#include "kernels_nh.hpp"
#include "stencil_common.hpp"

namespace gtfv3 {
namespace {

constexpr double GRAV = Constants::grav;
constexpr double RDGAS = Constants::rdgas;
constexpr double KAPPA = Constants::kappa;
constexpr double R3 = 1.0 / 3.0;
constexpr int BLOCK = 256;

struct RiemArgs {
  Dims d;
  int npz, ring, last_call, cgrid;
  double dt, ptop, p_fac, dz_min;
  const double *delp, *pt, *w_in, *phis;
  double* G;       // zh (heights, D-grid) or gz (heights in -> geopotential out, C-grid); L+1
  double* w_out;   // D-grid: w (in place); C-grid: null
  double* delz;    // D-grid only
  double* pout;    // C-grid: pef (full pressure); D-grid: ppe (perturbation); L+1
  double *pk3, *pe, *peln, *pk;  // D-grid only (pe/peln/pk on the last call)
  double* ws_out;  // D-grid: surface w for the remap (may be null)
  double *gam, *pp, *w2, *pl, *pm;  // scratch planes
};

// plane offset of this lane's column; false past the last column
__device__ __forceinline__ bool riem_column_of(const RiemArgs& a, int c, long& o) {
  const Dims& d = a.d;
  const int ni = d.nx + 2 * a.ring, nj = d.ny + 2 * a.ring;
  if (c >= ni * nj) return false;
  o = pidx(d, c % ni - a.ring, c / ni - a.ring);
  return true;
}

__global__ void __launch_bounds__(BLOCK) riem_pre_k(RiemArgs a) {
  long o;
  if (!riem_column_of(a, blockIdx.x * BLOCK + threadIdx.x, o)) return;
  const Dims& d = a.d;
  const int s = blockIdx.y, km = a.npz;
  const long P = d.plane;
  const long b1 = (long)s * (km + 1) * P + o, bk = (long)s * km * P + o;
  double* __restrict__ G = a.G + b1;
  double* __restrict__ PO = a.pout + b1;
  const double* __restrict__ DP = a.delp + bk;
  const double zs = a.phis[(long)s * P + o] * (1.0 / GRAV);
  double gb = G[km * P];
  if (a.ws_out) a.ws_out[(long)s * P + o] = (zs - gb) * (1.0 / a.dt);
  // dz_min clamp of the interface heights (bottom-up), in place; G[km] is not changed
#pragma unroll 4
  for (int k = km - 1; k >= 0; --k) {
    const double g = fmax(G[k * P], gb + a.dz_min);
    G[k * P] = g;
    gb = g;
  }
  // Lagrangian interface pressure, parked in the output array
  double pem = a.ptop;
  PO[0] = pem;
#pragma unroll 4
  for (int k = 0; k < km; ++k) {
    pem = pem + DP[k * P];
    PO[(k + 1) * P] = pem;
  }
}

// one lane per (column, level k in [0, km]): interface k and (k < km) layer k
__global__ void __launch_bounds__(BLOCK) riem_pt_k(RiemArgs a) {
  long o;
  if (!riem_column_of(a, blockIdx.x * BLOCK + threadIdx.x, o)) return;
  const Dims& d = a.d;
  const int k = blockIdx.y, s = blockIdx.z, km = a.npz;
  const long P = d.plane;
  const long i1 = ((long)s * (km + 1) + k) * P + o;
  const long ik = ((long)s * km + k) * P + o;
  const bool cg = a.cgrid != 0;
  const double pa = a.pout[i1];
  const double la = cg ? 0.0 : log(pa);
  if (!cg) {
    const double pkk = exp(KAPPA * la);
    a.pk3[i1] = pkk;
    if (a.last_call) {
      a.pe[i1] = pa;
      a.peln[i1] = la;
      a.pk[i1] = pkk;
    }
  }
  if (k == km) return;
  const double pb = a.pout[i1 + P];
  const double dpk = a.delp[ik];
  const double dm = dpk * (1.0 / GRAV);
  const double pm = cg ? dpk / log(pb / pa) : dpk / (log(pb) - la);
  const double dz = a.G[i1 + P] - a.G[i1];
  const double gama = 1.0 / (1.0 - KAPPA);
  a.pl[ik] = exp(gama * log(-dm / dz * RDGAS * a.pt[ik])) - pm;
  a.pm[ik] = pm;
}

template <bool CG>
__device__ __forceinline__ void riem_sweeps(const RiemArgs& a, int s, long o, double* __restrict__ G,
                                            double* __restrict__ GM, double* __restrict__ PO,
                                            double* __restrict__ PPc, double* __restrict__ W2c,
                                            const double* __restrict__ DP, const double* __restrict__ PT,
                                            const double* __restrict__ W1, const double* __restrict__ PL,
                                            const double* __restrict__ PM, double* __restrict__ WOUT,
                                            double* __restrict__ DELZ) {
  const Dims& d = a.d;
  const int km = a.npz;
  const long P = d.plane;
#define LP(k) PPc[(k) * P]
#define LW(k) W2c[(k) * P]
  const double dt = a.dt;
  const double hs = a.phis[(long)s * P + o];
  const double zs = hs * (1.0 / GRAV);
  const double gama = 1.0 / (1.0 - KAPPA);
  const double t1g = gama * 2.0 * dt * dt;
  const double rdt = 1.0 / dt;
  const double capa1 = KAPPA - 1.0;
  const double ws = (zs - G[km * P]) * (1.0 / dt);  // G[km] as before the clamp

  // S1: forward elimination for pp
  double dm_k = DP[0] * (1.0 / GRAV);
  double pl_k = PL[0];
  double bet = 0.0, pp_k = 0.0, g_prev = 0.0;
  LP(0) = 0.0;
#pragma unroll 2
  for (int k = 0; k < km; ++k) {
    double g = 0.0, bbk, ddk, dm_n = 0.0, pl_n = 0.0;
    if (k < km - 1) {
      dm_n = DP[(k + 1) * P] * (1.0 / GRAV);
      pl_n = PL[(k + 1) * P];
      g = dm_k / dm_n;
      bbk = 2.0 * (1.0 + g);
      ddk = 3.0 * (pl_k + g * pl_n);
    } else {
      bbk = 2.0;
      ddk = 3.0 * pl_k;
    }
    double ppn;
    if (k == 0) {
      bet = bbk;
      ppn = ddk / bet;
    } else {
      const double gm = g_prev / bet;
      GM[k * P] = gm;
      bet = bbk - gm;
      ppn = (ddk - pp_k) / bet;
    }
    LP(k + 1) = ppn;
    pp_k = ppn;
    g_prev = g;
    dm_k = dm_n;
    pl_k = pl_n;
  }
  // S2: back substitution for pp
  {
    double x = LP(km);
#pragma unroll 2
    for (int k = km - 1; k > 0; --k) {
      x = LP(k) - GM[k * P] * x;
      LP(k) = x;
    }
  }
  // S3: forward elimination for w (aa from dz, pem, pp on the fly; neighbours carried)
  {
    double g0 = G[0], g1 = G[P], g2 = G[2 * P];
    double dz_k = g1 - g0, dz_n = g2 - g1;  // dz[0], dz[1]
    double pp_k = LP(1);                    // pp[1]
    const double dm0 = DP[0] * (1.0 / GRAV);
    double aa_k = t1g / (dz_k + dz_n) * (PO[P] + pp_k);  // aa[1]
    bet = dm0 - aa_k;
    double w_prev = (dm0 * W1[0] + dt * pp_k) / bet;
    LW(0) = w_prev;
    g1 = g2;
#pragma unroll 2
    for (int k = 1; k < km - 1; ++k) {
      // here dz_n = dz[k], pp_k = pp[k], aa_k = aa[k]
      const double g_next = G[(k + 2) * P];
      const double dz_nn = g_next - g1;  // dz[k+1]
      const double pp_n = LP(k + 1);
      const double dmk = DP[k * P] * (1.0 / GRAV);
      const double aa_n = t1g / (dz_n + dz_nn) * (PO[(k + 1) * P] + pp_n);
      const double gm = aa_k / bet;
      GM[k * P] = gm;
      bet = dmk - (aa_k + aa_n + aa_k * gm);
      w_prev = (dmk * W1[k * P] + dt * (pp_n - pp_k) - aa_k * w_prev) / bet;
      LW(k) = w_prev;
      aa_k = aa_n;
      pp_k = pp_n;
      dz_n = dz_nn;
      g1 = g_next;
    }
    // dz_n = dz[km-1], pp_k = pp[km-1]
    const double dml = DP[(km - 1) * P] * (1.0 / GRAV);
    const double pp_b = LP(km);
    const double p1 = t1g / dz_n * (PO[km * P] + pp_b);
    const double gm = aa_k / bet;
    GM[(km - 1) * P] = gm;
    bet = dml - (aa_k + p1 + aa_k * gm);
    LW(km - 1) = (dml * W1[(km - 1) * P] + dt * (pp_b - pp_k) - p1 * ws - aa_k * w_prev) / bet;
  }
  // S4: back substitution for w
  {
    double x = LW(km - 1);
#pragma unroll 2
    for (int k = km - 2; k >= 0; --k) {
      x = LW(k) - GM[(k + 1) * P] * x;
      LW(k) = x;
    }
  }
  // S5: non-hydrostatic pressure perturbation at interfaces (pe replaces pp)
  {
    double pe_k = 0.0;
    LP(0) = 0.0;
#pragma unroll 2
    for (int k = 0; k < km; ++k) {
      const double w2 = LW(k);
      pe_k = pe_k + DP[k * P] * (1.0 / GRAV) * (w2 - W1[k * P]) * rdt;
      LP(k + 1) = pe_k;
      if (WOUT) WOUT[k * P] = w2;
    }
  }
  // S6: new layer thicknesses (bottom-up), heights / geopotential, pressures out
  {
    double g_out = CG ? hs : zs;
    double p1 = 0.0;
    double lp1 = LP(km), lp2 = 0.0;  // pe at interfaces k+1, k+2
    if (CG) PO[km * P] = lp1 + PO[km * P];
    else PO[km * P] = lp1;
    G[km * P] = g_out;
    double dm_b = 0.0;  // dm of layer k+1
#pragma unroll 2
    for (int k = km - 1; k >= 0; --k) {
      const double pem_t = PO[k * P];  // still the parked pem
      const double dmk = DP[k * P] * (1.0 / GRAV);
      const double pmk = PM[k * P];
      const double lp0 = LP(k);
      if (k == km - 1) {
        p1 = (lp0 + 2.0 * lp1) * R3;
      } else {
        const double g = dmk / dm_b;
        const double bbk = 2.0 * (1.0 + g);
        p1 = (lp0 + bbk * lp1 + g * lp2) * R3 - g * p1;
      }
      const double dz2 = -dmk * RDGAS * PT[k * P] * exp(capa1 * log(fmax(a.p_fac * pmk, p1 + pmk)));
      if (CG) {
        g_out = g_out - dz2 * GRAV;
        PO[k * P] = k == 0 ? a.ptop : lp0 + pem_t;
      } else {
        g_out = g_out - dz2;
        DELZ[k * P] = dz2;
        PO[k * P] = lp0;
      }
      G[k * P] = g_out;
      lp2 = lp1;
      lp1 = lp0;
      dm_b = dmk;
    }
  }
#undef LP
#undef LW
}

constexpr int RREG_BLOCK = 64;

// Register-resident form of riem_sweeps for a compile-time level count KM: the
// elimination factors and the pp / w2 / pe columns live in VGPR arrays (fully unrolled
// sweeps, static indices), so the only memory traffic is the inputs and outputs; the
// scratch planes of the streaming form (the dominant HBM traffic, ~3x the algorithmic
// bytes) disappear.  Fewer columns are in flight per CU (large VGPR footprint), which
// also keeps the repeated input reads of a column inside the Infinity Cache.  Same
// expressions as riem_sweeps (bit-identical).
template <int KM, bool CG>
__device__ __forceinline__ void riem_sweeps_reg(const RiemArgs& a, int s, long o, double* __restrict__ G,
                                                double* __restrict__ PO, const double* __restrict__ DP,
                                                const double* __restrict__ PT, const double* __restrict__ W1,
                                                const double* __restrict__ PL, const double* __restrict__ PM,
                                                double* __restrict__ WOUT, double* __restrict__ DELZ,
                                                double* gm) {
  const long P = a.d.plane;
  constexpr int km = KM;
  const double dt = a.dt;
  const double hs = a.phis[(long)s * P + o];
  const double zs = hs * (1.0 / GRAV);
  const double gama = 1.0 / (1.0 - KAPPA);
  const double t1g = gama * 2.0 * dt * dt;
  const double rdt = 1.0 / dt;
  const double capa1 = KAPPA - 1.0;
  const double ws = (zs - G[km * P]) * (1.0 / dt);
  double lp[KM + 1];  // pp (later pe)
  double lw[KM];      // w2
  // gm: the elimination factors, this lane's column of an LDS array (stride 64 lanes)

  // S1: forward elimination for pp
  {
    double dm_k = DP[0] * (1.0 / GRAV);
    double pl_k = PL[0];
    double bet = 0.0, pp_k = 0.0, g_prev = 0.0;
    lp[0] = 0.0;
#pragma unroll
    for (int k = 0; k < km; ++k) {
      double g = 0.0, bbk, ddk, dm_n = 0.0, pl_n = 0.0;
      if (k < km - 1) {
        dm_n = DP[(k + 1) * P] * (1.0 / GRAV);
        pl_n = PL[(k + 1) * P];
        g = dm_k / dm_n;
        bbk = 2.0 * (1.0 + g);
        ddk = 3.0 * (pl_k + g * pl_n);
      } else {
        bbk = 2.0;
        ddk = 3.0 * pl_k;
      }
      double ppn;
      if (k == 0) {
        bet = bbk;
        ppn = ddk / bet;
      } else {
        const double gmk = g_prev / bet;
        gm[k * RREG_BLOCK] = gmk;
        bet = bbk - gmk;
        ppn = (ddk - pp_k) / bet;
      }
      lp[k + 1] = ppn;
      pp_k = ppn;
      g_prev = g;
      dm_k = dm_n;
      pl_k = pl_n;
    }
  }
  // S2: back substitution for pp
  {
    double x = lp[km];
#pragma unroll
    for (int k = km - 1; k > 0; --k) {
      x = lp[k] - gm[k * RREG_BLOCK] * x;
      lp[k] = x;
    }
  }
  // S3: forward elimination for w
  {
    double g0 = G[0], g1 = G[P], g2 = G[2 * P];
    double dz_k = g1 - g0, dz_n = g2 - g1;
    double pp_k = lp[1];
    const double dm0 = DP[0] * (1.0 / GRAV);
    double aa_k = t1g / (dz_k + dz_n) * (PO[P] + pp_k);
    double bet = dm0 - aa_k;
    double w_prev = (dm0 * W1[0] + dt * pp_k) / bet;
    lw[0] = w_prev;
    g1 = g2;
#pragma unroll
    for (int k = 1; k < km - 1; ++k) {
      const double g_next = G[(k + 2) * P];
      const double dz_nn = g_next - g1;
      const double pp_n = lp[k + 1];
      const double dmk = DP[k * P] * (1.0 / GRAV);
      const double aa_n = t1g / (dz_n + dz_nn) * (PO[(k + 1) * P] + pp_n);
      const double gmk = aa_k / bet;
      gm[k * RREG_BLOCK] = gmk;
      bet = dmk - (aa_k + aa_n + aa_k * gmk);
      w_prev = (dmk * W1[k * P] + dt * (pp_n - pp_k) - aa_k * w_prev) / bet;
      lw[k] = w_prev;
      aa_k = aa_n;
      pp_k = pp_n;
      dz_n = dz_nn;
      g1 = g_next;
    }
    const double dml = DP[(km - 1) * P] * (1.0 / GRAV);
    const double pp_b = lp[km];
    const double p1 = t1g / dz_n * (PO[km * P] + pp_b);
    const double gmk = aa_k / bet;
    gm[(km - 1) * RREG_BLOCK] = gmk;
    bet = dml - (aa_k + p1 + aa_k * gmk);
    lw[km - 1] = (dml * W1[(km - 1) * P] + dt * (pp_b - pp_k) - p1 * ws - aa_k * w_prev) / bet;
  }
  // S4: back substitution for w
  {
    double x = lw[km - 1];
#pragma unroll
    for (int k = km - 2; k >= 0; --k) {
      x = lw[k] - gm[(k + 1) * RREG_BLOCK] * x;
      lw[k] = x;
    }
  }
  // S5: pressure perturbation at interfaces
  {
    double pe_k = 0.0;
    lp[0] = 0.0;
#pragma unroll
    for (int k = 0; k < km; ++k) {
      const double w2 = lw[k];
      pe_k = pe_k + DP[k * P] * (1.0 / GRAV) * (w2 - W1[k * P]) * rdt;
      lp[k + 1] = pe_k;
      if (WOUT) WOUT[k * P] = w2;
    }
  }
  // S6: new layer thicknesses (bottom-up), heights / geopotential, pressures out
  {
    double g_out = CG ? hs : zs;
    double p1 = 0.0;
    double lp1 = lp[km], lp2 = 0.0;
    if (CG) PO[km * P] = lp1 + PO[km * P];
    else PO[km * P] = lp1;
    G[km * P] = g_out;
    double dm_b = 0.0;
#pragma unroll
    for (int k = km - 1; k >= 0; --k) {
      const double pem_t = PO[k * P];
      const double dmk = DP[k * P] * (1.0 / GRAV);
      const double pmk = PM[k * P];
      const double lp0 = lp[k];
      if (k == km - 1) {
        p1 = (lp0 + 2.0 * lp1) * R3;
      } else {
        const double g = dmk / dm_b;
        const double bbk = 2.0 * (1.0 + g);
        p1 = (lp0 + bbk * lp1 + g * lp2) * R3 - g * p1;
      }
      const double dz2 = -dmk * RDGAS * PT[k * P] * exp(capa1 * log(fmax(a.p_fac * pmk, p1 + pmk)));
      if (CG) {
        g_out = g_out - dz2 * GRAV;
        PO[k * P] = k == 0 ? a.ptop : lp0 + pem_t;
      } else {
        g_out = g_out - dz2;
        DELZ[k * P] = dz2;
        PO[k * P] = lp0;
      }
      G[k * P] = g_out;
      lp2 = lp1;
      lp1 = lp0;
      dm_b = dmk;
    }
  }
}

template <int KM, bool CG>
__global__ void __launch_bounds__(RREG_BLOCK) riem_col_reg_k(RiemArgs a) {
  __shared__ double gm[(KM + 1) * RREG_BLOCK];
  long o;
  if (!riem_column_of(a, blockIdx.x * RREG_BLOCK + threadIdx.x, o)) return;
  const int s = blockIdx.y;
  const long P = a.d.plane;
  const long b1 = (long)s * (KM + 1) * P + o;
  const long bk = (long)s * KM * P + o;
  riem_sweeps_reg<KM, CG>(a, s, o, a.G + b1, a.pout + b1, a.delp + bk, a.pt + bk, a.w_in + bk, a.pl + bk,
                          a.pm + bk, a.w_out ? a.w_out + bk : nullptr, a.delz ? a.delz + bk : nullptr,
                          gm + threadIdx.x);
}

template <bool CG>
__global__ void __launch_bounds__(BLOCK) riem_col_k(RiemArgs a) {
  long o;
  if (!riem_column_of(a, blockIdx.x * BLOCK + threadIdx.x, o)) return;
  const int s = blockIdx.y, km = a.npz;
  const long P = a.d.plane;
  const long b1 = (long)s * (km + 1) * P + o;  // interface fields
  const long bk = (long)s * km * P + o;        // layer fields
  riem_sweeps<CG>(a, s, o, a.G + b1, a.gam + b1, a.pout + b1, a.pp + b1, a.w2 + b1, a.delp + bk, a.pt + bk,
                  a.w_in + bk, a.pl + bk, a.pm + bk, a.w_out ? a.w_out + bk : nullptr,
                  a.delz ? a.delz + bk : nullptr);
}

void launch_riem(const Ctx& c, const RiemArgs& a) {
  if (a.npz < 2) throw std::runtime_error("riem: npz >= 2 required");
  const int ncol = (c.d.nx + 2 * a.ring) * (c.d.ny + 2 * a.ring);
  const double km = a.npz, k1 = a.npz + 1, cols = (double)ncol * c.d.nsub;
  // algorithmic bytes per column: pre reads zh/gz (L+1) delp (L) phis, writes the clamped
  // heights and pem (L+1) (+ ws); pt reads pem, heights (L+1) delp pt (L), writes pl pm (L)
  // (+ pk3 (L+1), + pe peln pk on the last call); the sweeps read delp pt w pl pm (L)
  // heights pem (L+1) phis and write heights, pressure out (L+1) (+ w delz (L))
  GT_LAUNCH(riem_pre_k, dim3(cdiv(ncol, BLOCK), c.d.nsub), dim3(BLOCK), 0, c.st, a);
  HIP_LAUNCH_CHECK();
  ktimer_bytes(8.0 * cols * (3 * k1 + km + 1 + (a.ws_out ? 1 : 0)));
  GT_LAUNCH(riem_pt_k, dim3(cdiv(ncol, BLOCK), a.npz + 1, c.d.nsub), dim3(BLOCK), 0, c.st, a);
  HIP_LAUNCH_CHECK();
  ktimer_bytes(8.0 * cols * (2 * k1 + 4 * km + (a.cgrid ? 0 : (a.last_call ? 4 : 1) * k1)));
  if (a.npz == 72) {  // the Held-Suarez / Aquaplanet L72 configurations: register-resident sweeps
    if (a.cgrid) GT_LAUNCH((riem_col_reg_k<72, true>), dim3(cdiv(ncol, RREG_BLOCK), c.d.nsub), dim3(RREG_BLOCK), 0, c.st, a);
    else GT_LAUNCH((riem_col_reg_k<72, false>), dim3(cdiv(ncol, RREG_BLOCK), c.d.nsub), dim3(RREG_BLOCK), 0, c.st, a);
  } else if (a.cgrid) {
    GT_LAUNCH(riem_col_k<true>, dim3(cdiv(ncol, BLOCK), c.d.nsub), dim3(BLOCK), 0, c.st, a);
  } else {
    GT_LAUNCH(riem_col_k<false>, dim3(cdiv(ncol, BLOCK), c.d.nsub), dim3(BLOCK), 0, c.st, a);
  }
  HIP_LAUNCH_CHECK();
  ktimer_bytes(8.0 * cols * (5 * km + 4 * k1 + 1 + (a.cgrid ? 0 : 2 * km)));
}

}  // namespace

void riem_solver_c(const Ctx& c, int npz, double dt2, double ptop, double p_fac, double dz_min, const double* delpc,
                   const double* ptc, const double* wc, const double* phis, double* gz, double* pef,
                   const NhScratch& sc) {
  RiemArgs a{};
  a.d = c.d;
  a.npz = npz;
  a.ring = 1;
  a.cgrid = 1;
  a.dt = dt2;
  a.ptop = ptop;
  a.p_fac = p_fac;
  a.dz_min = dz_min;
  a.delp = delpc;
  a.pt = ptc;
  a.w_in = wc;
  a.phis = phis;
  a.G = gz;
  a.pout = pef;
  a.gam = sc.s[5];
  a.pp = sc.s[6];
  a.w2 = sc.s[13];
  a.pl = sc.s[7];
  a.pm = sc.s[8];
  launch_riem(c, a);
}

void riem_solver3(const Ctx& c, const Riem3Args& r, const NhScratch& sc) {
  RiemArgs a{};
  a.d = c.d;
  a.npz = r.npz;
  a.ring = 0;
  a.cgrid = 0;
  a.last_call = r.last_call;
  a.dt = r.dt;
  a.ptop = r.ptop;
  a.p_fac = r.p_fac;
  a.dz_min = r.dz_min;
  a.delp = r.delp;
  a.pt = r.pt;
  a.w_in = r.w;
  a.phis = r.phis;
  a.G = r.zh;
  a.w_out = r.w;
  a.delz = r.delz;
  a.pout = r.ppe;
  a.pk3 = r.pk3;
  a.pe = r.pe;
  a.peln = r.peln;
  a.pk = r.pk;
  a.ws_out = r.ws;
  a.gam = sc.s[5];
  a.pp = sc.s[6];
  a.w2 = sc.s[13];
  a.pl = sc.s[7];
  a.pm = sc.s[8];
  launch_riem(c, a);
}

}  // namespace gtfv3
