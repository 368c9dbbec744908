// riem.hip — riem_solver_c / riem_solver3 (FV3 nh_utils SIM1 semi-implicit vertical
// acoustic solve, a_imp = 1) as streaming column sweeps for gfx950.
//
// One column per lane, 256 columns per workgroup; a column's k-sweeps run in program
// order, so every k-plane access of a wave is a coalesced row read.  The kernel is
// latency bound (72-long dependent recurrences), so it is built for occupancy: no LDS,
// ~110 VGPRs, and only three work arrays that must survive between sweeps, kept as
// scratch planes (L2 / Infinity-Cache resident while a wave lives):
//   * pp / pe  (L+1),  w2 (L),  gam (L)
//   * the Lagrangian interface pressure pem is parked in the kernel's own output
//     array (pef for the C-grid solve, ppe for the D-grid one) and overwritten last.
// Everything else (dm, pm, dz, pl, g_rat, bb, dd, aa) is recomputed on the fly with
// the same expressions as the oracle (oracle/nh_core.py sim1_solver), so results are
// bit-identical to the previous scratch-plane version.
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
  double *gam, *pp, *w2;  // scratch, L+1 planes each
};

// The column body takes every array as a distinct __restrict__ pointer: the arrays never
// alias, and saying so lets the compiler hoist the loads of an unrolled group of levels
// above the stores of the previous ones (one memory latency per group of levels instead
// of one per level: the sweeps are otherwise a chain of dependent HBM / L2 round trips).
__device__ __forceinline__ void riem_column(const RiemArgs& a, int s, long o, double* __restrict__ G,
                                            double* __restrict__ GM, double* __restrict__ PO,
                                            double* __restrict__ PPc, double* __restrict__ W2c,
                                            const double* __restrict__ DP, const double* __restrict__ PT,
                                            const double* __restrict__ W1, double* __restrict__ PK3,
                                            double* __restrict__ PE, double* __restrict__ PELN,
                                            double* __restrict__ PK, double* __restrict__ WOUT,
                                            double* __restrict__ DELZ) {
  const Dims& d = a.d;
  const int km = a.npz;
  const long P = d.plane;
#define LP(k) PPc[(k) * P]
#define LW(k) W2c[(k) * P]

  const double dt = a.dt;
  const double hs = a.phis[(long)s * P + o];
  const double zs = hs * (1.0 / GRAV);
  const double ws = (zs - G[km * P]) * (1.0 / dt);
  if (a.ws_out) a.ws_out[(long)s * P + o] = ws;
  // S0: dz_min clamp of the interface heights (bottom-up), written back in place
  {
    double gb = G[km * P];
    _Pragma("unroll 2") for (int k = km - 1; k >= 0; --k) {
      double g = fmax(G[k * P], gb + a.dz_min);
      G[k * P] = g;
      gb = g;
    }
  }
  const double gama = 1.0 / (1.0 - KAPPA);
  const double t1g = gama * 2.0 * dt * dt;
  const double rdt = 1.0 / dt;
  const double capa1 = KAPPA - 1.0;
  const bool cg = a.cgrid != 0;

  // layer quantities: pm from pem (C grid: log of the ratio; D grid: difference of logs)
  auto pm_of = [&](double dpk, double pa, double pb, double la, double lb) {
    return cg ? dpk / log(pb / pa) : dpk / (lb - la);
  };
  auto pl_of = [&](double dm, double dz, double ptk, double pm) {
    return exp(gama * log(-dm / dz * RDGAS * ptk)) - pm;
  };

  // S1: pem / peln / pk3 prefix, pl, forward elimination for pp
  double pem0 = a.ptop, pln0 = cg ? 0.0 : log(a.ptop);
  PO[0] = pem0;  // park pem
  if (!cg) {
    const double ptk = exp(KAPPA * pln0);
    PK3[0] = ptk;
    if (a.last_call) {
      PE[0] = pem0;
      PELN[0] = pln0;
      PK[0] = ptk;
    }
  }
  auto advance = [&](int k, double pem_k, double& pem_n, double& pln_n) {
    // interface k+1 from interface k
    pem_n = pem_k + DP[k * P];
    PO[(k + 1) * P] = pem_n;
    if (!cg) {
      pln_n = log(pem_n);
      const double pkk = exp(KAPPA * pln_n);
      PK3[(k + 1) * P] = pkk;
      if (a.last_call) {
        PE[(k + 1) * P] = pem_n;
        PELN[(k + 1) * P] = pln_n;
        PK[(k + 1) * P] = pkk;
      }
    } else {
      pln_n = 0.0;
    }
  };
  double pem1, pln1;
  advance(0, pem0, pem1, pln1);
  double dpk = DP[0];
  double dm_k = dpk * (1.0 / GRAV);
  double pm_k = pm_of(dpk, pem0, pem1, pln0, pln1);
  double pl_k = pl_of(dm_k, G[P] - G[0], PT[0], pm_k);
  double pem_k1 = pem1, pln_k1 = pln1;  // interface k+1
  double bet = 0.0, pp_k = 0.0, g_prev = 0.0;
  LP(0) = 0.0;
  _Pragma("unroll 2") for (int k = 0; k < km; ++k) {
    double g = 0.0, bbk, ddk, dm_n = 0.0, pl_n = 0.0;
    if (k < km - 1) {
      double pem_k2, pln_k2;
      advance(k + 1, pem_k1, pem_k2, pln_k2);
      const double dpn = DP[(k + 1) * P];
      dm_n = dpn * (1.0 / GRAV);
      const double pm_n = pm_of(dpn, pem_k1, pem_k2, pln_k1, pln_k2);
      pl_n = pl_of(dm_n, G[(k + 2) * P] - G[(k + 1) * P], PT[(k + 1) * P], pm_n);
      g = dm_k / dm_n;
      bbk = 2.0 * (1.0 + g);
      ddk = 3.0 * (pl_k + g * pl_n);
      pem_k1 = pem_k2;
      pln_k1 = pln_k2;
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
    _Pragma("unroll 2") for (int k = km - 1; k > 0; --k) {
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
    _Pragma("unroll 2") for (int k = 1; k < km - 1; ++k) {
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
    _Pragma("unroll 2") for (int k = km - 2; k >= 0; --k) {
      x = LW(k) - GM[(k + 1) * P] * x;
      LW(k) = x;
    }
  }
  // S5: non-hydrostatic pressure perturbation at interfaces (pe replaces pp)
  {
    double pe_k = 0.0;
    LP(0) = 0.0;
    _Pragma("unroll 2") for (int k = 0; k < km; ++k) {
      const double w2 = LW(k);
      pe_k = pe_k + DP[k * P] * (1.0 / GRAV) * (w2 - W1[k * P]) * rdt;
      LP(k + 1) = pe_k;
      if (WOUT) WOUT[k * P] = w2;
    }
  }
  // S6: new layer thicknesses (bottom-up), heights / geopotential, pressures out
  {
    double pem_b = PO[km * P];  // interface k+1 (bottom first)
    double pln_b = cg ? 0.0 : log(pem_b);
    double g_out = cg ? hs : zs;
    double p1 = 0.0;
    double lp1 = LP(km), lp2 = 0.0;  // pe at interfaces k+1, k+2
    if (cg) PO[km * P] = lp1 + pem_b;
    else PO[km * P] = lp1;
    G[km * P] = g_out;
    double dm_b = 0.0;  // dm of layer k+1
    _Pragma("unroll 2") for (int k = km - 1; k >= 0; --k) {
      const double pem_t = PO[k * P];  // still the parked pem
      const double pln_t = cg ? 0.0 : log(pem_t);
      const double dpk2 = DP[k * P];
      const double dmk = dpk2 * (1.0 / GRAV);
      const double pmk = pm_of(dpk2, pem_t, pem_b, pln_t, pln_b);
      const double lp0 = LP(k);
      if (k == km - 1) {
        p1 = (lp0 + 2.0 * lp1) * R3;
      } else {
        const double g = dmk / dm_b;
        const double bbk = 2.0 * (1.0 + g);
        p1 = (lp0 + bbk * lp1 + g * lp2) * R3 - g * p1;
      }
      const double dz2 = -dmk * RDGAS * PT[k * P] * exp(capa1 * log(fmax(a.p_fac * pmk, p1 + pmk)));
      if (cg) {
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
      pem_b = pem_t;
      pln_b = pln_t;
      dm_b = dmk;
    }
  }
#undef LP
#undef LW
}

__global__ void __launch_bounds__(BLOCK) riem_col_k(RiemArgs a) {
  const Dims& d = a.d;
  const int km = a.npz, k1 = km + 1;
  const int ni = d.nx + 2 * a.ring, nj = d.ny + 2 * a.ring;
  const int c = blockIdx.x * BLOCK + threadIdx.x;
  const int s = blockIdx.y;
  if (c >= ni * nj) return;
  const int i = c % ni - a.ring, j = c / ni - a.ring;
  const long P = d.plane;
  const long o = pidx(d, i, j);
  const long b1 = (long)s * k1 * P + o;  // interface fields
  const long bk = (long)s * km * P + o;  // layer fields
  auto at = [](double* p, long off) { return p ? p + off : nullptr; };
  riem_column(a, s, o, a.G + b1, a.gam + b1, a.pout + b1, a.pp + b1, a.w2 + b1, a.delp + bk, a.pt + bk,
              a.w_in + bk, at(a.pk3, b1), at(a.pe, b1), at(a.peln, b1), at(a.pk, b1), at(a.w_out, bk),
              at(a.delz, bk));
}

void launch_riem(const Ctx& c, const RiemArgs& a) {
  if (a.npz < 2) throw std::runtime_error("riem: npz >= 2 required");
  const int ncol = (c.d.nx + 2 * a.ring) * (c.d.ny + 2 * a.ring);
  GT_LAUNCH(riem_col_k, dim3(cdiv(ncol, BLOCK), c.d.nsub), dim3(BLOCK), 0, c.st, a);
  HIP_LAUNCH_CHECK();
  // algorithmic bytes per column: C grid reads delpc ptc wc (L) gz (L+1) phis, writes gz pef (L+1);
  // D grid reads zh (L+1) delp pt w (L) phis, writes w delz (L) zh ppe pk3 (L+1) ws (+ pe peln pk)
  const double km = a.npz, k1 = a.npz + 1;
  const double per = a.cgrid ? 3 * km + 3 * k1 + 1 : 5 * km + (4 + (a.last_call ? 3 : 0)) * k1 + 2;
  ktimer_bytes(8.0 * ncol * c.d.nsub * per);
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
  launch_riem(c, a);
}

}  // namespace gtfv3
