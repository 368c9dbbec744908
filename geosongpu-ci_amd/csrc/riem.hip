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

int g_riem_variant = 0;

struct RiemArgs {
  Dims d;
  int npz, ring, last_call, cgrid, dump;
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

// ---------------- register-resident form (default) ----------------
//
// One wavefront owns 16 columns; its 64 lanes are 4 level blocks x 16 columns
// (lane = 16 b + column), block b holding layers [b M, b M + M) and interfaces
// b M .. b M + M of its column in registers (M = 18 at L72).  Every output is written
// once; inputs the registers cannot hold across all sweeps (DP, PT, W1, G) are re-read
// from cache where a later sweep needs them, and the clamped heights and interface
// pressures are recomputed there (nothing is parked in HBM and read back).
//
//   * pointwise work (the transcendentals of pm, pl, pk3, dz2; aa, the numerators) runs
//     on all 64 lanes at once;
//   * each recurrence (pem and pe prefixes, both Thomas eliminations and back
//     substitutions, the p1 recurrence, the height sums) runs block after block with its
//     carry handed to the next block by a lane shuffle (lane +- 16), so every value is
//     formed by the same operations in the same order as in riem_column: the results
//     are bit-identical to the column form (tests/test_gpu_riem.py compares them);
//   * the dz_min clamp (bottom-up max recurrence) runs on all blocks at once from the
//     unclamped interface below each block, then repeats only if a block's lower
//     neighbour changed that interface (exact; the clamp is rarely active).
// Two per-layer arrays that live from the first sweep to the last (pm, g_rat) are
// kept in LDS, the rest in VGPRs.
//
// A column whose level count is not a multiple of M (L137 = 7 x 18 + 11) runs as eight
// blocks of eight columns with a partial last block (PARTIAL, MV < M real layers, a template
// constant): its lanes' loads past the surface are masked to zero and their stores dropped,
// and every recurrence starts or stops at the real bottom MV instead of M.
constexpr int RB_WAVES = 4;
typedef unsigned int RbU2 __attribute__((ext_vector_type(2)));
// The pointwise loops are long straight-line runs of independent transcendentals; left
// alone the scheduler interleaves all M of them and runs out of registers.  A fence per
// level keeps one or two in flight (two waves per SIMD hide the latency instead).
#define RB_SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)

template <int NC>
__device__ __forceinline__ double rb_below(double v, int lane) { return __shfl(v, (lane + NC) & 63); }
template <int NC>
__device__ __forceinline__ double rb_above(double v, int lane) { return __shfl(v, (lane - NC) & 63); }

template <int M, bool CG, int NB = 4, int MV = M>
__global__ void __launch_bounds__(64 * RB_WAVES, 2) riem_blk_k(RiemArgs a) {
  constexpr int RB_NB = NB, RB_NC = 64 / NB;
  constexpr bool PARTIAL = MV < M;  // the last block holds MV < M layers (km = (nblk - 1) M + MV)
  auto from_below = [](double v, int ln) { return rb_below<RB_NC>(v, ln); };
  auto from_above = [](double v, int ln) { return rb_above<RB_NC>(v, ln); };
  __shared__ double lds_pm[RB_WAVES][M][64];
  __shared__ double lds_g[RB_WAVES][M][64];
  constexpr bool cg = CG;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int b = lane / RB_NC;
  const Dims& d = a.d;
  const int km = a.npz;
  const int nblk = (km + M - 1) / M;  // launch_riem: nblk <= NB, km = (nblk - 1) M + MV
  const int ni = d.nx + 2 * a.ring, nj = d.ny + 2 * a.ring;
  const int ncol = ni * nj;
  const int s = blockIdx.y;
  const int c0 = (blockIdx.x * RB_WAVES + wv) * RB_NC;
  if (c0 >= ncol) return;  // whole wavefront; no workgroup barrier in this kernel
  int c = c0 + (lane & (RB_NC - 1));
  const bool act = b < nblk;                // lanes of blocks past the column idle
  const bool valid = c < ncol && act;       // writes
  if (c >= ncol) c = ncol - 1;
  const int i = c % ni - a.ring, j = c / ni - a.ring;
  const long P = d.plane;
  const long o = pidx(d, i, j);
  const int kb0 = act ? b * M : 0;
  const bool lastblk = b == nblk - 1;
  double(&spm)[M][64] = lds_pm[wv];
  double(&sg)[M][64] = lds_g[wv];
  const double dt = a.dt;
  const double gama = 1.0 / (1.0 - KAPPA);
  const double t1g = gama * 2.0 * dt * dt;
  const double rdt = 1.0 / dt;
  const double capa1 = KAPPA - 1.0;

  // Memory: one buffer descriptor per array and sub-domain (wave-uniform SGPRs), a 32-bit
  // per-lane byte offset (the block's first level) and the level as the scalar offset.
  const uint32_t PB = (uint32_t)P * 8u;
  const uint32_t lo = (uint32_t)((o + (long)kb0 * P) * 8);
  const int li = (km + 1) * (int)PB, ll = km * (int)PB;  // bytes of a sub-domain's field
  auto rs = [&](const double* p, bool itf) {
    const long so = (long)s * (itf ? km + 1 : km) * P;
    return __builtin_amdgcn_make_buffer_rsrc((void*)(p + so), 0, itf ? li : ll, 0x00020000);
  };
  // itf: an interface field (levels 0 .. km).  In a partial block the levels past the surface
  // (static m >= MV, or > MV for interface fields) exist only for the other blocks' lanes: the
  // last block's lanes read zero there and store nothing (masked, no access).
  auto past = [&](int m, bool itf) { return PARTIAL && m >= MV + (itf ? 1 : 0); };
  auto ld = [&](__amdgpu_buffer_rsrc_t r, int m, bool itf = false) {
    if (past(m, itf)) {
      double v = 0.0;
      if (!lastblk) v = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, lo, (uint32_t)m * PB, 0));
      return v;
    }
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, lo, (uint32_t)m * PB, 0));
  };
  auto st = [&](__amdgpu_buffer_rsrc_t r, int m, double v, bool itf = false) {
    if (past(m, itf) && lastblk) return;
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(RbU2, v), r, lo, (uint32_t)m * PB, 0);
  };
  const auto rG = rs(a.G, true), rPO = rs(a.pout, true);
  const auto rDP = rs(a.delp, false), rPT = rs(a.pt, false), rW1 = rs(a.w_in, false);

  // ---- loads
  double gr[M + 1], DP[M];
#pragma unroll
  for (int m = 0; m <= M; ++m) gr[m] = ld(rG, m, true);
#pragma unroll
  for (int m = 0; m < M; ++m) DP[m] = ld(rDP, m);
  // surface values (re-read where used instead of held in registers)
  const uint32_t o8 = (uint32_t)o * 8u;
  const auto rPH = __builtin_amdgcn_make_buffer_rsrc((void*)(a.phis + (long)s * P), 0, (int)PB, 0x00020000);
  auto surf = [&](double& hs, double& zs, double& ws) {
    hs = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rPH, o8, 0, 0));
    zs = hs * (1.0 / GRAV);
    const double gbot = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rG, o8, (uint32_t)km * PB, 0));
    ws = (zs - gbot) * (1.0 / dt);
  };
  if (a.ws_out && valid && b == 0) {
    double hs, zs, ws;
    surf(hs, zs, ws);
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(RbU2, ws),
        __builtin_amdgcn_make_buffer_rsrc((void*)(a.ws_out + (long)s * P), 0, (int)PB, 0x00020000), o8, 0, 0);
  }

  // dz_min clamp of the heights g (bottom-up), speculative per block: each block clamps from
  // the unclamped interface below it, and repeats only if the block below changed it
  auto clamp = [&](const double (&g)[M + 1], double (&gl)[M + 1]) {
    double gin = g[M];  // unclamped interface kb1
    if (PARTIAL && lastblk) gin = ld(rG, MV, true);  // the partial block's is the surface at MV
    for (int it = 0; it <= RB_NB; ++it) {
      gl[M] = gin;
#pragma unroll
      for (int m = M - 1; m >= 0; --m)
        gl[m] = PARTIAL && lastblk && m >= MV ? gin : fmax(g[m], gl[m + 1] + a.dz_min);
      const double gn = from_below(gl[0], lane);
      const double want = lastblk || !act ? gin : gn;
      if (!__any(want != gin)) break;
      gin = want;
    }
  };
  // interface pressures pem = ptop + prefix sums of DP (top-down, block after block)
  auto prefix = [&](const double (&dpv)[M], double (&pe_)[M + 1]) {
#pragma unroll
    for (int m = 0; m <= M; ++m) pe_[m] = 0.0;
    double carry = a.ptop;
#pragma unroll 1
    for (int r = 0; r < nblk; ++r) {
      if (b == r) {
        pe_[0] = carry;
#pragma unroll
        for (int m = 0; m < M; ++m) pe_[m + 1] = pe_[m] + dpv[m];
      }
      carry = from_above(pe_[M], lane);
    }
  };
  // The clamped heights and pem are recomputed where S3 / S6 need them again (same
  // operations, same values) instead of being parked in HBM between the sweeps: the parked
  // copies cost a write and one or two re-reads per level (riem traffic was 2.4-3x its
  // algorithmic bytes).
  RB_SCHED_FENCE();
  // ---- S0: dz_min clamp
  double gl[M + 1];
  clamp(gr, gl);

  RB_SCHED_FENCE();
  // ---- S1a: pem prefix
  double pem[M + 1];
  prefix(DP, pem);

  RB_SCHED_FENCE();
  // ---- S1b: pointwise layer quantities
  double pl[M], dm[M];
  {
    double pln[M + 1];
    if (!cg) {
      const auto rK3 = rs(a.pk3, true);
#pragma unroll
      for (int m = 0; m <= M; ++m) {
        pln[m] = log(pem[m]);  // slot 0 of block 0: log(ptop)
        if (valid && (m < M || lastblk)) {
          RB_SCHED_FENCE();
          const double pkk = exp(KAPPA * pln[m]);
          st(rK3, m, pkk, true);
          if (a.last_call) {
            st(rs(a.pe, true), m, pem[m], true);
            st(rs(a.peln, true), m, pln[m], true);
            st(rs(a.pk, true), m, pkk, true);
          }
        }
      }
    }
#pragma unroll
    for (int m = 0; m < M; ++m) {
      dm[m] = DP[m] * (1.0 / GRAV);
      const double dz = gl[m + 1] - gl[m];
      const double pm = cg ? DP[m] / log(pem[m + 1] / pem[m]) : DP[m] / (pln[m + 1] - pln[m]);
      spm[m][lane] = pm;
      pl[m] = exp(gama * log(-dm[m] / dz * RDGAS * ld(rPT, m))) - pm;
      RB_SCHED_FENCE();
    }
  }
  // g_rat and the right-hand side of the pp system
  double dd[M], gprev;
  {
    const double dm_nb = from_below(dm[0], lane), pl_nb = from_below(pl[0], lane);
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const bool bot = lastblk && m == MV - 1;
      const double dmn = m + 1 < M ? dm[m + 1 < M ? m + 1 : 0] : dm_nb;
      const double pln_ = m + 1 < M ? pl[m + 1 < M ? m + 1 : 0] : pl_nb;
      const double g = bot ? 0.0 : dm[m] / dmn;
      sg[m][lane] = g;
      dd[m] = bot ? 3.0 * pl[m] : 3.0 * (pl[m] + g * pln_);
    }
    gprev = from_above(sg[M - 1][lane], lane);  // g_rat of layer kb0-1
  }

  RB_SCHED_FENCE();
  // ---- S1c: forward elimination for pp (top-down, block after block)
  double pp[M + 1], gam[M];
#pragma unroll
  for (int m = 0; m <= M; ++m) pp[m] = 0.0;
#pragma unroll
  for (int m = 0; m < M; ++m) gam[m] = 0.0;
  {
    double cbet = 0.0, cpp = 0.0;
#pragma unroll 1
    for (int r = 0; r < nblk; ++r) {
      double bet_o = 0.0;
      if (b == r) {
        double bet = cbet, ppk = cpp;
        pp[0] = cpp;
#pragma unroll
        for (int m = 0; m < M; ++m) {
          const bool bot = lastblk && m == MV - 1;
          const double g = sg[m][lane];
          const double bbk = bot ? 2.0 : 2.0 * (1.0 + g);
          double ppn;
          if (m == 0 && b == 0) {
            bet = bbk;
            ppn = dd[m] / bet;
          } else {
            const double gm = (m == 0 ? gprev : sg[m > 0 ? m - 1 : 0][lane]) / bet;
            gam[m] = gm;
            bet = bbk - gm;
            ppn = (dd[m] - ppk) / bet;
          }
          if (PARTIAL && lastblk && m >= MV) ppn = ppk;  // past the surface: pp[M] = pp[MV] for S2 and S3
          pp[m + 1] = ppn;
          ppk = ppn;
        }
        bet_o = bet;
      }
      cbet = from_above(bet_o, lane);
      cpp = from_above(pp[M], lane);
    }
  }
  RB_SCHED_FENCE();
  // ---- S2: back substitution for pp (bottom-up)
  {
    double cx = 0.0;
#pragma unroll 1
    for (int r = nblk - 1; r >= 0; --r) {
      if (b == r) {
        if (!lastblk) pp[M] = cx;
        double x = pp[M];
#pragma unroll
        for (int m = M - 1; m >= 0; --m) {
          if ((m > 0 || b > 0) && !(PARTIAL && lastblk && m >= MV)) {
            x = pp[m] - gam[m] * x;
            pp[m] = x;
          }
        }
      }
      cx = from_below(pp[0], lane);
    }
  }

  RB_SCHED_FENCE();
  // ---- S3: forward elimination for w (top-down)
  double aat[M], num[M], aab_last;
  {
    double pemr[M + 1], glr[M + 1], dz[M];
    {
      double dpv[M], g0[M + 1];
#pragma unroll
      for (int m = 0; m < M; ++m) dpv[m] = ld(rDP, m);
#pragma unroll
      for (int m = 0; m <= M; ++m) g0[m] = ld(rG, m, true);  // the unclamped heights (G is written in S6)
      prefix(dpv, pemr);
      clamp(g0, glr);
#pragma unroll
      for (int m = 0; m < M; ++m) dm[m] = dpv[m] * (1.0 / GRAV);
    }
#pragma unroll
    for (int m = 0; m < M; ++m) dz[m] = glr[m + 1] - glr[m];
    const double dz_ab = from_above(dz[M - 1], lane);
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const double dzu = m == 0 ? dz_ab : dz[m > 0 ? m - 1 : 0];
      aat[m] = t1g / (dzu + dz[m]) * (pemr[m] + pp[m]);  // aa at interface kb0+m (unused at 0)
      num[m] = dm[m] * ld(rW1, m) + dt * (pp[m + 1] - pp[m]);
    }
    // aa below the block's last layer: the next block's first aa, or p1 for the bottom
    const double aab_nb = from_below(aat[0], lane);
    double hs, zs, ws;
    surf(hs, zs, ws);
    double dzb = dz[M - 1];
    if (PARTIAL && lastblk) {  // the bottom layer MV-1 of the partial block, clamped as in clamp()
      const double gs = ld(rG, MV, true);
      dzb = gs - fmax(ld(rG, MV - 1, true), gs + a.dz_min);
    }
    const double p1 = t1g / dzb * (pemr[M] + pp[M]);  // pemr, pp constant past the surface
#pragma unroll
    for (int m = 0; m < M; ++m)
      if (lastblk && m == MV - 1) num[m] = num[m] - p1 * ws;
    aab_last = lastblk ? p1 : aab_nb;
  }
  double w2[M];
#pragma unroll
  for (int m = 0; m < M; ++m) w2[m] = 0.0;
  {
    double cbet = 0.0, cw = 0.0;
#pragma unroll 1
    for (int r = 0; r < nblk; ++r) {
      double bet_o = 0.0, w_o = 0.0;
      if (b == r) {
        double bet = cbet, wp = cw;
#pragma unroll
        for (int m = 0; m < M; ++m) {
          const double aab = m + 1 < M && !(PARTIAL && lastblk && m == MV - 1) ? aat[m + 1 < M ? m + 1 : 0] : aab_last;
          if (m == 0 && b == 0) {
            bet = dm[m] - aab;
            wp = num[m] / bet;
          } else {
            const double gm = aat[m] / bet;
            gam[m] = gm;
            bet = dm[m] - (aat[m] + aab + aat[m] * gm);
            wp = (num[m] - aat[m] * wp) / bet;
          }
          w2[m] = wp;
        }
        bet_o = bet;
        w_o = wp;
      }
      cbet = from_above(bet_o, lane);
      cw = from_above(w_o, lane);
    }
  }
  RB_SCHED_FENCE();
  // ---- S4: back substitution for w (bottom-up)
  {
    const double gam_nb = from_below(gam[0], lane);
    double cx = 0.0;
#pragma unroll 1
    for (int r = nblk - 1; r >= 0; --r) {
      if (b == r) {
        double x = cx;
#pragma unroll
        for (int m = M - 1; m >= 0; --m) {
          if (lastblk && m == MV - 1) {
            x = w2[m];
          } else if (!(PARTIAL && lastblk && m >= MV)) {
            x = w2[m] - (m + 1 < M ? gam[m + 1 < M ? m + 1 : 0] : gam_nb) * x;
            w2[m] = x;
          }
        }
      }
      cx = from_below(w2[0], lane);
    }
  }

  RB_SCHED_FENCE();
  // ---- S5: pe prefix (top-down); w out
#pragma unroll
  for (int m = 0; m < M; ++m) num[m] = ld(rDP, m) * (1.0 / GRAV) * (w2[m] - ld(rW1, m)) * rdt;
  if (a.w_out && valid) {
    const auto rW = rs(a.w_out, false);
#pragma unroll
    for (int m = 0; m < M; ++m) st(rW, m, w2[m]);
  }
  if (a.dump && valid) {  // debug: w2 and the final pp into the column kernel's scratch planes
    const auto rw = rs(a.w2, true), rg = rs(a.gam, true);
#pragma unroll
    for (int m = 0; m < M; ++m) {
      st(rw, m, w2[m], true);
      st(rg, m, gam[m], true);
    }
  }
  auto& pe = pp;  // pe replaces pp
  {
    double carry = 0.0;
#pragma unroll 1
    for (int r = 0; r < nblk; ++r) {
      if (b == r) {
        pe[0] = carry;
#pragma unroll
        for (int m = 0; m < M; ++m) pe[m + 1] = pe[m] + num[m];
      }
      carry = from_above(pe[M], lane);
    }
  }

  if (a.dump && valid) {
    const auto rp = rs(a.pp, true);
#pragma unroll
    for (int m = 0; m < M; ++m) st(rp, m, pe[m], true);
  }
  RB_SCHED_FENCE();
  // ---- S6: p1 recurrence, dz2, heights (bottom-up)
  {
    const double pe2_nb = from_below(pe[1], lane);  // pe at interface kb1+1
    double t[M];
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const double g = sg[m][lane];
      const double pe2 = m + 2 <= M ? pe[m + 2 <= M ? m + 2 : 0] : pe2_nb;
      if (lastblk && m == MV - 1) t[m] = (pe[m] + 2.0 * pe[m + 1]) * R3;
      else t[m] = (pe[m] + 2.0 * (1.0 + g) * pe[m + 1] + g * pe2) * R3;
    }
    double cp = 0.0;
#pragma unroll 1
    for (int r = nblk - 1; r >= 0; --r) {
      if (b == r) {
        double p1 = cp;
#pragma unroll
        for (int m = M - 1; m >= 0; --m) {
          if (PARTIAL && lastblk && m >= MV) continue;
          if (lastblk && m == MV - 1) p1 = t[m];
          else p1 = t[m] - sg[m][lane] * p1;
          t[m] = p1;
        }
      }
      cp = from_below(t[0], lane);
    }
    // dz2 (pointwise), then the height sums
    double dz2[M];
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const double pmk = spm[m][lane];
      dz2[m] = -(ld(rDP, m) * (1.0 / GRAV)) * RDGAS * ld(rPT, m) *
               exp(capa1 * log(fmax(a.p_fac * pmk, t[m] + pmk)));
      RB_SCHED_FENCE();
    }
    double gz[M + 1];
#pragma unroll
    for (int m = 0; m <= M; ++m) gz[m] = 0.0;
    double hs, zs, ws;
    surf(hs, zs, ws);
    double cg_in = cg ? hs : zs;
#pragma unroll 1
    for (int r = nblk - 1; r >= 0; --r) {
      if (b == r) {
        double go = cg_in;
        gz[M] = go;
#pragma unroll
        for (int m = M - 1; m >= 0; --m) {
          if (!(PARTIAL && lastblk && m >= MV)) go = cg ? go - dz2[m] * GRAV : go - dz2[m];
          gz[m] = go;  // the partial block: the surface up to MV
        }
      }
      cg_in = from_below(gz[0], lane);
    }
    // C grid: pem again for the full pressure (outside the divergent branch: the prefix
    // hands its carry between lanes)
    double pemr[M + 1];
    if (cg) {
      double dpv[M];
#pragma unroll
      for (int m = 0; m < M; ++m) dpv[m] = ld(rDP, m);
      prefix(dpv, pemr);
    } else {
#pragma unroll
      for (int m = 0; m <= M; ++m) pemr[m] = 0.0;
    }
    if (valid) {
      const auto rDZ = rs(a.delz, false);
#pragma unroll
      for (int m = 0; m < M; ++m) {
        st(rG, m, gz[m], true);
        if (cg) {
          st(rPO, m, m == 0 && b == 0 ? a.ptop : pe[m] + pemr[m], true);
        } else {
          st(rDZ, m, dz2[m]);
          st(rPO, m, pe[m], true);
        }
      }
      if (lastblk) {
        st(rG, M, cg ? hs : zs, true);
        st(rPO, M, cg ? pe[M] + pemr[M] : pe[M], true);
      }
    }
  }
}


void launch_riem(const Ctx& c, const RiemArgs& a) {
  if (a.npz < 2) throw std::runtime_error("riem: npz >= 2 required");
  const int km = a.npz;
  const int ncol = (c.d.nx + 2 * a.ring) * (c.d.ny + 2 * a.ring);
  const dim3 gb(cdiv(cdiv(ncol, 16), RB_WAVES), c.d.nsub);
  const dim3 gb8(cdiv(cdiv(ncol, 8), RB_WAVES), c.d.nsub);
  const dim3 tb(64 * RB_WAVES);
  // blocked form when the column splits into at most four blocks of an instantiated size
  // (16 columns a wave), or into up to eight blocks of 18 with a partial last one (8 columns)
  auto fits = [&](int m) { return km % m == 0 && km / m <= 4; };
  const bool blk = riem_variant() != 1;
  const bool part = blk && km == 7 * 18 + 11;  // L137
  if (blk && fits(3)) {
    if (a.cgrid) GT_LAUNCH((riem_blk_k<3, true>), gb, tb, 0, c.st, a);
    else GT_LAUNCH((riem_blk_k<3, false>), gb, tb, 0, c.st, a);
  } else if (blk && fits(5)) {
    if (a.cgrid) GT_LAUNCH((riem_blk_k<5, true>), gb, tb, 0, c.st, a);
    else GT_LAUNCH((riem_blk_k<5, false>), gb, tb, 0, c.st, a);
  } else if (blk && fits(18)) {
    if (a.cgrid) GT_LAUNCH((riem_blk_k<18, true>), gb, tb, 0, c.st, a);
    else GT_LAUNCH((riem_blk_k<18, false>), gb, tb, 0, c.st, a);
  } else if (part) {
    if (a.cgrid) GT_LAUNCH((riem_blk_k<18, true, 8, 11>), gb8, tb, 0, c.st, a);
    else GT_LAUNCH((riem_blk_k<18, false, 8, 11>), gb8, tb, 0, c.st, a);
  } else {
    GT_LAUNCH(riem_col_k, dim3(cdiv(ncol, BLOCK), c.d.nsub), dim3(BLOCK), 0, c.st, a);
  }
  HIP_LAUNCH_CHECK();
  // algorithmic bytes per column: C grid reads delpc ptc wc (L) gz (L+1) phis, writes gz pef (L+1);
  // D grid reads zh (L+1) delp pt w (L) phis, writes w delz (L) zh ppe pk3 (L+1) ws (+ pe peln pk)
  const double L = km, L1 = km + 1;
  const double per = a.cgrid ? 3 * L + 3 * L1 + 1 : 5 * L + (4 + (a.last_call ? 3 : 0)) * L1 + 2;
  ktimer_bytes(8.0 * ncol * c.d.nsub * per);
}

}  // namespace

void set_riem_variant(int v) { g_riem_variant = v; }
int riem_variant() { return g_riem_variant; }

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
  a.dump = riem_variant() == 2;
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
