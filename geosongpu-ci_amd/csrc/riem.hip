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
#include "blockscan.hpp"
#include "kernels_nh.hpp"
#include "stencil_common.hpp"

namespace gtfv3 {
namespace {

constexpr double GRAV = Constants::grav;
constexpr double RDGAS = Constants::rdgas;
constexpr double KAPPA = Constants::kappa;
constexpr double R3 = 1.0 / 3.0;
constexpr int BLOCK = 256;

int g_riem_variant = -1;  // -1: not set, GTFV3_RIEM decides

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

// ---------------- level-block scan form (default) ----------------
//
// One wavefront owns NC = 64 / NB columns; lane = NB * column + b, block b holding layers
// [b M, b M + M) and interfaces b M .. b M + M of its column in registers (L72: M = 9, NB = 8,
// eight columns a wave; L137: M = 9, NB = 16 with a partial last block).  A column's blocks sit
// in consecutive lanes of one 16-lane DPP row, so every hand-over between neighbouring blocks
// is a DPP row shift (no LDS, no ds_bpermute).
//
// Every sweep runs on all 64 lanes at once:
//   * pointwise work: the logs / exps of pln, pk3, pl and dz2, the layer quantities;
//   * prefix sums (pem, pe, the heights): each block sums its layers, a Kogge-Stone scan of the
//     block totals over the NB lanes (log2 NB DPP shifts) gives each block its carry-in, and the
//     block runs its recurrence from that carry;
//   * the two tridiagonal solves (pp, then w) as a partitioned Thomas algorithm (tri_solve):
//     the pivots bet_k = d_k - a_k c_{k-1} / bet_{k-1} are a Möbius recurrence, a product of 2x2
//     matrices [[d_k, -a_k c_{k-1}], [1, 0]]: each block multiplies its M, a scan multiplies the
//     block products, block b reads its incoming pivot off the product of blocks 0..b-1 and
//     eliminates from it; the forward-substituted right-hand side y_k = (r_k - a_k y_{k-1}) / bet_k
//     and the back substitution x_k = y_k - gam_{k+1} x_{k+1} are affine recurrences, each run as
//     a block pass with a zero carry (giving the block's affine map), a scan of the maps and a
//     second block pass from the true carry;
//   * the p1 recurrence (bottom-up affine) and the dz_min clamp (bottom-up max recurrence,
//     speculative per block, repeated only where a block below changed its bottom interface).
// The w system is nearly singular (the acoustic coupling aa ~ 1e8 against layer masses ~ 1e2):
// scanned (Moebius-product) pivots would carry the cancellation of the matrix products
// (~1e-13 relative), so the w solve hands its pivots block to block serially
// (tri_solve<M, NB, false>: block b eliminates from block b-1's last pivot, NB dependent DPP
// steps) -- the column sweep's pivot sequence -- and only the right-hand side and the back
// substitution are scanned; no refinement step.  Measured against the oracle's column solve:
// w within 1e-11 of its scale at L7 .. L137 (tests/test_gpu_riem.py).
// Sums and products are associated differently from the column sweep (riem_col_k): the
// results agree with it and with the oracle to rounding (tests/test_gpu_riem.py), not bit for
// bit.  Transcendentals and divisions come from fastmath.hpp (~1 ulp; a third of ocml's log).
// Each input is read once (G, DP, PT, W1, phis) and each output written once.
constexpr int RS_WAVES = 4;
typedef unsigned int RbU2 __attribute__((ext_vector_type(2)));

template <int M, int NB, bool PART, bool CG>
__global__ void __launch_bounds__(64 * RS_WAVES, 2) riem_scan_k(RiemArgs a) {
  constexpr int NC = 64 / NB;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int b = lane & (NB - 1);
  const bool last = b == NB - 1;
  const Dims& d = a.d;
  const int km = a.npz;  // launch_riem: km = (NB - 1) M + nv_last, 1 <= nv_last <= M
  const int nv = PART && last ? km - (NB - 1) * M : M;  // real layers of this block
  auto real = [&](int m) { return !PART || m < nv; };
  auto isbot = [&](int m) { return last && m == nv - 1; };
  const int ni = d.nx + 2 * a.ring, nj = d.ny + 2 * a.ring;
  const int ncol = ni * nj;
  const int s = blockIdx.y;
  // XCD-aware order (xcd_block): a wave's 8 columns are 64 B of each level's 128-B lines, the
  // other half read by the neighbouring wave; with each XCD on a contiguous run of workgroups
  // the neighbours that share lines sit behind one L2
  const int c0 = ((int)xcd_block() * RS_WAVES + wv) * NC;
  if (c0 >= ncol) return;  // whole wavefront; no workgroup barrier in this kernel
  int c = c0 + lane / NB;
  const bool valid = c < ncol;  // writes
  if (!valid) c = ncol - 1;
  const int i = c % ni - a.ring, j = c / ni - a.ring;
  const long P = d.plane;
  const long o = pidx(d, i, j);
  const double dt = a.dt, rdt = 1.0 / dt;
  const double gama = 1.0 / (1.0 - KAPPA);
  const double t1g = gama * 2.0 * dt * dt;
  const double capa1 = KAPPA - 1.0;

  // Memory: one buffer descriptor per array and sub-domain (wave-uniform SGPRs), a 32-bit
  // per-lane byte offset (the block's first level) and the level as the scalar offset.  The
  // scalar offset is excluded from the descriptor's range check, so the levels past the
  // bottom (a partial block's) take an out-of-range per-lane offset instead: their loads read
  // zero and their stores are dropped, whatever the level offset.
  const uint32_t PB = (uint32_t)P * 8u;
  const uint32_t lo = (uint32_t)((o + (long)(b * M) * P) * 8);
  const uint32_t o8 = (uint32_t)o * 8u;
  const int li = (km + 1) * (int)PB, ll = km * (int)PB;
  auto rs = [&](const double* p, bool itf) {
    const long so = (long)s * (itf ? km + 1 : km) * P;
    return __builtin_amdgcn_make_buffer_rsrc((void*)(p + so), 0, itf ? li : ll, 0x00020000);
  };
  constexpr uint32_t OOB = 0x80000000u;
  auto lom = [&](int m) { return real(m) ? lo : OOB; };
  auto ld = [&](__amdgpu_buffer_rsrc_t r, int m) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, lom(m), (uint32_t)m * PB, 0));
  };
  auto st = [&](__amdgpu_buffer_rsrc_t r, int m, double v) {  // layer m of the block
    if (valid) __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(RbU2, v), r, lom(m), (uint32_t)m * PB, 0);
  };
  // interface m of the block: real up to the block's bottom interface (m <= nv)
  auto loi = [&](int m) { return m == 0 || real(m - 1) ? lo : OOB; };
  auto sti = [&](__amdgpu_buffer_rsrc_t r, int m, double v) {
    if (valid) __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(RbU2, v), r, loi(m), (uint32_t)m * PB, 0);
  };
  // the column's bottom interface (level km), written by the last block
  auto st_bot = [&](__amdgpu_buffer_rsrc_t r, double v) {
    if (valid && last) __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(RbU2, v), r, o8, (uint32_t)km * PB, 0);
  };
  const auto rG = rs(a.G, true), rPO = rs(a.pout, true);
  const auto rDP = rs(a.delp, false), rPT = rs(a.pt, false), rW1 = rs(a.w_in, false);

  // ---- loads (W1 after the pp solve)
  double G[M + 1], DP[M], PT[M];
#pragma unroll
  for (int m = 0; m <= M; ++m)  // G[M] is the block's bottom interface: real when its top layer is
    G[m] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rG, loi(m), (uint32_t)m * PB, 0));
#pragma unroll
  for (int m = 0; m < M; ++m) DP[m] = ld(rDP, m);
#pragma unroll
  for (int m = 0; m < M; ++m) PT[m] = ld(rPT, m);
  const double hs = __builtin_bit_cast(
      double, __builtin_amdgcn_raw_buffer_load_b64(
                  __builtin_amdgcn_make_buffer_rsrc((void*)(a.phis + (long)s * P), 0, (int)PB, 0x00020000), o8, 0, 0));
  const double gsurf = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rG, o8, (uint32_t)km * PB, 0));
  const double zs = hs * (1.0 / GRAV);
  const double ws = (zs - gsurf) * (1.0 / dt);
  if (a.ws_out && valid && b == 0)
    __builtin_amdgcn_raw_buffer_store_b64(
        __builtin_bit_cast(RbU2, ws),
        __builtin_amdgcn_make_buffer_rsrc((void*)(a.ws_out + (long)s * P), 0, (int)PB, 0x00020000), o8, 0, 0);

  // ---- S0: dz_min clamp (bottom-up max recurrence): each block clamps from the unclamped
  // interface below it and repeats only if the block below changed that interface (exact)
  double gl[M + 1];
  {
    double gin = PART && last ? gsurf : G[M];
    for (int it = 0; it <= NB; ++it) {
      gl[M] = gin;
#pragma unroll
      for (int m = M - 1; m >= 0; --m) gl[m] = real(m) ? fmax(G[m], gl[m + 1] + a.dz_min) : gin;
      const double gn = blk_next(gl[0]);
      const double want = last ? gin : gn;
      if (!__any(want != gin)) break;
      gin = want;
    }
  }

  // ---- S1: pem = ptop + DP[0] + DP[1] + ... summed top-down in level order, block after
  // block (the carry handed down by DPP): bit for bit the sum pk3_pe_halo forms for the halo
  // columns, so pk3 / pe agree across a sub-domain edge (the step is then the same on 1x1 and
  // 2x2 / 1x4 sub-domains); M dependent adds per block, NB blocks in turn
  double pem[M + 1];
  {
    double carry = a.ptop;
#pragma unroll 1
    for (int r = 0; r < NB; ++r) {
      if (b == r) {
        pem[0] = carry;
#pragma unroll
        for (int m = 0; m < M; ++m) pem[m + 1] = pem[m] + DP[m];
      }
      const double nx = blk_prev(pem[M]);  // all lanes, outside the branch (blockscan.hpp)
      carry = b == r + 1 ? nx : carry;
    }
  }

  // ---- S1b: pointwise layer quantities (and pk3 / pe / peln / pk on the D grid)
  // per-layer values that live from the first sweep to the last, in LDS: pm, q = dm RDGAS pt
  // (dz2's factor) and g_rat
  __shared__ double lds_rs[3][RS_WAVES][M][64];
  double(&Spm)[M][64] = lds_rs[0][wv];
  double(&Sq)[M][64] = lds_rs[1][wv];
  double(&Sg)[M][64] = lds_rs[2][wv];
  double dm[M], dz[M], pl[M];
  {
    double pln[M + 1];
    if constexpr (!CG) {
      const double lpt = fm_log(a.ptop);
#pragma unroll
      for (int m = 1; m <= M; ++m) pln[m] = fm_log(pem[m]);
      const double plu = blk_prev(pln[M]);
      pln[0] = b == 0 ? lpt : plu;
      const auto rK3 = rs(a.pk3, true);
#pragma unroll
      for (int m = 0; m <= M; ++m) {
        if (m > 0 || b == 0) {  // interface 0 of block b > 0 is written by block b - 1
          const double pkk = fm_exp(KAPPA * pln[m]);
          sti(rK3, m, pkk);
          if (a.last_call) {
            sti(rs(a.pe, true), m, pem[m]);
            sti(rs(a.peln, true), m, pln[m]);
            sti(rs(a.pk, true), m, pkk);
          }
        }
      }
    }
#pragma unroll
    for (int m = 0; m < M; ++m) {
      dm[m] = DP[m] * (1.0 / GRAV);
      dz[m] = gl[m + 1] - gl[m];
      double pmv;
      if constexpr (CG) pmv = fm_div(DP[m], fm_log(fm_div(pem[m + 1], pem[m])));
      else pmv = fm_div(DP[m], pln[m + 1] - pln[m]);
      const double plv = fm_exp(gama * fm_log(fm_div(-dm[m], dz[m]) * RDGAS * PT[m])) - pmv;
      Spm[m][lane] = real(m) ? pmv : 0.0;
      Sq[m][lane] = dm[m] * RDGAS * PT[m];
      pl[m] = real(m) ? plv : 0.0;
    }
  }

  // ---- S1c/S2: the pp system (rows: interfaces 1..km), g_rat
  double pp[M];  // pp[m] = pp at interface b M + m + 1
  {
    const double dmn_b = blk_next(dm[0]), pln_b = blk_next(pl[0]);
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const double dmn = m + 1 < M ? dm[m + 1 < M ? m + 1 : 0] : dmn_b;
      const double pn = m + 1 < M ? pl[m + 1 < M ? m + 1 : 0] : pln_b;
      const bool bt = isbot(m);
      const double gv = bt || !real(m) ? 0.0 : fm_div(dm[m], dmn);
      Sg[m][lane] = gv;
      // (rows past a partial block's bottom: 0 by a select -- pn there is the next column's
      // value, and 0 * NaN would carry a garbage column's NaN into this one)
      pp[m] = !real(m) ? 0.0 : (bt ? 3.0 * pl[m] : 3.0 * (pl[m] + gv * pn));
    }
    double dd[M];
#pragma unroll
    for (int m = 0; m < M; ++m) dd[m] = pp[m];
    auto row = [&](int m, double& am, double& dg, double& cm) {
      am = (b == 0 && m == 0) || !real(m) ? 0.0 : 1.0;
      const double gv = Sg[m][lane];
      dg = !real(m) ? 1.0 : (isbot(m) ? 2.0 : 2.0 * (1.0 + gv));
      cm = gv;
    };
    tri_solve<M, NB, true>(row, [&](int m) { return dd[m]; }, pp, b, last);
  }

  // ---- S3/S4: the w system
  double W1[M];
#pragma unroll
  for (int m = 0; m < M; ++m) W1[m] = ld(rW1, m);
  double w2[M];
  {
    // pp and dz at the block's interfaces / layers above
    const double ppu = blk_prev(pp[M - 1]);
    const double pp_up = b == 0 ? 0.0 : ppu;  // pp at interface b M
    const double dz_up = blk_prev(dz[M - 1]);
    auto ppi = [&](int m) { return m > 0 ? pp[m > 0 ? m - 1 : 0] : pp_up; };  // pp at interface m
    double aat[M];  // aa at interface b M + m (0 at the column's top)
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const double dzu = m > 0 ? dz[m > 0 ? m - 1 : 0] : dz_up;
      const double v = fm_div(t1g, dzu + dz[m]) * (pem[m] + ppi(m));
      aat[m] = (b == 0 && m == 0) || !real(m) ? 0.0 : v;
    }
    // aa below the block's last real layer: the next block's first, or p1 at the surface
    const double aab_nb = blk_next(aat[0]);
    double p1 = 0.0;
    if (last) {
      double dzb = dz[M - 1], pemb = pem[M], ppb = pp[M - 1];
      if constexpr (PART) {
#pragma unroll
        for (int m = 0; m < M; ++m)
          if (m == nv - 1) {
            dzb = dz[m];
            pemb = pem[m + 1];
            ppb = pp[m];
          }
      }
      p1 = fm_div(t1g, dzb) * (pemb + ppb);
    }
    auto aab = [&](int m) { return isbot(m) ? p1 : (m + 1 < M ? aat[m + 1 < M ? m + 1 : 0] : aab_nb); };
    auto row = [&](int m, double& am, double& dg, double& cm) {
      am = aat[m];
      const double ab = aab(m);
      dg = real(m) ? dm[m] - (aat[m] + ab) : 1.0;
      cm = isbot(m) || !real(m) ? 0.0 : ab;
    };
    auto rhs = [&](int m) {
      const double v = dm[m] * W1[m] + dt * (pp[m] - ppi(m));
      return isbot(m) ? v - p1 * ws : (real(m) ? v : 0.0);
    };
    tri_solve<M, NB, false>(row, rhs, w2, b, last);
  }

  // ---- S5: pe prefix (top-down); w out
  double pe[M + 1];  // pe at interfaces b M .. b M + M
  {
    double num[M], tot = 0.0;
#pragma unroll
    for (int m = 0; m < M; ++m) {
      num[m] = dm[m] * (w2[m] - W1[m]) * rdt;
      tot += num[m];
    }
    const double ex = blk_prev(scan_sum<NB, true>(tot, b));
    pe[0] = b == 0 ? 0.0 : ex;
#pragma unroll
    for (int m = 0; m < M; ++m) pe[m + 1] = pe[m] + num[m];
    if (a.w_out) {
      const auto rW = rs(a.w_out, false);
#pragma unroll
      for (int m = 0; m < M; ++m) st(rW, m, w2[m]);
    }
  }

  // ---- S6: p1 recurrence (bottom-up affine), dz2, heights
  {
    const double pe2_nb = blk_next(pe[1]);  // pe at interface b M + M + 1
    double p1v[M];
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const double pe2 = m + 2 <= M ? pe[m + 2 <= M ? m + 2 : 0] : pe2_nb;
      const double gv = Sg[m][lane];
      const double t = isbot(m) ? (pe[m] + 2.0 * pe[m + 1]) * R3 : (pe[m] + 2.0 * (1.0 + gv) * pe[m + 1] + gv * pe2) * R3;
      p1v[m] = real(m) ? t : 0.0;
    }
    // p1_k = t_k - g_k p1_{k+1}: block pass with a zero carry, scan of the maps, second pass
    double ph = 0.0, Cc = 1.0;
#pragma unroll
    for (int m = M - 1; m >= 0; --m) {
      const double gv = Sg[m][lane];
      ph = __builtin_fma(-gv, ph, p1v[m]);
      Cc = -gv * Cc;
    }
    const Aff H = scan_aff<NB, false>(Aff{Cc, ph}, b);
    const double pnd = blk_next(H.B);
    double pin = last ? 0.0 : pnd;
#pragma unroll
    for (int m = M - 1; m >= 0; --m) {
      pin = __builtin_fma(-Sg[m][lane], pin, p1v[m]);
      p1v[m] = pin;
    }
    double dz2[M], tot = 0.0;
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const double pmk = Spm[m][lane];
      const double v = -Sq[m][lane] * fm_exp(capa1 * fm_log(fmax(a.p_fac * pmk, p1v[m] + pmk)));
      dz2[m] = real(m) ? v : 0.0;
      tot += CG ? dz2[m] * GRAV : dz2[m];
    }
    // heights bottom-up from the surface
    const double incl = scan_sum<NB, false>(tot, b);
    const double base = CG ? hs : zs;
    const double incl_d = blk_next(incl);
    double gz = last ? base : base - incl_d;
    double gzo[M];
#pragma unroll
    for (int m = M - 1; m >= 0; --m) {
      gz = CG ? gz - dz2[m] * GRAV : gz - dz2[m];
      gzo[m] = gz;
    }
#pragma unroll
    for (int m = 0; m < M; ++m) sti(rG, m, gzo[m]);
    st_bot(rG, base);
    if constexpr (CG) {
#pragma unroll
      for (int m = 0; m < M; ++m) sti(rPO, m, b == 0 && m == 0 ? a.ptop : pe[m] + pem[m]);
      double peb = pe[M] + pem[M];
      if constexpr (PART) {
#pragma unroll
        for (int m = 0; m < M; ++m)
          if (m == nv - 1) peb = pe[m + 1] + pem[m + 1];
      }
      st_bot(rPO, peb);
    } else {
      const auto rDZ = rs(a.delz, false);
#pragma unroll
      for (int m = 0; m < M; ++m) {
        st(rDZ, m, dz2[m]);
        sti(rPO, m, pe[m]);
      }
      double peb = pe[M];
      if constexpr (PART) {
#pragma unroll
        for (int m = 0; m < M; ++m)
          if (m == nv - 1) peb = pe[m + 1];
      }
      st_bot(rPO, peb);
    }
  }
}

void launch_riem(const Ctx& c, const RiemArgs& a) {
  if (a.npz < 2) throw std::runtime_error("riem: npz >= 2 required");
  const int km = a.npz;
  const int ncol = (c.d.nx + 2 * a.ring) * (c.d.ny + 2 * a.ring);
  const dim3 tb(64 * RS_WAVES);
  // scan form when the column splits into NB blocks of an instantiated M (all but the last
  // block full): (NB - 1) M < km <= NB M
  auto fits = [&](int m, int nb) { return (nb - 1) * m < km && km <= nb * m; };
  auto grid = [&](int nb) {
    return dim3(xcd_pad(cdiv(cdiv(ncol, 64 / nb), RS_WAVES)), c.d.nsub);
  };
  const bool scan = riem_variant() != 1;
#define RIEM_SCAN(M_, NB_, PART_)                                                                   \
  do {                                                                                              \
    if (a.cgrid) GT_LAUNCH((riem_scan_k<M_, NB_, PART_, true>), grid(NB_), tb, 0, c.st, a);        \
    else GT_LAUNCH((riem_scan_k<M_, NB_, PART_, false>), grid(NB_), tb, 0, c.st, a);               \
  } while (0)
  if (scan && km == 72) RIEM_SCAN(9, 8, false);
  else if (scan && fits(9, 8)) RIEM_SCAN(9, 8, true);
  else if (scan && fits(9, 16)) RIEM_SCAN(9, 16, true);
  else if (scan && fits(6, 16)) RIEM_SCAN(6, 16, true);
  else if (scan && fits(5, 4)) RIEM_SCAN(5, 4, true);
  else if (scan && fits(3, 4)) RIEM_SCAN(3, 4, true);
  else if (scan && fits(2, 4)) RIEM_SCAN(2, 4, true);
  else GT_LAUNCH(riem_col_k, dim3(cdiv(ncol, BLOCK), c.d.nsub), dim3(BLOCK), 0, c.st, a);
#undef RIEM_SCAN
  HIP_LAUNCH_CHECK();
  // algorithmic bytes per column: C grid reads delpc ptc wc (L) gz (L+1) phis, writes gz pef (L+1);
  // D grid reads zh (L+1) delp pt w (L) phis, writes w delz (L) zh ppe pk3 (L+1) ws (+ pe peln pk)
  const double L = km, L1 = km + 1;
  const double per = a.cgrid ? 3 * L + 3 * L1 + 1 : 5 * L + (4 + (a.last_call ? 3 : 0)) * L1 + 2;
  ktimer_bytes(8.0 * ncol * c.d.nsub * per);
}

}  // namespace

void set_riem_variant(int v) { g_riem_variant = v; }
// GTFV3_RIEM=1: the column sweeps on the step (A/B and fault isolation); the stencil
// interface's explicit variant parameter overrides it
int riem_variant() {
  static const int env = [] {
    const char* e = std::getenv("GTFV3_RIEM");
    return e ? std::atoi(e) : 0;
  }();
  return g_riem_variant >= 0 ? g_riem_variant : env;
}

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
