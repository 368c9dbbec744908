// tp.hip — fv_tp_2d (Lin & Rood 1996 two-dimensional flux-form PPM transport,
// FV3 tp_core) and the tracer_2d_1l pieces (FV3 fv_tracer2d), HIP for gfx950.
//
// fv_tp_2d (HBM-bound, no MFMA) is one column-marching kernel computing:
//   fx2 = xppm(q, crx) [x-corner-filled q]   fy2 = yppm(q, cry) [y-corner-filled q]
//   q_i = (q*area + yfx*fy2|j - yfx*fy2|j+1)/ra_y    q_j = (q*area + xfx*fx2|i - ...)/ra_x
//   fx = 0.5*(xppm(q_i) + fx2)*mfx     fy = 0.5*(yppm(q_j) + fy2)*mfy
// Operation order inside each expression follows the Fortran so the fp64
// numpy oracle (oracle/tp_core.py) matches to the last bits.
#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include <vector>

#include "kernels.hpp"
#include "stencil_common.hpp"

namespace gtfv3 {
namespace {

constexpr int ZMAX = 65535;

// ---------------- fv_tp_2d, column-marching form (default) ----------------
//
// One wavefront owns a strip of 64 columns x = a-3 .. a+60 of one (sub-domain, level)
// and marches up a segment of rows [j0, j1): lane L holds column a-3+L, so every row
// access is one coalesced 64-wide load.  Per row r it
//   * loads q (x- and y-corner-filled where the row crosses a cube-corner halo),
//   * computes the inner x flux fx2 and q_j on row r (x neighbours by DPP lane shifts:
//     no LDS, no barrier, the four waves of a workgroup are independent),
//   * keeps q (y fill) and q_j of rows r-5..r in registers, so the y fluxes fy2 and fy
//     on edge r-2 and q_i on row r-3 need no neighbour exchange at all,
//   * writes fx on row r-3 (x-PPM of q_i through the LDS row) and fy on edge r-2.
// The outputs are the 58 edges / columns a..a+57 (the outer three lanes on each side
// are the x halo); the y halo costs six extra rows per segment.  Each step's loads are
// issued ahead (MarchIn) so their latency overlaps the previous rows' work.  Every
// expression follows tp_core / the oracle (bit-identical results); q, the Courant
// numbers, the fluxes and the area terms stream through HBM once per strip and segment.
// (An LDS-tiled form with 64 x 8 tiles, the first fused version, gave bit-identical
// results and ran 1.9x slower at C180; removed with the ra_x / ra_y planes it read.)
constexpr int MW = 64, MOUT = MW - 6, MWAVES = 4;
// Output spans (round 5).  A row of a sub-domain's outputs (x-edges / columns 0 .. nx) is cut
// into spans, each one wave's strip of lanes: the tile-edge PPM forms (ppm_al at g = -1, 0, 1
// and N-1, N, N+1) reach only the outputs 0 .. 2 and N-3 .. N of a tile (edges g - 1 .. g + 1,
// cells through their two edges), so a sub-domain at a west tile edge has a 3-output tile-edge
// span [0, 2], one at an east tile edge a 4-output span [nx-3, nx], and everything between is
// cut into interior strips of MOUT outputs (C180: 3 + 3 x 58 + 4 = 181, no short strip).  A
// span of at most 26 outputs runs two levels per wave (lanes 0-31 level k, 32-63 level k+1),
// one of at most 10 four levels (16-lane groups): each group is a strip with three halo lanes
// on either side, so the DPP shifts that cross groups reach only halo lanes.  Round 4 cut
// rows at multiples of 58 (C180: 58 58 58 7), which ran two of four strips per level in the
// tile-edge form and one with 7 outputs.
constexpr int MAXSPAN = 192;
// span entry: sub-domain, tile-edge form, first output column, output count (1 .. MOUT)
__host__ __device__ constexpr int span_enc(int s, bool ex, int a0, int nout) {
  return (s << 19) | ((ex ? 1 : 0) << 18) | (a0 << 6) | (nout - 1);
}
__host__ __device__ inline int span_s(int e) { return e >> 19; }
__host__ __device__ inline bool span_ex(int e) { return ((e >> 18) & 1) != 0; }
__host__ __device__ inline int span_a0(int e) { return (e >> 6) & 4095; }
__host__ __device__ inline int span_nout(int e) { return (e & 63) + 1; }
// levels per wave of a span: class 0 one (> 26 outputs), 1 two (<= 26), 2 four (<= 10).
// (Capping the tile-edge spans at two / one levels per wave measured 34.0-34.2 / 35.5 ms per
// step against 33.1-33.2: the four-level waves stay)
inline int span_class(int nout) { return nout <= MW / 4 - 6 ? 2 : (nout <= MW / 2 - 6 ? 1 : 0); }
// DXL (the thermo march's tile-edge strips): the dxa of the <= 8 tile-edge columns a strip
// can hold (I = -2 .. 1, N-2 .. N+1) for the segment's rows live in LDS, one region per wave,
// instead of two dxa loads per row step in the prefetch buffers: 8 fewer VGPRs, which puts
// the tile-edge kernel at two waves per SIMD without scratch
constexpr int DXL_ROWS = 64;
typedef unsigned int TpU2 __attribute__((ext_vector_type(2)));

// NF fields per wave (field group g of a sub-domain = fields g*NF .. g*NF+NF-1, field f
// of the group at qf[f] / fxf[f] / fyf[f] + the group's plane offset); ntg groups
struct TpM {
  Dims d;
  const SubInfo* subs;
  const double* M;
  const double* area4;  // [nsub][4][plane]: the cell area once per level group of a wave
  const double* qf[3];
  double* qo[3];  // TM = 1: the updated delp, w, pt; TM = 2: the updated tracers
  // TM = 2 (tracer_2d_1l update fused): dp1 in, dp2 out (written by field group 0), the
  // per-level sub-step counts and this sub-step (levels with it >= nsplt[k] are copied)
  const double* dp1;
  double* dp2o;
  const int* nsplt;
  int it;
  int nt, nk, ntg;
  const double *crx, *cry, *xfx, *yfx, *mx, *my;
  double* fxf[3];
  double* fyf[3];
  int nz, nseg, seg;
  // the launch's spans (span_enc), by class: nspan[0] one-level spans, then nspan[1] two-level
  // and nspan[2] four-level ones; a wave's span index runs fastest, so the four waves of a
  // workgroup all have work (a workgroup holds its CU slots until its last wave ends)
  int nspan[3];
  int spans[MAXSPAN];
  // TM = 3 (d_sw's ds_uv fused): corner kinetic energy; u, v updated in place
  const double* ke;
  double *uu, *vv;
};

// Wavefront-wide lane shifts through DPP (no LDS): dpp_prev(v) in lane L is v of lane
// L-1 (column x-1), dpp_next(v) is v of lane L+1; the lanes shifted in at the ends read 0.
template <int CTRL>
__device__ __forceinline__ double dpp_shift(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, true);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double dpp_prev(double v) { return dpp_shift<0x138>(v); }  // wave_shr:1
__device__ __forceinline__ double dpp_next(double v) { return dpp_shift<0x130>(v); }  // wave_shl:1

// n / d for several numerators over one denominator: rd = 1 / d (a correctly rounded division,
// once), then per numerator q = n rd and one fused correction, q + (n - d q) rd -- the
// correctly rounded n / d whenever rd is the correctly rounded reciprocal and q is within an
// ulp of n / d (Markstein's theorem; normal-range operands), so the bits of n / d at three
// instructions instead of a full division sequence.  0 mismatches against n / d in 2e8
// random pairs on the host, the march's operand ranges included.
__device__ __forceinline__ double div_rcp(double n, double d, double rd) {
  const double q = n * rd;
  return fma(fma(-d, q, n), rd, q);
}

// PPM split into per-interface and per-cell pieces so neighbours share them (the same
// expressions as ppm_flux, so results are bit-identical):
//   al(g)                 interface value (ppm_al, tile-edge forms near g = 0, N)
//   cell c: bl = al(c) - q, br = al(c+1) - q, b0 = bl + br, s = the ORD smoothness test
//   flux at edge g from cell m = g-1 (upwind for c > 0) and cell 0 = g (c <= 0).
struct PpmCell {
  double q, bl, br, b0;
  bool s;
};
template <int ORD>
__device__ __forceinline__ PpmCell ppm_cell(double q, double al_l, double al_r) {
  PpmCell c;
  c.q = q;
  c.bl = al_l - q;
  c.br = al_r - q;
  c.b0 = c.bl + c.br;
  c.s = ORD == 5 ? c.bl * c.br < 0.0 : 3.0 * fabs(c.b0) < fabs(c.bl - c.br);
  return c;
}
// Both upwind candidates are evaluated and one is selected (no lane-divergent branch:
// neighbouring lanes see Courant numbers of both signs); each candidate is the
// expression of the branch it replaces, so results are unchanged.
__device__ __forceinline__ double ppm_edge_flux(const PpmCell& m, const PpmCell& z, double c) {
  const bool smooth = m.s || z.s;
  const double fm = (1.0 - c) * (m.br - c * m.b0);
  const double fz = (1.0 + c) * (z.bl + c * z.b0);
  const double vm = m.q + (smooth ? fm : 0.0);
  const double vz = z.q + (smooth ? fz : 0.0);
  return c > 0.0 ? vm : vz;
}

// x-PPM flux at the lane's edge (interface g = I, between cells x-1 and x), cells held
// one per lane: the lane computes al at its own interface and its own cell, and takes
// the neighbours' pieces by DPP.  EX: the strip reaches the tile edges (tile-edge al).
template <int ORD, bool EX>
__device__ __forceinline__ double ppm_x_dpp(double q, double dx, int g, int N, double c) {
  const double qm1 = dpp_prev(q), qm2 = dpp_prev(qm1), qp1 = dpp_next(q);
  double al;
  if (EX) {
    // ppm_al with the tile-edge form at g = 0, N, 0.5 * (Q1 + Q2), evaluated with ONE
    // division per lane instead of two: the edge lane divides for Q1 (its cells g-2, g-1)
    // and its right neighbour (g = 1, N+1) divides for the edge lane's Q2 (cells g, g+1,
    // held by that neighbour as its own g-1, g); Q2 then comes back by DPP.  Same operands
    // and operation order as ppm_al, so the same values.  (All DPP outside any
    // lane-divergent branch: every source lane must be active.)
    const double dxm1 = dpp_prev(dx), dxm2 = dpp_prev(dxm1);
    const bool e0 = g == 0 || g == N, e1 = g == 1 || g == N + 1;
    const double num = e0 ? (2.0 * dxm1 + dxm2) * qm1 - dxm1 * qm2 : (2.0 * dxm1 + dx) * qm1 - dxm1 * q;
    const double den = e0 ? dxm2 + dxm1 : dxm1 + dx;
    const double qd = (e0 || e1) ? num / den : 0.0;
    const double q2 = dpp_next(qd);
    if (g == -1 || g == N - 1) al = C1 * qm2 + C2 * qm1 + C3 * q;
    else if (e1) al = C3 * qm1 + C2 * q + C1 * qp1;
    else if (e0) al = 0.5 * (qd + q2);
    else al = P1 * (qm1 + q) + P2 * (qm2 + qp1);
  } else {
    al = P1 * (qm1 + q) + P2 * (qm2 + qp1);
  }
  const double alp = dpp_next(al);
  const PpmCell z = ppm_cell<ORD>(q, al, alp);
  PpmCell m;
  m.q = qm1;
  m.br = dpp_prev(z.br);
  m.b0 = dpp_prev(z.b0);
  m.s = __builtin_amdgcn_update_dpp(0, (int)z.s, 0x138, 0xF, 0xF, true) != 0;
  m.bl = 0.0;  // unused for the cell upwind of a positive Courant number
  return ppm_edge_flux(m, z, c);
}

// everything one row step reads from HBM, prefetched one step ahead
// (ra_x / ra_y are not read: the march forms them from area and the fluxes it already
// holds, ra_x = area + xfx|i - xfx|i+1 (x neighbour by DPP), ra_y = area + yfx|j - yfx|j+1
// (previous row step), the expressions of ds_ra / ra_k / tracer_ra_k; without separate
// mass fluxes (MF = false) mfx, mfy are xfx, yfx and come from registers too)
template <int NF>
struct MarchIn {
  double qx[NF], qy[NF];            // row r, per field (x- / y-corner fill)
  double crx, xfx, area_r, dxr;     // row r
  double cry, yfx, my;              // edge r-2
  double mx, dxm;                   // row r-3
  double dp1;                       // row r-3 (TM = 2)
};

// y-direction PPM state rolled along the march: al at the last interface computed and
// the last cell, so each row step adds one interface value and one cell.
struct YRoll {
  double al;
  PpmCell cell;
};

// TM = 0: fv_tp_2d proper, the NF fields' fluxes fx, fy are written.
// TM = 1: d_sw's thermodynamic transport fused (NF = 3: delp, w, pt): delp's fluxes (mass
//   fluxes xfx / yfx) stay in registers and are the mass fluxes of w and pt at the same
//   edge in the same row step (fv_tp_2d(w | pt, ..., mfx = fx, mfy = fy)); they are
//   accumulated into mfx / mfy (MX / MY planes, read-modify-write: the flux capacitor),
//   and the three fields are updated on row r-3 from the fluxes of its four edges
//   (ds_thermo's expressions) into qo -- no flux plane is written or re-read.
// TM = 2: tracer_2d_1l's update fused (NF tracers with the mass fluxes mfx / mfy): dp2 of
//   row r-3 is formed from the mass fluxes the march holds (tracer_dp2's expression) and the
//   tracers are updated from their outer fluxes (tracer_update's expression) into qo.
// TM = 3: d_sw's vorticity transport with ds_uv fused (NF = 1, no mass fluxes): u on row
//   r-2 takes the outer y flux of that edge, v on row r-3 the outer x flux of that row, with
//   the corner kinetic energy of rows r-3 / r-2 (ds_uv's expressions); no flux plane.
// lv: levels per wave (1, 2, 4: lane group gi of MW / lv lanes runs level k + gi); nvl of
// them exist (a group past the last level repeats level k and stores nothing); the span's
// outputs are columns a0 .. a0 + nout - 1 of every group
template <int ORD, bool EX, bool AHEAD2, bool MF, int NF, int TM>
__device__ void tp_march_strip(const TpM& a, int z, int a0, int nout, int j0, int j1, int lv, int nvl) {
  static_assert(TM == 0 || (TM == 1 && NF == 3 && MF) || (TM == 2 && MF) || ((TM == 3 || TM == 4) && NF == 1 && !MF),
                "thermo march: delp, w, pt with the accumulators as MX / MY; tracer march: mass fluxes; "
                "ds_uv and height marches: one field, no mass fluxes");
  const Dims& d = a.d;
  const int lane = threadIdx.x & (MW - 1);
  const int gw = MW / lv;                     // lanes per level group
  const int gi = lane / gw, hl = lane % gw;   // group, lane within the group's strip
  const bool lvl_ok = gi < nvl;
  const int gl = lvl_ok ? gi : 0;             // the group's level offset
  // z: (sub-domain, level, field group), the field group fastest: the groups of one level
  // share the Courant numbers and fluxes (loaded once per wave for its NF fields), and with
  // the groups of a level adjacent in launch order those planes are re-read from the
  // Infinity Cache, not HBM (54 tracers: 27 groups per level)
  const int tg = z % a.ntg, k = (z / a.ntg) % a.nk, s = z / a.ntg / a.nk;
  const SubInfo sub = a.subs[s];
  const int nx = d.nx, ny = d.ny, N = sub.N;
  const bool last = j1 >= ny;
  const int x = a0 - NG + hl;
  const int I = x + sub.ioff;
  const int xc = x < -NG ? -NG : (x > nx + NG ? nx + NG : x);  // addressable column
  const long pitch = d.pitch;
  const long zo = ((long)(s * a.nt + tg * NF) * a.nk + k) * d.plane, fo = ((long)s * a.nk + k) * d.plane;
  const double* dxa = met(a.M, d, M_DXA, s);
  const double* dya = met(a.M, d, M_DYA, s);
  const bool cin = x >= -NG && x < nx + NG;              // q exists (cell halo)
  // owns an output edge / column (a group past the last level owns nothing)
  const bool out_lane = lvl_ok && hl >= NG && hl < NG + nout;
  const long xo = xc + NG;
  // Buffer descriptors (wave-uniform) for every plane the march reads or writes; a lane
  // addresses column xo of row r with the constant voffset vx and the row offset as the
  // scalar offset, so the loads of a row step cost no vector address arithmetic.
  const int PBy = (int)(d.plane * 8);
  // metric planes: one plane; level fields: the wave's nvl planes
  const int PBf = nvl * PBy;
  auto rsrc = [&](const double* p) { return __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, PBy, 0x00020000); };
  auto rsrcf = [&](const double* p) { return __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, PBf, 0x00020000); };
  __amdgpu_buffer_rsrc_t rQ[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) rQ[f] = rsrcf(a.qf[f] + zo);
  const auto rCRX = rsrcf(a.crx + fo), rCRY = rsrcf(a.cry + fo), rXFX = rsrcf(a.xfx + fo);
  const auto rYFX = rsrcf(a.yfx + fo);
  // the area through the level fields' offset: area4 holds it once per level group
  const auto rMX = rsrcf(a.mx + fo), rMY = rsrcf(a.my + fo), rDXA = rsrc(dxa);
  const auto rAR = __builtin_amdgcn_make_buffer_rsrc((void*)(a.area4 + (long)s * 4 * d.plane), 0, 4 * PBy, 0x00020000);
  const auto rDP1 = rsrcf(TM == 2 ? a.dp1 + fo : a.mx + fo);
  const auto rDP2 = rsrcf(TM == 2 ? a.dp2o + fo : a.mx + fo);
  const bool dp2_group = TM == 2 && tg == 0;  // one field group writes dp2
  // TM = 2, several levels per wave: a group whose level has had its sub-steps carries its
  // tracers (and dp1 as dp2) over unchanged -- the march's own copy of the old values
  const bool tdone = TM == 2 && lv > 1 && a.it >= a.nsplt[k + gl];
  // TM = 3: ke, u, v (level fields), dx, dy (metric planes)
  const auto rKE = rsrcf(TM == 3 ? a.ke + fo : a.crx + fo), rU = rsrcf(TM == 3 ? a.uu + fo : a.crx + fo);
  const auto rV = rsrcf(TM == 3 ? a.vv + fo : a.crx + fo);
  const auto rDX = rsrc(met(a.M, d, M_DX, s)), rDY = rsrc(met(a.M, d, M_DY, s));
  const uint32_t vx = (uint32_t)xo * 8u;  // metric planes
  const uint32_t vf = vx + (uint32_t)gl * (uint32_t)PBy;  // level fields
  // dxa only enters the tile-edge interface values (ppm_al at g = 0, N reads the four
  // cells g-2 .. g+1): the other lanes read one shared word instead of their own column
  const bool dx_lane = (I >= -2 && I <= 1) || (I >= N - 2 && I <= N + 1);
  const uint32_t vxd = dx_lane ? vx : 0u;
  const uint32_t rowb = (uint32_t)pitch * 8u;
  constexpr bool DXL = EX && TM == 1;
  const int r_lo = j0 - NG, r_hi = j1 + 2;
  // DXL: rows rb .. rb+DXL_ROWS-1 of the tile-edge columns' dxa (every row a step reads:
  // r_lo-3 .. r_hi+1, clamped to the plane) at sdx[wave][row - rb][slot]
  __shared__ double sdx[DXL ? MWAVES * DXL_ROWS * 8 : 1];
  const int rb = r_lo - 3 > -NG ? r_lo - 3 : -NG;
  const int dslot = I <= 1 ? I + 2 : I - (N - 2) + 4;
  double* const sdw = sdx + (DXL ? (threadIdx.x / MW) * DXL_ROWS * 8 + dslot : 0);
  if constexpr (DXL) {
    const int rt = r_hi + 1 < ny + NG ? r_hi + 1 : ny + NG;
    // sixteen rows' loads in flight at once, then their LDS writes (one row per round trip
    // was ~50 dependent L2 / HBM latencies at the start of every tile-edge wave)
    if (dx_lane)
      for (int r0 = rb; r0 <= rt; r0 += 16) {
        double v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int rr = r0 + u <= rt ? r0 + u : rt;
          v[u] = dxa[(long)(rr + NG) * pitch + xo];
        }
#pragma unroll
        for (int u = 0; u < 16; ++u)
          if (r0 + u <= rt) sdw[(r0 + u - rb) * 8] = v[u];
      }
    __builtin_amdgcn_wave_barrier();
  }
  // dxa of row r (clamped as the loads clamp) for the tile-edge PPM forms
  auto dxl = [&](int r) {
    const int rr = r < -NG ? -NG : (r > ny + NG ? ny + NG : r);
    return dx_lane ? sdw[(rr - rb) * 8] : 0.0;
  };
  auto bl = [&](__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
  };

  // Every load below is issued unconditionally (addresses clamped into the plane,
  // values masked afterwards): with a fixed count of loads per step the compiler's
  // vmcnt bookkeeping lets the next step's prefetch stay in flight across this step.
  auto load = [&](int r) {
    MarchIn<NF> v;
    const int rr = r < ny + NG ? r : ny + NG;  // last plane row
    const uint32_t so = (uint32_t)(rr + NG) * rowb;
    const int J = r + sub.joff;
    const bool qin = cin && r >= -NG && r < ny + NG;
    if (EX && (J < 0 || J >= N)) {  // cube-corner halo cells read the copy_corners source
      const bool cc = qin && (I < 0 || I >= N);
      const uint32_t hof = vf - vx;
      const uint32_t ox = cc ? (uint32_t)cc_off(d, sub, x, r, 1) * 8u + hof : vf + so;
      const uint32_t oy = cc ? (uint32_t)cc_off(d, sub, x, r, 2) * 8u + hof : vf + so;
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        const double q1 = bl(rQ[f], ox, 0), q2 = bl(rQ[f], oy, 0);
        v.qx[f] = qin ? q1 : 0.0;
        v.qy[f] = qin ? q2 : 0.0;
      }
    } else {
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        const double q1 = bl(rQ[f], vf, so);
        v.qx[f] = qin ? q1 : 0.0;
        v.qy[f] = v.qx[f];
      }
    }
    v.crx = bl(rCRX, vf, so);
    v.xfx = bl(rXFX, vf, so);
    v.area_r = bl(rAR, vf, so);
    v.dxr = EX && !DXL ? bl(rDXA, vxd, so) : 0.0;
    const int re = r - 2 < -NG ? -NG : r - 2;
    const uint32_t se = (uint32_t)(re + NG) * rowb;
    v.cry = bl(rCRY, vf, se);
    v.yfx = bl(rYFX, vf, se);
    v.my = MF ? bl(rMY, vf, se) : 0.0;
    const int rm = r - 3 < -NG ? -NG : r - 3;
    const uint32_t sm = (uint32_t)(rm + NG) * rowb;
    v.mx = MF ? bl(rMX, vf, sm) : 0.0;
    v.dxm = EX && !DXL ? bl(rDXA, vxd, sm) : 0.0;
    v.dp1 = TM == 2 ? bl(rDP1, vf, sm) : 0.0;
    return v;
  };

  // al at interface g = r-1 (global G) from rows r-3 .. r of a column window
  auto y_al = [&](const double* w, int G, long o_r) {
    if (G == 0 || G == N) {
      double dv[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) dv[m] = dya[o_r + (m - 3) * pitch];
      return ppm_al(G, N, w, dv);
    }
    if (G == -1 || G == N - 1 || G == 1 || G == N + 1) return ppm_al(G, N, w, w);
    return P1 * (w[1] + w[2]) + P2 * (w[0] + w[3]);
  };

  double qyw[NF][4], qjw[NF][4];  // rows r-3 .. r
  double hf2[NF][4], hcx[4];      // fx2 and crx of rows r-3 .. r
  double arw[4];                  // cell area of rows r-3 .. r (read once per row)
  double hxf[4];                  // xfx of rows r-3 .. r (the mass flux mfx when MF = false)
  YRoll ry[NF], rj[NF];           // q (y fill) and q_j
  double fyy_prev[NF];
  double fyo_prev[NF];            // TM = 1, 2: outer y flux of edge r-3
  double my_prev = 0.0;           // TM = 2: mfy of edge r-3
#pragma unroll
  for (int m = 0; m < 4; ++m) hcx[m] = arw[m] = hxf[m] = 0.0;
#pragma unroll
  for (int f = 0; f < NF; ++f) {
#pragma unroll
    for (int m = 0; m < 4; ++m) qyw[f][m] = qjw[f][m] = hf2[f][m] = 0.0;
    ry[f] = YRoll{};
    rj[f] = YRoll{};
    fyy_prev[f] = 0.0;
    fyo_prev[f] = 0.0;
  }
  double yfx_prev = 0.0;  // yfx at edge r-3 (the previous row step's edge r-2)
  double ke_m = 0.0;      // TM = 3: ke of row r-3 (the previous row step's row r-2)

  // lane predicates (constant along the march)
  const bool l_fx2 = x >= 0 && x <= nx, l_qj = x >= 0 && x < nx;
  const bool l_fy2 = x >= -NG && x <= nx + NG - 1;
  const bool s_fy = out_lane && x < nx, s_fx = out_lane && x <= nx;
  __amdgpu_buffer_rsrc_t rFX[NF], rFY[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    if (TM == 0) {
      rFX[f] = rsrcf(a.fxf[f] + zo);
      rFY[f] = rsrcf(a.fyf[f] + zo);
    } else if (TM == 1) {
      rFX[f] = rsrcf(a.qo[f] + fo);  // updated field f (TM = 1 groups are one field each)
    } else {
      rFX[f] = rsrcf(a.qo[f] + zo);  // updated tracer f of the group
    }
  }
  auto bst = [&](__amdgpu_buffer_rsrc_t r, uint32_t soff, double v) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(TpU2, v), r, vf, soff, 0);
  };
  // lane-predicated store without a branch: a lane that must not store addresses past the
  // end of the plane (the descriptor's range check drops the write), so the steady rows
  // stay one basic block the scheduler can interleave across the three unrolled rows
  constexpr uint32_t OOB = 0x80000000u;
  const uint32_t vfy = s_fy ? vf : OOB, vfx = s_fx ? vf : OOB;
  auto bstv = [&](__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, double v) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(TpU2, v), r, voff, soff, 0);
  };

  // One row step.  GEN: the generic step (row clamps, segment ends, tile-edge rows of the
  // y interpolant, cube-corner fills); steady rows (most of a segment) need none of those
  // checks, so their step is branch-free apart from the two output stores.
  // steady load of the step for row rl (rows rl, rl-2, rl-3 inside the plane, away
  // from the cube corners)
  auto load_steady = [&](int rl, MarchIn<NF>& nxt) {
      const uint32_t so = (uint32_t)(rl + NG) * rowb;
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        nxt.qx[f] = bl(rQ[f], vf, so);
        if (!cin) nxt.qx[f] = 0.0;
        nxt.qy[f] = nxt.qx[f];
      }
      nxt.crx = bl(rCRX, vf, so);
      nxt.xfx = bl(rXFX, vf, so);
      nxt.area_r = bl(rAR, vf, so);
      nxt.dxr = EX && !DXL ? bl(rDXA, vxd, so) : 0.0;
      const uint32_t se = so - 2 * rowb, sm = so - 3 * rowb;
      nxt.cry = bl(rCRY, vf, se);
      nxt.yfx = bl(rYFX, vf, se);
      nxt.my = MF ? bl(rMY, vf, se) : 0.0;
      nxt.mx = MF ? bl(rMX, vf, sm) : 0.0;
      nxt.dxm = EX && !DXL ? bl(rDXA, vxd, sm) : 0.0;
      nxt.dp1 = TM == 2 ? bl(rDP1, vf, sm) : 0.0;
  };
  // ahead: how many rows ahead the steady step prefetches (1, or 2 in the three-buffer loop)
  auto step = [&](auto gen, int r, const MarchIn<NF>& cur, MarchIn<NF>& nxt, int ahead) {
    constexpr bool GEN = decltype(gen)::value;
    if (GEN) nxt = load(r + 1);
    else load_steady(r + ahead, nxt);
    // TM = 3: this step's ke / u / dx (row r-2) and v / dy (row r-3), issued here so their
    // latency overlaps the step's PPM work (not prefetched: three row buffers would cost the
    // march its third wave per SIMD)
    double t_ke = 0.0, t_u = 0.0, t_dx = 0.0, t_v = 0.0, t_dy = 0.0;
    if constexpr (TM == 3) {
      const int re = r - 2 < -NG ? -NG : r - 2, rm = r - 3 < -NG ? -NG : r - 3;
      const uint32_t se3 = (uint32_t)(re + NG) * rowb, sm3 = (uint32_t)(rm + NG) * rowb;
      t_ke = bl(rKE, vf, se3);
      t_u = bl(rU, vf, se3);
      t_dx = bl(rDX, vx, se3);
      t_v = bl(rV, vf, sm3);
      t_dy = bl(rDY, vx, sm3);
    }
    const long o = (long)(r + NG) * pitch + xo;
    const double rax = cur.area_r + cur.xfx - dpp_next(cur.xfx);
    // ---- row r: inner x flux fx2, q_j (per field)
    double fx2[NF], qj[NF];
    const double rrax = NF > 1 ? 1.0 / rax : 0.0;
    const double dxr = DXL ? dxl(r) : cur.dxr, dxm = DXL ? dxl(r - 3) : cur.dxm;
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      {
        const double v = ppm_x_dpp<ORD, EX>(cur.qx[f], dxr, I, N, cur.crx);
        const bool ok = GEN ? l_fx2 && r >= -NG && r <= ny + NG - 1 : l_fx2;
        fx2[f] = ok ? v : 0.0;
      }
      const double fxx = cur.xfx * fx2[f];
      const double fxx_e = dpp_next(fxx);
      const double nxq = cur.qx[f] * cur.area_r + fxx - fxx_e;
      const double v = NF > 1 ? div_rcp(nxq, rax, rrax) : nxq / rax;
      const bool ok = GEN ? l_qj && r >= -NG && r < ny + NG : l_qj;
      qj[f] = ok ? v : 0.0;
    }
#pragma unroll
    for (int m = 0; m < 3; ++m) {
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        qyw[f][m] = qyw[f][m + 1];
        qjw[f][m] = qjw[f][m + 1];
        hf2[f][m] = hf2[f][m + 1];
      }
      hcx[m] = hcx[m + 1];
      arw[m] = arw[m + 1];
      hxf[m] = hxf[m + 1];
    }
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      qyw[f][3] = cur.qy[f];
      qjw[f][3] = qj[f];
      hf2[f][3] = fx2[f];
    }
    hcx[3] = cur.crx;
    arw[3] = cur.area_r;
    hxf[3] = cur.xfx;
    const double my = MF ? cur.my : cur.yfx, mx = MF ? cur.mx : hxf[0];

    // ---- y PPM pieces: interface r-1, cell r-2 (both windows, per field)
    const int e = r - 2;
    PpmCell cy[NF], cj[NF], cym[NF], cjm[NF];
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      double aly, alj;
      if (GEN) {
        const int E = e + sub.joff;
        aly = y_al(qyw[f], E + 1, o);
        alj = y_al(qjw[f], E + 1, o);
      } else {
        aly = P1 * (qyw[f][1] + qyw[f][2]) + P2 * (qyw[f][0] + qyw[f][3]);
        alj = P1 * (qjw[f][1] + qjw[f][2]) + P2 * (qjw[f][0] + qjw[f][3]);
      }
      cy[f] = ppm_cell<ORD>(qyw[f][1], ry[f].al, aly);
      cj[f] = ppm_cell<ORD>(qjw[f][1], rj[f].al, alj);
      cym[f] = ry[f].cell;
      cjm[f] = rj[f].cell;
      ry[f].al = aly;
      ry[f].cell = cy[f];
      rj[f].al = alj;
      rj[f].cell = cj[f];
    }

    if (!GEN || e >= j0) {
      const uint32_t se = (uint32_t)(e + NG) * rowb;
      const int mrow = r - 3;
      const double ray = arw[0] + yfx_prev - cur.yfx;
      const double rray = NF > 1 ? 1.0 / ray : 0.0;
      const bool rowm = !GEN || (mrow >= j0 && mrow < ny);  // wave-uniform
      double fyo[NF], fxo[NF];
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        // ---- edge e: inner y flux fy2, outer y flux fy
        double fy2 = ppm_edge_flux(cym[f], cy[f], cur.cry);
        if (!(GEN ? e <= ny && l_fy2 : l_fy2)) fy2 = 0.0;
        const double fyy = !GEN || e <= ny ? cur.yfx * fy2 : 0.0;
        // TM = 1: w and pt take delp's flux (field 0, this edge) as their mass flux
        const double myf = TM == 1 ? (f == 0 ? cur.yfx : fyo[0]) : my;
        fyo[f] = 0.5 * (ppm_edge_flux(cjm[f], cj[f], cur.cry) + fy2) * myf;
        if (TM == 0) {
          if (GEN) {
            if (s_fy && e <= ny && (e < j1 || last)) bst(rFY[f], se, fyo[f]);
          } else {
            bstv(rFY[f], vfy, se, fyo[f]);
          }
        }
        // ---- row m = r-3: q_i, outer x flux fx
        if (rowm) {
          const double ny_ = qyw[f][0] * arw[0] + fyy_prev[f] - fyy;
          const double v = NF > 1 ? div_rcp(ny_, ray, rray) : ny_ / ray;
          const double qi = cin ? v : 0.0;
          const double fo_ = ppm_x_dpp<ORD, EX>(qi, dxm, I, N, hcx[0]);
          const double mxf = TM == 1 ? (f == 0 ? hxf[0] : fxo[0]) : mx;
          fxo[f] = 0.5 * (fo_ + hf2[f][0]) * mxf;
          if (TM == 0) {
            if (GEN) {
              if (s_fx && mrow < j1) bst(rFX[f], se - rowb, fxo[f]);
            } else {
              bstv(rFX[f], vfx, se - rowb, fxo[f]);
            }
          }
        }
        fyy_prev[f] = fyy;
      }
      if constexpr (TM == 3) {
        // ds_uv: u on edge e with this edge's outer y flux, v on row m with this row's outer
        // x flux; ke of row m (carried from the previous step) and row e, x neighbour by DPP;
        // ds_uv's expressions and order
        const double ke_e1 = dpp_next(t_ke);
        const double un = t_u * t_dx + t_ke - ke_e1 + fyo[0];
        if (GEN) {
          if (s_fy && e <= ny && (e < j1 || last)) bst(rU, se, un);
        } else {
          bstv(rU, vfy, se, un);
        }
        if (rowm) {
          const double vn = t_v * t_dy + ke_m - t_ke - fxo[0];
          if (GEN) {
            if (s_fx && mrow < j1) bst(rV, se - rowb, vn);
          } else {
            bstv(rV, vfx, se - rowb, vn);
          }
        }
      }
      if constexpr (TM == 1) {
        // flux capacitor (ds_accum): mfy on edge e, mfx on row m (cur.my / cur.mx hold them)
        if (GEN) {
          if (s_fy && e <= ny && (e < j1 || last)) bst(rMY, se, cur.my + fyo[0]);
        } else {
          bstv(rMY, vfy, se, cur.my + fyo[0]);
        }
        if (rowm) {
          if (GEN) {
            if (s_fx && mrow < j1) bst(rMX, se - rowb, cur.mx + fxo[0]);
          } else {
            bstv(rMX, vfx, se - rowb, cur.mx + fxo[0]);
          }
          // ds_thermo on row m: flux differences of the cell's four edges (x neighbour by
          // DPP, edge m from the previous row step), same expressions and order
          const double ra = 1.0 / arw[0];  // == rarea (grid.cpp: 1 / area, both IEEE)
          double num[NF];
#pragma unroll
          for (int f = 0; f < NF; ++f) num[f] = fxo[f] - dpp_next(fxo[f]) + fyo_prev[f] - fyo[f];
          const double dp = qyw[0][0];
          const double dpn = dp + num[0] * ra;
          const double wn = dp * qyw[1][0] + num[1] * ra;
          const double ptn = qyw[2][0] * dp + num[2] * ra;
          const double rdpn = 1.0 / dpn;
          const double wq = div_rcp(wn, dpn, rdpn), ptq = div_rcp(ptn, dpn, rdpn);
          if (GEN) {
            if (s_fy && mrow < j1) {
              bst(rFX[0], se - rowb, dpn);
              bst(rFX[1], se - rowb, wq);
              bst(rFX[2], se - rowb, ptq);
            }
          } else {
            bstv(rFX[0], vfy, se - rowb, dpn);
            bstv(rFX[1], vfy, se - rowb, wq);
            bstv(rFX[2], vfy, se - rowb, ptq);
          }
        }
#pragma unroll
        for (int f = 0; f < NF; ++f) fyo_prev[f] = fyo[f];
      }
      if constexpr (TM == 2) {
        if (rowm) {
          // tracer_dp2 then tracer_update on row m (same expressions and order)
          const double ra = 1.0 / arw[0];  // == rarea
          const double dp1 = cur.dp1;
          const double dp2 = dp1 + (cur.mx - dpp_next(cur.mx) + my_prev - cur.my) * ra;
          double qn[NF];
          const double rdp2 = NF > 1 ? 1.0 / dp2 : 0.0;
#pragma unroll
          for (int f = 0; f < NF; ++f) {
            const double nq = qyw[f][0] * dp1 + (fxo[f] - dpp_next(fxo[f]) + fyo_prev[f] - fyo[f]) * ra;
            qn[f] = NF > 1 ? div_rcp(nq, dp2, rdp2) : nq / dp2;
            if (tdone) qn[f] = qyw[f][0];
          }
          const double dp2o = tdone ? dp1 : dp2;
          if (GEN) {
            if (s_fy && mrow < j1) {
#pragma unroll
              for (int f = 0; f < NF; ++f) bst(rFX[f], se - rowb, qn[f]);
              if (dp2_group) bst(rDP2, se - rowb, dp2o);
            }
          } else {
#pragma unroll
            for (int f = 0; f < NF; ++f) bstv(rFX[f], vfy, se - rowb, qn[f]);
            if (dp2_group) bstv(rDP2, vfy, se - rowb, dp2o);
          }
        }
#pragma unroll
        for (int f = 0; f < NF; ++f) fyo_prev[f] = fyo[f];
        my_prev = cur.my;
      }
      if constexpr (TM == 4) {
        if (rowm) {
          // zh_update on row m (same expressions and order): the x fluxes of the cell's two
          // edges (x neighbour by DPP), the y fluxes of edges m (previous step) and m + 1, the
          // area fluxes xfx of row m and yfx of edges m, m + 1
          const double area = arw[0];
          const double rxm = area + hxf[0] - dpp_next(hxf[0]);
          const double fxe = dpp_next(fxo[0]);
          const double zn = (qyw[0][0] * area + fxo[0] - fxe + fyo_prev[0] - fyo[0]) / (rxm + ray - area);
          if (GEN) {
            if (s_fy && mrow < j1) bst(rFX[0], se - rowb, zn);
          } else {
            bstv(rFX[0], vfy, se - rowb, zn);
          }
        }
        fyo_prev[0] = fyo[0];
      }
    }
    yfx_prev = cur.yfx;
    if constexpr (TM == 3) ke_m = t_ke;
  };

  // steady rows: 2 <= G <= N-2 for the y interpolant's interface G = r-1, rows r+1 (the
  // prefetch), r-2, r-3 inside the plane and the tile (no corner fills), edge e = r-2 and
  // row r-3 inside the segment's outputs
  int rs0 = j0 + 3, rs1 = j1 + 1;  // [rs0, rs1] candidate steady rows
  rs0 = rs0 > 3 - sub.joff ? rs0 : 3 - sub.joff;
  rs1 = rs1 < N - 2 - sub.joff ? rs1 : N - 2 - sub.joff;
  rs1 = rs1 < ny + NG - 2 ? rs1 : ny + NG - 2;
  if (rs1 < rs0) rs1 = rs0 - 1;
  const std::integral_constant<bool, true> G1{};
  const std::integral_constant<bool, false> G0{};
  MarchIn<NF> cur = load(r_lo), nxt;
  int r = r_lo;
  for (; r < rs0; ++r) {
    step(G1, r, cur, nxt, 1);
    cur = nxt;
  }
  // steady rows whose two-ahead loads stay in the steady range: three rotating buffers,
  // each step prefetching two rows ahead (one more step of HBM latency covered)
  // steady rows hold no cube-corner fill, so their x- and y-filled q are one value: with
  // that stated at the loop entry the loop carries one register set for both
  if (r <= rs1) {
#pragma unroll
    for (int f = 0; f < NF; ++f) cur.qy[f] = cur.qx[f];
  }
  {
    const int lmax = ny + NG - 1 < N - 1 - sub.joff ? ny + NG - 1 : N - 1 - sub.joff;
    const int rs1b = rs1 < lmax - 2 ? rs1 : lmax - 2;
    if (AHEAD2 && r + 2 <= rs1b) {
      MarchIn<NF> b0 = cur, b1, b2;
      load_steady(r + 1, b1);
      for (; r + 2 <= rs1b; r += 3) {
        step(G0, r, b0, b2, 2);
        step(G0, r + 1, b1, b0, 2);
        step(G0, r + 2, b2, b1, 2);
      }
      cur = b0;
    }
  }
  for (; r <= rs1; ++r) {
    step(G0, r, cur, nxt, 1);
    cur = nxt;
  }
  for (; r <= r_hi; ++r) {
    step(G1, r, cur, nxt, 1);
    cur = nxt;
  }
}

// AHEAD2: steady rows prefetch two rows ahead (three row buffers, 149 VGPRs, three
// waves per SIMD); otherwise one row ahead (two buffers, <= 128 VGPRs, four waves)
// copy of the strip's output cells of rows [j0, j1) from the tracers to qo (and dp1 to dp2)
template <int NF>
__device__ void tracer_carry(const TpM& a, int z, int a0, int nout, int j0, int j1) {
  const Dims& d = a.d;
  const int lane = threadIdx.x & (MW - 1);
  const int tg = z % a.ntg, k = (z / a.ntg) % a.nk, s = z / a.ntg / a.nk;
  const int x = a0 - NG + lane;
  if (!(lane >= NG && lane < NG + nout && x < d.nx)) return;
  const long zo = ((long)(s * a.nt + tg * NF) * a.nk + k) * d.plane, fo = ((long)s * a.nk + k) * d.plane;
  const long tstride = (long)a.nk * d.plane;
  const double* __restrict__ qi = a.qf[0] + zo;
  double* __restrict__ qo = a.qo[0] + zo;
  const double* __restrict__ di = a.dp1 + fo;
  double* __restrict__ dout = a.dp2o + fo;
  // four rows' loads in flight before their stores (the planes do not overlap)
  for (int j = j0; j < j1; j += 4) {
    double v[4][NF], w[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long o = (long)((j + u < j1 ? j + u : j1 - 1) + NG) * d.pitch + x + NG;
#pragma unroll
      for (int f = 0; f < NF; ++f) v[u][f] = qi[f * tstride + o];
      w[u] = tg == 0 ? di[o] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (j + u >= j1) break;
      const long o = (long)(j + u + NG) * d.pitch + x + NG;
#pragma unroll
      for (int f = 0; f < NF; ++f) qo[f * tstride + o] = v[u][f];
      if (tg == 0) dout[o] = w[u];
    }
  }
}

// OCC: minimum workgroups per CU the register budget must allow (0: 1 with AHEAD2, else 4)
// EXS: 1 = only the strips reaching a tile edge (tile-edge PPM forms), 2 = only interior
// strips (fewer registers, so more waves per SIMD), 0 = both; the other waves leave at once
template <int ORD, bool AHEAD2, bool MF, int NF, int TM = 0, int OCC = 0, int EXS = 0>
__global__ void __launch_bounds__(MW * MWAVES, OCC ? OCC : (AHEAD2 ? 1 : 4)) tp_march(TpM a) {
  // wave index through readfirstlane: everything derived from it (plane, strip, segment,
  // buffer descriptors, row offsets) is then provably wave-uniform (SGPRs, no waterfalls)
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / MW);
  unsigned w = blockIdx.x * MWAVES + wv;  // < 2^31 (launch_tp checks)
  // span class (levels per wave 1, 2, 4), then field group (fastest), span, segment, level
  // slot: the groups of one (span, segment, level) are neighbouring waves of one workgroup, so
  // the Courant / flux rows they all read come from HBM once (one CU's L1, one XCD's L2)
  // instead of once per group on different XCDs
  // (the four-level spans first: their waves take the longest, so they start in the first
  // round instead of trailing the launch)
  int cls = 2, first = a.nspan[0] + a.nspan[1];
  for (; cls >= 0; --cls) {
    const unsigned slots = (unsigned)((a.nk + (1 << cls) - 1) >> cls);
    const unsigned nw = (unsigned)a.nspan[cls] * (unsigned)a.nseg * (unsigned)a.ntg * slots;
    if (w < nw) break;
    w -= nw;
    if (cls > 0) first -= a.nspan[cls - 1];
  }
  if (cls < 0) return;  // whole wavefront leaves; no workgroup barrier follows
  const int tg = (int)(w % (unsigned)a.ntg);
  unsigned t = w / (unsigned)a.ntg;
  const unsigned p = t % (unsigned)a.nspan[cls];
  t /= (unsigned)a.nspan[cls];
  const int seg = (int)(t % (unsigned)a.nseg);
  const int k = (int)(t / (unsigned)a.nseg) << cls;
  const int e = a.spans[first + (int)p];
  const int s = span_s(e), a0 = span_a0(e), nout = span_nout(e);
  const bool ex = span_ex(e);
  const int lv = 1 << cls, nvl = a.nk - k < lv ? a.nk - k : lv;
  const int z = (s * a.nk + k) * a.ntg + tg;
  const int j0 = seg * a.seg;
  const int j1 = j0 + a.seg < a.d.ny ? j0 + a.seg : a.d.ny;
  if constexpr (TM == 2) {
    // tracer sub-steps past this level's count: the level's tracers carry over unchanged
    // (several levels per wave: per group, inside the march)
    if (lv == 1 && a.it >= a.nsplt[k]) {
      tracer_carry<NF>(a, z, a0, nout, j0, j1);
      return;
    }
  }
  if constexpr (EXS == 1) {
    if (ex) tp_march_strip<ORD, true, AHEAD2, MF, NF, TM>(a, z, a0, nout, j0, j1, lv, nvl);
  } else if constexpr (EXS == 2) {
    if (!ex) tp_march_strip<ORD, false, AHEAD2, MF, NF, TM>(a, z, a0, nout, j0, j1, lv, nvl);
  } else {
    if (ex) tp_march_strip<ORD, true, AHEAD2, MF, NF, TM>(a, z, a0, nout, j0, j1, lv, nvl);
    else tp_march_strip<ORD, false, AHEAD2, MF, NF, TM>(a, z, a0, nout, j0, j1, lv, nvl);
  }
}

// The output spans of every local sub-domain (see MAXSPAN): tile-edge spans [0, 2] at a west
// tile edge and [nx-3, nx] at an east one, interior strips of MOUT outputs between them (a
// sub-domain too narrow for both runs one tile-edge span over all its outputs).  `ex` /
// `in` receive the spans of each form.  Returns the tile-edge spans' share of the outputs.
double plan_spans(const Ctx& c, std::vector<int>& ex, std::vector<int>& in) {
  const Dims& d = c.d;
  long nex = 0, nall = 0;
  if (d.nx + 1 > 4095) throw std::runtime_error("fv_tp_2d: sub-domain too wide for the span encoding");
  for (int s = 0; s < d.nsub; ++s) {
    const SubInfo& h = c.hsubs[s];
    const bool we = h.ioff == 0, ee = h.ioff + d.nx == h.N;
    int lo = we ? 3 : 0, hi = ee ? d.nx - 4 : d.nx;
    nall += d.nx + 1;
    if (hi < lo) {
      if (d.nx + 1 > MOUT) throw std::runtime_error("fv_tp_2d: no span plan for this sub-domain");
      ex.push_back(span_enc(s, true, 0, d.nx + 1));
      nex += d.nx + 1;
      continue;
    }
    if (we) {
      ex.push_back(span_enc(s, true, 0, 3));
      nex += 3;
    }
    for (int a0 = lo; a0 <= hi; a0 += MOUT) in.push_back(span_enc(s, false, a0, std::min(MOUT, hi - a0 + 1)));
    if (ee) {
      ex.push_back(span_enc(s, true, d.nx - 3, 4));
      nex += 4;
    }
  }
  return (double)nex / (double)nall;
}

// fill m's span list from `spans` (any order; sorted into the three classes); returns the
// launch's wave count
long set_spans(TpM& m, const std::vector<int>& spans) {
  if ((int)spans.size() > MAXSPAN) throw std::runtime_error("fv_tp_2d: too many spans for one launch");
  auto cls_of = [](int e) { return span_class(span_nout(e)); };
  int n = 0;
  for (int cls = 0; cls < 3; ++cls) {
    m.nspan[cls] = 0;
    for (int e : spans)
      if (cls_of(e) == cls) {
        m.spans[n++] = e;
        ++m.nspan[cls];
      }
  }
  long waves = 0;
  for (int cls = 0; cls < 3; ++cls)
    waves += (long)m.nspan[cls] * m.nseg * m.ntg * ((m.nk + (1 << cls) - 1) >> cls);
  if (waves >= (1L << 31)) throw std::runtime_error("fv_tp_2d: too many strips for one launch");
  return waves;
}

// waves per (sub-domain, level, field group) plane of a span list: the segment heuristic's
// strip count
double span_waves_per_plane(const std::vector<int>& spans, int nsub) {
  double w = 0.0;
  for (int e : spans) w += 1.0 / (1 << span_class(span_nout(e)));
  return w / nsub;
}

// One march as two kernels: the tile-edge spans (EX forms, their register count) and the
// interior strips (A2_IN prefetch depth, OCC_IN workgroups per CU).  Each launch registers its
// share of the algorithmic bytes (by output columns).
template <int ORD, bool MF, int NF, int TM, int OCC_IN, bool A2_IN, int OCC_EX = 0, bool A2_EX = true>
void march2(const Ctx& c, const TpM& m0, double bytes, const char* name_ex, const char* name_in) {
  std::vector<int> pex, pin;
  const double fex = plan_spans(c, pex, pin);
  // (shorter segments for the tile-edge launch, 15 or 23 rows against the interior's 45,
  // measured 32.12 / 32.02 against 32.00 ms per step: not kept)
  // a launch carries at most MAXSPAN spans in its arguments; more (many sub-domains in one
  // process: C720 at 1x4 is 24 x 15) go as consecutive launches of disjoint spans
  auto go = [&](const std::vector<int>& pr, bool ex, hipStream_t st) {
    for (size_t b0 = 0; b0 < pr.size(); b0 += MAXSPAN) {
      const std::vector<int> part(pr.begin() + b0, pr.begin() + std::min(pr.size(), b0 + MAXSPAN));
      TpM m = m0;
      const long waves = set_spans(m, part);
      const dim3 g(cdiv(waves, MWAVES)), b(MW * MWAVES);
      if (ex) GT_LAUNCH_N(name_ex, (tp_march<ORD, A2_EX, MF, NF, TM, OCC_EX, 1>), g, b, 0, st, m);
      else GT_LAUNCH_N(name_in, (tp_march<ORD, A2_IN, MF, NF, TM, OCC_IN, 2>), g, b, 0, st, m);
      HIP_LAUNCH_CHECK();
    }
  };
  // The tile-edge kernel's few waves (one per SIMD at most, ~1000 at C180) each march a whole
  // segment: alone, the chip idles behind them for its length.  With a side stream (Ctx::side)
  // it runs there, beside the interior kernel (disjoint outputs and accumulator points).
  const bool side = c.side && !pex.empty() && !pin.empty();
  if (side) {
    HIP_CHECK(hipEventRecord(c.side_fork, c.st));
    HIP_CHECK(hipStreamWaitEvent(c.side, c.side_fork, 0));
  }
  if (!pex.empty()) {
    go(pex, true, side ? c.side : c.st);
    ktimer_bytes(bytes * fex);
  }
  if (!pin.empty()) {
    go(pin, false, c.st);
    ktimer_bytes(bytes * (1.0 - fex));
  }
  if (side) {
    HIP_CHECK(hipEventRecord(c.side_join, c.side));
    HIP_CHECK(hipStreamWaitEvent(c.st, c.side_join, 0));
  }
}

// ---------------- tracer_2d_1l ----------------

__device__ __forceinline__ void atomic_max_pos(double* addr, double v) {
  // non-negative doubles order like their bit patterns
  atomicMax(reinterpret_cast<unsigned long long*>(addr), (unsigned long long)__double_as_longlong(v));
}

// Each thread walks TP_RPT rows so one workgroup covers 4*TP_RPT rows of the plane:
// the per-level Courant maximum then costs one atomic per workgroup (a few per level
// and sub-domain) instead of one per wavefront.
constexpr int TP_RPT = 12;
__global__ void __launch_bounds__(256) tracer_prep_k(Dims d, const double* __restrict__ M, int npz,
                                                     const double* __restrict__ cx, const double* __restrict__ cy,
                                                     double* __restrict__ xfx, double* __restrict__ yfx,
                                                     double* __restrict__ cmax) {
  __shared__ double wmax[4];
  const int z = blockIdx.z, k = z % npz, s = z / npz;
  const long fo = (long)z * d.plane;
  const int i = blockIdx.x * BX + threadIdx.x - NG;
  const double* dxa = met(M, d, M_DXA, s);
  const double* dya = met(M, d, M_DYA, s);
  const double* dx = met(M, d, M_DX, s);
  const double* dy = met(M, d, M_DY, s);
  double cm = 0.0;
  for (int rr = 0; rr < TP_RPT; ++rr) {
    const int j = (blockIdx.y * TP_RPT + rr) * BY + threadIdx.y - NG;
    if (i > d.nx + NG || j > d.ny + NG) continue;
    const long o = pidx(d, i, j);
    if (i >= 0 && i <= d.nx && j >= -NG && j <= d.ny + NG - 1) {
      double c = cx[fo + o];
      double v;
      if (c > 0.0)
        v = c * dxa[pidx(d, i - 1, j)] * dy[o] * met(M, d, M_SIN3, s)[pidx(d, i - 1, j)];
      else
        v = c * dxa[o] * dy[o] * met(M, d, M_SIN1, s)[o];
      xfx[fo + o] = v;
    }
    if (j >= 0 && j <= d.ny && i >= -NG && i <= d.nx + NG - 1) {
      double c = cy[fo + o];
      double v;
      if (c > 0.0)
        v = c * dya[pidx(d, i, j - 1)] * dx[o] * met(M, d, M_SIN4, s)[pidx(d, i, j - 1)];
      else
        v = c * dya[o] * dx[o] * met(M, d, M_SIN2, s)[o];
      yfx[fo + o] = v;
    }
    if (i >= 0 && i < d.nx && j >= 0 && j < d.ny) {
      double a = fmax(fabs(cx[fo + o]), fabs(cy[fo + o]));
      if (!(k + 1 < npz / 6)) a = a + 1.0 - met(M, d, M_SIN5, s)[o];
      cm = fmax(cm, a);
    }
  }
  // wave reduction, workgroup reduction, one atomic per workgroup
  for (int off = 32; off > 0; off >>= 1) cm = fmax(cm, __shfl_xor(cm, off));
  const int w = (threadIdx.y * BX + threadIdx.x) >> 6;
  if ((threadIdx.x & 63) == 0) wmax[w] = cm;
  __syncthreads();
  if (threadIdx.x == 0 && threadIdx.y == 0) {
    double m = wmax[0];
    for (int q = 1; q < (BX * BY) / 64; ++q) m = fmax(m, wmax[q]);
    atomic_max_pos(&cmax[k], m);
  }
}

__global__ void __launch_bounds__(256) tracer_split_k(Dims d, const double* __restrict__ M, int npz,
                                                      const int* __restrict__ nsplt, double* __restrict__ cx,
                                                      double* __restrict__ cy, double* __restrict__ xfx,
                                                      double* __restrict__ yfx, double* __restrict__ mfx,
                                                      double* __restrict__ mfy) {
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

__global__ void tracer_nsplt_k(int npz, const double* __restrict__ cmax, int* __restrict__ nsplt) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < npz) nsplt[k] = (int)(1.0 + cmax[k]);
}

__global__ void copy_k(long n, const double* __restrict__ a, double* __restrict__ b) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long stride = (long)gridDim.x * blockDim.x;
  for (; i < n; i += stride) b[i] = a[i];
}

}  // namespace

void fv_tp_2d(const Ctx& c, const TpArgs& a) {
  const Dims& d = c.d;
  if (a.ord != 5 && a.ord != 6) throw std::runtime_error("fv_tp_2d: hord must be 5 or 6");
  // field pairs share a wave (and the Courant / flux loads): a second field array (q2), or
  // consecutive tracers when their count is even
  const bool pair2 = a.q2 != nullptr;
  if (pair2 && a.nt != 1) throw std::runtime_error("fv_tp_2d: a second field array needs nt = 1");
  // fields per wave: a.nf when given (1, 2 or 3, dividing nt), else 2 for pairs / even nt
  if (a.nf != 0 && (pair2 || a.nf < 1 || a.nf > 3 || a.nt % a.nf != 0 || (a.nf == 3 && !a.q_out)))
    throw std::runtime_error("fv_tp_2d: nf must be 1, 2 or 3 (3 only for the tracer update) and divide nt");
  const int NFw = a.nf != 0 ? a.nf : (pair2 || (a.nt % 2 == 0) ? 2 : 1);
  const int nfields = pair2 ? 2 : a.nt;
  {
    static const int seg_env = [] {
      const char* e = getenv("GTFV3_TP_SEG");  // tuning override of the default segment
      return e ? atoi(e) : 0;
    }();
    TpM m{};
    m.d = d;
    m.subs = c.subs;
    m.M = c.met;
  m.area4 = c.area4;
    const long tstride = (long)a.nk * d.plane;  // next tracer of the same sub-domain
    // field f of a group at slot f (the group's plane offset is added in the kernel); every
    // slot below NFw must be set: a null or stale slot is an out-of-bounds access
    m.qf[0] = a.q;
    m.qf[1] = pair2 ? a.q2 : a.q + tstride;
    m.qf[2] = pair2 ? nullptr : a.q + 2 * tstride;
    m.fxf[0] = a.fx;
    m.fyf[0] = a.fy;
    m.fxf[1] = pair2 ? a.fx_2 : (a.fx ? a.fx + tstride : nullptr);
    m.fyf[1] = pair2 ? a.fy_2 : (a.fy ? a.fy + tstride : nullptr);
    m.fxf[2] = pair2 || !a.fx ? nullptr : a.fx + 2 * tstride;
    m.fyf[2] = pair2 || !a.fy ? nullptr : a.fy + 2 * tstride;
    const bool tupd = a.q_out != nullptr;
    if (tupd) {
      if (pair2 || !a.mfx || !a.dp1 || !a.dp2 || !a.nsplt)
        throw std::runtime_error("fv_tp_2d tracer update: tracer array, mass fluxes, dp1, dp2, nsplt needed");
      m.qo[0] = a.q_out;
      m.qo[1] = a.q_out + tstride;
      m.qo[2] = a.q_out + 2 * tstride;
      m.dp1 = a.dp1;
      m.dp2o = a.dp2;
      m.nsplt = a.nsplt;
      m.it = a.it;
    }
    const bool zup = a.zh_out != nullptr;
    if (zup) {
      if (pair2 || tupd || a.nt != 1 || a.mfx || a.u_uv)
        throw std::runtime_error("fv_tp_2d with the height update: one field, no mass fluxes");
      m.qo[0] = a.zh_out;
    }
    const bool uv = a.u_uv != nullptr;
    if (uv) {
      if (pair2 || tupd || a.nt != 1 || a.mfx || !a.ke_uv || !a.v_uv)
        throw std::runtime_error("fv_tp_2d with the u, v update: one field, no mass fluxes, ke, u and v needed");
      m.ke = a.ke_uv;
      m.uu = a.u_uv;
      m.vv = a.v_uv;
    }
    for (int f = 0; f < NFw; ++f)
      if (!m.qf[f] || (tupd || zup ? !m.qo[f] : (!uv && (!m.fxf[f] || !m.fyf[f]))))
        throw std::runtime_error("fv_tp_2d: field slot " + std::to_string(f) + " of a " + std::to_string(NFw) +
                                 "-field group is not set");
    m.nt = a.nt;
    m.nk = a.nk;
    m.ntg = pair2 ? 1 : a.nt / NFw;
    m.crx = a.crx; m.cry = a.cry; m.xfx = a.xfx; m.yfx = a.yfx;
    m.mx = a.mfx ? a.mfx : a.xfx;
    m.my = a.mfy ? a.mfy : a.yfx;
    const long nz = (long)d.nsub * m.ntg * a.nk;
    m.nz = (int)nz;
    // Default: segments of <= 45 rows, more (down to 15 rows) when the launch would
    // otherwise have fewer than ~6900 field-waves (the C180 count on one GPU; small
    // sub-domains, as on 4-8 GPUs, need the shorter segments to fill the chip).
    std::vector<int> spans;
    // (the round-4 layout -- strips of MOUT from the first column, the tile-edge ones in the
    // edge form -- measured 32.43 / 32.34 / 32.45 ms per step for the uv / zh / tracer marches
    // against 32.33-32.40 with the spans: not kept)
    plan_spans(c, spans, spans);
    const double wpp = span_waves_per_plane(spans, d.nsub);
    int seg = a.cfg >= 8 ? a.cfg : seg_env;
    if (seg < 8) {
      const long fw = std::max<long>(1, (long)(nz * NFw * wpp));
      const long want = (6912 + fw - 1) / fw;
      const long nseg = std::max<long>((d.ny + 44) / 45, std::min<long>((d.ny + 14) / 15, want));
      seg = (int)((d.ny + nseg - 1) / nseg);
    }
    m.seg = seg;
    m.nseg = (d.ny + seg - 1) / seg;
    // algorithmic bytes: q read + fx, fy written per field plane; crx cry xfx yfx (+ mfx mfy)
    // read once per (sub-domain, level) however many fields share them (ra_x, ra_y are
    // formed in the kernel, the 2-D area plane is not counted)
    const Ext e = ext(d);
    const double bytes = tupd
        // per tracer q read and written; crx cry xfx yfx mfx mfy dp1 read, dp2 written once
        ? 8.0 * a.nk * (nfields * 2 * e.C + 3 * (e.X + e.Y) + 2 * e.C)
        : 8.0 * a.nk * (nfields * (e.C + e.X + e.Y) + (a.mfx ? 3 : 2) * (e.X + e.Y));
    // (the one-row-ahead form measured 3 % slower at C180; tile-edge and interior strips
    // as two kernels -- the interior one at four waves per SIMD for single fields --
    // measured 314 against 245 us per single-field launch at C180: two launch tails, and
    // the interior strips' rows are not 128-B aligned, so they are no cheaper)
    // MF: separate mass fluxes (w, pt and the tracers) or xfx / yfx themselves
    // (the paired last strip of the split thermo march measured 7 us slower per launch here,
    // 242 -> 249 us at C180, in either wave order: single-kernel marches keep one level per wave)
    // a launch carries at most MAXSPAN spans in its arguments; more (many sub-domains in one
    // process: C720 at 1x4 is 24 x 15) go as consecutive launches of disjoint spans, the
    // algorithmic bytes registered with the last
    const size_t nchunk = (spans.size() + MAXSPAN - 1) / MAXSPAN;
    for (size_t ci = 0; ci < nchunk; ++ci) {
      const std::vector<int> part(spans.begin() + ci * MAXSPAN,
                                  spans.begin() + std::min(spans.size(), (ci + 1) * MAXSPAN));
      const double share = ci + 1 == nchunk ? 1.0 : 0.0;
      const long waves = set_spans(m, part);
      const dim3 g(cdiv(waves, MWAVES)), b(MW * MWAVES);
#define TP_GO(O, M_, F_)                                                                           \
  do {                                                                                             \
    GT_LAUNCH_N("tp_march<" #O ", " #M_ ", " #F_ ">", (tp_march<O, true, M_, F_>), g, b, 0, c.st, m); \
    HIP_LAUNCH_CHECK();                                                                            \
    gt_bytes(share * bytes / 8.0);                                                                 \
  } while (0)
      if (uv) {
        // q read; crx cry xfx yfx read; ke, u, v read, u, v written; dx, dy once
        const double ub = 8.0 * a.nk * ((e.C + 2 * (e.X + e.Y)) + e.K + 2 * (e.X + e.Y)) + 16.0 * e.C;
        if (a.ord == 5) GT_LAUNCH_N("tp_march_uv<5>", (tp_march<5, true, false, 1, 3>), g, b, 0, c.st, m);
        else GT_LAUNCH_N("tp_march_uv<6>", (tp_march<6, true, false, 1, 3>), g, b, 0, c.st, m);
        HIP_LAUNCH_CHECK();
        gt_bytes(share * ub / 8.0);
        continue;
      }
      if (zup) {
        // zh read and written; crx cry xfx yfx read (the 2-D area plane not counted)
        const double zb = 8.0 * a.nk * (2 * e.C + 2 * (e.X + e.Y));
        if (a.ord == 5) GT_LAUNCH_N("tp_march_zh<5>", (tp_march<5, true, false, 1, 4>), g, b, 0, c.st, m);
        else GT_LAUNCH_N("tp_march_zh<6>", (tp_march<6, true, false, 1, 4>), g, b, 0, c.st, m);
        HIP_LAUNCH_CHECK();
        gt_bytes(share * zb / 8.0);
        continue;
      }
      if (tupd) {
#define TQ_GO(O, F_)                                                                                  \
  do {                                                                                                \
    GT_LAUNCH_N("tp_march_tracer<" #O ", " #F_ ">", (tp_march<O, true, true, F_, 2>), g, b, 0, c.st, m); \
    HIP_LAUNCH_CHECK();                                                                               \
    gt_bytes(share * bytes / 8.0);                                                                    \
  } while (0)
        if (NFw == 3) { if (a.ord == 5) TQ_GO(5, 3); else TQ_GO(6, 3); }
        else if (NFw == 2) { if (a.ord == 5) TQ_GO(5, 2); else TQ_GO(6, 2); }
        else { if (a.ord == 5) TQ_GO(5, 1); else TQ_GO(6, 1); }
#undef TQ_GO
      } else if (a.mfx) {
        if (NFw == 2) { if (a.ord == 5) TP_GO(5, true, 2); else TP_GO(6, true, 2); }
        else { if (a.ord == 5) TP_GO(5, true, 1); else TP_GO(6, true, 1); }
      } else {
        if (NFw == 2) { if (a.ord == 5) TP_GO(5, false, 2); else TP_GO(6, false, 2); }
        else { if (a.ord == 5) TP_GO(5, false, 1); else TP_GO(6, false, 1); }
      }
    }
#undef TP_GO
  }
}

void d_sw_thermo_march(const Ctx& c, const ThermoArgs& a) {
  const Dims& d = c.d;
  if (a.ord != 5 && a.ord != 6) throw std::runtime_error("d_sw thermo march: hord must be 5 or 6");
  TpM m{};
  m.d = d;
  m.subs = c.subs;
  m.M = c.met;
  m.area4 = c.area4;
  m.qf[0] = a.delp; m.qf[1] = a.w; m.qf[2] = a.pt;
  m.qo[0] = a.delp_o; m.qo[1] = a.w_o; m.qo[2] = a.pt_o;
  m.nt = 1;
  m.nk = a.npz;
  m.ntg = 1;
  m.crx = a.crx; m.cry = a.cry; m.xfx = a.xfx; m.yfx = a.yfx;
  m.mx = a.mfx;  // accumulators, read-modify-write
  m.my = a.mfy;
  const long nz = (long)d.nsub * a.npz;
  m.nz = (int)nz;
  std::vector<int> pex, pin;
  plan_spans(c, pex, pin);
  pex.insert(pex.end(), pin.begin(), pin.end());
  const long fw = std::max<long>(1, (long)(nz * 3 * span_waves_per_plane(pex, d.nsub)));
  const long want = (6912 + fw - 1) / fw;
  const long nseg = std::max<long>((d.ny + 44) / 45, std::min<long>((d.ny + 14) / 15, want));
  m.seg = (int)((d.ny + nseg - 1) / nseg);
  static const int seg_env = [] {
    const char* e = getenv("GTFV3_TP_SEG");  // tuning override of the default segment
    return e ? atoi(e) : 0;
  }();
  if (seg_env >= 8) m.seg = seg_env;
  m.nseg = (d.ny + m.seg - 1) / m.seg;
  if (m.seg + 10 > DXL_ROWS) throw std::runtime_error("d_sw thermo march: segment longer than the LDS dxa rows");
  // delp w pt read and written, crx cry xfx yfx read, mfx mfy read and written; the
  // interior strips prefetch one row ahead to fit two waves per SIMD (233 VGPRs; the
  // tile-edge form takes 292 with the two-ahead prefetch)
  const Ext e = ext(d);
  const double bytes = 8.0 * a.npz * (6 * e.C + 4 * (e.X + e.Y));
  if (a.ord == 5) march2<5, true, 3, 1, 2, false, 2, false>(c, m, bytes, "tp_march_thermo<5, ex>", "tp_march_thermo<5, in>");
  else march2<6, true, 3, 1, 2, false, 2, false>(c, m, bytes, "tp_march_thermo<6, ex>", "tp_march_thermo<6, in>");
}

void tracer_prep(const Ctx& c, int npz, const double* cx, const double* cy, double* xfx, double* yfx,
                 double* cmax_dev) {
  const Dims& d = c.d;
  HIP_CHECK(hipMemsetAsync(cmax_dev, 0, sizeof(double) * npz, c.st));
  Launch2D L{-NG, -NG, d.nx + 2 * NG + 1, d.ny + 2 * NG + 1};
  GT_LAUNCH(tracer_prep_k, dim3(cdiv(L.ni, BX), cdiv(L.nj, BY * TP_RPT), d.nsub * npz), dim3(BX, BY), 0, c.st, d,
                     c.met, npz, cx, cy, xfx, yfx, cmax_dev);
  HIP_LAUNCH_CHECK();
  const Ext e = ext(d);
  gt_bytes(npz * (2 * e.X + 2 * e.Y) + 4 * e.C);
}

void tracer_nsplt(const Ctx& c, int npz, const double* cmax_dev, int* nsplt_dev) {
  GT_LAUNCH(tracer_nsplt_k, dim3(cdiv(npz, 64)), dim3(64), 0, c.st, npz, cmax_dev, nsplt_dev);
  HIP_LAUNCH_CHECK();
}

void tracer_split(const Ctx& c, int npz, const int* nsplt_dev, double* cx, double* cy, double* xfx, double* yfx,
                  double* mfx, double* mfy) {
  const Dims& d = c.d;
  Launch2D L{-NG, -NG, d.nx + 2 * NG + 1, d.ny + 2 * NG + 1};
  GT_LAUNCH(tracer_split_k, plane_grid(L, d.nsub * npz), dim3(BX, BY), 0, c.st, d,
                     c.met, npz, nsplt_dev, cx, cy, xfx, yfx, mfx, mfy);
  HIP_LAUNCH_CHECK();
  // (no ra_x / ra_y planes: fv_tp_2d forms them from area and the split fluxes)
}

void tracer_dp2(const Ctx& c, int npz, const double* dp1, const double* mfx, const double* mfy, double* dp2) {
  const Dims& d = c.d;
  GT_LAUNCH(tracer_dp2_k, plane_grid(Launch2D{0, 0, d.nx, d.ny}, d.nsub * npz), dim3(BX, BY), 0, c.st, d,
                     c.met, npz, dp1, mfx, mfy, dp2);
  HIP_LAUNCH_CHECK();
  const Ext e = ext(d);
  gt_bytes(npz * (2 * e.C + e.X + e.Y) + e.C);
}

void tracer_update(const Ctx& c, int npz, int nq, double* q, const double* qn, const double* dp1, const double* dp2,
                   const double* fx, const double* fy, const int* nsplt_dev, int it) {
  (void)qn;
  const Dims& d = c.d;
  long nz = (long)d.nsub * nq * npz;
  GT_LAUNCH(tracer_update_k, plane_grid(Launch2D{0, 0, d.nx, d.ny}, nz < ZMAX ? nz : ZMAX),
                     dim3(BX, BY), 0, c.st, d, c.met, npz, nq, q, dp1, dp2, fx, fy, nsplt_dev, it, (int)nz);
  HIP_LAUNCH_CHECK();
  const Ext e = ext(d);
  gt_bytes((double)nq * npz * (4 * e.C + e.X + e.Y) + e.C);
}

void copy_levels(const Ctx& c, long n, const double* src, double* dst) {
  GT_LAUNCH(copy_k, dim3(cdiv(n, 256) < 8192 ? cdiv(n, 256) : 8192), dim3(256), 0, c.st, n, src, dst);
  HIP_LAUNCH_CHECK();
  gt_bytes(2.0 * n);
}

}  // namespace gtfv3
