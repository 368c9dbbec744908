// csw_march.hip — c_sw's first stage as ONE column-marching kernel for gfx950:
// d2a2c_vect (utmp / vtmp, the generic ua / va, the cube-corner fixes, uc / vc and the
// contravariant ut / vt scaled by dt2 * dy * sin_sg), the half-step upwind transport of
// delp / pt / w (delpc, ptc, wc) and the cell kinetic energy ke.  It replaces the chain
// cs_tmp -> cs_corner_fix -> cs_cgrid -> cs_transport_ke (sw.hip, kept as the checked
// default form; this one with GTFV3_CSW_FUSED=1) with the same expressions in the same order,
// so every output is bit-identical to the chain's (tests/test_gpu_sw.py compares them).
// Measured C180 L72 on one MI355X: 5.26 ms per step against the chain's 5.25 (877 us per
// launch, 70 % of wave cycles waiting on memory at 3 waves per SIMD): the halved field
// passes do not pay while each row step waits out its loads, so the chain stays the default.
//
// One wavefront owns a strip of 64 columns (lane L: column x = a - 3 + L; the 57 output
// columns are lanes 3 .. 59) of one (sub-domain, level) plane and marches up a segment of
// rows.  x neighbours come from DPP lane shifts, y neighbours from register windows rolled
// row by row, so u, v, delp, pt and w are read once per strip and segment and utmp / vtmp
// never reach HBM (the chain wrote and re-read them, and re-read u, v, ua, va, uc, vc, ut,
// vt between its kernels: 31 field passes per level, 15 here).  Row step R computes
//   stage 1 on row R     utmp, vtmp, ua, va   (u rows R-1 .. R+2, v row R and lanes x-1 .. x+2)
//   stage 2 on row R-1   uc, ut, vc, vt       (utmp / ua lanes x-2 .. x+1, vtmp / va rows R-3 .. R)
//   stage 3 on row R-2   delpc, ptc, wc, ke   (ut / uc lanes x, x+1, vt / vc rows R-2, R-1)
// The cube-corner fixes of d2a2c_vect overwrite utmp / vtmp / ua / va at a few halo points
// next to an owned cube corner with the (negated) generic value at a transposed source point;
// a lane holding a target evaluates that source's generic value directly from u and v in HBM
// (the same expressions), so the fixed values enter the later stages like any other.
#include <cmath>
#include <cstdlib>

#include "kernels_sw.hpp"
#include "stencil_common.hpp"

namespace gtfv3 {
namespace {

// debugging build (make BOUNDS=1): every plane-relative offset checked against the plane
#ifdef GTFV3_BOUNDS
#define CK(o) ck_plane((long)(o), d.plane, __LINE__)
#define CKS(o) (zo + ck_plane((long)(o) - zo, d.plane, __LINE__))
__device__ __forceinline__ long ck_plane(long o, long n, int line) {
  if (o < 0 || o >= n) {
    printf("csw_march line %d: offset %ld outside the plane (%ld) block %d thread %d\n", line, o, n, blockIdx.x, threadIdx.x);
    return o < 0 ? 0 : n - 1;
  }
  return o;
}
#else
#define CK(o) (o)
#define CKS(o) (o)
#endif

constexpr double A1 = 0.5625, A2 = -0.0625;
constexpr double BIG = 1.0e8;
constexpr int CW_OUT = 57, CW_L = 3;  // outputs per strip, halo lanes on the left
constexpr int CW_WAVES = 4;

struct CsM {
  Dims d;
  const SubInfo* subs;
  const double* M;
  int npz;
  double dt2;
  const double *u, *v, *delp, *pt, *w;
  double *ua, *va, *uc, *vc, *ut, *vt, *delpc, *ptc, *wc, *ke;
  int nstrip, nseg, seg;
  long nwaves;
};

__device__ __forceinline__ double ei4(double u0, double u1, double u2, double u3, double d0, double d1, double d2,
                                      double d3) {
  double t1 = d0 + d1;
  double t2 = d2 + d3;
  return 0.5 * (((t1 + d1) * u1 - d1 * u0) / t1 + ((t2 + d2) * u2 - d2 * u3) / t2);
}

// d2a2c_vect part 1 at local (i, j) (cs_tmp's branches): which forms apply
struct TmpForm {
  bool in, rows, cols, two;
};
__device__ __forceinline__ TmpForm tmp_form(int i, int j, const SubInfo& sub, int nx, int ny) {
  TmpForm f{false, false, false, false};
  const int N = sub.N, io = sub.ioff, jo = sub.joff, I = i + io, J = j + jo;
  f.in = i <= nx + NG - 1 && j <= ny + NG - 1;
  if (!f.in) return f;
  f.rows = J >= max(3, jo - 1) && J <= min(N - 4, jo + ny);
  f.cols = I >= max(3, io - 1) && I <= min(N - 4, io + nx);
  const int jsd = jo - NG, jed = jo + ny + NG - 1, isd = io - NG, ied = io + nx + NG - 1;
  const bool mid = J >= max(3, jsd) && J <= min(N - 4, jed);
  if (J >= jsd && J <= 2) f.two = true;
  if (J >= N - 3 && J <= jed) f.two = true;
  if (mid && I >= isd && I <= 2) f.two = true;
  if (mid && I >= N - 3 && I <= ied) f.two = true;
  return f;
}
// uy[0..3] = u(i, j-1 .. j+2), vx[0..3] = v(i-1 .. i+2, j); cs_tmp's expressions
__device__ __forceinline__ void tmp_eval(const TmpForm& f, const double* uy, const double* vx, double& ut,
                                         double& vt) {
  ut = BIG;
  vt = BIG;
  if (f.in) {
    if (f.rows) ut = A2 * (uy[0] + uy[3]) + A1 * (uy[1] + uy[2]);
    if (f.cols) vt = A2 * (vx[0] + vx[3]) + A1 * (vx[1] + vx[2]);
    if (f.two) {
      ut = 0.5 * (uy[1] + uy[2]);
      vt = 0.5 * (vx[1] + vx[2]);
    }
  }
}
__device__ __forceinline__ bool uava_in(int i, int j, int nx, int ny) {
  return i >= -2 && i <= nx + 1 && j >= -2 && j <= ny + 1;
}

// generic utmp / vtmp / ua / va at tile-global (Is, Js) read from HBM (a corner-fix source)
struct Gen {
  const Dims& d;
  const SubInfo& sub;
  const double* U;
  const double* V;
  const double* cs;  // cosa_s plane
  const double* r2;  // rsin2 plane
  __device__ void tmp(int Is, int Js, double& ut, double& vt) const {
    const int i = Is - sub.ioff, j = Js - sub.joff;
    const TmpForm f = tmp_form(i, j, sub, d.nx, d.ny);
    const long o = pidx(d, i, j);
    double uy[4] = {0, 0, 0, 0}, vx[4] = {0, 0, 0, 0};
    if (f.in && (f.rows || f.two)) {
      uy[1] = U[CK(o)];
      uy[2] = U[CK(o + d.pitch)];
      if (f.rows) {
        uy[0] = U[CK(o - d.pitch)];
        uy[3] = U[CK(o + 2 * d.pitch)];
      }
    }
    if (f.in && (f.cols || f.two)) {
      vx[1] = V[CK(o)];
      vx[2] = V[CK(o + 1)];
      if (f.cols) {
        vx[0] = V[CK(o - 1)];
        vx[3] = V[CK(o + 2)];
      }
    }
    tmp_eval(f, uy, vx, ut, vt);
  }
  __device__ double ua(int Is, int Js) const {
    double ut, vt;
    tmp(Is, Js, ut, vt);
    const int i = Is - sub.ioff, j = Js - sub.joff;
    if (!uava_in(i, j, d.nx, d.ny)) return 0.0;
    const long o = pidx(d, i, j);
    return (ut - vt * cs[CK(o)]) * r2[CK(o)];
  }
  __device__ double va(int Is, int Js) const {
    double ut, vt;
    tmp(Is, Js, ut, vt);
    const int i = Is - sub.ioff, j = Js - sub.joff;
    if (!uava_in(i, j, d.nx, d.ny)) return 0.0;
    const long o = pidx(d, i, j);
    return (vt - ut * cs[CK(o)]) * r2[CK(o)];
  }
};

__global__ void __launch_bounds__(64 * CW_WAVES) cs_march_k(CsM a) {
  // wave index through readfirstlane: the plane, strip, segment and every pointer derived
  // from it stay in SGPRs
  const long wid = (long)blockIdx.x * CW_WAVES + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (wid >= a.nwaves) return;  // whole wave; no workgroup barrier in this kernel
  const int lane = threadIdx.x & 63;
  const int strip = (int)(wid % a.nstrip);
  const long t = wid / a.nstrip;
  const int sg = (int)(t % a.nseg);
  const int z = (int)(t / a.nseg);
  const int s = z / a.npz;
  const Dims& d = a.d;
  const SubInfo sub = a.subs[s];
  const int nx = d.nx, ny = d.ny, N = sub.N, io = sub.ioff, jo = sub.joff;
  const long pitch = d.pitch;
  const long zo = (long)z * d.plane;
  const int x = -NG + strip * CW_OUT - CW_L + lane;
  const int I = x + io;
  const int xc = x < -NG ? -NG : (x > nx + NG ? nx + NG : x);
  const long xo = xc + NG;
  const bool out_lane = lane >= CW_L && lane < CW_L + CW_OUT && x <= nx + NG;
  const int j0 = -NG + sg * a.seg;
  const int j1 = min(j0 + a.seg, ny + NG + 1);
  const double dt2 = a.dt2, dt4 = 0.5 * dt2;

  const double* U = a.u + zo;
  const double* V = a.v + zo;
  const double* QD = a.delp + zo;
  const double* QP = a.pt + zo;
  const double* QW = a.w + zo;
  auto MP = [&](int m) { return met(a.M, d, m, s); };
  const double *mCS = MP(M_COSA_S), *mR2 = MP(M_RSIN2), *mCU = MP(M_COSA_U), *mRU = MP(M_RSIN_U);
  const double *mCV = MP(M_COSA_V), *mRV = MP(M_RSIN_V), *mDX = MP(M_DX), *mDY = MP(M_DY);
  const double *mS1 = MP(M_SIN1), *mS2 = MP(M_SIN2), *mS3 = MP(M_SIN3), *mS4 = MP(M_SIN4);
  const double *mC1 = MP(M_COS1), *mC2 = MP(M_COS2), *mC3 = MP(M_COS3), *mC4 = MP(M_COS4);
  const double *mDXA = MP(M_DXA), *mDYA = MP(M_DYA), *mRA = MP(M_RAREA);
  const Gen gen{d, sub, U, V, mCS, mR2};

  auto rc = [&](int r) { return r < -NG ? -NG : (r > ny + NG ? ny + NG : r); };
  auto ro = [&](int r) { return (long)(rc(r) + NG) * pitch + xo; };  // this lane's column, row r (clamped)
  // the strip reaches a tile edge (ei4 forms at I = 0, N; sin / cos of the edge columns)
  const int xs0 = -NG + strip * CW_OUT - CW_L;
  const bool EX = (0 - io >= xs0 - 2 && 0 - io <= xs0 + 65) || (N - io >= xs0 - 2 && N - io <= xs0 + 65);
  const bool own00 = io <= 0 && 0 <= io + nx && jo <= 0 && 0 <= jo + ny;
  const bool ownN0 = io <= N && N <= io + nx && jo <= 0 && 0 <= jo + ny;
  const bool ownNN = io <= N && N <= io + nx && jo <= N && N <= jo + ny;
  const bool own0N = io <= 0 && 0 <= io + nx && jo <= N && N <= jo + ny;
  const bool anyown = own00 || ownN0 || ownNN || own0N;
  const bool ccol = I < 0 || I >= N;  // a column of the cube-corner halo (with a halo row)

  // windows (index 0 = oldest row)
  double uw[5], vw[3];          // u rows R-2 .. R+2, v rows R-2 .. R
  double tmu[2], tmv[4];        // utmp rows R-1, R; vtmp rows R-3 .. R
  double uaw[3], vaw[4];        // ua rows R-2 .. R; va rows R-3 .. R
  double uc2[2], ut2[2], vc2[2], vt2[2];  // stage-2 outputs, rows R-2, R-1
  double s4w[2], s1w[2], s3w[2], s2w[2];  // sin4 / sin1 / sin3 / sin2, rows R-2, R-1
  double qy[3][3];              // delp, pt, w (y-sweep corner fill), rows R-3 .. R-1
#pragma unroll
  for (int m = 0; m < 2; ++m) tmu[m] = uc2[m] = ut2[m] = vc2[m] = vt2[m] = s4w[m] = s1w[m] = s3w[m] = s2w[m] = 0.0;
#pragma unroll
  for (int m = 0; m < 4; ++m) tmv[m] = vaw[m] = 0.0;
#pragma unroll
  for (int m = 0; m < 3; ++m) {
    uaw[m] = vw[m] = 0.0;
    qy[0][m] = qy[1][m] = qy[2][m] = 0.0;
  }
  const int R_lo = j0 - 2, R_hi = j1 + 1;
#pragma unroll
  for (int m = 1; m < 5; ++m) uw[m] = U[CK(ro(R_lo - 3 + m))];
  uw[0] = 0.0;
  // the field rows of a row step (u row R+2, v row R, delp / pt / w row R-1 with the y-sweep
  // corner fill) are loaded one row step ahead, so a step waits on the metric loads only
  // (L2 / Infinity-Cache hits) instead of an HBM round trip
  auto q_off = [&](int r) -> long {
    const int Jr = r + jo;
    return (Jr < 0 || Jr >= N) && ccol && r >= -NG && r <= ny + NG - 1 && x >= -NG && x <= nx + NG - 1
               ? cc_off(d, sub, x, r, 2)
               : ro(r);
  };
  double nU = U[CK(ro(R_lo + 2))], nV = V[CK(ro(R_lo))];
  double nQ[3];
  {
    const long oq = q_off(R_lo - 1);
    nQ[0] = QD[CK(oq)];
    nQ[1] = QP[CK(oq)];
    nQ[2] = QW[CK(oq)];
  }

  for (int R = R_lo; R <= R_hi; ++R) {
    // ---- roll the windows, load the new rows
#pragma unroll
    for (int m = 0; m < 4; ++m) uw[m] = uw[m + 1];
    uw[4] = nU;
    vw[0] = vw[1];
    vw[1] = vw[2];
    vw[2] = nV;
    const int r2 = R - 1, r3 = R - 2;
    const int J = R + jo, J2 = r2 + jo, J3 = r3 + jo;
    const long o2 = ro(r2), o3 = ro(r3);
    s4w[0] = s4w[1];
    s1w[0] = s1w[1];
    s3w[0] = s3w[1];
    s2w[0] = s2w[1];
    s4w[1] = mS4[CK(o2)];
    s1w[1] = mS1[CK(o2)];
    s3w[1] = mS3[CK(o2)];
    s2w[1] = mS2[CK(o2)];
    // delp / pt / w: y-sweep fill of row r2 (stage 3's row r3 + 1; q_off: the cube-corner
    // remap applies to the cells' halo, i, j in [-NG, n + NG - 1]; the extra staggered column /
    // row of the padded plane has no corner source and keeps its own, never output, value)
#pragma unroll
    for (int f = 0; f < 3; ++f) {
      qy[f][0] = qy[f][1];
      qy[f][1] = qy[f][2];
    }
#pragma unroll
    for (int f = 0; f < 3; ++f) qy[f][2] = nQ[f];
    // the next row step's field rows
    nU = U[CK(ro(R + 3))];
    nV = V[CK(ro(R + 1))];
    {
      const long oq = q_off(R);
      nQ[0] = QD[CK(oq)];
      nQ[1] = QP[CK(oq)];
      nQ[2] = QW[CK(oq)];
    }

    // ---- stage 1, row R: utmp, vtmp and the generic ua, va
    double utn, vtn, uan, van;
    {
      const double vm1 = lane_prev(vw[2]), vp1 = lane_next(vw[2]), vp2 = lane_next(vp1);
      const double uy[4] = {uw[1], uw[2], uw[3], uw[4]};
      const double vx[4] = {vm1, vw[2], vp1, vp2};
      const TmpForm tf = tmp_form(x, R, sub, nx, ny);
      tmp_eval(tf, uy, vx, utn, vtn);
      uan = van = 0.0;
      if (uava_in(x, R, nx, ny)) {
        const long o1 = ro(R);
        const double cs = mCS[CK(o1)], r2v = mR2[CK(o1)];
        uan = (utn - vtn * cs) * r2v;
        van = (vtn - utn * cs) * r2v;
      }
      // cube-corner fixes (cs_corner_fix's targets; the sources are generic values): each
      // output has at most one fix per lane, so the source point and sign are chosen first and
      // the generic value is evaluated once
      if (anyown && (J <= -1 || J >= N)) {
        int us = 0, vs = 0, as = 0, bs = 0;              // sign (0: no fix)
        int uI = 0, uJ = 0, vI = 0, vJ = 0, aI = 0, aJ = 0, bI = 0, bJ = 0;  // source points
        if (J == -1 && own00 && I >= -3 && I <= -1) { us = -1; uI = -1; uJ = -I - 1; }
        if (J == -1 && ownN0 && I >= N && I <= N + 2) { us = 1; uI = N; uJ = I - N; }
        if (J == N && ownNN && I >= N && I <= N + 2) { us = -1; uI = N; uJ = N - 1 - (I - N); }
        if (J == N && own0N && I >= -3 && I <= -1) { us = 1; uI = -1; uJ = N + I; }
        if (I == -1 && own00 && J >= -3 && J <= -1) { vs = -1; vI = -J - 1; vJ = -1; }
        if (I == N && ownN0 && J >= -3 && J <= -1) { vs = 1; vI = N + J; vJ = -1; }
        if (I == N && ownNN && J >= N && J <= N + 2) { vs = -1; vI = N - (J - N) - 1; vJ = N; }
        if (I == -1 && own0N && J >= N && J <= N + 2) { vs = 1; vI = J - N; vJ = N; }
        if (own00 && J == -1 && I == -2) { as = -1; aI = -1; aJ = 1; }
        if (own00 && J == -1 && I == -1) { as = -1; aI = -1; aJ = 0; }
        if (ownN0 && J == -1 && I == N) { as = 1; aI = N; aJ = 0; }
        if (ownN0 && J == -1 && I == N + 1) { as = 1; aI = N; aJ = 1; }
        if (ownNN && J == N && I == N) { as = -1; aI = N; aJ = N - 1; }
        if (ownNN && J == N && I == N + 1) { as = -1; aI = N; aJ = N - 2; }
        if (own0N && J == N && I == -2) { as = 1; aI = -1; aJ = N - 2; }
        if (own0N && J == N && I == -1) { as = 1; aI = -1; aJ = N - 1; }
        if (own00 && I == -1 && J == -2) { bs = -1; bI = 1; bJ = -1; }
        if (own00 && I == -1 && J == -1) { bs = -1; bI = 0; bJ = -1; }
        if (ownN0 && I == N && J == -1) { bs = 1; bI = N - 1; bJ = -1; }
        if (ownN0 && I == N && J == -2) { bs = 1; bI = N - 2; bJ = -1; }
        if (ownNN && I == N && J == N) { bs = -1; bI = N - 1; bJ = N; }
        if (ownNN && I == N && J == N + 1) { bs = -1; bI = N - 2; bJ = N; }
        if (own0N && I == -1 && J == N) { bs = 1; bI = 0; bJ = N; }
        if (own0N && I == -1 && J == N + 1) { bs = 1; bI = 1; bJ = N; }
        // utmp takes the source's vtmp, vtmp the source's utmp; ua the source's va, va its ua
        if (us != 0) { double a_, b_; gen.tmp(uI, uJ, a_, b_); utn = us > 0 ? b_ : -b_; }
        if (vs != 0) { double a_, b_; gen.tmp(vI, vJ, a_, b_); vtn = vs > 0 ? a_ : -a_; }
        if (as != 0) { const double g = gen.va(aI, aJ); uan = as > 0 ? g : -g; }
        if (bs != 0) { const double g = gen.ua(bI, bJ); van = bs > 0 ? g : -g; }
      }
    }
    tmu[0] = tmu[1];
    tmu[1] = utn;
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      tmv[m] = tmv[m + 1];
      vaw[m] = vaw[m + 1];
    }
    tmv[3] = vtn;
    vaw[3] = van;
    uaw[0] = uaw[1];
    uaw[1] = uaw[2];
    uaw[2] = uan;
    if (out_lane && R >= j0 && R < j1 && R <= ny + NG) {
      const long o1 = (long)(R + NG) * pitch + xo;
      a.ua[CKS(zo + o1)] = uan;
      a.va[CKS(zo + o1)] = van;
    }

    // ---- stage 2, row r2: uc, ut (x-edges of y-direction faces) and vc, vt
    {
      const double tm = tmu[0], tm_m1 = lane_prev(tm), tm_m2 = lane_prev(tm_m1), tm_p1 = lane_next(tm);
      const double sin3m = lane_prev(s3w[1]);
      double ex = 0.0;
      if (EX) {
        const double ua0 = uaw[1], ua_m1 = lane_prev(ua0), ua_m2 = lane_prev(ua_m1), ua_p1 = lane_next(ua0);
        const double dx0 = mDXA[CK(o2)], dx_m1 = lane_prev(dx0), dx_m2 = lane_prev(dx_m1), dx_p1 = lane_next(dx0);
        if (I == 0 || I == N) ex = ei4(ua_m2, ua_m1, ua0, ua_p1, dx_m2, dx_m1, dx0, dx_p1);
      }
      double ucv = 0.0, utv = 0.0;
      if (x >= -1 && x <= nx + 1 && r2 >= -1 && r2 <= ny) {
        if (I == 0 || I == N) {
          ucv = ex * (ex > 0.0 ? sin3m : s1w[1]);
          utv = ex;
        } else {
          if (I == -1 || I == N - 1) ucv = C1 * tm_m2 + C2 * tm_m1 + C3 * tm;
          else if (I == 1) ucv = C1 * tm_p1 + C2 * tm + C3 * tm_m1;
          else if (I == N + 1) ucv = C3 * tm_m1 + C2 * tm + C1 * tm_p1;
          else ucv = A2 * (tm_m2 + tm_p1) + A1 * (tm_m1 + tm);
          utv = (ucv - vw[1] * mCU[CK(o2)]) * mRU[CK(o2)];
        }
        const double dy = mDY[CK(o2)];
        utv = utv > 0.0 ? dt2 * utv * dy * sin3m : dt2 * utv * dy * s1w[1];
      }
      double vcv = 0.0, vtv = 0.0;
      if (x >= -1 && x <= nx && r2 >= -1 && r2 <= ny + 1) {
        if (J2 == 0 || J2 == N) {
          const double e = ei4(vaw[0], vaw[1], vaw[2], vaw[3], mDYA[CK(o2 - 2 * pitch)], mDYA[CK(o2 - pitch)], mDYA[CK(o2)],
                               mDYA[CK(o2 + pitch)]);
          vcv = e * (e > 0.0 ? s4w[0] : s2w[1]);
          vtv = e;
        } else {
          if (J2 == -1 || J2 == N - 1) vcv = C1 * tmv[0] + C2 * tmv[1] + C3 * tmv[2];
          else if (J2 == 1 || J2 == N + 1) vcv = C1 * tmv[3] + C2 * tmv[2] + C3 * tmv[1];
          else vcv = A2 * (tmv[0] + tmv[3]) + A1 * (tmv[1] + tmv[2]);
          vtv = (vcv - uw[1] * mCV[CK(o2)]) * mRV[CK(o2)];
        }
        const double dx = mDX[CK(o2)];
        vtv = vtv > 0.0 ? dt2 * vtv * dx * s4w[0] : dt2 * vtv * dx * s2w[1];
      }
      uc2[0] = uc2[1];
      ut2[0] = ut2[1];
      vc2[0] = vc2[1];
      vt2[0] = vt2[1];
      uc2[1] = ucv;
      ut2[1] = utv;
      vc2[1] = vcv;
      vt2[1] = vtv;
      if (out_lane && r2 >= j0 && r2 < j1 && r2 >= -NG && r2 <= ny + NG) {
        const long oo = zo + o2;
        a.uc[CKS(oo)] = ucv;
        a.ut[CKS(oo)] = utv;
        a.vc[CKS(oo)] = vcv;
        a.vt[CKS(oo)] = vtv;
      }
    }

    // ---- stage 3, row r3: delpc, ptc, wc and ke
    {
      // x-sweep fill of row r3 (differs from the y-sweep one only in cube-corner halo cells)
      double qx[3] = {qy[0][1], qy[1][1], qy[2][1]};
      const bool crow3 = J3 < 0 || J3 >= N;
      if (crow3 && r3 >= -NG && r3 <= ny + NG - 1) {
        const bool cc = ccol && x >= -NG && x <= nx + NG - 1;
        const long oq = cc ? cc_off(d, sub, x, r3, 1) : o3;
        if (__any(cc)) {
          qx[0] = QD[CK(oq)];
          qx[1] = QP[CK(oq)];
          qx[2] = QW[CK(oq)];
        }
      }
      // x faces: the lane's face x (upwind cell x-1 or x), face x+1 from the next lane
      const double c = ut2[0];
      double f1, fp, fw;
      {
        const double dm = lane_prev(qx[0]), pm = lane_prev(qx[1]), wm = lane_prev(qx[2]);
        const double dps = c > 0.0 ? dm : qx[0];
        const double pps = c > 0.0 ? pm : qx[1];
        const double wws = c > 0.0 ? wm : qx[2];
        f1 = c * dps;
        fp = f1 * pps;
        fw = f1 * wws;
      }
      const double f1n = lane_next(f1), fpn = lane_next(fp), fwn = lane_next(fw);
      const double ucn = lane_next(uc2[0]), vn = lane_next(vw[0]);
      double s1c = 0.0, c1c = 0.0, s3c = 0.0, c3c = 0.0;
      if (EX) {
        s1c = s1w[0];
        s3c = s3w[0];
        c1c = mC1[CK(o3)];
        c3c = mC3[CK(o3)];
      }
      if (x >= -1 && x <= nx && r3 >= -1 && r3 <= ny) {
        // y faces r3 (cells r3-1 | r3) and r3+1 (cells r3 | r3+1)
        double g1[2], gp[2], gw[2];
#pragma unroll
        for (int f = 0; f < 2; ++f) {
          const double cy = f == 0 ? vt2[0] : vt2[1];
          const int lo_ = f, hi_ = f + 1;  // qy rows r3-1+f, r3+f
          const double dps = cy > 0.0 ? qy[0][lo_] : qy[0][hi_];
          const double pps = cy > 0.0 ? qy[1][lo_] : qy[1][hi_];
          const double wws = cy > 0.0 ? qy[2][lo_] : qy[2][hi_];
          g1[f] = cy * dps;
          gp[f] = g1[f] * pps;
          gw[f] = g1[f] * wws;
        }
        const double ra = mRA[CK(o3)];
        const double dpo = qy[0][1], ppo = qy[1][1], wwo = qy[2][1];
        const double dpc = dpo + (f1 - f1n + g1[0] - g1[1]) * ra;
        const long oo = zo + o3;
        // kinetic energy
        double kk, vv;
        const double uaa = uaw[0], vaa = vaw[1];
        if (uaa > 0.0) {
          if (I == 0 || I == N) kk = uc2[0] * s1c + vw[0] * c1c;
          else kk = uc2[0];
        } else {
          if (I == -1 || I == N - 1) kk = ucn * s3c + vn * c3c;
          else kk = ucn;
        }
        if (vaa > 0.0) {
          if (J3 == 0 || J3 == N) vv = vc2[0] * s2w[0] + uw[0] * mC2[CK(o3)];
          else vv = vc2[0];
        } else {
          if (J3 == -1 || J3 == N - 1) vv = vc2[1] * s4w[0] + uw[1] * mC4[CK(o3)];
          else vv = vc2[1];
        }
        if (out_lane && r3 >= j0 && r3 < j1) {
          a.delpc[CKS(oo)] = dpc;
          a.ptc[CKS(oo)] = (ppo * dpo + (fp - fpn + gp[0] - gp[1]) * ra) / dpc;
          a.wc[CKS(oo)] = (wwo * dpo + (fw - fwn + gw[0] - gw[1]) * ra) / dpc;
          a.ke[CKS(oo)] = dt4 * (uaa * kk + vaa * vv);
        }
      }
    }
  }
}

}  // namespace

bool c_sw_fused() {
  static const bool on = [] {
    const char* e = std::getenv("GTFV3_CSW_FUSED");
    return e && e[0] == '1';
  }();
  return on;
}

// c_sw's first stage as one march (the chain's outputs uc, vc, ua, va, ut, vt, delpc, ptc,
// wc, ke; utmp / vtmp are not formed in HBM)
void c_sw_transport_march(const Ctx& c, const CswArgs& a) {
  const Dims& d = c.d;
  CsM m{};
  m.d = d;
  m.subs = c.subs;
  m.M = c.met;
  m.npz = a.npz;
  m.dt2 = a.dt2;
  m.u = a.u; m.v = a.v; m.delp = a.delp; m.pt = a.pt; m.w = a.w;
  m.ua = a.ua; m.va = a.va; m.uc = a.uc; m.vc = a.vc; m.ut = a.ut; m.vt = a.vt;
  m.delpc = a.delpc; m.ptc = a.ptc; m.wc = a.wc; m.ke = a.ke;
  const int cols = d.nx + 2 * NG + 1, rows = d.ny + 2 * NG + 1;
  m.nstrip = (cols + CW_OUT - 1) / CW_OUT;
  const long planes = (long)d.nsub * a.npz;
  // segments: enough waves to fill the chip (~8 per SIMD), at least 12 rows each
  const long want = 8192;
  int nseg = (int)std::max<long>(1, (want + planes * m.nstrip - 1) / (planes * m.nstrip));
  nseg = std::min(nseg, std::max(1, rows / 12));
  m.seg = (rows + nseg - 1) / nseg;
  m.nseg = (rows + m.seg - 1) / m.seg;
  m.nwaves = planes * m.nstrip * m.nseg;
  GT_LAUNCH(cs_march_k, dim3((unsigned)((m.nwaves + CW_WAVES - 1) / CW_WAVES)), dim3(64 * CW_WAVES), 0, c.st, m);
  HIP_LAUNCH_CHECK();
  const Ext e = ext(d);
  const double L = a.npz;
  // reads u, v, delp, pt, w; writes ua, va, uc, vc, ut, vt, delpc, ptc, wc, ke; metric planes once
  gt_bytes(L * (e.X + e.Y + 3 * e.C) + L * (2 * e.C + 2 * e.X + 2 * e.Y + 4 * e.C) + 22 * e.C);
}

}  // namespace gtfv3
