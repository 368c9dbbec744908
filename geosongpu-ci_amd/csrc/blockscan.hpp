// blockscan.hpp — a column split into NB level blocks on NB consecutive lanes of one
// 16-lane DPP row (lane = NB * column + block): neighbour hand-overs by DPP row shifts,
// Kogge-Stone scans of block sums / affine maps / Möbius (2x2) maps over the NB blocks, and
// the partitioned Thomas solve built on them (riem.hip's SIM1 solver).  Every lane of the
// wave must execute these (no lane-divergent branch around a shift: a DPP read of an
// exec-disabled lane returns 0).  CPU emulation of the same arithmetic, against a
// sequential sweep: tests/test_blockscan_emul.py.
#pragma once
#include <type_traits>

#include "fastmath.hpp"
#include "stencil_common.hpp"

namespace gtfv3 {

// Rule for every shift below: evaluate it into a variable BEFORE any lane-divergent `?:` that
// uses it.  Written inside an arm (`b == 0 ? x : blk_prev(v)`), clang emits the arm as a
// branch, the convergent DPP call stays inside it, and the source lanes the condition
// disables read as 0 there (block 1 then read block 0's value as 0).
template <int CTRL>
__device__ __forceinline__ double dpp_pinned(double v) {
  return lane_shift<CTRL>(v);
}
template <int S>
__device__ __forceinline__ double row_shr(double v) { return dpp_pinned<0x110 + S>(v); }
template <int S>
__device__ __forceinline__ double row_shl(double v) { return dpp_pinned<0x100 + S>(v); }
// value of the block above (lane b - 1) / below (lane b + 1) in the same column
__device__ __forceinline__ double blk_prev(double v) { return row_shr<1>(v); }
__device__ __forceinline__ double blk_next(double v) { return row_shl<1>(v); }

// affine map x_out = A x_in + B of a block
struct Aff {
  double A, B;
};
// 2x2 matrix [[p11, p12], [p21, p22]] acting on (u, v), bet = u / v
struct Mob {
  double p11, p12, p21, p22;
};
// member-wise selects (a select of whole structs compiles to a select of stack addresses)
__device__ __forceinline__ double ks_sel(bool c, double x, double y) { return c ? x : y; }
__device__ __forceinline__ Aff ks_sel(bool c, Aff x, Aff y) { return Aff{c ? x.A : y.A, c ? x.B : y.B}; }
__device__ __forceinline__ Mob ks_sel(bool c, Mob x, Mob y) {
  return Mob{c ? x.p11 : y.p11, c ? x.p12 : y.p12, c ? x.p21 : y.p21, c ? x.p22 : y.p22};
}

// Kogge-Stone over the NB blocks of a column.  DN: lane b ends with the fold of blocks 0..b
// (neighbour b - s); UP: of blocks b..NB-1 (neighbour b + s).  comb(self, other) folds the
// neighbour's partial into this lane's.
template <int NB, bool DN, int S, class St, class Sh, class Comb>
__device__ __forceinline__ void ks_step(St& v, int b, Sh shift, Comb comb) {
  if constexpr (S < NB) {
    const St o = shift(std::integral_constant<int, S>{}, v);
    const bool on = DN ? b >= S : b + S < NB;
    v = ks_sel(on, comb(v, o), v);
    ks_step<NB, DN, 2 * S>(v, b, shift, comb);
  }
}

template <int NB, bool DN>
__device__ __forceinline__ double scan_sum(double v, int b) {
  auto sh = [](auto sc, double x) {
    constexpr int S = decltype(sc)::value;
    return DN ? row_shr<S>(x) : row_shl<S>(x);
  };
  ks_step<NB, DN, 1>(v, b, sh, [](double x, double y) { return DN ? y + x : x + y; });
  return v;
}

template <int NB, bool DN>
__device__ __forceinline__ Aff scan_aff(Aff v, int b) {
  auto sh = [](auto sc, Aff x) {
    constexpr int S = decltype(sc)::value;
    return DN ? Aff{row_shr<S>(x.A), row_shr<S>(x.B)} : Aff{row_shl<S>(x.A), row_shl<S>(x.B)};
  };
  // self after the neighbour's blocks: (A, B) o (A', B') = (A A', A B' + B)
  ks_step<NB, DN, 1>(v, b, sh, [](Aff f, Aff g) { return Aff{f.A * g.A, __builtin_fma(f.A, g.B, f.B)}; });
  return v;
}

__device__ __forceinline__ Mob mob_norm(Mob t) {
  const double sc = fm_rcp(fabs(t.p11) + fabs(t.p12) + fabs(t.p21) + fabs(t.p22));
  return Mob{t.p11 * sc, t.p12 * sc, t.p21 * sc, t.p22 * sc};
}
template <int NB>
__device__ __forceinline__ Mob scan_mob(Mob v, int b) {
  auto sh = [](auto sc, Mob x) {
    constexpr int S = decltype(sc)::value;
    return Mob{row_shr<S>(x.p11), row_shr<S>(x.p12), row_shr<S>(x.p21), row_shr<S>(x.p22)};
  };
  // self (later blocks) on the left
  ks_step<NB, true, 1>(v, b, sh, [](Mob f, Mob g) {
    return mob_norm(Mob{__builtin_fma(f.p11, g.p11, f.p12 * g.p21), __builtin_fma(f.p11, g.p12, f.p12 * g.p22),
                        __builtin_fma(f.p21, g.p11, f.p22 * g.p21), __builtin_fma(f.p21, g.p12, f.p22 * g.p22)});
  });
  return v;
}

// Partitioned Thomas solve of a column's tridiagonal system, rows in blocks of M on the NB
// lanes of the column.  Row k: a_k x_{k-1} + d_k x_k + c_k x_{k+1} = r_k, with a = 0 on the
// column's first row and c = 0 on its last (rows past the bottom of a partial block: a = c =
// r = 0, d = 1).  row(m, a, d, c) gives the coefficients of the block's row m, rhs(m) its r;
// x returns the solution.
// Pivots bet_k = d_k - a_k c_{k-1} / bet_{k-1}:
//   * MOBIUS: each block multiplies its M Möbius matrices [[d, -a c_{k-1}], [1, 0]], a scan
//     multiplies the block products, block b reads its incoming pivot off blocks 0..b-1 and
//     eliminates from it.  Exact for well-separated eigenvalues (the pp system: d ~ 4, a c ~ 1);
//   * serial (MOBIUS = false): block after block, the incoming pivot handed down by DPP (1/NB
//     lane use for this one recurrence).  Needed for the w system: it is nearly a scaled
//     discrete Laplacian (acoustic coupling ~1e8 against layer masses ~1e2), whose matrices
//     [[2, -1], [1, 0]] are a Jordan block -- products of normalised block products cancel
//     (first KS step ~0.2, third ~5e-5 of their inputs' size) and a column's pivot came out
//     0 / 0 on the GPU.
// The forward substitution y_k = (r_k - a_k y_{k-1}) / bet_k and the back substitution
// x_k = y_k - gam_{k+1} x_{k+1} are affine recurrences: a block pass with a zero carry gives
// the block's map, a scan composes the maps, a second pass runs from the true carry (as
// accurate as the sequential sweep: ~1e-14 of the mean |x| on both systems in a numpy model).
// The pivots depend on the rows only: tri_factor forms them (gam_k = c_{k-1} / bet_{k-1}, rbs_k
// = 1 / bet_k) once, tri_apply solves for a right-hand side -- several right-hand sides of one
// system (remap_blk_k's tracers) share one factorisation.
template <int M, int NB, bool MOBIUS, class Row>
__device__ __forceinline__ void tri_factor(Row row, double (&gam)[M], double (&rbs)[M], int b) {
  auto cof = [&](int m, double& a_, double& d_, double& c_) { row(m, a_, d_, c_); };
  auto c_of = [&](int m) { double a_, d_, c_; cof(m, a_, d_, c_); return c_; };
  const double cprev_ = blk_prev(c_of(M - 1));
  const double cprev = b == 0 ? 0.0 : cprev_;  // c of the row above the block
  auto c_up = [&](int m) { return m > 0 ? c_of(m > 0 ? m - 1 : 0) : cprev; };
  // the block's elimination from an incoming 1 / pivot
  auto eliminate = [&](double rb) {
#pragma unroll
    for (int m = 0; m < M; ++m) {
      double a_, d_, c_;
      cof(m, a_, d_, c_);
      const double gm = c_up(m) * rb;
      rb = fm_rcp(__builtin_fma(-a_, gm, d_));
      gam[m] = gm;
      rbs[m] = rb;
    }
  };
  if constexpr (MOBIUS) {
    Mob T{1.0, 0.0, 0.0, 1.0};
#pragma unroll
    for (int m = 0; m < M; ++m) {
      double a_, d_, c_;
      cof(m, a_, d_, c_);
      const double e = a_ * c_up(m);
      T = Mob{__builtin_fma(d_, T.p11, -e * T.p21), __builtin_fma(d_, T.p12, -e * T.p22), T.p11, T.p12};
    }
    T = scan_mob<NB>(mob_norm(T), b);
    // incoming pivot: blocks 0..b-1 applied to (1, 0) (the top row has a = 0)
    const double pu = blk_prev(T.p11), pv = blk_prev(T.p21);
    eliminate(b == 0 ? 0.0 : fm_div(pv, pu));
  } else {
    double rb_in = 0.0;
#pragma unroll 1
    for (int r = 0; r < NB; ++r) {
      if (b == r) eliminate(rb_in);
      const double nx = blk_prev(rbs[M - 1]);
      rb_in = b == r + 1 ? nx : rb_in;
    }
  }
}

template <int M, int NB, class Row, class Rhs>
__device__ __forceinline__ void tri_apply(Row row, Rhs rhs, const double (&gam)[M], const double (&rbs)[M],
                                          double (&x)[M], int b, bool last) {
  auto a_of = [&](int m) { double a_, d_, c_; row(m, a_, d_, c_); return a_; };
  // y with a zero carry, and its coefficient on the carry
  double yh = 0.0, A = 1.0;
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const double a_ = a_of(m);
    yh = __builtin_fma(-a_, yh, rhs(m)) * rbs[m];
    A = -a_ * A * rbs[m];
  }
  const double gam_nb = blk_next(gam[0]);
  auto gnext = [&](int m) { return m + 1 < M ? gam[m + 1 < M ? m + 1 : 0] : (last ? 0.0 : gam_nb); };
  double Bc = 1.0;  // back-substitution coefficient of the block's top row on the carry below
#pragma unroll
  for (int m = M - 1; m >= 0; --m) Bc = -gnext(m) * Bc;
  const Aff F = scan_aff<NB, true>(Aff{A, yh}, b);
  const double yu = blk_prev(F.B);
  double y = b == 0 ? 0.0 : yu;
#pragma unroll
  for (int m = 0; m < M; ++m) {
    y = __builtin_fma(-a_of(m), y, rhs(m)) * rbs[m];
    x[m] = y;
  }
  double xh = 0.0;
#pragma unroll
  for (int m = M - 1; m >= 0; --m) xh = __builtin_fma(-gnext(m), xh, x[m]);
  const Aff H = scan_aff<NB, false>(Aff{Bc, xh}, b);
  const double xd = blk_next(H.B);
  double xi = last ? 0.0 : xd;
#pragma unroll
  for (int m = M - 1; m >= 0; --m) {
    xi = __builtin_fma(-gnext(m), xi, x[m]);
    x[m] = xi;
  }
}

template <int M, int NB, bool MOBIUS, class Row, class Rhs>
__device__ __forceinline__ void tri_solve(Row row, Rhs rhs, double (&x)[M], int b, bool last) {
  double gam[M], rbs[M];
  tri_factor<M, NB, MOBIUS>(row, gam, rbs, b);
  tri_apply<M, NB>(row, rhs, gam, rbs, x, b, last);
}

}  // namespace gtfv3
