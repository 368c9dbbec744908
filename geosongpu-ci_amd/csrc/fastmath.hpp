// fastmath.hpp — fp64 log / exp / reciprocal / division for gfx950 kernels that are
// bound by their transcendentals (the SIM1 Riemann solver: three logs and three exps per
// level).
//
// ocml's log_f64 carries its result in double-double (≈98 VALU instructions, 43 of them
// v_add_f64) and exp_f64 ≈42; both are ~0.5 ulp.  The forms here are ~1 ulp and a third to
// a half of that:
//   * fm_log: fdlibm's __ieee754_log reduction and its minimax polynomial in s = f/(2+f)
//     (Lg1..Lg7; < 1 ulp in fdlibm), the division by fm_div; ~37 instructions.
//   * fm_exp: Cody–Waite reduction by ln2 (fdlibm's ln2_hi / ln2_lo split), Taylor series to
//     r^13 on |r| <= ln2/2 (truncation < 5e-18 relative), ldexp; ~19 instructions.
//   * fm_rcp / fm_div: v_rcp_f64 + two Newton steps (+ one residual correction for the
//     quotient), without div_scale / div_fixup: valid for normal operands away from the
//     exponent extremes (|x| in [2^-1000, 2^1000]), which every caller guarantees.
// Arguments are finite and positive (log) / |x| < 700 (exp); no special-value handling.
// CPU restatement of the same arithmetic: tests/test_fastmath.py (ulp error against
// numpy over the ranges the solver uses).
#pragma once
#include <hip/hip_runtime.h>

namespace gtfv3 {

__device__ __forceinline__ double fm_rcp(double x) {
  double r = __builtin_amdgcn_rcp(x);
  double e = __builtin_fma(-x, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-x, r, 1.0);
  return __builtin_fma(r, e, r);
}

__device__ __forceinline__ double fm_div(double a, double b) {
  const double r = fm_rcp(b);
  const double q = a * r;
  const double e = __builtin_fma(-b, q, a);
  return __builtin_fma(r, e, q);
}

__device__ __forceinline__ double fm_log(double x) {
  constexpr double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
  constexpr double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01, Lg3 = 2.857142874366239149e-01,
                   Lg4 = 2.222219843214978396e-01, Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
                   Lg7 = 1.479819860511658591e-01;
  double m = __builtin_amdgcn_frexp_mant(x);  // [0.5, 1)
  int e = __builtin_amdgcn_frexp_exp(x);
  const bool lo = m < 0.70710678118654752440;
  m = lo ? m + m : m;  // [sqrt(1/2), sqrt(2))
  e = lo ? e - 1 : e;
  const double f = m - 1.0;
  const double s = fm_div(f, 2.0 + f);
  const double dk = (double)e;
  const double z = s * s, w = z * z;
  const double t1 = w * __builtin_fma(w, __builtin_fma(w, Lg6, Lg4), Lg2);
  const double t2 = z * __builtin_fma(w, __builtin_fma(w, __builtin_fma(w, Lg7, Lg5), Lg3), Lg1);
  const double R = t2 + t1;
  const double hfsq = 0.5 * f * f;
  return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
}

__device__ __forceinline__ double fm_exp(double x) {
  constexpr double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
  const double k = __builtin_rint(x * 1.44269504088896338700e+00);
  double r = __builtin_fma(-k, ln2_hi, x);
  r = __builtin_fma(-k, ln2_lo, r);
  double p = 1.0 / 6227020800.0;  // 1/13!
  p = __builtin_fma(p, r, 1.0 / 479001600.0);
  p = __builtin_fma(p, r, 1.0 / 39916800.0);
  p = __builtin_fma(p, r, 1.0 / 3628800.0);
  p = __builtin_fma(p, r, 1.0 / 362880.0);
  p = __builtin_fma(p, r, 1.0 / 40320.0);
  p = __builtin_fma(p, r, 1.0 / 5040.0);
  p = __builtin_fma(p, r, 1.0 / 720.0);
  p = __builtin_fma(p, r, 1.0 / 120.0);
  p = __builtin_fma(p, r, 1.0 / 24.0);
  p = __builtin_fma(p, r, 1.0 / 6.0);
  p = __builtin_fma(p, r, 0.5);
  p = __builtin_fma(p, r, 1.0);
  p = __builtin_fma(p, r, 1.0);
  return __builtin_amdgcn_ldexp(p, (int)k);
}

// x^y for x > 0 as FV3 writes it, exp(y * log(x))
__device__ __forceinline__ double fm_pow(double x, double y) { return fm_exp(y * fm_log(x)); }

}  // namespace gtfv3
