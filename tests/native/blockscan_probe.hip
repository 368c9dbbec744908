// blockscan_probe.hip — test-only shared library (tests/native/bin/libblockscan_probe.so)
// that runs the device helpers of csrc/fastmath.hpp and csrc/blockscan.hpp on given host
// arrays, for tests/test_gpu_fastmath.py to compare against numpy:
//   probe_math(kind, x, y, out, n):  kind 0 fm_log(x), 1 fm_exp(x), 2 fm_div(x, y), 3 fm_rcp(x)
//   probe_shift(in, out): per 64-lane wave, out[0..63] = blk_prev, [64..] blk_next, [128..]
//     scan_sum<8, DN>, [192..] scan_sum<8, UP>, [256..] row_shr<4>, [320..] scan_sum<16, DN>
//   probe_tri(ncol, a, d, c, r, x, mobius): ncol columns of 72 rows (NB = 8 blocks of 9) solved by
//     tri_solve (Möbius-scan or serial pivots); arrays [ncol][72]
#include <hip/hip_runtime.h>

#include <cstdio>

#include "../../geosongpu-ci_amd/csrc/blockscan.hpp"

using namespace gtfv3;

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      return 1;                                                             \
    }                                                                       \
  } while (0)

__global__ void k_math(int kind, const double* x, const double* y, double* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double v = 0.0;
  if (kind == 0) v = fm_log(x[i]);
  else if (kind == 1) v = fm_exp(x[i]);
  else if (kind == 2) v = fm_div(x[i], y[i]);
  else v = fm_rcp(x[i]);
  out[i] = v;
}

__global__ void k_shift(const double* in, double* out) {
  const int lane = threadIdx.x;
  const double v = in[lane];
  out[lane] = blk_prev(v);
  out[64 + lane] = blk_next(v);
  out[128 + lane] = scan_sum<8, true>(v, lane & 7);
  out[192 + lane] = scan_sum<8, false>(v, lane & 7);
  out[256 + lane] = row_shr<4>(v);
  out[320 + lane] = scan_sum<16, true>(v, lane & 15);
}

template <bool MOBIUS>
__global__ void k_tri(int ncol, const double* A, const double* D, const double* C, const double* R, double* X) {
  constexpr int M = 9, NB = 8;
  const int lane = threadIdx.x & 63;
  const int b = lane & (NB - 1);
  int col = (blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)) * (64 / NB) + lane / NB;
  const bool valid = col < ncol;
  if (!valid) col = ncol - 1;
  const long base = (long)col * 72 + b * M;
  double x[M];
  auto row = [&](int m, double& a_, double& d_, double& c_) {
    a_ = A[base + m];
    d_ = D[base + m];
    c_ = C[base + m];
  };
  tri_solve<M, NB, MOBIUS>(row, [&](int m) { return R[base + m]; }, x, b, b == NB - 1);
  if (valid)
    for (int m = 0; m < M; ++m) X[base + m] = x[m];
}

extern "C" int probe_math(int kind, const double* x, const double* y, double* out, int n) {
  double *dx, *dy, *dout;
  CK(hipMalloc(&dx, n * 8));
  CK(hipMalloc(&dy, n * 8));
  CK(hipMalloc(&dout, n * 8));
  CK(hipMemcpy(dx, x, n * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dy, y, n * 8, hipMemcpyHostToDevice));
  k_math<<<(n + 255) / 256, 256>>>(kind, dx, dy, dout, n);
  CK(hipGetLastError());
  CK(hipMemcpy(out, dout, n * 8, hipMemcpyDeviceToHost));
  CK(hipFree(dx));
  CK(hipFree(dy));
  CK(hipFree(dout));
  return 0;
}

extern "C" int probe_shift(const double* in, double* out) {
  double *din, *dout;
  CK(hipMalloc(&din, 64 * 8));
  CK(hipMalloc(&dout, 384 * 8));
  CK(hipMemcpy(din, in, 64 * 8, hipMemcpyHostToDevice));
  k_shift<<<1, 64>>>(din, dout);
  CK(hipGetLastError());
  CK(hipMemcpy(out, dout, 384 * 8, hipMemcpyDeviceToHost));
  CK(hipFree(din));
  CK(hipFree(dout));
  return 0;
}

extern "C" int probe_tri(int ncol, const double* a, const double* d, const double* c, const double* r, double* x,
                         int mobius) {
  const size_t n = (size_t)ncol * 72 * 8;
  double *da, *dd, *dc, *dr, *dx;
  CK(hipMalloc(&da, n));
  CK(hipMalloc(&dd, n));
  CK(hipMalloc(&dc, n));
  CK(hipMalloc(&dr, n));
  CK(hipMalloc(&dx, n));
  CK(hipMemcpy(da, a, n, hipMemcpyHostToDevice));
  CK(hipMemcpy(dd, d, n, hipMemcpyHostToDevice));
  CK(hipMemcpy(dc, c, n, hipMemcpyHostToDevice));
  CK(hipMemcpy(dr, r, n, hipMemcpyHostToDevice));
  const int blocks = (ncol + 31) / 32;  // 4 waves x 8 columns
  if (mobius) k_tri<true><<<blocks, 256>>>(ncol, da, dd, dc, dr, dx);
  else k_tri<false><<<blocks, 256>>>(ncol, da, dd, dc, dr, dx);
  CK(hipGetLastError());
  CK(hipMemcpy(x, dx, n, hipMemcpyDeviceToHost));
  CK(hipFree(da));
  CK(hipFree(dd));
  CK(hipFree(dc));
  CK(hipFree(dr));
  CK(hipFree(dx));
  return 0;
}
