// column.hip — K-column primitives with the GT4Py interval semantics the reference's
// DSL pattern tests pin (dsl_patterns/*.py), HIP for gfx950.
//
// One lane per (sub-domain, i, j) column over the compute domain; lanes are i-fastest
// so every level's load is a coalesced 64-wide row, and k runs sequentially in
// registers (the K axis is never split).  These are the building blocks
// of the moist column kernels (top-of-column reads, level searches, index gathers).
//
//   column_top       FORWARD interval(-1, None): tmp2d = in;  PARALLEL: out = tmp2d
//                    (Do__get_top_of_the_column.py:33-38)
//   column_while_lt  out[k] = smallest lev >= 0 with in[k + lev] >= thr (K-relative
//                    offset evaluated per level, Do__while_in_gt_functions.py:23-32);
//                    the search stops at the last level (lev = nk-1-k there)
//   column_gather_k  FORWARD interval(...): if kmask[k] == kidx: out2d = data[k]
//                    (WIP__hybrid_index_2dout.py:34-42; exact compare, last match wins)
#include "kernels_column.hpp"
#include "stencil_common.hpp"

namespace gtfv3 {
namespace {

struct ColPt {
  int s;
  long o;
};

__device__ __forceinline__ bool column_point(const Dims& d, ColPt& c) {
  const int i = blockIdx.x * BX + threadIdx.x, j = blockIdx.y * BY + threadIdx.y;
  c.s = blockIdx.z;
  c.o = pidx(d, i, j);
  return i < d.nx && j < d.ny;
}

__global__ void __launch_bounds__(256) col_top_k(Dims d, int nk, const double* __restrict__ in,
                                                 double* __restrict__ out) {
  ColPt c;
  if (!column_point(d, c)) return;
  const long base = (long)c.s * nk * d.plane + c.o;
  const double top = in[base + (long)(nk - 1) * d.plane];
  for (int k = 0; k < nk; ++k) out[base + (long)k * d.plane] = top;
}

__global__ void __launch_bounds__(256) col_while_k(Dims d, int nk, double thr, const double* __restrict__ in,
                                                   double* __restrict__ out) {
  ColPt c;
  if (!column_point(d, c)) return;
  const long base = (long)c.s * nk * d.plane + c.o;
  // sweep from the top of the column down: the answer at k is 0 where in[k] >= thr,
  // otherwise one more than at k+1 (the same as the per-level forward search)
  int lev = 0;
  for (int k = nk - 1; k >= 0; --k) {
    const double v = in[base + (long)k * d.plane];
    lev = (v >= thr || k == nk - 1) ? 0 : lev + 1;
    out[base + (long)k * d.plane] = (double)lev;
  }
}

__global__ void __launch_bounds__(256) col_gather_k(Dims d, int nk, const double* __restrict__ data,
                                                    const double* __restrict__ kmask,
                                                    const double* __restrict__ kidx, double* __restrict__ out) {
  ColPt c;
  if (!column_point(d, c)) return;
  const long base = (long)c.s * nk * d.plane + c.o;
  const long b2 = (long)c.s * d.plane + c.o;
  const double want = kidx[b2];
  double r = out[b2];
  for (int k = 0; k < nk; ++k) {
    const long q = base + (long)k * d.plane;
    if (kmask[q] == want) r = data[q];
  }
  out[b2] = r;
}

inline dim3 colgrid(const Dims& d) { return dim3(cdiv(d.nx, BX), cdiv(d.ny, BY), d.nsub); }

}  // namespace

void column_top(const Ctx& c, int nk, const double* in, double* out) {
  GT_LAUNCH(col_top_k, colgrid(c.d), dim3(BX, BY), 0, c.st, c.d, nk, in, out);
  HIP_LAUNCH_CHECK();
}

void column_while_lt(const Ctx& c, int nk, double thr, const double* in, double* out) {
  GT_LAUNCH(col_while_k, colgrid(c.d), dim3(BX, BY), 0, c.st, c.d, nk, thr, in, out);
  HIP_LAUNCH_CHECK();
}

void column_gather_k(const Ctx& c, int nk, const double* data, const double* kmask, const double* kidx,
                     double* out) {
  GT_LAUNCH(col_gather_k, colgrid(c.d), dim3(BX, BY), 0, c.st, c.d, nk, data, kmask, kidx, out);
  HIP_LAUNCH_CHECK();
}

}  // namespace gtfv3
