// kernels.hpp — host launchers of the FV3 stencil kernels (HIP, gfx950).
// Every launcher enqueues on `st`, never synchronises, never allocates.
#pragma once
#include <hip/hip_runtime.h>

#include "gtfv3.hpp"

namespace gtfv3 {

struct Ctx {
  Dims d;
  const SubInfo* subs;     // device [nsub]
  const SubInfo* hsubs;    // host copy
  const double* met;       // device [NMETRIC][nsub][plane]
  const double* cornerw;   // device [nsub][12]
  double da_min, da_min_c;
  hipStream_t st;
};

// fv_tp_2d: nt fields q[s][t][k] advected with fluxes [s][k]; fx/fy [s][t][k]
struct TpArgs {
  const double* q;
  const double* q2 = nullptr;                // optional second field (nt = 1) sharing the fluxes
  double *fx_2 = nullptr, *fy_2 = nullptr;   // its fluxes
  int nt, nk;
  const double *crx, *cry, *xfx, *yfx;  // (ra_x, ra_y are formed from area, xfx, yfx)
  const double *mfx, *mfy;  // nullable: use xfx/yfx
  double *fx, *fy;
  int ord;
  int cfg = -1;  // tile variant (tuning); -1: default
};
void fv_tp_2d(const Ctx& c, const TpArgs& a);

// tracer_2d_1l pieces
void tracer_prep(const Ctx& c, int npz, const double* cx, const double* cy, double* xfx, double* yfx,
                 double* cmax_dev);
void tracer_split(const Ctx& c, int npz, const int* nsplt_dev, double* cx, double* cy, double* xfx, double* yfx,
                  double* mfx, double* mfy);
void tracer_dp2(const Ctx& c, int npz, const double* dp1, const double* mfx, const double* mfy, double* dp2);
void tracer_update(const Ctx& c, int npz, int nq, double* q, const double* qn, const double* dp1,
                   const double* dp2, const double* fx, const double* fy, const int* nsplt_dev, int it);
void copy_levels(const Ctx& c, long n_elems, const double* src, double* dst);

}  // namespace gtfv3
