// kernels_moist.hpp — launchers of the moist column physics (moist.hip).
// Layer fields [sub][k][plane] (k = 0 top); 2-D outputs [sub][plane].
#pragma once
#include "kernels.hpp"

namespace gtfv3 {

// saturation specific humidity over water / ice (GFDL table form) and d(qsw)/dT
void moist_qsat(const Ctx& c, int nk, const double* t, const double* p, double* qsw, double* qsi, double* dqsw);
// column fill of negative q keeping sum(q dp); fill = -sum(min(q,0) dp)
void fillq2zero(const Ctx& c, int nk, double* q, const double* dp, double* fill);

struct Gfdl1mArgs {
  int nk;
  int qsub = 0;  // levels per sub-domain of the species arrays (0: nk; nq*nk for slices of the tracer array q)
  double dt;
  double *T, *qv, *ql, *qr, *qi, *qs, *qg;  // updated in place
  const double *dp, *dz;                   // delp (Pa), delz (m, < 0)
  const double *pm = nullptr, *pe = nullptr;  // layer pressure (Pa), or interface pressure (L+1)
  double *pr, *ps, *pg, *pi;               // surface rain / snow / graupel / ice (kg m-2 per step)
};
void gfdl_1m(const Ctx& c, const Gfdl1mArgs& a);

// parcel buoyancy (per level), CAPE, CIN and the LCL level index (-1: none)
void buoyancy(const Ctx& c, int nk, const double* t, const double* qv, const double* pm, const double* zm,
              double* by, double* cape, double* cin, double* klcl);

}  // namespace gtfv3
