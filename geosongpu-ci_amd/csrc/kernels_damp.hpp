// kernels_damp.hpp — launchers of d_sw's damping options (damp.hip): higher-order divergence
// damping (nord 1..3), vorticity damping (vtdm4, nord_v) and the d_con heating / diss_est.
#pragma once
#include "kernels.hpp"

namespace gtfv3 {

// c_sw's divergence_corner (nord > 0): rarea_c * the dual-cell divergence at compute corners
void divergence_corner(const Ctx& c, int npz, const double* u, const double* v, const double* ua, const double* va,
                       double* divg);

struct DampArgs {
  int npz, nord;
  double dt, dddmp, d2_bg, d4_bg;
  const double* divg;  // c_sw's corner divergence, halo exchanged (kept: it is delpc)
  const double* wk;    // relative vorticity at cell centres (halo included)
  double* ke;          // += the corner damping term
  double* vd;          // out: the corner damping term (d_con heat)
  double *dd, *vcx, *ucy, *vort, *qx, *qy;  // scratch planes (npz levels)
};
void divergence_damping(const Ctx& c, const DampArgs& a);
void vorticity_wk(const Ctx& c, int npz, const double* u, const double* v, double* wk);
// del-(2 nord + 2) diffusive fluxes of wk: fx2 on y-edges, fy2 on x-edges (nord 0..2)
void del6_vt_flux(const Ctx& c, int npz, int nord, double damp, const double* wk, double* d2, double* fx2,
                  double* fy2);
// heat += delp * (-0.25 d_con rsin2 ...), diss += -rsin2 ... on compute cells (fx2 / fy2 nullable)
void damping_heat(const Ctx& c, int npz, double d_con, const double* u, const double* v, const double* vd,
                  const double* fx2, const double* fy2, const double* delp, double* heat, double* diss);
void vorticity_damping_apply(const Ctx& c, int npz, const double* fx2, const double* fy2, double* u, double* v);
void damping_heat_apply(const Ctx& c, int npz, double delt, const double* heat, const double* delp, const double* delz,
                        double* pt);

}  // namespace gtfv3
