// kernels_moist.hpp — launchers of the moist column physics (moist.hip).
// Layer fields [sub][k][plane] (k = 0 top); 2-D outputs [sub][plane].
#pragma once
#include "kernels.hpp"

namespace gtfv3 {

// saturation specific humidity over water / ice (GFDL table form) and d(qsw)/dT
void moist_qsat(const Ctx& c, int nk, const double* t, const double* p, double* qsw, double* qsi, double* dqsw);
// column fill of negative q keeping sum(q dp); fill = -sum(min(q,0) dp)
void fillq2zero(const Ctx& c, int nk, double* q, const double* dp, double* fill);

// GFDL single-moment cloud microphysics (gfdl_cloud_microphys_driver -> mpdrv per column:
// neg_adj, terminal_fall with Lagrangian PPM sedimentation + sedi_heat, warm_rain, icloud)
struct Gfdl1mArgs {
  int nk;
  int qsub = 0;  // levels per sub-domain of the species arrays (0: nk; nq*nk for slices of the tracer array q)
  double dt;
  double *T, *qv, *ql, *qr, *qi, *qs, *qg;  // updated in place
  const double *dp, *dz;                   // delp (Pa), delz (m, < 0)
  double* scr;                             // gfdl_mp_scratch_levels(nk) planes per sub-domain
  double *pr, *ps, *pg, *pi;               // surface rain / snow / graupel / ice (kg m-2 per step)
  int variant = 0;                         // 0: the level-block form where instantiated, 1: the column driver
};
int gfdl_mp_scratch_levels(int nk);
void gfdl_1m(const Ctx& c, const Gfdl1mArgs& a);

// GEOS evap_subl_pdf loop: MELTFRZ of anvil and large-scale condensate, EVAP3 / SUBL3 of the
// anvil condensate, hystpdf large-scale condensation (uniform PDF); all in place
struct EvapSublArgs {
  int nk;
  double dt;
  double *T, *qv, *qlls, *qils, *qlcn, *qicn, *clls, *clcn;
  long qv_sub = 0, ql_sub = 0, qi_sub = 0;  // levels per sub-domain of qv / qlls / qils (0: nk)
  const double *pl, *nactl, *nacti;
};
void evap_subl_pdf(const Ctx& c, const EvapSublArgs& a);

// GEOS RADCOUPLE: in-cloud water contents, total cloud fraction and effective radii
struct RadcoupleArgs {
  int nk;
  long qv_sub = 0, ql_sub = 0, qi_sub = 0, qr_sub = 0, qs_sub = 0, qg_sub = 0;
  const double *T, *pl, *cf, *af, *qv, *qlls, *qils, *qlcn, *qicn, *qr, *qs, *qg, *nl;
  double *rqv, *rql, *rqi, *rqr, *rqs, *rqg, *rcf, *rrl, *rri;
};
void radcouple(const Ctx& c, const RadcoupleArgs& a);

// aerosol activation (Abdul-Razzak & Ghan 2000, three lognormal modes) and ice nuclei
void aer_activation(const Ctx& c, int nk, long qv_sub, const double* pl, const double* t, const double* qv,
                    const double* zm, const double* w, double* nactl, double* nacti, double* smax);

// GEOS cup_gf_sh shallow cumulus (Grell-Freitas shallow plume): source level, cloud base,
// entraining updraft, cloud top, convective-velocity closure, flux-form tendencies of T and
// qv, detrained condensate added to qlcn / qicn, convective cloud fraction, index fields
struct GfShArgs {
  int nk;
  long qv_sub = 0;  // levels per sub-domain of qv (0: nk)
  double dt;
  double *T, *qv;                             // updated in place
  const double *pl, *zm, *dp;                 // layer pressure (Pa), mid heights (m), delp (Pa)
  const double *kpbl, *hfx;                   // 2-D: PBL-top level index, sensible heat flux (W m-2)
  double *qlcn, *qicn;                        // detrained condensate added
  double *cf, *mb, *k22, *kbcon, *ktop;       // cloud fraction (L); 2-D mass flux and indices (-1: none)
  double* scr;                                // gf_scratch_levels(nk) planes per sub-domain
};
int gf_scratch_levels(int nk);
// uniform surface sensible heat flux (W m-2) of the Aquaplanet coupling when no "hfx" field
// was uploaded (no surface model on this path)
constexpr double kSurfaceHfx = 15.0;
void cup_gf_sh(const Ctx& c, const GfShArgs& a);

// layer pressure from the interfaces pe, layer-mid heights from delz (surface at 0) and the
// PBL-top level index (the highest level below 1 km)
void moist_prep(const Ctx& c, int nk, const double* pe, const double* dz, double* pl, double* zm, double* kpbl);

// parcel buoyancy (per level), CAPE, CIN and the LCL level index (-1: none)
void buoyancy(const Ctx& c, int nk, const double* t, const double* qv, const double* pm, const double* zm,
              double* by, double* cape, double* cin, double* klcl);

}  // namespace gtfv3
