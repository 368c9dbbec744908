// kernels_sw.hpp — launchers of the shallow-water core (sw.hip) and the
// non-hydrostatic / vertical pieces (nh.hip, remap.hip).
#pragma once
#include "kernels.hpp"
#include "kernels_damp.hpp"

namespace gtfv3 {

struct CswArgs {
  int npz;
  double dt2;
  const double *delp, *pt, *w, *u, *v;
  double *uc, *vc, *ua, *va, *ut, *vt;  // outputs (ut, vt: dt2 * area fluxes)
  double *delpc, *ptc, *wc;
  double *utmp, *vtmp, *ke, *vort;  // scratch
  // optional: d_sw's cell vorticity + Coriolis of this sub-step's starting u, v (ds_vort's
  // expressions), formed by d2a2c's first kernel, which reads those u, v already
  double* dvort = nullptr;
};
void c_sw(const Ctx& c, const CswArgs& a);            // the two stages in order
// d2a2c_vect, delpc / ptc / wc, ke.  part (the interior / boundary split of the u, v exchange,
// Dycore::step): 0 everything; 1 cs_tmp on the points that read no halo value only (while the
// exchange's messages fly); 2 the rest -- cs_tmp's boundary frame and the stages after it
void c_sw_transport(const Ctx& c, const CswArgs& a, int part = 0);
// the split needs sub-domains of at least 6 x 6 cells
bool split_fits(const Dims& d);
void c_sw_winds(const Ctx& c, const CswArgs& a);      // vorticity, uc / vc update
int kloop_levels();                                          // GTFV3_KLOOP (stencil_common.hpp)

struct DswArgs {
  int npz;
  double dt, dddmp;  // (d2_bg per level: lv[k].d2_divg)
  int hord_mt, hord_vt, hord_tm, hord_dp;
  double *delp, *pt, *w, *u, *v;      // updated in place (u, v left multiplied by dx, dy)
  // optional: delp, pt, w updated into these (fused thermo march, d_sw_thermo_fused) --
  // the caller then takes them as the new fields
  double *delp_o = nullptr, *pt_o = nullptr, *w_o = nullptr;
  const double *uc, *vc, *ua, *va;
  double *crx, *cry, *xfx, *yfx;      // per level, saved for update_dz_d
  double *cx, *cy, *mfx, *mfy;        // accumulated
  double *ut, *vt, *fx, *fy, *gwx, *gwy, *gtx, *gty, *ke, *vort;  // scratch
  double *gvx, *gvy;  // vorticity fluxes (own planes: the wind stage may run beside the thermo stage)
  // damping (damp.hip): the column of per-level parameters (column_damping; device table lv,
  // its host copy hlv, npz entries each) -- required -- and the namelist-wide switches
  const LevelDamp* lv = nullptr;
  const LevelDamp* hlv = nullptr;
  int nord = 0;         // the namelist nord (c_sw's divg exists when > 0)
  double d4_bg = 0.0;
  double d_con = 0.0;   // the namelist d_con: > 1e-5 sums the heat / diss_est of every level
  double ke_dt = 0.0;   // ke_bg |dt| (the w damping's background heat)
  const double* divg = nullptr;  // nord > 0: c_sw's corner divergence, halo exchanged
  double *wk = nullptr, *vd = nullptr;  // cell vorticity; the corner damping term (d_con)
  double *dd = nullptr, *dvcx = nullptr, *ducy = nullptr, *dvort = nullptr, *dqx = nullptr, *dqy = nullptr;
  double *d2 = nullptr, *fx2 = nullptr, *fy2 = nullptr;  // vorticity damping (winds stage)
  // del-n of delp / pt / w (thermo stage): scratch, the w increment and its heat
  double *td2 = nullptr, *tfx2 = nullptr, *tfy2 = nullptr, *dw = nullptr, *hw = nullptr;
  double *heat = nullptr, *diss = nullptr;               // d_con: summed over the sub-steps
};
void d_sw(const Ctx& c, const DswArgs& a);  // the three stages in order
// ut, vt, Courant numbers and area fluxes; utvt_done (optional) is recorded once ut / vt are
// written (d_sw's kinetic energy needs those, not the Courant numbers)
// part as c_sw_transport's, for the uc, vc exchange: 1 ds_utvt1 on the points that read no
// halo value, 2 its boundary frame and the stages after it
void d_sw_courant(const Ctx& c, const DswArgs& a, hipEvent_t utvt_done = nullptr, int part = 0);
void d_sw_thermo(const Ctx& c, const DswArgs& a);   // delp / w / pt transport, flux accumulation
// kinetic energy, vorticity transport, u, v.  vort_done: the cell vorticity was formed already
// (d_sw_vort, from the same u, v); the stream waits for the nwait events of march_wait before
// the vorticity march (which needs the Courant numbers)
void d_sw_winds(const Ctx& c, const DswArgs& a, bool vort_done = false, const hipEvent_t* march_wait = nullptr,
                int nwait = 0);
void d_sw_vort(const Ctx& c, const DswArgs& a);  // d_sw's cell vorticity of the old u, v (ds_vort)
// after both stages (needs the updated delp): d_con heat / diss_est, vorticity-damping fluxes
void d_sw_post(const Ctx& c, const DswArgs& a);
bool d_sw_post_needed(const DswArgs& a);
bool d_sw_thermo_fused(const DswArgs& a);           // delp/w/pt go to *_o (one march)

}  // namespace gtfv3
