// kernels_nh.hpp — launchers of the non-hydrostatic (nh.hip) and remap (remap.hip) kernels.
#pragma once
#include "kernels.hpp"

namespace gtfv3 {

struct LevelDamp;  // kernels_damp.hpp

// per-column work planes (each npz+1 levels, [sub][k][plane])
struct NhScratch {
  double* s[14];
};

void update_dz_c(const Ctx& c, int npz, const double* dp0, const double* ut, const double* vt, const double* gz,
                 double* gz_out);
// clamp + ws + SIM1 on the C-grid half step; gz: heights in, geopotential out
void riem_solver_c(const Ctx& c, int npz, double dt2, double ptop, double p_fac, double dz_min, const double* delpc,
                   const double* ptc, const double* wc, const double* phis, double* gz, double* pef,
                   const NhScratch& sc);
void p_grad_c(const Ctx& c, int npz, double dt2, const double* delpc, const double* pkc, const double* gz, double* uc,
              double* vc);

struct UdzdArgs {
  int npz, hord;
  const double* dp0;
  const double *crx, *cry, *xfx, *yfx;
  double *crx_e, *cry_e, *xfx_e, *yfx_e;
  const double* zh;
  double* zh_out;  // the updated heights (out of place: the march reads zh's neighbours)
  // damp_vt of the heights (FV3 update_dz_d's del6_vt_flux of zh): the npz+1-level column of
  // kernels_damp.hpp height_damping, device and host copies; null: no level damps.  d2, fx2,
  // fy2: npz+1-level scratch planes
  const LevelDamp* lv = nullptr;
  const LevelDamp* hlv = nullptr;
  double *d2 = nullptr, *fx2 = nullptr, *fy2 = nullptr;
};
void update_dz_d(const Ctx& c, const UdzdArgs& a);
// update_dz_d's edge_profile of (crx, xfx) on x-face and (cry, yfx) on y-face columns.
// variant: 0 = by level count (register column for 3 <= npz <= 80, blocked above),
// 1 = force the blocked form edge_prof_k (the bitwise reference of the register form)
void edge_profile(const Ctx& c, int npz, const double* dp0, const double* crx, const double* xfx, const double* cry,
                  const double* yfx, double* crx_e, double* xfx_e, double* cry_e, double* yfx_e, int variant = 0);

struct Riem3Args {
  int npz;
  double dt, ptop, p_fac, dz_min;
  int last_call;
  const double *delp, *pt, *phis;
  double *w, *delz, *zh, *ppe, *pk3, *pe, *peln, *pk;
  double* ws;  // surface w (dz/dt of the ground), consumed by the remap; may be null
};
void riem_solver3(const Ctx& c, const Riem3Args& a, const NhScratch& sc);
// Riemann kernel form: 0 = register-resident level blocks (default), 1 = column sweeps
// through scratch planes (riem_col_k, kept as the bitwise reference of the blocked form)
void set_riem_variant(int v);
int riem_variant();
void pk3_pe_halo(const Ctx& c, int npz, double ptop, bool do_pe, const double* delp, double* pk3, double* pe);
void a2b_ord4(const Ctx& c, int nk, const double* q, double* qout, double* qx, double* qy);
// up to four fields in one launch (same result as one a2b_ord4 call per field)
// scale (optional, per field): each field is multiplied by it as it is loaded
void a2b_ord4_multi(const Ctx& c, int nf, const int* nk, const double* const* q, double* const* qout,
                    const double* scale = nullptr);

struct NhPgArgs {
  int npz;
  double dt, ptop;
  const double *pp, *pk3, *gz, *delp;
  double *ppb, *pkb, *gzb, *wk1, *qx, *qy;
  double *u, *v;
  // gz enters a2b_ord4 multiplied by this as it is loaded (the step passes zh and grav)
  double gz_scale = 1.0;
};
void nh_p_grad(const Ctx& c, const NhPgArgs& a);
void scale_field(const Ctx& c, long n, double a, const double* x, double* y);

struct RemapState {
  double *pe, *peln, *pk, *pkz, *delp, *delz, *pt, *w, *q, *u, *v, *ps, *ws;
};
struct RemapScratch {
  double* s[3];  // q edges, gam, source copy: remap_scratch_slots(nq) * (npz+1) levels each
};
int remap_jobs(int nq);
int remap_scratch_slots(int nq);  // scratch column sets (jobs run in chunks of this many)
// variant: 0 = the level-block form (remap_blkq_k tracers) where a shape is instantiated, else
// the scratch-column jobs (remap_job_k, the generic form for any level count); 3 = the level
// blocks one tracer per wave; 1 = the scratch-column jobs
int remap_variant();  // GTFV3_REMAP (default 0: the level-block form where instantiated)
void lagrangian_to_eulerian(const Ctx& c, int npz, int nq, double ptop, bool fill, const double* ak_dev,
                            const double* bk_dev, const RemapState& S, const RemapScratch& R, int variant = 0,
                            int phase = 0);  // 1: prep + T_v/delz/w/winds, 2: tracers + finish

}  // namespace gtfv3
