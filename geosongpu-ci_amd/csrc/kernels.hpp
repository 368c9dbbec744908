// kernels.hpp — host launchers of the FV3 stencil kernels (HIP, gfx950).
// Every launcher enqueues on `st`, never synchronises, never allocates.
#pragma once
#include <hip/hip_runtime.h>

#include "gtfv3.hpp"
#include "hip_util.hpp"

namespace gtfv3 {

// Algorithmic bytes of one launch (bytes_manifest.yaml at the repo root):
// fp64 fields over the compute domain of every local sub-domain, each counted once per
// level read and once per level written -- cells C = nx*ny, x-edges X = (nx+1)*ny,
// y-edges Y = nx*(ny+1), corners K = (nx+1)*(ny+1) -- and 2-D metric planes once per
// launch (counted as C); halo re-reads and kernel-internal temporaries are not counted.
struct Ext {
  double C, X, Y, K;
};
inline Ext ext(const Dims& d) {
  const double n = d.nsub;
  return Ext{n * d.nx * d.ny, n * (d.nx + 1) * d.ny, n * d.nx * (d.ny + 1), n * (d.nx + 1) * (d.ny + 1)};
}
// register `doubles` fp64 values moved by the launch just issued
inline void gt_bytes(double doubles) { ktimer_bytes(8.0 * doubles); }

struct Ctx {
  Dims d;
  const SubInfo* subs;     // device [nsub]
  const SubInfo* hsubs;    // host copy
  const double* met;       // device [NMETRIC][nsub][plane]
  const double* cornerw;   // device [nsub][12]
  const double* area4;     // device [nsub][4][plane]: the cell area four times (tp_march lane groups)
  double da_min, da_min_c;
  hipStream_t st;
  // optional side stream of a stage whose launches split into independent parts (the thermo
  // march's tile-edge kernel beside its interior one): fork / join events; null: one stream
  hipStream_t side = nullptr;
  hipEvent_t side_fork = nullptr, side_join = nullptr;
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
  int nf = 0;    // fields per wave (1, 2, 3 dividing nt; 3 only with q_out); 0: 2 for even nt, else 1
  // tracer_2d_1l update fused into the march (mfx / mfy required): the nt tracers are
  // updated into q_out (no flux planes), dp2 = dp1 + mass-flux divergence written to dp2;
  // levels with it >= nsplt[k] are copied unchanged
  double* q_out = nullptr;
  const double* dp1 = nullptr;
  double* dp2 = nullptr;
  const int* nsplt = nullptr;
  int it = 0;
  // d_sw's u, v update fused into the vorticity march (nt = 1, no mass fluxes): u += ... + fy,
  // v += ... - fx with the corner kinetic energy ke (ds_uv's expressions); no flux plane
  const double* ke_uv = nullptr;
  double *u_uv = nullptr, *v_uv = nullptr;
  // update_dz_d's height update fused into the march (nt = 1, no mass fluxes): zh_out =
  // (zh area + flux divergence) / (area + area-flux divergence), zh_update's expressions; no
  // flux plane
  double* zh_out = nullptr;
};
void fv_tp_2d(const Ctx& c, const TpArgs& a);

// d_sw's thermodynamic transport in one march (tp.hip, tp_march<.., 3, TM = 1>): fv_tp_2d
// of delp (mass fluxes xfx / yfx), of w and pt with delp's fluxes as mass fluxes, the
// flux-capacitor accumulation mfx += fx, mfy += fy, and the delp / w / pt update, the
// fluxes never leaving registers.  New values go to *_o (the inputs are the march's halo
// sources for neighbouring waves, so the update cannot be in place).
struct ThermoArgs {
  int npz, ord;
  const double *delp, *w, *pt;
  double *delp_o, *w_o, *pt_o;
  const double *crx, *cry, *xfx, *yfx;
  double *mfx, *mfy;
};
void d_sw_thermo_march(const Ctx& c, const ThermoArgs& a);

// tracer_2d_1l pieces
void tracer_prep(const Ctx& c, int npz, const double* cx, const double* cy, double* xfx, double* yfx,
                 double* cmax_dev);
// per-level sub-step counts nsplt[k] = int(1 + cmax[k]) (fv_tracer2d), on the device
void tracer_nsplt(const Ctx& c, int npz, const double* cmax_dev, int* nsplt_dev);
void tracer_split(const Ctx& c, int npz, const int* nsplt_dev, double* cx, double* cy, double* xfx, double* yfx,
                  double* mfx, double* mfy);
void tracer_dp2(const Ctx& c, int npz, const double* dp1, const double* mfx, const double* mfy, double* dp2);
void tracer_update(const Ctx& c, int npz, int nq, double* q, const double* qn, const double* dp1,
                   const double* dp2, const double* fx, const double* fy, const int* nsplt_dev, int it);
void copy_levels(const Ctx& c, long n_elems, const double* src, double* dst);

}  // namespace gtfv3
