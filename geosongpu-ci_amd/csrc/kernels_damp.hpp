// kernels_damp.hpp — launchers of d_sw's damping options (damp.hip): the per-level parameters
// of FV3 dyn_core's k loop (sponge layers included), higher-order divergence damping (nord
// 1..3), vorticity damping, the del-n flux damping of delp / pt inside fv_tp_2d, the w damping,
// and the d_con heating / diss_est with its del2_cubed smoothing.
#pragma once
#include <functional>
#include <vector>

#include "kernels.hpp"

namespace gtfv3 {

// d_sw's parameters of one level (FV3 dyn_core before each d_sw call; oracle
// sw_core.column_namelist), with the damping coefficients formed once on the host:
// a coefficient is 0 where its branch is off at that level.
struct LevelDamp {
  double d2_divg;  // nord == 0 divergence damping background (d2_bg; sponge: d2_bg_k1 / k2)
  double vt4;      // vorticity damping: (damp_vt da_min_c)^(nord_v+1), damp_vt > 1e-5
  double dp4;      // delp's del-n mass-flux damping in fv_tp_2d: (damp_vt da_min)^(nord_v+1), damp_vt > 1e-4
  double w4;       // w damping: (damp_w da_min_c)^(nord_w+1), damp_w > 1e-5
  double pt4;      // pt's mass-weighted del-n damping: (damp_t da_min)^(nord_t+1), damp_t > 1e-4
  double d_con;    // d_con_k (0 in the sponge layers)
  int nord, nord_v, nord_w, nord_t;
};
// the column from the namelist (vtdm4 / nord_v as in Namelist: vtdm4 is the namelist value,
// acting only with do_vort_damp)
std::vector<LevelDamp> column_damping(const Namelist& nl, double da_min, double da_min_c);
// FV3 dyn_core n_con: the top levels whose dissipated kinetic energy heats the air
int heat_levels(const Namelist& nl);
bool any_level(const LevelDamp* lv, int n, double LevelDamp::*coef);

// c_sw's divergence_corner (nord > 0): rarea_c * the dual-cell divergence at compute corners
void divergence_corner(const Ctx& c, int npz, const double* u, const double* v, const double* ua, const double* va,
                       double* divg);

struct DampArgs {
  int npz, nord;
  double dt, dddmp, d4_bg;
  const LevelDamp* lv;  // device table: levels with lv[k].nord == 0 take no corner term here
  const double* divg;  // c_sw's corner divergence, halo exchanged (kept: it is delpc)
  const double* wk;    // relative vorticity at cell centres (halo included)
  double* ke;          // += the corner damping term
  double* vd;          // out: the corner damping term (d_con heat)
  double *dd, *vcx, *ucy, *vort, *qx, *qy;  // scratch planes (npz levels)
};
void divergence_damping(const Ctx& c, const DampArgs& a);
void vorticity_wk(const Ctx& c, int npz, const double* u, const double* v, double* wk);

// which coefficient of LevelDamp scales the del-n field d2 = coef * q (DL_ONE: d2 = q, the
// mass-weighted form)
enum DelnCoef : int { DL_VT4 = 0, DL_DP4 = 1, DL_W4 = 2, DL_ONE = 3 };
// tp_core deln_flux's diffusive fluxes of levels [k0, k0+nk) of the cell field q: fx2 on
// y-edges, fy2 on x-edges, del-(2 nord + 2), nord 0..2 (d2: scratch)
void deln_fluxes(const Ctx& c, int npz, int k0, int nk, int nord, const LevelDamp* lv, int coef, const double* q,
                 double* d2, double* fx2, double* fy2);
// fx += fx2 / fy += fy2 on the flux regions (mass null), or the mass-weighted
// fx += 0.5 lv[k].pt4 (mass(i-1) + mass(i)) fx2
void deln_add(const Ctx& c, int npz, int k0, int nk, const LevelDamp* lv, const double* fx2, const double* fy2,
              const double* mass, double* fx, double* fy);
// the w damping: dw = div(fx2, fy2) rarea, hw = ke_dt - dw (w + dw / 2) on compute cells
void w_damping(const Ctx& c, int npz, int k0, int nk, double ke_dt, const double* fx2, const double* fy2,
               const double* w, double* dw, double* hw);
void w_damping_add(const Ctx& c, int npz, int k0, int nk, const double* dw, double* w);
// q += (fx2 - fx2(i+1) + fy2 - fy2(j+1)) rarea on compute cells of levels [k0, k0+nk)
// (update_dz_d's height damping)
void deln_div_add(const Ctx& c, int npz, int k0, int nk, const double* fx2, const double* fy2, double* q);
// update_dz_d's per-interface column (npz+1 levels): the d_sw column with the bottom level's
// (nord_v, damp_vt) repeated for the surface interface (FV3: damp(km+1) = damp(km))
std::vector<LevelDamp> height_damping(const std::vector<LevelDamp>& col);
// nord_w = 0 levels after the fused thermo march, one pass: dw from the old w, w_new += dw,
// hw (nullable) its heat -- bit-identical to deln_fluxes + w_damping + w_damping_add
void w_damping0_fused(const Ctx& c, int npz, int k0, int nk, const LevelDamp* lv, double ke_dt, const double* w,
                      double* w_new, double* hw);
// heat += delp (hw - 0.25 d_con_k rsin2 ...), diss += hw - rsin2 ... on compute cells (levels with
// d_con_k <= 1e-5: heat += hw, diss += hw); vorticity-damping fluxes where lv[k].vt4 > 0, hw where
// lv[k].w4 > 0 (hw nullable when no level has it)
void damping_heat(const Ctx& c, int npz, const LevelDamp* lv, const double* u, const double* v, const double* vd,
                  const double* fx2, const double* fy2, const double* hw, const double* delp, double* heat,
                  double* diss);
// u += fy2, v -= fx2 on the levels with lv[k].vt4 > 0
void vorticity_damping_apply(const Ctx& c, int npz, const LevelDamp* lv, const double* fx2, const double* fy2,
                             double* u, double* v);
// FV3 del2_cubed on levels [k0, k0+nk) of a cell field whose halo is filled: min(3, nmax)
// del-2 passes with coefficient cd, the cube-corner cells averaged first (fx, fy: scratch)
void del2_cubed(const Ctx& c, int npz, int k0, int nk, int nmax, double cd, double* q, double* fx, double* fy);
// after the acoustic sub-steps, levels [0, n_con): pt += sign(min(lim, |dT|), dT) / pkz with
// dT = heat / (cv_air delp)
void damping_heat_apply(const Ctx& c, int npz, int n_con, double delt, const double* heat, const double* delp,
                        const double* delz, double* pt);

// contiguous runs of levels where sel(level) >= 0, grouped by that value (a nord):
// fn(k0, nk, value)
template <class F>
void level_runs(const LevelDamp* lv, int n, F sel, const std::function<void(int, int, int)>& fn) {
  int k = 0;
  while (k < n) {
    const int key = sel(lv[k]);
    int e = k + 1;
    while (e < n && sel(lv[e]) == key) ++e;
    if (key >= 0) fn(k, e - k, key);
    k = e;
  }
}

}  // namespace gtfv3
