// kernels_misc.hpp — launchers of the pointwise fv_dynamics pieces (misc.hip).
#pragma once
#include "kernels.hpp"

namespace gtfv3 {

// zvir: Constants::zvir with moist physics, 0 for adiabatic (dry) dynamics
void fv_prep(const Ctx& c, int npz, int nq, double zvir, const double* delp, const double* delz, const double* q, double* pt,
             double* pkz);
void zh_init(const Ctx& c, int npz, const double* phis, const double* delz, double* zh);
void fv_wrapup(const Ctx& c, int npz, int nq, double zvir, const double* q, const double* delp, const double* delz,
               const double* w, double* pt, double* omga);
void c2l_ord4(const Ctx& c, int npz, const double* u, const double* v, double* ua, double* va);
void held_suarez(const Ctx& c, int npz, double dt, const double* pe, double* pt, double* u, double* v);
// copy the NG-wide halo ring of nplanes planes (every level of every sub-domain) src -> dst
void copy_halo_ring(const Ctx& c, int nplanes, const double* src, double* dst);
// per tracer: sum(q * delp * area), min, max, count of non-finite values over the compute
// domain of every local sub-domain; part: nq * nsub * npz * 4 doubles, out: nq * 4
void tracer_stats(const Ctx& c, int npz, int nq, const double* q, const double* delp, double* part, double* out);
void fill_field(const Ctx& c, long n, double a, double* x);
// y = max(y, x) elementwise
void max_field(const Ctx& c, long n, const double* x, double* y);

}  // namespace gtfv3
