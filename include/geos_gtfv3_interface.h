/* geos_gtfv3_interface.h — C ABI of libgeos_gtfv3_interface.so, the MI355X-native
 * drop-in for the geos_gtfv3 bridge of GEOS-ESM/geosongpu-ci.
 *
 * Reference interfaces replaced (paths relative to the reference repo):
 *   - symbol names  : src/tcn/py_ftn_interface/templates/interface.c.jinja2:8
 *                     ("{{prefix}}_{{function.name}}_c") and interface.f90.jinja2:39
 *                     (bind(c, name='{{prefix}}_{{function.name}}_c'))
 *   - argument lists: src/tcn/py_ftn_interface/example_def_dycore.yaml:4-71
 *                     (inputs first, then inouts, YAML order: interface.c.jinja2:10-20)
 *   - type mapping  : src/tcn/py_ftn_interface/argument.py:54-86
 *                     (int -> int by value, float -> float by value, array_float -> float*,
 *                      MPI -> void* in C; Fortran passes it as integer(c_int), value)
 *   - library name  : src/tcn/py_ftn_interface/templates/cmake.jinja2:44-52 (lib<prefix>_interface.so)
 * Error convention: the reference entry points return void and a
 * Python exception is printed and swallowed (interface.py.jinja2:26-51).  These
 * keep void, record the error (geos_gtfv3_last_error) and, unless
 * GTFV3_NONFATAL=1, abort the process on a fatal error instead of swallowing it.
 */
#ifndef GEOS_GTFV3_INTERFACE_H
#define GEOS_GTFV3_INTERFACE_H

#ifdef __cplusplus
extern "C" {
#endif

/* example_def_dycore.yaml:4-20 */
void geos_gtfv3_init_c(void* comm, int npx, int npy, int npz, int ntiles, int is, int ie, int js, int je,
                       int isd, int ied, int jsd, int jed, float bdt, int nq_tot);

/* example_def_dycore.yaml:21-70 — fp32 Fortran buffers, updated in place. */
void geos_gtfv3_run_c(void* comm, int npx, int npy, int npz, int ntiles, int is, int ie, int js, int je, int isd,
                      int ied, int jsd, int jed, float bdt, int nq_tot, int ng, float ptop, int ks, int layout_1,
                      int layout_2, int adiabatic, float* ak, float* bk, float* u, float* v, float* w,
                      float* delz, float* pt, float* delp, float* q, float* ps, float* pe, float* pk,
                      float* peln, float* pkz, float* phis, float* q_con, float* omga, float* ua, float* va,
                      float* uc, float* vc, float* mfx, float* mfy, float* cx, float* cy, float* diss_est);

/* example_def_dycore.yaml:71 */
void geos_gtfv3_finalize_c(void);

/* fp64 twin of geos_gtfv3_run_c (PACE_FLOAT_PRECISION=64): same argument order. */
void geos_gtfv3_run_f64_c(void* comm, int npx, int npy, int npz, int ntiles, int is, int ie, int js, int je,
                          int isd, int ied, int jsd, int jed, float bdt, int nq_tot, int ng, float ptop, int ks,
                          int layout_1, int layout_2, int adiabatic, double* ak, double* bk, double* u, double* v,
                          double* w, double* delz, double* pt, double* delp, double* q, double* ps, double* pe,
                          double* pk, double* peln, double* pkz, double* phis, double* q_con, double* omga,
                          double* ua, double* va, double* uc, double* vc, double* mfx, double* mfy, double* cx,
                          double* cy, double* diss_est);

/* Added error channel: copies the last error message, returns its length (0 = none). */
int geos_gtfv3_last_error(char* buf, int len);

#ifdef __cplusplus
}
#endif
#endif
