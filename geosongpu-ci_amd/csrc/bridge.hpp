// bridge.hpp — Fortran-buffer side of geos_gtfv3_{init,run,finalize}_c.
// Replaces the CFFI hook + FortranPythonConversion of the reference
// (templates/data_conversion.py:59-191, hook.py.jinja2:11-34): Fortran
// column-major buffers are copied host->device once per call and scattered into
// the padded HBM layout by a kernel (i fastest in both, so no transpose; pe and
// peln carry k in the middle and are permuted by the same kernel), and written
// back in place with sizeof(T) per element (the reference copies 4*size bytes
// whatever the dtype, data_conversion.py:95).
#pragma once
#include <string>

namespace gtfv3 {

template <typename T>
struct BridgeArgs {
  void* comm;
  int npx, npy, npz, ntiles, is, ie, js, je, isd, ied, jsd, jed;
  float bdt;
  int nq_tot, ng;
  float ptop;
  int ks, layout_1, layout_2, adiabatic;
  T *ak, *bk, *u, *v, *w, *delz, *pt, *delp, *q, *ps, *pe, *pk, *peln, *pkz, *phis, *q_con, *omga, *ua, *va, *uc,
      *vc, *mfx, *mfy, *cx, *cy, *diss_est;
};

struct Namelist;
// "key=value;..." namelist items applied on top of `base` (capi.cpp; the bridge reads them from
// GTFV3_CONFIG: the FV3 namelist options pyFV3 takes from input.nml's fv_core_nml)
Namelist parse_config(const char* cfg, const Namelist& base);

void bridge_init(void* comm, int npx, int npy, int npz, int ntiles, int is, int ie, int js, int je, int isd, int ied,
                 int jsd, int jed, float bdt, int nq_tot);
template <typename T>
void bridge_run(const BridgeArgs<T>& a);
void bridge_finalize();
// rank 0's ncclUniqueId file, if this process published one (finalize removes it too)
void bridge_remove_id_file();
// last run call: out[0..5] = upload ms (the part before the step), step ms, download ms,
// host bytes uploaded, host bytes downloaded, Fortran arrays page-locked
void bridge_stats(double* out);
void bridge_fatal(const std::string& msg);
// rank / size of the job: from the caller's Fortran MPI communicator when MPI is in the
// process, else from the launcher's environment
void job_rank_size(void* comm, int* rank, int* nranks);
// rank 0's 128-byte ncclUniqueId to every rank (MPI_Bcast over `comm`, else a job-stamped file)
void share_unique_id(void* comm, int rank, int nranks, unsigned char* id);
class Dycore;
Dycore* bridge_dycore();  // process-global context (nullptr before init)

}  // namespace gtfv3
