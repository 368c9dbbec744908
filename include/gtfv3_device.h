/* gtfv3_device.h — device-resident API of libgeos_gtfv3_interface.so.
 *
 * Used by the Python hook (geosongpu-ci_amd/hook.py, mirror of
 * templates/hook.py.jinja2:11-34), the NDSL-style stencil surface
 * (geosongpu-ci_amd/stencils.py, call shape of dsl_patterns/Do__get_top_of_the_column.py:28-55)
 * and bench.py.  All functions return 0 on success and -1 on error
 * (message: geos_gtfv3_last_error).  Fields live in HBM in the padded
 * layout [sub][level][j][i] described in DESIGN.md; host buffers passed to
 * upload/download use that same layout, fp64.
 */
#ifndef GTFV3_DEVICE_H
#define GTFV3_DEVICE_H

#ifdef __cplusplus
extern "C" {
#endif

/* config: "key=value;..." (npx, npz, nq, layout_x, layout_y, dt, n_split, k_split,
 * hord_*, kord_*, dddmp, d2_bg, p_fac, fill, adiabatic, ptop).  nccl_id: 128-byte
 * ncclUniqueId shared by all ranks (NULL when nranks == 1). */
void* gtfv3_create(const char* config, int rank, int nranks, const void* nccl_id);
void gtfv3_destroy(void* h);
int gtfv3_get_unique_id(void* out128);
/* The bridge's id bootstrap on its own (no GPU): rank/size from the Fortran MPI handle
 * `comm` when MPI is initialised in the process, else from the launcher environment; rank 0's
 * id128 (filled by the caller) reaches every rank by MPI_Bcast, else through the job-stamped
 * GTFV3_NCCL_ID_FILE.  gtfv3_bootstrap_done removes rank 0's id file and nothing else (a live bridge context stays). */
int gtfv3_bootstrap_id(void* comm, unsigned char* id128, int* rank, int* nranks);
int gtfv3_bootstrap_done(void);
/* the bridge's last geos_gtfv3_run call: out[0..5] = host->device ms before the step starts,
 * step ms (incl. waiting for the tracers that upload beside it), device->host ms, host bytes
 * uploaded, host bytes downloaded, number of page-locked Fortran arrays */
int gtfv3_bridge_stats(double* out);

/* out[0..9] = nx, ny, pitch, nj, nsub, npz, N, layout_x, layout_y, nq */
int gtfv3_dims(void* h, int* out);
/* out[0..7] per local sub-domain s: tile, ioff, joff, N, flags, gid */
int gtfv3_sub_info(void* h, int s, int* out);

int gtfv3_field_create(void* h, const char* name, int nk);
int gtfv3_field_nk(void* h, const char* name);
int gtfv3_field_upload(void* h, const char* name, int nk, const double* host);
int gtfv3_field_download(void* h, const char* name, double* host);
/* levels [k0, k0+nk) of an existing field from host (nsub, nk, nj, pitch) */
int gtfv3_field_upload_levels(void* h, const char* name, int k0, int nk, const double* host);
/* levels [k0, k0+nk) of every sub-domain of an existing field into host (nsub, nk, nj, pitch) */
int gtfv3_field_download_levels(void* h, const char* name, int k0, int nk, double* host);
/* raw device pointer of a field (for zero-copy interop), NULL if missing.  Valid until the
 * next gtfv3_step: the step ping-pongs q (tracer_2d) between two allocations, so take the
 * pointer again after each step. */
void* gtfv3_field_ptr(void* h, const char* name);

/* metric plane(s) [nsub][plane] by name (see grid.cpp kMetricNames) */
int gtfv3_get_metric(void* h, const char* name, double* out);
/* corner points xyz [nsub][ny+2*NG+3][nx+2*NG+3][3] and scalars da_min, da_min_c */
int gtfv3_get_xyz(void* h, double* out);
int gtfv3_get_scalars(void* h, double* out);
/* the column of d_sw damping parameters of the namelist (FV3 dyn_core's k loop, sponge layers
 * included): 10 doubles per level {d2_divg, vt4, dp4, w4, pt4, d_con, nord, nord_v, nord_w,
 * nord_t} (the coefficients as (damp * da_min[_c])^(n+1), 0 where the branch is off; written
 * when cap >= npz); returns n_con, the number of top levels the d_con heat reaches. */
int gtfv3_level_damping(void* h, double* out, int cap);

/* host copy of the same-rank halo table of a kind (0 cell, 1 corner, 2 D-grid, 3 C-grid,
 * 4 A-grid, 5 C-grid tile-edge sync, 6 = 5 then 3 as one exchange): 6 ints per entry
 * {dst_sub, dst_off, src_sub, src_off, comp, sign}; returns the entry count (writes only
 * when cap >= count). */
int gtfv3_halo_table(void* h, int kind, int* out, int cap);
/* cross-rank halo tables (dir 0 = pack/send, 1 = unpack/recv): entries of 6 ints
 * (sub, plane offset, component, sign, position in the peer's segment, peer rank);
 * returns the entry count (copies when cap >= 6*count) */
int gtfv3_halo_remote(void* h, int kind, int dir, int* out, int cap);

/* halo update, spec "name:kind,..." kind c=cell b=corner d=D-grid pair C=C-grid pair a=A-grid pair
 * S=C-grid tile-edge sync pair X=sync and C-grid halo in one exchange (a pair lists x then y
 * component, e.g. "u:d,v:d") */
int gtfv3_halo_update(void* h, const char* spec);

/* run one named stencil on named fields: NDSL-style `stencil(*fields, params)` */
int gtfv3_stencil(void* h, const char* name, const char* fields_csv, const double* params, int nparams);

int gtfv3_set_vertical(void* h, const double* ak, const double* bk, int ks);
/* nsteps fv_dynamics calls on the device-resident state */
int gtfv3_step(void* h, int nsteps);
int gtfv3_sync(void* h);
/* hipStream_t of the dycore */
void* gtfv3_stream(void* h);
/* accumulated per-phase timers (ms), "name=value;..." into buf */
int gtfv3_timers(void* h, char* buf, int len);
/* device time (ms) of each step completed since the last reset, oldest first: HIP events on the
 * library stream around one fv_dynamics call (first to last kernel).  Returns the count and
 * copies when cap >= count; reset != 0 clears the record afterwards. */
int gtfv3_step_times(void* h, double* out, int cap, int reset);
/* per-kernel HIP-event timing (off by default); enabling resets the statistics */
int gtfv3_kernel_timing(void* h, int on);
/* time only this kernel family (name without template arguments, e.g. "tp_march"); NULL or "": all */
int gtfv3_kernel_timing_filter(void* h, const char* kernel);
/* streams of the step: 1 = every kernel on the library stream; 3 (the default) = c_sw's and
   d_sw's wind stages, update_dz_d and the tracer transport forked onto two side streams */
int gtfv3_set_streams(void* h, int n);
/* per-kernel totals since enabling, "kernel=ms,launches;..." into buf */
int gtfv3_kernel_stats(void* h, char* buf, int len);

#ifdef __cplusplus
}
#endif
#endif
