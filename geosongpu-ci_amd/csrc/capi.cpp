// capi.cpp — extern "C" boundary of libgeos_gtfv3_interface.so.
// See include/geos_gtfv3_interface.h (reference symbols) and include/gtfv3_device.h.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <mutex>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/geos_gtfv3_interface.h"
#include "../../include/gtfv3_device.h"
#include "bridge.hpp"
#include "dycore.hpp"
#include "hip_util.hpp"
#include "stencils_registry.hpp"

namespace gtfv3 {
namespace {
std::mutex g_err_mu;
std::string g_err;
}  // namespace
std::string last_error() {
  std::lock_guard<std::mutex> l(g_err_mu);
  return g_err;
}
void set_error(const std::string& m) {
  std::lock_guard<std::mutex> l(g_err_mu);
  g_err = m;
}

// GTFV3_CONFIG: `key=value` items separated by ',' or ';' (whitespace around items, keys
// and values ignored).  A value must be a number consumed whole (integer keys: an integer);
// anything else is an error, never a silently truncated option.
Namelist parse_config(const char* cfg, const Namelist& base) {
  Namelist nl = base;
  std::string s = cfg ? cfg : "";
  for (char& ch : s)
    if (ch == ';') ch = ',';
  auto trim = [](std::string t) {
    const auto a = t.find_first_not_of(" \t\n\r"), b = t.find_last_not_of(" \t\n\r");
    return a == std::string::npos ? std::string() : t.substr(a, b - a + 1);
  };
  std::stringstream ss(s);
  std::string item;
  bool nord_v_given = false;
  while (std::getline(ss, item, ',')) {
    item = trim(item);
    if (item.empty()) continue;
    auto eq = item.find('=');
    if (eq == std::string::npos) throw std::runtime_error("config item without '=': " + item);
    std::string k = trim(item.substr(0, eq)), v = trim(item.substr(eq + 1));
    size_t used = 0;
    double x = 0.0;
    try {
      x = std::stod(v, &used);
    } catch (const std::exception&) {
      used = 0;
    }
    if (v.empty() || used != v.size()) throw std::runtime_error("config value of " + k + " is not a number: '" + v + "'");
    int ix = (int)x;
    static const char* real_keys[] = {"dt", "dddmp", "d2_bg", "d4_bg", "vtdm4", "d_con", "delt_max", "p_fac",
                                      "dz_min", "ptop", "d2_bg_k1", "d2_bg_k2", "ke_bg"};
    bool is_real = false;
    for (const char* rk : real_keys) is_real = is_real || k == rk;
    if (!is_real && (double)ix != x) throw std::runtime_error("config value of " + k + " must be an integer: '" + v + "'");
    if (k == "nord_v") nord_v_given = true;
    if (k == "npx") nl.npx = nl.npy = ix;
    else if (k == "npz") nl.npz = ix;
    else if (k == "nq") nl.nq = ix;
    else if (k == "layout_x") nl.layout_x = ix;
    else if (k == "layout_y") nl.layout_y = ix;
    else if (k == "dt") nl.dt_atmos = x;
    else if (k == "k_split") nl.k_split = ix;
    else if (k == "n_split") nl.n_split = ix;
    else if (k == "hord_mt") nl.hord_mt = ix;
    else if (k == "hord_vt") nl.hord_vt = ix;
    else if (k == "hord_tm") nl.hord_tm = ix;
    else if (k == "hord_dp") nl.hord_dp = ix;
    else if (k == "hord_tr") nl.hord_tr = ix;
    else if (k == "kord_mt") nl.kord_mt = ix;
    else if (k == "kord_wz") nl.kord_wz = ix;
    else if (k == "kord_tr") nl.kord_tr = ix;
    else if (k == "kord_tm") nl.kord_tm = ix;
    else if (k == "dddmp") nl.dddmp = x;
    else if (k == "d2_bg") nl.d2_bg = x;
    else if (k == "nord") nl.nord = ix;
    else if (k == "d4_bg") nl.d4_bg = x;
    else if (k == "vtdm4") nl.vtdm4 = x;
    else if (k == "nord_v") nl.nord_v = ix;
    else if (k == "d_con") nl.d_con = x;
    else if (k == "delt_max") nl.delt_max = x;
    else if (k == "p_fac") nl.p_fac = x;
    else if (k == "dz_min") nl.dz_min = x;
    else if (k == "fill") nl.fill = ix != 0;
    else if (k == "adiabatic") nl.adiabatic = ix != 0;
    else if (k == "ptop") nl.ptop = x;
    else if (k == "host_only") nl.host_only = ix != 0;
    else if (k == "loopback") nl.loopback = ix;
    else if (k == "rccl_self") nl.rccl_self = ix != 0;
    else if (k == "ipc") nl.ipc = ix != 0;
    else if (k == "do_vort_damp") nl.do_vort_damp = ix != 0;
    else if (k == "n_sponge") nl.n_sponge = ix;
    else if (k == "d2_bg_k1") nl.d2_bg_k1 = x;
    else if (k == "d2_bg_k2") nl.d2_bg_k2 = x;
    else if (k == "ke_bg") nl.ke_bg = x;
    else if (k == "convert_ke") nl.convert_ke = ix != 0;
    else throw std::runtime_error("unknown config key: " + k);
  }
  // fv_core_nml semantics: the vorticity damping order follows nord (FV3 dyn_core:
  // nord_v = min(2, nord)) unless given; vtdm4 damps vorticity, delp, w and pt only with
  // do_vort_damp (damp.hip column_damping), while vtdm4 > 1e-4 alone still puts the d_con heat
  // on every level (heat_levels) -- said once on stderr, since that combination is easy to
  // write by accident
  if (!nord_v_given) nl.nord_v = nl.nord < 2 ? nl.nord : 2;
  if (nl.vtdm4 > 0.0 && !nl.do_vort_damp)
    std::fprintf(stderr,
                 "gtfv3: vtdm4 = %g without do_vort_damp = 1: no vorticity / delp / w / pt del-n damping "
                 "(FV3 fv_core_nml semantics); d_con heat on every level\n",
                 nl.vtdm4);
  for (int h : {nl.hord_mt, nl.hord_vt, nl.hord_tm, nl.hord_dp, nl.hord_tr})
    if (h != 5 && h != 6) throw std::runtime_error("hord must be 5 or 6");
  // the remap implements FV3's kord = 9 profile only (remap.hip): any other order is refused
  // rather than run as kord 9 (kord_tm = -9: the same profile for T in log p)
  for (int kd : {nl.kord_mt, nl.kord_wz, nl.kord_tr})
    if (kd != 9) throw std::runtime_error("kord_mt / kord_wz / kord_tr must be 9 (the implemented PPM remap)");
  if (nl.kord_tm != -9) throw std::runtime_error("kord_tm must be -9 (the implemented PPM remap of T in log p)");
  if (nl.nord < 0 || nl.nord > 3) throw std::runtime_error("nord must be 0 .. 3");
  if (nl.nord_v < 0 || nl.nord_v > 2) throw std::runtime_error("nord_v must be 0 .. 2");
  return nl;
}

}  // namespace gtfv3

using namespace gtfv3;

#define API_TRY try {
#define API_CATCH                      \
  }                                    \
  catch (const std::exception& e) {    \
    set_error(e.what());               \
    return -1;                         \
  }                                    \
  return 0;

static Dycore* D(void* h) {
  if (!h) throw std::runtime_error("null dycore handle");
  return static_cast<Dycore*>(h);
}

extern "C" {

int geos_gtfv3_last_error(char* buf, int len) {
  std::string e = last_error();
  if (buf && len > 0) {
    std::strncpy(buf, e.c_str(), (size_t)len - 1);
    buf[len - 1] = 0;
  }
  return (int)e.size();
}

void* gtfv3_create(const char* config, int rank, int nranks, const void* nccl_id) {
  try {
    Namelist nl = parse_config(config, Namelist());
    return new Dycore(nl, rank, nranks, nccl_id);
  } catch (const std::exception& e) {
    set_error(e.what());
    return nullptr;
  }
}

void gtfv3_destroy(void* h) { delete static_cast<Dycore*>(h); }

int gtfv3_get_unique_id(void* out) {
  API_TRY
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) throw std::runtime_error("ncclGetUniqueId failed");
  std::memcpy(out, &id, sizeof(id));
  API_CATCH
}

int gtfv3_bootstrap_id(void* comm, unsigned char* id128, int* rank, int* nranks) {
  API_TRY
  job_rank_size(comm, rank, nranks);
  share_unique_id(comm, *rank, *nranks, id128);
  API_CATCH
}

int gtfv3_bootstrap_done(void) {
  API_TRY
  bridge_remove_id_file();
  API_CATCH
}

int gtfv3_bridge_stats(double* out) {
  API_TRY
  bridge_stats(out);
  API_CATCH
}

int gtfv3_dims(void* h, int* out) {
  API_TRY
  Dycore* d = D(h);
  int v[10] = {d->d.nx, d->d.ny, d->d.pitch, d->d.nj, d->d.nsub, d->d.npz, d->dc.N, d->dc.lx, d->dc.ly, d->nl.nq};
  std::memcpy(out, v, sizeof(v));
  API_CATCH
}

int gtfv3_sub_info(void* h, int s, int* out) {
  API_TRY
  Dycore* d = D(h);
  if (s < 0 || s >= d->d.nsub) throw std::runtime_error("sub index out of range");
  const SubInfo& si = d->hsubs[s];
  int v[8] = {si.tile, si.ioff, si.joff, si.N, si.flags, si.gid, 0, 0};
  std::memcpy(out, v, sizeof(v));
  API_CATCH
}

int gtfv3_field_create(void* h, const char* name, int nk) {
  API_TRY
  D(h)->field(name, nk);
  API_CATCH
}

int gtfv3_field_nk(void* h, const char* name) {
  try {
    Field* f = D(h)->find(name);
    return f ? f->nk : 0;
  } catch (const std::exception& e) {
    set_error(e.what());
    return -1;
  }
}

int gtfv3_field_upload(void* h, const char* name, int nk, const double* host) {
  API_TRY
  D(h)->upload(name, host, nk);
  API_CATCH
}

int gtfv3_field_upload_levels(void* h, const char* name, int k0, int nk, const double* host) {
  API_TRY
  D(h)->upload_levels(name, host, k0, nk);
  API_CATCH
}

int gtfv3_field_download_levels(void* h, const char* name, int k0, int nk, double* host) {
  API_TRY
  D(h)->download_levels(name, host, k0, nk);
  API_CATCH
}

int gtfv3_field_download(void* h, const char* name, double* host) {
  API_TRY
  D(h)->download(name, host);
  API_CATCH
}

void* gtfv3_field_ptr(void* h, const char* name) {
  try {
    Field* f = D(h)->find(name);
    return f ? f->p : nullptr;
  } catch (...) {
    return nullptr;
  }
}

int gtfv3_get_metric(void* h, const char* name, double* out) {
  API_TRY
  Dycore* d = D(h);
  for (int m = 0; m < NMETRIC; ++m)
    if (std::strcmp(kMetricNames[m], name) == 0) {
      std::memcpy(out, d->hm.at(m, 0), sizeof(double) * d->d.nsub * d->d.plane);
      return 0;
    }
  throw std::runtime_error(std::string("unknown metric ") + name);
  API_CATCH
}

int gtfv3_get_xyz(void* h, double* out) {
  API_TRY
  Dycore* d = D(h);
  std::memcpy(out, d->hm.xyz.data(), sizeof(double) * d->hm.xyz.size());
  API_CATCH
}

int gtfv3_get_scalars(void* h, double* out) {
  API_TRY
  Dycore* d = D(h);
  out[0] = d->hm.da_min;
  out[1] = d->hm.da_min_c;
  for (size_t i = 0; i < d->hm.corner_w.size(); ++i) out[2 + i] = d->hm.corner_w[i];
  API_CATCH
}

int gtfv3_level_damping(void* h, double* out, int cap) {
  try {
    Dycore* d = D(h);
    const std::vector<LevelDamp> col = column_damping(d->nl, d->hm.da_min, d->hm.da_min_c);
    if (out && cap >= (int)col.size())
      for (size_t k = 0; k < col.size(); ++k) {
        const LevelDamp& l = col[k];
        const double row[10] = {l.d2_divg, l.vt4, l.dp4, l.w4, l.pt4, l.d_con,
                                (double)l.nord, (double)l.nord_v, (double)l.nord_w, (double)l.nord_t};
        std::memcpy(out + 10 * k, row, sizeof(row));
      }
    return heat_levels(d->nl);
  } catch (const std::exception& e) {
    set_error(e.what());
    return -1;
  }
}

int gtfv3_halo_table(void* h, int kind, int* out, int cap) {
  try {
    const auto& t = D(h)->halo.local_table(kind);
    int n = (int)t.size();
    if (out && cap >= n) std::memcpy(out, t.data(), sizeof(HaloEntry) * n);
    return n;
  } catch (const std::exception& e) {
    set_error(e.what());
    return -1;
  }
}

int gtfv3_halo_remote(void* h, int kind, int dir, int* out, int cap) {
  try {
    std::vector<int> t = D(h)->halo.remote_table(kind, dir);
    int n = (int)t.size() / 6;
    if (out && cap >= (int)t.size()) std::memcpy(out, t.data(), sizeof(int) * t.size());
    return n;
  } catch (const std::exception& e) {
    set_error(e.what());
    return -1;
  }
}

int gtfv3_halo_update(void* h, const char* spec) {
  API_TRY
  std::vector<std::pair<std::string, char>> items;
  std::stringstream ss(spec);
  std::string it;
  while (std::getline(ss, it, ',')) {
    auto c = it.find(':');
    if (c == std::string::npos || c + 1 >= it.size()) throw std::runtime_error("halo spec item: " + it);
    items.push_back({it.substr(0, c), it[c + 1]});
  }
  D(h)->halo_update(items);
  API_CATCH
}

int gtfv3_stencil(void* h, const char* name, const char* fields_csv, const double* params, int np) {
  API_TRY
  std::vector<std::string> names;
  std::stringstream ss(fields_csv ? fields_csv : "");
  std::string it;
  while (std::getline(ss, it, ',')) names.push_back(it);
  std::vector<double> p(params, params + (np > 0 ? np : 0));
  run_registered_stencil(*D(h), name, names, p);
  API_CATCH
}

int gtfv3_set_vertical(void* h, const double* ak, const double* bk, int ks) {
  API_TRY
  D(h)->set_vertical(ak, bk, ks);
  API_CATCH
}

int gtfv3_step(void* h, int nsteps) {
  API_TRY
  for (int n = 0; n < nsteps; ++n) D(h)->step();
  API_CATCH
}

int gtfv3_sync(void* h) {
  API_TRY
  HIP_CHECK(hipStreamSynchronize(D(h)->st));
  API_CATCH
}

void* gtfv3_stream(void* h) {
  try {
    return (void*)D(h)->st;
  } catch (...) {
    return nullptr;
  }
}

int gtfv3_step_times(void* h, double* out, int cap, int reset) {
  API_TRY
  D(h)->flush_all_timers();
  std::vector<double>& v = D(h)->step_ms;
  const int n = (int)v.size();
  if (out && cap >= n) std::copy(v.begin(), v.end(), out);
  if (reset) v.clear();
  return n;
  API_CATCH
}

int gtfv3_timers(void* h, char* buf, int len) {
  API_TRY
  D(h)->flush_all_timers();
  std::string s;
  for (auto& kv : D(h)->timers) s += kv.first + "=" + std::to_string(kv.second) + ";";
  if (buf && len > 0) {
    std::strncpy(buf, s.c_str(), (size_t)len - 1);
    buf[len - 1] = 0;
  }
  API_CATCH
}

int gtfv3_kernel_timing(void* h, int on) {
  API_TRY
  (void)D(h);
  gtfv3::ktimer_reset();
  gtfv3::ktimer_enable(on != 0);
  API_CATCH
}

int gtfv3_kernel_timing_filter(void* h, const char* kernel) {
  API_TRY
  (void)D(h);
  gtfv3::ktimer_filter(kernel);
  API_CATCH
}

int gtfv3_set_streams(void* h, int n) {
  API_TRY
  if (n != 1 && n != 3) throw std::runtime_error("set_streams: 1 or 3 streams");
  D(h)->fork_substep = n == 3;
  API_CATCH
}

int gtfv3_kernel_stats(void* h, char* buf, int len) {
  API_TRY
  HIP_CHECK(hipStreamSynchronize(D(h)->st));
  gtfv3::ktimer_flush();
  std::string s;
  for (auto& kv : gtfv3::ktimer_stats())
    s += kv.first + "=" + std::to_string(kv.second.ms) + "," + std::to_string(kv.second.launches) + "," +
         std::to_string(kv.second.bytes) + ";";
  if (buf && len > 0) {
    std::strncpy(buf, s.c_str(), (size_t)len - 1);
    buf[len - 1] = 0;
  }
  API_CATCH
}

// ---------------- reference bridge symbols ----------------

void geos_gtfv3_init_c(void* comm, int npx, int npy, int npz, int ntiles, int is, int ie, int js, int je, int isd,
                       int ied, int jsd, int jed, float bdt, int nq_tot) {
  try {
    bridge_init(comm, npx, npy, npz, ntiles, is, ie, js, je, isd, ied, jsd, jed, bdt, nq_tot);
  } catch (const std::exception& e) {
    bridge_fatal(e.what());
  }
}

void geos_gtfv3_run_c(void* comm, int npx, int npy, int npz, int ntiles, int is, int ie, int js, int je, int isd,
                      int ied, int jsd, int jed, float bdt, int nq_tot, int ng, float ptop, int ks, int layout_1,
                      int layout_2, int adiabatic, float* ak, float* bk, float* u, float* v, float* w, float* delz,
                      float* pt, float* delp, float* q, float* ps, float* pe, float* pk, float* peln, float* pkz,
                      float* phis, float* q_con, float* omga, float* ua, float* va, float* uc, float* vc,
                      float* mfx, float* mfy, float* cx, float* cy, float* diss_est) {
  try {
    BridgeArgs<float> a{comm, npx, npy, npz, ntiles, is, ie, js, je, isd, ied, jsd, jed, bdt, nq_tot, ng, ptop, ks,
                        layout_1, layout_2, adiabatic, ak, bk, u, v, w, delz, pt, delp, q, ps, pe, pk, peln, pkz,
                        phis, q_con, omga, ua, va, uc, vc, mfx, mfy, cx, cy, diss_est};
    bridge_run(a);
  } catch (const std::exception& e) {
    bridge_fatal(e.what());
  }
}

void geos_gtfv3_run_f64_c(void* comm, int npx, int npy, int npz, int ntiles, int is, int ie, int js, int je, int isd,
                          int ied, int jsd, int jed, float bdt, int nq_tot, int ng, float ptop, int ks, int layout_1,
                          int layout_2, int adiabatic, double* ak, double* bk, double* u, double* v, double* w,
                          double* delz, double* pt, double* delp, double* q, double* ps, double* pe, double* pk,
                          double* peln, double* pkz, double* phis, double* q_con, double* omga, double* ua,
                          double* va, double* uc, double* vc, double* mfx, double* mfy, double* cx, double* cy,
                          double* diss_est) {
  try {
    BridgeArgs<double> a{comm, npx, npy, npz, ntiles, is, ie, js, je, isd, ied, jsd, jed, bdt, nq_tot, ng, ptop, ks,
                         layout_1, layout_2, adiabatic, ak, bk, u, v, w, delz, pt, delp, q, ps, pe, pk, peln, pkz,
                         phis, q_con, omga, ua, va, uc, vc, mfx, mfy, cx, cy, diss_est};
    bridge_run(a);
  } catch (const std::exception& e) {
    bridge_fatal(e.what());
  }
}

void geos_gtfv3_finalize_c(void) {
  try {
    bridge_finalize();
  } catch (const std::exception& e) {
    bridge_fatal(e.what());
  }
}

}  // extern "C"
