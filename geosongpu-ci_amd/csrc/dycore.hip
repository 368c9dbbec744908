// dycore.hip — Dycore context: decomposition, grid upload, named device
// fields, halo groups, and the per-step algorithm sequence (fv_dynamics).
#include "dycore.hpp"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <stdexcept>

#include "hip_util.hpp"
#include "kernels_damp.hpp"
#include "kernels_misc.hpp"
#include "kernels_moist.hpp"
#include "kernels_nh.hpp"
#include "kernels_sw.hpp"

namespace gtfv3 {

long Field::elems() const { return 0; }

namespace {
constexpr size_t kGuardElems = 2048;  // 16 KiB guard zones in GTFV3_SYNC_LAUNCH=1 mode
// every field allocation ends in this many spare planes: the level-block kernels' loads of a
// partial last block (remap_blkq_k: the level in the scalar offset, which the buffer range
// check does not cover) may read up to a block (<= 16 levels) past the last sub-domain's
// bottom level; those values are discarded, and the pad keeps them inside the allocation
constexpr int kFieldTailPlanes = 16;
}  // namespace

Dycore::Dycore(const Namelist& nl_, int rank, int nranks, const void* nccl_id) : nl(nl_) {
  if (nl.ntiles != 6) throw std::runtime_error("only the 6-tile cubed sphere is supported");
  if (nl.npx != nl.npy) throw std::runtime_error("npx must equal npy");
  dc.N = nl.npx - 1;
  dc.lx = nl.layout_x;
  dc.ly = nl.layout_y;
  dc.nranks = nranks;
  dc.rank = rank;
  if (dc.N % dc.lx || dc.N % dc.ly) throw std::runtime_error("layout must divide the tile size");
  if (dc.nsub_total() % nranks) throw std::runtime_error("6*layout_x*layout_y must be a multiple of the rank count");
  if (dc.sub_nx() < NG + 1 || dc.sub_ny() < NG + 1) throw std::runtime_error("sub-domain smaller than the halo");
  d = make_dims(dc, nl.npz);
  cs = std::make_unique<CubedSphere>(dc.N);
  for (int s = 0; s < d.nsub; ++s) hsubs.push_back(dc.sub(rank * d.nsub + s));
  hm.dims = d;
  build_metrics(*cs, dc, hsubs, hm);

  int max_nk = std::max(nl.npz + 1, nl.npz * std::max(nl.nq, 1));
  if (nl.host_only) {
    halo.set_self_messages(nl.rccl_self);  // (the tables only: no communicator)
    halo.build(*cs, dc, d, max_nk, 8, false);
    return;
  }
  // the step's three streams, default priority (dispatch priorities measured no gain at C180
  // and starved the side streams at the 8-rank share: 7.0 -> 12.1-12.7 ms)
  HIP_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  HIP_CHECK(hipStreamCreateWithFlags(&st_b, hipStreamNonBlocking));
  HIP_CHECK(hipStreamCreateWithFlags(&st_c, hipStreamNonBlocking));
  HIP_CHECK(hipStreamCreateWithFlags(&st_d, hipStreamNonBlocking));
  for (hipEvent_t* e : {&ev_fork, &ev_b, &ev_c, &ev_ut, &ev_df, &ev_dj})
    HIP_CHECK(hipEventCreateWithFlags(e, hipEventDisableTiming));
  {
    const char* e = std::getenv("GTFV3_STREAMS");
    // several rank processes sharing a GPU (the IPC transport): one stream each by default --
    // every process's queues compete for the GPU's hardware queues
    fork_substep = e ? e[0] == '1' : !nl.ipc;
    const char* w = std::getenv("GTFV3_EARLY_WINDS");  // 0: the wind stage after the Courant numbers
    early_winds = w && *w && w[0] == '0' ? 0 : 1;
  }
  HIP_CHECK(hipMalloc(&dsubs, sizeof(SubInfo) * d.nsub));
  HIP_CHECK(hipMemcpy(dsubs, hsubs.data(), sizeof(SubInfo) * d.nsub, hipMemcpyHostToDevice));
  HIP_CHECK(hipMalloc(&dmet, sizeof(double) * hm.m.size()));
  HIP_CHECK(hipMemcpy(dmet, hm.m.data(), sizeof(double) * hm.m.size(), hipMemcpyHostToDevice));
  HIP_CHECK(hipMalloc(&dcornerw, sizeof(double) * hm.corner_w.size()));
  HIP_CHECK(hipMemcpy(dcornerw, hm.corner_w.data(), sizeof(double) * hm.corner_w.size(), hipMemcpyHostToDevice));
  {
    // the cell area four times per sub-domain, so a march wave whose lane groups run two or
    // four levels addresses it with the level fields' per-lane offset (tp.hip output spans)
    std::vector<double> a4(4 * (size_t)d.nsub * d.plane);
    for (int s = 0; s < d.nsub; ++s)
      for (int h = 0; h < 4; ++h)
        std::memcpy(a4.data() + ((size_t)s * 4 + h) * d.plane, hm.m.data() + ((size_t)M_AREA * d.nsub + s) * d.plane,
                    sizeof(double) * d.plane);
    HIP_CHECK(hipMalloc(&darea4, sizeof(double) * a4.size()));
    HIP_CHECK(hipMemcpy(darea4, a4.data(), sizeof(double) * a4.size(), hipMemcpyHostToDevice));
  }
  debug_canary("subs", dsubs, hsubs.data(), sizeof(SubInfo) * d.nsub);
  debug_canary("metrics", dmet, hm.m.data(), sizeof(double) * hm.m.size());
  debug_canary("corner_w", dcornerw, hm.corner_w.data(), sizeof(double) * hm.corner_w.size());

  if (nl.rccl_self) {
    // one rank talking to itself over RCCL (Namelist::rccl_self): a size-1 communicator
    if (nranks != 1 || nl.loopback) throw std::runtime_error("rccl_self needs one rank and no loopback group");
    comm = make_nccl_transport(1, 0, nullptr);
    halo.set_transport(comm.get());
    halo.set_self_messages(true);
  } else if (nranks > 1) {
    comm = nl.loopback ? make_loopback_transport(nl.loopback, nranks, rank)
           : nl.ipc    ? make_ipc_transport(nranks, rank, nccl_id)
                       : make_nccl_transport(nranks, rank, nccl_id);
    halo.set_transport(comm.get());
  }
  halo.build(*cs, dc, d, max_nk, 8);
  // the null-stream copies and memsets above complete before the non-blocking streams run
  HIP_CHECK(hipDeviceSynchronize());
}

Dycore::~Dycore() {
  // nothing of this context may still run when its memory is released (every stream,
  // including the halo exchanger's comm stream)
  if (st) (void)hipDeviceSynchronize();
  if (ac_exec) (void)hipGraphExecDestroy(ac_exec);
  for (auto& kv : fields) {
    if (debug_sync_launch()) {
      double* base = kv.second.p - kGuardElems;
      debug_canary_drop(base);
      debug_canary_drop(guard_hi(kv.second.p, kv.second.nk));
      (void)hipFree(base);
    } else {
      (void)hipFree(kv.second.p);
    }
  }
  debug_canary_drop(dsubs);
  debug_canary_drop(dmet);
  debug_canary_drop(dcornerw);
  if (h_cmax) (void)hipHostFree(h_cmax);
  if (ev_cmax) (void)hipEventDestroy(ev_cmax);
  if (dsubs) (void)hipFree(dsubs);
  if (dlevel) (void)hipFree(dlevel);
  if (dlevel_zh) (void)hipFree(dlevel_zh);
  if (dmet) (void)hipFree(dmet);
  if (dcornerw) (void)hipFree(dcornerw);
  if (darea4) (void)hipFree(darea4);
  for (hipEvent_t e : {ev_fork, ev_b, ev_c, ev_ut, ev_df, ev_dj})
    if (e) (void)hipEventDestroy(e);
  for (auto& set : ev_ph)
    for (hipEvent_t e : set)
      if (e) (void)hipEventDestroy(e);
  if (st_b) (void)hipStreamDestroy(st_b);
  if (st_c) (void)hipStreamDestroy(st_c);
  if (st_d) (void)hipStreamDestroy(st_d);
  if (st) (void)hipStreamDestroy(st);
}

Field& Dycore::field(const std::string& name, int nk) {
  if (nl.host_only) throw std::runtime_error("host-only dycore has no device fields");
  auto it = fields.find(name);
  if (it != fields.end()) {
    if (it->second.nk != nk) throw std::runtime_error("field '" + name + "' exists with a different level count");
    return it->second;
  }
  Field f;
  f.nk = nk;
  ++field_gen;
  size_t bytes = sizeof(double) * (size_t)field_elems(nk);
  const size_t pad = sizeof(double) * (size_t)kFieldTailPlanes * d.plane;
  if (debug_sync_launch()) {
    // debug mode: guard zones either side of the field, checked after every launch; the
    // high guard sits after the tail pad the level-block loads may read into (not in it)
    const size_t gb = sizeof(double) * kGuardElems;
    double* base = nullptr;
    HIP_CHECK(hipMalloc(&base, bytes + pad + 2 * gb));
    HIP_CHECK(hipMemset(base, 0xA5, bytes + pad + 2 * gb));
    f.p = base + kGuardElems;
    HIP_CHECK(hipMemset(f.p, 0, bytes + pad));
    const std::vector<unsigned char> pat(gb, 0xA5);
    debug_canary(("guard-lo " + name).c_str(), base, pat.data(), gb);
    debug_canary(("guard-hi " + name).c_str(), guard_hi(f.p, nk), pat.data(), gb);
    return fields[name] = f;
  }
  HIP_CHECK(hipMalloc(&f.p, bytes + pad));
  HIP_CHECK(hipMemsetAsync(f.p, 0, bytes + pad, st));
  return fields[name] = f;
}

double* Dycore::guard_hi(double* p, int nk) const { return p + field_elems(nk) + (long)kFieldTailPlanes * d.plane; }

Field* Dycore::find(const std::string& name) {
  auto it = fields.find(name);
  return it == fields.end() ? nullptr : &it->second;
}

Ctx Dycore::ctx() const {
  Ctx c;
  c.d = d;
  c.subs = dsubs;
  c.hsubs = hsubs.data();
  c.met = dmet;
  c.cornerw = dcornerw;
  c.area4 = darea4;
  c.da_min = hm.da_min;
  c.da_min_c = hm.da_min_c;
  c.st = st;
  return c;
}

void Dycore::upload(const std::string& name, const double* host, int nk) {
  Field& f = field(name, nk);
  HIP_CHECK(hipMemcpyAsync(f.p, host, sizeof(double) * field_elems(nk), hipMemcpyHostToDevice, st));
  HIP_CHECK(hipStreamSynchronize(st));
}

void Dycore::upload_levels(const std::string& name, const double* host, int k0, int nk) {
  Field* f = find(name);
  if (!f) throw std::runtime_error("no field '" + name + "'");
  if (k0 < 0 || nk < 1 || k0 + nk > f->nk) throw std::runtime_error("upload_levels: level range outside the field");
  // host (nsub, nk, plane) -> levels k0 .. k0+nk-1 of every sub-domain
  HIP_CHECK(hipMemcpy2DAsync(f->p + (long)k0 * d.plane, sizeof(double) * f->nk * d.plane, host,
                             sizeof(double) * nk * d.plane, sizeof(double) * nk * d.plane, d.nsub,
                             hipMemcpyHostToDevice, st));
  HIP_CHECK(hipStreamSynchronize(st));
}

void Dycore::download_levels(const std::string& name, double* host, int k0, int nk) {
  Field* f = find(name);
  if (!f) throw std::runtime_error("no field '" + name + "'");
  if (k0 < 0 || nk < 1 || k0 + nk > f->nk) throw std::runtime_error("download_levels: level range outside the field");
  HIP_CHECK(hipMemcpy2DAsync(host, sizeof(double) * nk * d.plane, f->p + (long)k0 * d.plane,
                             sizeof(double) * f->nk * d.plane, sizeof(double) * nk * d.plane, d.nsub,
                             hipMemcpyDeviceToHost, st));
  HIP_CHECK(hipStreamSynchronize(st));
}

void Dycore::download(const std::string& name, double* host) {
  Field* f = find(name);
  if (!f) throw std::runtime_error("no field '" + name + "'");
  HIP_CHECK(hipMemcpyAsync(host, f->p, sizeof(double) * field_elems(f->nk), hipMemcpyDeviceToHost, st));
  HIP_CHECK(hipStreamSynchronize(st));
}

void Dycore::halo_update(const std::vector<std::pair<std::string, char>>& items) {
  const std::vector<HaloField> hf = halo_fields(items);
  halo.exchange(hf.data(), (int)hf.size(), st);
}

void Dycore::halo_begin(const std::vector<std::pair<std::string, char>>& items) {
  const std::vector<HaloField> hf = halo_fields(items);
  halo.exchange_begin(hf.data(), (int)hf.size(), st);
}

void Dycore::halo_end() { halo.exchange_end(st); }

std::vector<HaloField> Dycore::halo_fields(const std::vector<std::pair<std::string, char>>& items) {
  std::vector<HaloField> hf;
  for (size_t n = 0; n < items.size(); ++n) {
    const auto& it = items[n];
    HaloField h{};
    char k = it.second;
    if (k == 'c' || k == 'b') {
      Field* f = find(it.first);
      if (!f) throw std::runtime_error("halo: no field '" + it.first + "'");
      h.p[0] = f->p;
      h.p[1] = nullptr;
      h.nk = f->nk;
      h.kind = k == 'c' ? H_CELL : H_CORNER;
    } else {
      // vector pair: this item names the x component, the next item the y component
      if (n + 1 >= items.size()) throw std::runtime_error("halo: vector pair incomplete");
      Field* fx = find(it.first);
      Field* fy = find(items[n + 1].first);
      if (!fx || !fy) throw std::runtime_error("halo: missing vector component");
      h.p[0] = fx->p;
      h.p[1] = fy->p;
      h.nk = fx->nk;
      h.kind = k == 'd' ? H_DGRID : k == 'C' ? H_CGRID : k == 'S' ? H_CSYNC : k == 'X' ? H_CSC : H_AGRID;
      ++n;
    }
    hf.push_back(h);
  }
  return hf;
}

void Dycore::allreduce_max(double* dev, int n) {
  if (comm) comm->allreduce_max(dev, n, st);
}

void Dycore::set_vertical(const double* ak_, const double* bk_, int ks_) {
  // a caller that passes the same table every step (the bridge) uploads it once
  const bool same = (int)ak.size() == nl.npz + 1 && std::equal(ak.begin(), ak.end(), ak_) &&
                    std::equal(bk.begin(), bk.end(), bk_);
  if (same && ks == ks_) return;
  ak.assign(ak_, ak_ + nl.npz + 1);
  bk.assign(bk_, bk_ + nl.npz + 1);
  ks = ks_;
  vert_dirty = true;
}

// tracer_2d_1l (FV3 fv_tracer2d): large-time-step transport of nq tracers with
// the mass fluxes (mfx,mfy) and Courant numbers (cx,cy) accumulated over the
// acoustic sub-steps; dp1 = delp at the start of the step.
void Dycore::tracer_2d(int nq, double /*dt*/, int fused_mode, int nf) {
  const int npz = nl.npz;
  Ctx c = ctx();
  Field& q = field("q", nq * npz);
  Field& dp1 = field("dp1", npz);
  Field& cx = field("cx", npz);
  Field& cy = field("cy", npz);
  Field& mfx = field("mfx", npz);
  Field& mfy = field("mfy", npz);
  Field& xfx = field("tr_xfx", npz);
  Field& yfx = field("tr_yfx", npz);
  Field& dp2 = field("tr_dp2", npz);
  Field& cmax = field("tr_cmax", 1);  // first npz doubles used
  Field& nspl = field("tr_nsplt", 1);
  if ((long)npz > d.plane) throw std::runtime_error("tracer cmax scratch too small");
  static const bool fused_env = [] {
    const char* e = getenv("GTFV3_TRACER_FUSED");  // 0: flux planes + tracer_dp2 + tracer_update
    return !(e && e[0] == '0');
  }();
  const bool fused = fused_mode < 0 ? fused_env : fused_mode != 0;

  tracer_prep(c, npz, cx.p, cy.p, xfx.p, yfx.p, cmax.p);
  allreduce_max(cmax.p, npz);
  // nsplt[k] = int(1 + cmax[k]) on the device; the host needs only the largest count (the
  // number of sub-steps to launch): it comes through pinned memory, and the host waits for
  // it only after the first sub-step is queued, so the GPU does not idle on the round trip
  int* dns = reinterpret_cast<int*>(nspl.p);
  tracer_nsplt(c, npz, cmax.p, dns);
  if (!h_cmax) {
    HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h_cmax), sizeof(double) * std::max(npz, 1)));
    HIP_CHECK(hipEventCreateWithFlags(&ev_cmax, hipEventDisableTiming));
  }
  HIP_CHECK(hipMemcpyAsync(h_cmax, cmax.p, sizeof(double) * npz, hipMemcpyDeviceToHost, st));
  HIP_CHECK(hipEventRecord(ev_cmax, st));
  tracer_split(c, npz, dns, cx.p, cy.p, xfx.p, yfx.p, mfx.p, mfy.p);
  // the last writer of cx, cy, mfx, mfy (the bridge copies them back from here on)
  record_mark(SM_FLUXES, st);
  int nmax = -1;
  auto sub_steps = [&]() {
    if (nmax < 0) {
      HIP_CHECK(hipEventSynchronize(ev_cmax));
      nmax = 1;
      for (int k = 0; k < npz; ++k) nmax = std::max(nmax, (int)(1.0 + h_cmax[k]));
    }
    return nmax;
  };
  TpArgs a{};
  a.nt = nq; a.nk = npz;
  a.crx = cx.p; a.cry = cy.p; a.xfx = xfx.p; a.yfx = yfx.p;
  a.mfx = mfx.p; a.mfy = mfy.p;
  a.ord = nl.hord_tr;
  static const int nf_env = [] {
    const char* e = getenv("GTFV3_TRACER_NF");
    return e ? atoi(e) : 0;
  }();
  a.nf = nf != 0 ? nf : (nf_env > 0 && nq % nf_env == 0 && (fused || nf_env < 3) ? nf_env : 0);
  if (fused) {
    // each sub-step updates the tracers into a second set of planes, which then become "q"
    // (the march reads neighbouring columns' tracers as its halo: no in-place update)
    Field& qa = field("_q_alt", nq * npz);
    for (int it = 0; it < (it == 0 ? 1 : sub_steps()); ++it) {
      if (it > 0) copy_levels(c, field_elems(npz), dp2.p, dp1.p);
      halo_update({{"q", 'c'}});
      a.q = q.p; a.q_out = qa.p;
      a.dp1 = dp1.p; a.dp2 = dp2.p; a.nsplt = dns; a.it = it;
      fv_tp_2d(c, a);
      std::swap(q.p, qa.p);
    }
    // the march writes the compute domain only: give the new planes the halo ring of the
    // last exchange (FV3's q leaves tracer_2d with those halo values, and the bridge copies
    // q's halo back to the caller).  "q" may now live in the other allocation: device
    // pointers taken before step() are not stable (gtfv3_device.h gtfv3_field_ptr).
    copy_halo_ring(c, d.nsub * nq * npz, qa.p, q.p);
    return;
  }
  Field& fx = field("tr_fx", nq * npz);
  Field& fy = field("tr_fy", nq * npz);
  halo_update({{"q", 'c'}});
  for (int it = 0; it < (it == 0 ? 1 : sub_steps()); ++it) {
    tracer_dp2(c, npz, dp1.p, mfx.p, mfy.p, dp2.p);
    a.q = q.p;
    a.fx = fx.p; a.fy = fy.p;
    fv_tp_2d(c, a);
    tracer_update(c, npz, nq, q.p, nullptr, dp1.p, dp2.p, fx.p, fy.p, dns, it);
    if (it + 1 < sub_steps()) {
      copy_levels(c, field_elems(npz), dp2.p, dp1.p);
      halo_update({{"q", 'c'}});
    }
  }
}

void Dycore::record_mark(int m, hipStream_t s) {
  if (!marks) return;
  HIP_CHECK(hipEventRecord(marks[m], s));
  if (on_mark) on_mark(m);
}

Field& Dycore::need(const std::string& name, int nk) {
  Field* f = find(name);
  if (!f) throw std::runtime_error("step: state field '" + name + "' was never uploaded");
  if (f->nk != nk) throw std::runtime_error("step: field '" + name + "' has the wrong level count");
  return *f;
}

// Device copies of ak, bk and the reference layer thickness dp_ref = dak + dbk*1e5.
const double* Dycore::vertical_dev() {
  const int k1 = nl.npz + 1;
  if ((int)ak.size() != k1) throw std::runtime_error("step: set_vertical() was not called");
  if (3L * k1 > d.plane) throw std::runtime_error("vertical table larger than one plane");
  Field& v = field("_vert", 1);
  if (!vert_dirty) return v.p;  // uploaded once per set_vertical(), not per step
  std::vector<double> h(3 * k1, 0.0);
  for (int k = 0; k < k1; ++k) {
    h[k] = ak[k];
    h[k1 + k] = bk[k];
  }
  for (int k = 0; k < nl.npz; ++k) h[2 * k1 + k] = (ak[k + 1] - ak[k]) + (bk[k + 1] - bk[k]) * 1.0e5;
  HIP_CHECK(hipMemcpyAsync(v.p, h.data(), sizeof(double) * h.size(), hipMemcpyHostToDevice, st));
  HIP_CHECK(hipStreamSynchronize(st));
  vert_dirty = false;
  return v.p;
}

const LevelDamp* Dycore::level_table(const std::vector<LevelDamp>& t, int slot) {
  std::vector<LevelDamp>& h = slot ? hlevel_zh : hlevel;
  LevelDamp*& dv = slot ? dlevel_zh : dlevel;
  size_t& cap = slot ? dlevel_zh_cap : dlevel_cap;
  const size_t bytes = sizeof(LevelDamp) * t.size();
  if (dv && t.size() == h.size() && std::memcmp(t.data(), h.data(), bytes) == 0) return dv;
  if (t.size() > cap) {
    // nothing queued may still read the old table
    if (dv) {
      HIP_CHECK(hipDeviceSynchronize());
      HIP_CHECK(hipFree(dv));
    }
    HIP_CHECK(hipMalloc(&dv, bytes));
    cap = t.size();
  }
  h = t;
  HIP_CHECK(hipMemcpyAsync(dv, h.data(), bytes, hipMemcpyHostToDevice, st));
  HIP_CHECK(hipStreamSynchronize(st));
  return dv;
}

// One fv_dynamics call (FV3 fv_dynamics.F90 / dyn_core.F90 sequence, non-hydrostatic,
// k_split remap cycles of n_split acoustic sub-steps, tracer_2d_1l, Lagrangian-to-
// Eulerian remap, then T/omega/A-grid winds for the caller).
// Aquaplanet moist physics on the device-resident state after
// fv_dynamics, in the order of GEOS's moist run (GFDL_1M.drawio): aerosol activation, the
// shallow cumulus (cup_gf_sh), the evap_subl_pdf loop (anvil evaporation / sublimation, large-scale PDF condensation),
// the GFDL cloud microphysics driver, RADCOUPLE.  T = pt, species = tracers 0..5 (qv ql qr
// qi qs qg; ql / qi are the large-scale condensate), anvil condensate and the cloud
// fractions in their own fields (qlcn, qicn, clcn, clls), surface precipitation into
// prec_{rain,snow,graupel,ice}, the radiation's view into rad_*.
void Dycore::moist_physics(double dt) {
  const int npz = nl.npz, nq = nl.nq;
  if (nq < 6) throw std::runtime_error("moist_physics: needs nq >= 6 (qv ql qr qi qs qg)");
  Ctx c = ctx();
  Field& q = need("q", nq * npz);
  const long sp = (long)npz * d.plane;  // one species of sub-domain 0
  const long qsub = (long)nq * npz;
  double* qv = q.p;
  double *ql = q.p + sp, *qr = q.p + 2 * sp, *qi = q.p + 3 * sp, *qs = q.p + 4 * sp, *qg = q.p + 5 * sp;
  double* T = need("pt", npz).p;
  const double* delz = need("delz", npz).p;
  auto F = [&](const char* n) { return field(n, npz).p; };
  double *pl = F("_m_pl"), *zm = F("_m_zm"), *nactl = F("nactl"), *nacti = F("nacti"), *smax = F("_m_smax");
  double *qlcn = F("qlcn"), *qicn = F("qicn"), *clls = F("clls"), *clcn = F("clcn");
  double* kpbl = field("_m_kpbl", 1).p;
  if (!find("hfx")) {  // no surface model here: a uniform sensible heat flux drives the shallow plumes
    Field& h = field("hfx", 1);
    fill_field(c, field_elems(1), kSurfaceHfx, h.p);
  }
  moist_prep(c, npz, need("pe", npz + 1).p, delz, pl, zm, kpbl);
  aer_activation(c, npz, qsub, pl, T, qv, zm, need("w", npz).p, nactl, nacti, smax);
  GfShArgs gf{};
  gf.nk = npz;
  gf.qv_sub = qsub;
  gf.dt = dt;
  gf.T = T; gf.qv = qv; gf.pl = pl; gf.zm = zm; gf.dp = need("delp", npz).p;
  gf.kpbl = kpbl; gf.hfx = need("hfx", 1).p; gf.qlcn = qlcn; gf.qicn = qicn;
  gf.cf = F("_m_cfcn"); gf.mb = field("gf_mb", 1).p; gf.k22 = field("gf_k22", 1).p;
  gf.kbcon = field("gf_kbcon", 1).p; gf.ktop = field("gf_ktop", 1).p;
  gf.scr = field("_gf_scr", gf_scratch_levels(npz)).p;
  cup_gf_sh(c, gf);
  max_field(c, field_elems(npz), gf.cf, clcn);  // convective cloud fraction into the anvil fraction
  EvapSublArgs e{};
  e.nk = npz;
  e.dt = dt;
  e.T = T; e.qv = qv; e.qlls = ql; e.qils = qi; e.qlcn = qlcn; e.qicn = qicn; e.clls = clls; e.clcn = clcn;
  e.qv_sub = e.ql_sub = e.qi_sub = qsub;
  e.pl = pl; e.nactl = nactl; e.nacti = nacti;
  evap_subl_pdf(c, e);
  Gfdl1mArgs g{};
  g.nk = npz;
  g.qsub = (int)qsub;
  g.dt = dt;
  g.T = T;
  g.qv = qv; g.ql = ql; g.qr = qr; g.qi = qi; g.qs = qs; g.qg = qg;
  g.dp = need("delp", npz).p;
  g.dz = delz;
  g.scr = field("_mp_scr", gfdl_mp_scratch_levels(npz)).p;
  g.pr = field("prec_rain", 1).p; g.ps = field("prec_snow", 1).p; g.pg = field("prec_graupel", 1).p;
  g.pi = field("prec_ice", 1).p;
  gfdl_1m(c, g);
  RadcoupleArgs r{};
  r.nk = npz;
  r.qv_sub = r.ql_sub = r.qi_sub = r.qr_sub = r.qs_sub = r.qg_sub = qsub;
  r.T = T; r.pl = pl; r.cf = clls; r.af = clcn; r.qv = qv; r.qlls = ql; r.qils = qi; r.qlcn = qlcn; r.qicn = qicn;
  r.qr = qr; r.qs = qs; r.qg = qg; r.nl = nactl;
  r.rqv = F("rad_qv"); r.rql = F("rad_ql"); r.rqi = F("rad_qi"); r.rqr = F("rad_qr"); r.rqs = F("rad_qs");
  r.rqg = F("rad_qg"); r.rcf = F("rad_cf"); r.rrl = F("rad_rl"); r.rri = F("rad_ri");
  radcouple(c, r);
}

// GTFV3_HALO_SPLIT (read per step): the interior / boundary split of the uc / vc and u / v
// exchanges.  Unset: on where the messages cross GPUs (RCCL with several ranks), off for the
// null / loopback transports and the one-rank RCCL self messages, whose messages are device
// copies that take less than the split's two cross-queue hand-offs (the 8-rank share on the
// null transport: 5.91 ms whole exchanges, 6.37 ms split with four-rectangle frames);
// "1" on, "0" off wherever the exchanges carry messages.
static int halo_split_mode() {
  const char* e = std::getenv("GTFV3_HALO_SPLIT");
  return e && *e ? (e[0] == '0' ? 0 : 1) : -1;
}

// GTFV3_GRAPH=1: the acoustic sub-steps replayed as one captured HIP graph (read per step).
// Off by default: measured on one MI355X, the graph saves the launch gaps of the small
// per-rank shares (rank 0 of the 8-rank layout alone: 6.91 -> 6.66 ms per step) but loses
// to the three-stream launches at C180 on one GPU (38.23 -> 38.60 ms), and the RCCL
// transport of real multi-GPU runs is not captured (profiles/r03g_*)
static bool graph_enabled() {
  const char* e = std::getenv("GTFV3_GRAPH");
  return e && e[0] == '1';
}

// GTFV3_EDGE_SIDE (default 1): the thermo march's tile-edge kernel on its own stream beside the
// interior kernel; 0: in series
static bool edge_side() {
  const char* e = std::getenv("GTFV3_EDGE_SIDE");
  return !(e && e[0] == '0');
}

void Dycore::step() {
  if (nl.host_only) throw std::runtime_error("host-only dycore cannot step");
  if (nl.k_split != 1) throw std::runtime_error("step: only k_split = 1 is supported");
  const int npz = nl.npz, k1 = npz + 1, nq = nl.nq;
  if (nq < 1) throw std::runtime_error("step: nq >= 1 required (tracer 0 is specific humidity)");
  Ctx c = ctx();
  const double bdt = nl.dt_atmos;
  const double mdt = bdt / nl.k_split;
  const double dt = mdt / nl.n_split, dt2 = 0.5 * dt;
  const double ptop = ak[0];
  // adiabatic (the bridge's `adiabatic` argument, example_def_dycore.yaml:40): dry
  // dynamics, no moisture in the virtual temperature (FV3 moist_phys = .false.)
  const double zvir = nl.adiabatic ? 0.0 : Constants::zvir;
  const double* vert = vertical_dev();
  const double* ak_dev = vert;
  const double* bk_dev = vert + k1;
  const double* dp_ref = vert + 2 * k1;

  // phase events in a two-step ring: the slot's previous step (two steps ago) has completed
  // by now -- the tracer step's pinned-memory read waits for its own step mid-way, so the
  // host is never more than one step ahead -- and its times are read without a stall
  const int slot = ev_slot;
  ev_slot ^= 1;
  if (ev_pending[slot]) flush_timers(slot);
  if (!ev_ph[slot][0])
    for (auto& e : ev_ph[slot]) HIP_CHECK(hipEventCreate(&e));
  hipEvent_t* ev = ev_ph[slot];
  HIP_CHECK(hipEventRecord(ev[0], st));

  Field& u = need("u", npz);
  Field& v = need("v", npz);
  Field& w = need("w", npz);
  Field& delz = need("delz", npz);
  Field& pt = need("pt", npz);
  Field& delp = need("delp", npz);
  Field& q = need("q", nq * npz);
  Field& phis = need("phis", 1);
  auto S = [&](const char* n, int nk) { return field(n, nk).p; };
  double* pe = S("pe", k1);
  double* peln = S("peln", k1);
  double* pk = S("pk", k1);
  double* pkz = S("pkz", npz);
  double* ps = S("ps", 1);
  double* omga = S("omga", npz);
  double* ua = S("ua", npz);
  double* va = S("va", npz);
  double* uc = S("uc", npz);
  double* vc = S("vc", npz);
  double* mfx = S("mfx", npz);
  double* mfy = S("mfy", npz);
  double* cx = S("cx", npz);
  double* cy = S("cy", npz);
  double* dp1 = S("dp1", npz);

  fv_prep(c, npz, nq, zvir, delp.p, delz.p, q.p, pt.p, pkz);
  copy_levels(c, field_elems(npz), delp.p, dp1);
  for (double* x : {mfx, mfy, cx, cy}) fill_field(c, field_elems(npz), 0.0, x);

  // ---- dyn_core ----
  double* zh = S("zh", k1);
  double* gzc = S("_gzc", k1);
  double* pef = S("_pef", k1);
  double* ppe = S("ppe", k1);
  double* pk3 = S("_pk3", k1);
  double* ws = S("ws", 1);
  NhScratch nsc;
  for (int n = 0; n < 14; ++n) nsc.s[n] = S(("_nh" + std::to_string(n)).c_str(), k1);

  CswArgs ca{};
  ca.npz = npz;
  ca.dt2 = dt2;
  ca.delp = delp.p; ca.pt = pt.p; ca.w = w.p; ca.u = u.p; ca.v = v.p;
  ca.uc = uc; ca.vc = vc; ca.ua = ua; ca.va = va;
  ca.ut = S("_ut", npz); ca.vt = S("_vt", npz);
  ca.delpc = S("_delpc", npz); ca.ptc = S("_ptc", npz); ca.wc = S("_wc", npz);
  ca.utmp = S("_cs_utmp", npz); ca.vtmp = S("_cs_vtmp", npz); ca.ke = S("_cs_ke", npz); ca.vort = S("_cs_vort", npz);

  DswArgs da{};
  da.npz = npz;
  da.dt = dt; da.dddmp = nl.dddmp;
  da.hord_mt = nl.hord_mt; da.hord_vt = nl.hord_vt; da.hord_tm = nl.hord_tm; da.hord_dp = nl.hord_dp;
  da.delp = delp.p; da.pt = pt.p; da.w = w.p; da.u = u.p; da.v = v.p;
  da.uc = uc; da.vc = vc; da.ua = ua; da.va = va;
  da.crx = S("crx", npz); da.cry = S("cry", npz); da.xfx = S("xfx", npz); da.yfx = S("yfx", npz);
  da.cx = cx; da.cy = cy; da.mfx = mfx; da.mfy = mfy;
  da.ut = S("_ds_ut", npz); da.vt = S("_ds_vt", npz);
  da.fx = S("_ds_fx", npz); da.fy = S("_ds_fy", npz); da.gwx = S("_ds_gwx", npz); da.gwy = S("_ds_gwy", npz);
  da.gtx = S("_ds_gtx", npz); da.gty = S("_ds_gty", npz); da.ke = S("_ds_ke", npz); da.vort = S("_ds_vort", npz);
  // d_sw's cell vorticity formed by c_sw's cs_tmp, which reads the same starting u, v (a
  // ds_vort launch and its reads of u, v less per sub-step: 31.48-31.53 -> 31.33-31.43 ms in
  // one box's A/B)
  ca.dvort = da.vort;
  // d_sw's damping (damp.hip): the column of per-level parameters of FV3 dyn_core (the sponge
  // layers' divergence and w damping at the top in the Held-Suarez namelist)
  const std::vector<LevelDamp> col = column_damping(nl, c.da_min, c.da_min_c);
  da.lv = level_table(col);
  da.hlv = hlevel.data();
  da.nord = nl.nord; da.d4_bg = nl.d4_bg; da.d_con = nl.d_con;
  da.ke_dt = nl.ke_bg * std::fabs(dt);
  const bool dcon = nl.d_con > 1e-5;
  const bool vdamp = any_level(col.data(), npz, &LevelDamp::vt4);
  const bool tdamp = vdamp || any_level(col.data(), npz, &LevelDamp::w4) ||
                     any_level(col.data(), npz, &LevelDamp::dp4) || any_level(col.data(), npz, &LevelDamp::pt4);
  if (nl.nord > 0) {
    da.divg = S("divgd", npz);
    da.dd = S("_dd_dd", npz); da.dvcx = S("_dd_vcx", npz); da.ducy = S("_dd_ucy", npz);
    da.dvort = S("_dd_vort", npz); da.dqx = S("_dd_qx", npz); da.dqy = S("_dd_qy", npz);
  }
  if (nl.nord > 0 || vdamp) da.wk = S("_dd_wk", npz);
  if (vdamp) {
    da.d2 = S("_dd_d2", npz); da.fx2 = S("_dd_fx2", npz); da.fy2 = S("_dd_fy2", npz);
  }
  if (tdamp) {
    da.td2 = S("_dl_d2", npz); da.tfx2 = S("_dl_fx2", npz); da.tfy2 = S("_dl_fy2", npz);
    da.dw = S("_dl_dw", npz); da.hw = S("_dl_hw", npz);
  }
  if (dcon) {
    // heat source and the dissipation estimate summed over this call's acoustic sub-steps
    da.vd = S("_dd_vd", npz); da.heat = S("_dd_heat", npz); da.diss = S("diss_est", npz);
    fill_field(c, field_elems(npz), 0.0, da.heat);
    fill_field(c, field_elems(npz), 0.0, da.diss);
  }

  UdzdArgs za{};
  za.npz = npz;
  za.hord = nl.hord_tm;
  za.dp0 = dp_ref;
  za.crx = da.crx; za.cry = da.cry; za.xfx = da.xfx; za.yfx = da.yfx;
  za.crx_e = S("_ud_crx", k1); za.cry_e = S("_ud_cry", k1); za.xfx_e = S("_ud_xfx", k1); za.yfx_e = S("_ud_yfx", k1);
  za.zh = zh;
  // update_dz_d writes the new heights into a second set of planes (the march reads the
  // old heights' neighbours), which then become "zh" (pointer swap, as the thermo fields)
  za.zh_out = S("_zh_alt", k1);
  if (vdamp) {
    // damp_vt on the heights too (FV3 dyn_core: "for delp, delz, and vorticity")
    za.lv = level_table(height_damping(col), 1);
    za.hlv = hlevel_zh.data();
    za.d2 = S("_ud_d2", k1); za.fx2 = S("_ud_fx2", k1); za.fy2 = S("_ud_fy2", k1);
  }

  Riem3Args ra{};
  ra.npz = npz;
  ra.dt = dt; ra.ptop = ptop; ra.p_fac = nl.p_fac; ra.dz_min = nl.dz_min;
  ra.delp = delp.p; ra.pt = pt.p; ra.phis = phis.p;
  ra.w = w.p; ra.delz = delz.p; ra.zh = zh; ra.ppe = ppe; ra.pk3 = pk3; ra.pe = pe; ra.peln = peln; ra.pk = pk;
  ra.ws = ws;

  NhPgArgs pa{};
  pa.npz = npz;
  pa.dt = dt; pa.ptop = ptop;
  pa.pp = ppe; pa.pk3 = pk3; pa.delp = delp.p;
  // gz = grav * zh, formed as nh_p_grad's a2b_ord4 loads zh (the same product, no pass)
  pa.gz = zh;
  pa.gz_scale = Constants::grav;
  pa.ppb = S("_pg_pp", k1); pa.pkb = S("_pg_pk", k1); pa.gzb = S("_pg_gz", k1); pa.wk1 = S("_pg_wk", npz);
  pa.qx = S("_pg_qx", k1); pa.qy = S("_pg_qy", k1);
  pa.u = u.p; pa.v = v.p;

  // fused d_sw thermo march: delp / w / pt are updated into a second set of planes, which
  // then become the fields (pointer swap; n_split even ends on the original planes).  The
  // second set takes the first's halo ring, so the halo points no exchange fills (the
  // cube-corner regions) match whichever set is current; the march writes every compute
  // point (a whole-plane copy, 0.15 ms per C180 step, was not needed).
  DswArgs probe{};
  probe.hord_vt = nl.hord_vt; probe.hord_tm = nl.hord_tm; probe.hord_dp = nl.hord_dp;
  probe.delp_o = probe.w_o = probe.pt_o = delp.p;  // (only their presence is tested)
  probe.npz = npz;
  probe.hlv = da.hlv;
  const bool tfused = d_sw_thermo_fused(probe);
  Field* alt[3] = {nullptr, nullptr, nullptr};
  Field* cur3[3] = {&delp, &w, &pt};
  double* orig3[3] = {delp.p, w.p, pt.p};
  if (tfused) {
    const char* an[3] = {"_delp_alt", "_w_alt", "_pt_alt"};
    for (int f = 0; f < 3; ++f) {
      alt[f] = &field(an[f], npz);
      copy_halo_ring(c, d.nsub * npz, cur3[f]->p, alt[f]->p);
    }
  }
  auto zh_swap = [&]() {
    Field& fz = field("zh", k1);
    Field& fa = field("_zh_alt", k1);
    std::swap(fz.p, fa.p);
    zh = fz.p;
    za.zh = zh;
    za.zh_out = fa.p;
    ra.zh = zh;
    pa.gz = zh;
  };
  auto thermo_swap = [&]() {
    for (int f = 0; f < 3; ++f) std::swap(cur3[f]->p, alt[f]->p);
    ca.delp = da.delp = delp.p;
    ra.delp = pa.delp = delp.p;
    ca.pt = da.pt = pt.p;
    ra.pt = pt.p;
    ca.w = da.w = ra.w = w.p;
    da.delp_o = alt[0]->p; da.w_o = alt[1]->p; da.pt_o = alt[2]->p;
  };
  if (tfused) {
    da.delp_o = alt[0]->p; da.w_o = alt[1]->p; da.pt_o = alt[2]->p;
  }

  zh_init(c, npz, phis.p, delz.p, zh);  // compute domain: reads no halo
  halo_update({{"u", 'd'}, {"v", 'd'}, {"delp", 'c'}, {"pt", 'c'}, {"w", 'c'}, {"phis", 'c'}, {"zh", 'c'}});
  // the height planes alternate with _zh_alt (the march writes compute points only): give the
  // second set the halo ring of the first, so a halo point no exchange fills (the cube-corner
  // regions) holds the same value whichever set is current -- the in-place update's semantics
  copy_halo_ring(c, d.nsub * k1, zh, za.zh_out);
  bool in_graph = false;  // the loop is being captured: no event records inside
  // Interior / boundary split of the exchanges with messages (several ranks, or RCCL self
  // messages; GTFV3_HALO_SPLIT=0: off): the uc / vc and the u / v exchanges begin (pack, same-rank
  // gather, messages on the exchange's communication stream), the stencil that consumes them
  // runs on the points that read no halo value -- ds_utvt1 after uc / vc, cs_tmp after u / v --
  // while the messages fly, then the exchange ends (unpack) and the boundary frame follows.
  const int split_mode = halo_split_mode();
  // the thermo march's tile-edge kernel on stream d beside its interior kernel (tp.hip march2)
  Ctx ct = c;
  if (fork_substep && edge_side()) {
    ct.side = st_d;
    ct.side_fork = ev_df;
    ct.side_join = ev_dj;
  }
  const bool split = halo.remote() && split_fits(d) && kloop_levels() > 0 &&
                     (split_mode == 1 || (split_mode < 0 && dc.nranks > 1 && !nl.loopback));
  auto acoustic = [&]() {
  const bool early = fork_substep && early_winds != 0;
  bool uv_open = false;  // the previous sub-step's u, v exchange has begun and not ended
  for (int it = 0; it < nl.n_split; ++it) {
    const bool last = it == nl.n_split - 1;
    if (uv_open) {
      c_sw_transport(c, ca, 1);  // cs_tmp's interior beside the messages
      halo_end();
      uv_open = false;
    }
    const int csw_part = split && it > 0 ? 2 : 0;
    c_sw_transport(c, ca, csw_part);
    // nord > 0: c_sw's divergence_corner from the D-grid winds and d2a2c's ua, va
    if (nl.nord > 0) divergence_corner(c, npz, u.p, v.p, ua, va, const_cast<double*>(da.divg));
    // c_sw's wind stage (vorticity, uc / vc) beside update_dz_c + riem_solver_c: they share
    // no field; joined before p_grad_c, which needs both
    if (fork_substep) {
      HIP_CHECK(hipEventRecord(ev_fork, st));
      HIP_CHECK(hipStreamWaitEvent(st_b, ev_fork, 0));
      Ctx cb = c;
      cb.st = st_b;
      c_sw_winds(cb, ca);
      HIP_CHECK(hipEventRecord(ev_b, st_b));
    } else {
      c_sw_winds(c, ca);
    }
    update_dz_c(c, npz, dp_ref, ca.ut, ca.vt, zh, gzc);
    riem_solver_c(c, npz, dt2, ptop, nl.p_fac, nl.dz_min, ca.delpc, ca.ptc, ca.wc, phis.p, gzc, pef, nsc);
    if (fork_substep) HIP_CHECK(hipStreamWaitEvent(st, ev_b, 0));
    p_grad_c(c, npz, dt2, ca.delpc, pef, gzc, uc, vc);
    // one value per shared tile-edge point: the east / north edges take the C-grid winds
    // the neighbouring tile computed there (otherwise the two tiles' winds differ next to
    // the cube corners -- the corner circulation of c_sw -- and so do their mass fluxes:
    // a dry-mass drift of 3e-7 per step, 1.5e-11 with the sync); the sync and the C halo
    // as one exchange (H_CSC, bit-identical to 'S' then 'C')
    {
      std::vector<std::pair<std::string, char>> cx = {{"uc", 'X'}, {"vc", 'X'}};
      if (nl.nord > 0) cx.push_back({"divgd", 'b'});
      if (split) {
        halo_begin(cx);
        d_sw_courant(c, da, nullptr, 1);  // ds_utvt1's interior beside the messages
        halo_end();
      } else {
        halo_update(cx);
      }
    }
    if (last && !in_graph) record_mark(SM_CWINDS, st);
    // fork: after the Courant numbers, the wind stage of d_sw (stream b) and update_dz_d
    // (stream c) run beside the mass / thermodynamic transport (and the wind stage on beside
    // riem_solver3 and the exchange of delp, pt, zh, ppe, w).  Default on (GTFV3_STREAMS=0: one
    // stream): with the thermo march at one or two waves per SIMD the side streams fill
    // the chip -- C180 on one GPU 43.8 -> 42.4 ms per step.
    d_sw_courant(c, da, early ? ev_ut : nullptr, split ? 2 : 0);
    if (!fork_substep) {
      d_sw_thermo(ct, da);
      if (tfused) thermo_swap();
      d_sw_winds(c, da, true);
      update_dz_d(c, za);
      zh_swap();
    } else {
    HIP_CHECK(hipEventRecord(ev_fork, st));
    HIP_CHECK(hipStreamWaitEvent(st_c, ev_fork, 0));
    {
      Ctx cb = c, cc = c;
      cb.st = st_b;
      cc.st = st_c;
      if (early) {
        // the kinetic energy needs ut / vt, not the Courant numbers: it starts beside
        // ds_courant, and the vorticity march waits for those and the vorticity
        HIP_CHECK(hipStreamWaitEvent(st_b, ev_ut, 0));
        d_sw_winds(cb, da, true, &ev_fork, 1);
      } else {
        HIP_CHECK(hipStreamWaitEvent(st_b, ev_fork, 0));
        d_sw_winds(cb, da, true);
      }
      update_dz_d(cc, za);
      zh_swap();
    }
    d_sw_thermo(ct, da);
    if (tfused) thermo_swap();
    HIP_CHECK(hipEventRecord(ev_b, st_b));
    HIP_CHECK(hipEventRecord(ev_c, st_c));
    // riem_solver3 needs update_dz_d's heights, not d_sw's winds: the wind stage (u, v) keeps
    // running beside the Riemann solver, the halo updates, pk3 and gz, and is joined only
    // before nh_p_grad, which updates u and v
    HIP_CHECK(hipStreamWaitEvent(st, ev_c, 0));
    }
    ra.last_call = last ? 1 : 0;
    riem_solver3(c, ra, nsc);
    // delp / pt (d_sw's thermodynamic update) join riem_solver3's fields in one exchange:
    // nothing between reads their halos (riem_solver3 works on the compute domain; the wind
    // stage and update_dz_d do not read them), pk3_pe_halo and the next c_sw do
    halo_update({{"delp", 'c'}, {"pt", 'c'}, {"zh", 'c'}, {"ppe", 'c'}, {"w", 'c'}});
    pk3_pe_halo(c, npz, ptop, last, delp.p, pk3, pe);
    if (fork_substep) HIP_CHECK(hipStreamWaitEvent(st, ev_b, 0));
    if (d_sw_post_needed(da)) d_sw_post(c, da);  // the new delp and u, v: after both d_sw stages
    nh_p_grad(c, pa);
    if (!last) {
      if (split) {
        halo_begin({{"u", 'd'}, {"v", 'd'}});
        uv_open = true;
      } else {
        halo_update({{"u", 'd'}, {"v", 'd'}});
      }
    }
  }
  };
  // The n_split acoustic sub-steps (~40 launches each, on three streams, with their halo
  // exchanges) replayed as one HIP graph (GTFV3_GRAPH=1): the per-launch gaps between
  // dependent kernels (~9 us median at the 8-rank share, 11 % of its step) become graph edges.  Captured only
  // where nothing in the loop waits on the host (one rank, or a capturable transport: RCCL
  // and the loopback test transport are not), with an even n_split (the thermo ping-pong
  // then ends on the planes it started from, so the host's pointers match the graph's), and
  // without per-kernel timing.  The key holds everything the captured launches bake in.
  const bool graph = graph_enabled() && nsteps > 0 && nl.n_split % 2 == 0 && !ktimer_enabled() &&
                     !debug_sync_launch() && halo.capturable();
  if (graph) {
    std::vector<double> key = {(double)field_gen, dt, dt2, ptop, (double)fork_substep, (double)tfused,
                               (double)nl.n_split, nl.dddmp, nl.d2_bg, nl.p_fac, nl.dz_min, nl.d4_bg, nl.vtdm4,
                               nl.d_con, (double)nl.nord, (double)nl.nord_v, (double)nl.hord_mt, (double)nl.hord_vt,
                               (double)nl.n_sponge, nl.d2_bg_k1, nl.d2_bg_k2, nl.ke_bg, (double)nl.do_vort_damp,
                               (double)nl.hord_tm, (double)nl.hord_dp, (double)early_winds,
                               // launch-shape switches read at every launch (tests flip them in-process)
                               (double)kloop_levels(),
                               (double)riem_variant(), (double)remap_variant(), (double)halo_split_mode(),
                               (double)edge_side()};
    for (const Field* f : {&u, &v, &w, &delz, &pt, &delp, &phis})
      key.push_back((double)reinterpret_cast<uintptr_t>(f->p));
    for (const double* p : {vert, dp_ref}) key.push_back((double)reinterpret_cast<uintptr_t>(p));
    if (!ac_exec || key != ac_key) {
      if (ac_exec) HIP_CHECK(hipGraphExecDestroy(ac_exec));
      ac_exec = nullptr;
      hipGraph_t g = nullptr;
      HIP_CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed));
      in_graph = true;
      acoustic();
      in_graph = false;
      HIP_CHECK(hipStreamEndCapture(st, &g));
      HIP_CHECK(hipGraphInstantiate(&ac_exec, g, nullptr, nullptr, 0));
      HIP_CHECK(hipGraphDestroy(g));
      ac_key = key;
    }
    HIP_CHECK(hipGraphLaunch(ac_exec, st));
  } else {
    acoustic();
  }
  ++nsteps;
  // odd n_split: the fields end on the second planes; copy back to the caller's planes
  if (tfused && delp.p != orig3[0]) {
    for (int f = 0; f < 3; ++f) copy_levels(c, field_elems(npz), cur3[f]->p, alt[f]->p);
    thermo_swap();
  }
  // d_con: the damped kinetic energy, summed over the sub-steps, into the potential temperature
  // of the top n_con levels, smoothed first by del2_cubed (FV3 dyn_core "Add dissipative heating")
  const int n_con = heat_levels(nl);
  if (dcon && n_con > 0) {
    halo_update({{"_dd_heat", 'c'}});
    del2_cubed(c, npz, 0, n_con, std::min(3, nl.nord + 1), 0.2 * c.da_min, da.heat, S("_dd_h2x", npz),
               S("_dd_h2y", npz));
    damping_heat_apply(c, npz, n_con, std::fabs(bdt * nl.delt_max), da.heat, delp.p, delz.p, pt.p);
  }
  HIP_CHECK(hipEventRecord(ev[1], st));
  auto mark = [&](int m) { record_mark(m, st); };
  if (graph) mark(SM_CWINDS);  // (not recorded inside the replayed loop)
  mark(SM_ACOUSTIC);

  // ---- tracer transport with the accumulated mass fluxes, beside the remap of T_v, delz,
  // w and the winds (which touch none of the tracer step's fields); the tracer remap and
  // the remap's finish wait for both ----
  RemapScratch rsc;
  for (int n = 0; n < 3; ++n) rsc.s[n] = S(("_rmj" + std::to_string(n)).c_str(), remap_scratch_slots(nq) * k1);
  if (fork_substep) {
    HIP_CHECK(hipEventRecord(ev_fork, st));
    HIP_CHECK(hipStreamWaitEvent(st_b, ev_fork, 0));
    std::swap(st, st_b);  // tracer_2d enqueues (kernels, halo updates, copies) on the side stream
    if (tracer_wait) HIP_CHECK(hipStreamWaitEvent(st, tracer_wait, 0));
    tracer_2d(nq, mdt);  // records SM_FLUXES
    std::swap(st, st_b);
    HIP_CHECK(hipEventRecord(ev_b, st_b));
    RemapState rs1{pe, peln, pk, pkz, delp.p, delz.p, pt.p, w.p, q.p, u.p, v.p, ps, ws};
    lagrangian_to_eulerian(c, npz, nq, ptop, nl.fill != 0, ak_dev, bk_dev, rs1, rsc, remap_variant(), 1);
    HIP_CHECK(hipStreamWaitEvent(st, ev_b, 0));
  } else {
    if (tracer_wait) HIP_CHECK(hipStreamWaitEvent(st, tracer_wait, 0));
    tracer_2d(nq, mdt);  // records SM_FLUXES
  }
  HIP_CHECK(hipEventRecord(ev[2], st));

  // ---- vertical remap to the hybrid Eulerian coordinate ----
  RemapState rs{pe, peln, pk, pkz, delp.p, delz.p, pt.p, w.p, q.p, u.p, v.p, ps, ws};
  lagrangian_to_eulerian(c, npz, nq, ptop, nl.fill != 0, ak_dev, bk_dev, rs, rsc, remap_variant(), fork_substep ? 2 : 0);
  HIP_CHECK(hipEventRecord(ev[3], st));
  mark(SM_REMAP);

  // ---- exit: T, omega, A-grid winds ----
  if (exit_wait) HIP_CHECK(hipStreamWaitEvent(st, exit_wait, 0));
  fv_wrapup(c, npz, nq, zvir, q.p, delp.p, delz.p, w.p, pt.p, omga);
  mark(SM_WRAPUP);
  halo_update({{"u", 'd'}, {"v", 'd'}});
  mark(SM_WINDS);
  c2l_ord4(c, npz, u.p, v.p, ua, va);
  HIP_CHECK(hipEventRecord(ev[4], st));
  ev_pending[slot] = true;
  if (ktimer_enabled()) ktimer_flush();
}

void Dycore::flush_timers(int slot) {
  hipEvent_t* ev = ev_ph[slot];
  HIP_CHECK(hipEventSynchronize(ev[4]));
  const char* names[4] = {"dyn_core", "tracer_2d", "remap", "exit"};
  for (int n = 0; n < 4; ++n) {
    float ms = 0;
    HIP_CHECK(hipEventElapsedTime(&ms, ev[n], ev[n + 1]));
    timers[names[n]] += ms;
  }
  float tot = 0;
  HIP_CHECK(hipEventElapsedTime(&tot, ev[0], ev[4]));
  timers["fv_dynamics"] += tot;
  step_ms.push_back(tot);
  timers["steps"] += 1;
  ev_pending[slot] = false;
}

void Dycore::flush_all_timers() {
  // oldest first
  for (int n = 0; n < 2; ++n) {
    const int slot = (ev_slot + n) & 1;
    if (ev_pending[slot]) flush_timers(slot);
  }
}

}  // namespace gtfv3
