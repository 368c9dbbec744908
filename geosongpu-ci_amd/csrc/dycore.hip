// dycore.hip — Dycore context: decomposition, grid upload, named device
// fields, halo groups, and the per-step algorithm sequence (fv_dynamics).
#include "dycore.hpp"

#include <algorithm>
#include <cstring>
#include <stdexcept>

#include "hip_util.hpp"

namespace gtfv3 {

long Field::elems() const { return 0; }

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
    halo.build(*cs, dc, d, max_nk, 8, false);
    return;
  }
  HIP_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  HIP_CHECK(hipMalloc(&dsubs, sizeof(SubInfo) * d.nsub));
  HIP_CHECK(hipMemcpy(dsubs, hsubs.data(), sizeof(SubInfo) * d.nsub, hipMemcpyHostToDevice));
  HIP_CHECK(hipMalloc(&dmet, sizeof(double) * hm.m.size()));
  HIP_CHECK(hipMemcpy(dmet, hm.m.data(), sizeof(double) * hm.m.size(), hipMemcpyHostToDevice));
  HIP_CHECK(hipMalloc(&dcornerw, sizeof(double) * hm.corner_w.size()));
  HIP_CHECK(hipMemcpy(dcornerw, hm.corner_w.data(), sizeof(double) * hm.corner_w.size(), hipMemcpyHostToDevice));

  if (nranks > 1) {
    if (!nccl_id) throw std::runtime_error("multi-rank run needs an ncclUniqueId");
    ncclUniqueId id;
    std::memcpy(&id, nccl_id, sizeof(id));
    if (ncclCommInitRank(&comm, nranks, id, rank) != ncclSuccess) throw std::runtime_error("ncclCommInitRank failed");
    halo.set_comm(comm);
  }
  halo.build(*cs, dc, d, max_nk, 8);
}

Dycore::~Dycore() {
  for (auto& kv : fields) (void)hipFree(kv.second.p);
  if (dsubs) (void)hipFree(dsubs);
  if (dmet) (void)hipFree(dmet);
  if (dcornerw) (void)hipFree(dcornerw);
  if (comm) ncclCommDestroy(comm);
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
  size_t bytes = sizeof(double) * (size_t)field_elems(nk);
  HIP_CHECK(hipMalloc(&f.p, bytes));
  HIP_CHECK(hipMemsetAsync(f.p, 0, bytes, st));
  return fields[name] = f;
}

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

void Dycore::download(const std::string& name, double* host) {
  Field* f = find(name);
  if (!f) throw std::runtime_error("no field '" + name + "'");
  HIP_CHECK(hipMemcpyAsync(host, f->p, sizeof(double) * field_elems(f->nk), hipMemcpyDeviceToHost, st));
  HIP_CHECK(hipStreamSynchronize(st));
}

void Dycore::halo_update(const std::vector<std::pair<std::string, char>>& items) {
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
      h.kind = k == 'd' ? H_DGRID : (k == 'C' ? H_CGRID : H_AGRID);
      ++n;
    }
    hf.push_back(h);
  }
  halo.exchange(hf.data(), (int)hf.size(), st);
}

void Dycore::allreduce_max(double* dev, int n) {
  if (!comm) return;
  if (ncclAllReduce(dev, dev, n, ncclDouble, ncclMax, comm, st) != ncclSuccess)
    throw std::runtime_error("ncclAllReduce failed");
}

void Dycore::set_vertical(const double* ak_, const double* bk_, int ks_) {
  ak.assign(ak_, ak_ + nl.npz + 1);
  bk.assign(bk_, bk_ + nl.npz + 1);
  ks = ks_;
}

// tracer_2d_1l (FV3 fv_tracer2d): large-time-step transport of nq tracers with
// the mass fluxes (mfx,mfy) and Courant numbers (cx,cy) accumulated over the
// acoustic sub-steps; dp1 = delp at the start of the step.
void Dycore::tracer_2d(int nq, double /*dt*/) {
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
  Field& ra_x = field("tr_ra_x", npz);
  Field& ra_y = field("tr_ra_y", npz);
  Field& dp2 = field("tr_dp2", npz);
  Field& cmax = field("tr_cmax", 1);  // first npz doubles used
  Field& nspl = field("tr_nsplt", 1);
  Field& fx = field("tr_fx", nq * npz);
  Field& fy = field("tr_fy", nq * npz);
  Field& fx2 = field("tr_fx2", nq * npz);
  Field& fy2 = field("tr_fy2", nq * npz);
  Field& qi = field("tr_qi", nq * npz);
  Field& qj = field("tr_qj", nq * npz);
  if ((long)npz > d.plane) throw std::runtime_error("tracer cmax scratch too small");

  tracer_prep(c, npz, cx.p, cy.p, xfx.p, yfx.p, ra_x.p, ra_y.p, cmax.p);
  allreduce_max(cmax.p, npz);
  std::vector<double> hcm(npz);
  HIP_CHECK(hipMemcpyAsync(hcm.data(), cmax.p, sizeof(double) * npz, hipMemcpyDeviceToHost, st));
  HIP_CHECK(hipStreamSynchronize(st));
  std::vector<int> ns(npz);
  int nmax = 1;
  for (int k = 0; k < npz; ++k) {
    ns[k] = (int)(1.0 + hcm[k]);
    nmax = std::max(nmax, ns[k]);
  }
  int* dns = reinterpret_cast<int*>(nspl.p);
  HIP_CHECK(hipMemcpyAsync(dns, ns.data(), sizeof(int) * npz, hipMemcpyHostToDevice, st));
  tracer_split(c, npz, dns, cx.p, cy.p, xfx.p, yfx.p, mfx.p, mfy.p, ra_x.p, ra_y.p);
  halo_update({{"q", 'c'}});
  for (int it = 0; it < nmax; ++it) {
    tracer_dp2(c, npz, dp1.p, mfx.p, mfy.p, dp2.p);
    TpArgs a{};
    a.q = q.p; a.nt = nq; a.nk = npz;
    a.crx = cx.p; a.cry = cy.p; a.xfx = xfx.p; a.yfx = yfx.p; a.ra_x = ra_x.p; a.ra_y = ra_y.p;
    a.mfx = mfx.p; a.mfy = mfy.p;
    a.fx = fx.p; a.fy = fy.p; a.fx2 = fx2.p; a.fy2 = fy2.p; a.qi = qi.p; a.qj = qj.p;
    a.ord = nl.hord_tr;
    fv_tp_2d(c, a);
    tracer_update(c, npz, nq, q.p, nullptr, dp1.p, dp2.p, fx.p, fy.p, dns, it);
    if (it + 1 < nmax) {
      copy_levels(c, field_elems(npz), dp2.p, dp1.p);
      halo_update({{"q", 'c'}});
    }
  }
}

void Dycore::step() { throw std::runtime_error("step: not built yet"); }

}  // namespace gtfv3
