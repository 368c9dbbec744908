// stencils_registry.cpp — named stencil entry points (gtfv3_stencil).
#include "stencils_registry.hpp"

#include <functional>
#include <map>
#include <stdexcept>

#include "dycore.hpp"
#include "kernels.hpp"

namespace gtfv3 {

namespace {

using Fn = std::function<void(Dycore&, const std::vector<std::string>&, const std::vector<double>&)>;

Field& F(Dycore& dy, const std::string& n) {
  Field* f = dy.find(n);
  if (!f) throw std::runtime_error("stencil: unknown field '" + n + "'");
  return *f;
}

void need(const std::vector<std::string>& f, size_t n, const char* who) {
  if (f.size() != n) throw std::runtime_error(std::string(who) + ": expected " + std::to_string(n) + " fields");
}

std::map<std::string, Fn>& reg() {
  static std::map<std::string, Fn> r = {
      // fv_tp_2d(q, crx, cry, xfx, yfx, ra_x, ra_y, mfx|-, mfy|-, fx, fy) params: ord, nt
      {"fv_tp_2d",
       [](Dycore& dy, const std::vector<std::string>& f, const std::vector<double>& p) {
         need(f, 11, "fv_tp_2d");
         int ord = p.size() > 0 ? (int)p[0] : 6;
         int nt = p.size() > 1 ? (int)p[1] : 1;
         Field& q = F(dy, f[0]);
         int nk = q.nk / nt;
         TpArgs a{};
         a.q = q.p; a.nt = nt; a.nk = nk;
         a.crx = F(dy, f[1]).p; a.cry = F(dy, f[2]).p; a.xfx = F(dy, f[3]).p; a.yfx = F(dy, f[4]).p;
         a.ra_x = F(dy, f[5]).p; a.ra_y = F(dy, f[6]).p;
         a.mfx = f[7] == "-" ? nullptr : F(dy, f[7]).p;
         a.mfy = f[8] == "-" ? nullptr : F(dy, f[8]).p;
         a.fx = dy.field(f[9], q.nk).p; a.fy = dy.field(f[10], q.nk).p;
         a.fx2 = dy.field("_tp_fx2", q.nk).p; a.fy2 = dy.field("_tp_fy2", q.nk).p;
         a.qi = dy.field("_tp_qi", q.nk).p; a.qj = dy.field("_tp_qj", q.nk).p;
         a.ord = ord;
         fv_tp_2d(dy.ctx(), a);
       }},
      // tracer_2d_1l: uses state fields q, dp1, cx, cy, mfx, mfy. params: nq
      {"tracer_2d_1l",
       [](Dycore& dy, const std::vector<std::string>& f, const std::vector<double>& p) {
         (void)f;
         int nq = p.size() > 0 ? (int)p[0] : dy.nl.nq;
         dy.tracer_2d(nq, dy.nl.dt_atmos);
       }},
  };
  return r;
}

}  // namespace

void register_dynamics_stencils(std::map<std::string, Fn>& r);

void run_registered_stencil(Dycore& dy, const std::string& name, const std::vector<std::string>& fields,
                            const std::vector<double>& params) {
  auto& r = reg();
  auto it = r.find(name);
  if (it == r.end()) throw std::runtime_error("unknown stencil '" + name + "'");
  it->second(dy, fields, params);
}

std::vector<std::string> registered_stencils() {
  std::vector<std::string> v;
  for (auto& kv : reg()) v.push_back(kv.first);
  return v;
}

}  // namespace gtfv3
