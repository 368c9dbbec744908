// stencils_registry.cpp — named stencil entry points (gtfv3_stencil).
#include "stencils_registry.hpp"

#include <functional>
#include <map>
#include <stdexcept>

#include "dycore.hpp"
#include "kernels.hpp"
#include "kernels_column.hpp"
#include "kernels_damp.hpp"
#include "kernels_misc.hpp"
#include "kernels_moist.hpp"
#include "kernels_nh.hpp"
#include "kernels_sw.hpp"

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
      // fv_tp_2d(q, crx, cry, xfx, yfx, ra_x, ra_y, mfx|-, mfy|-, fx, fy) params: ord, nt, cfg
      // (FV3 argument list; ra_x / ra_y are formed in the kernel from area, xfx, yfx and not read)
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
         // ra_x, ra_y: not read (may be "-"); when named they must exist
         if (f[5] != "-") (void)F(dy, f[5]);
         if (f[6] != "-") (void)F(dy, f[6]);
         a.mfx = f[7] == "-" ? nullptr : F(dy, f[7]).p;
         a.mfy = f[8] == "-" ? nullptr : F(dy, f[8]).p;
         a.fx = dy.field(f[9], q.nk).p; a.fy = dy.field(f[10], q.nk).p;
         a.ord = ord;
         a.cfg = p.size() > 2 ? (int)p[2] : -1;
         fv_tp_2d(dy.ctx(), a);
       }},
      // fv_tp_2d_pair(q, q2, crx, cry, xfx, yfx, mfx|-, mfy|-, fx, fy, fx_2, fy_2) params: ord
      // two fields with shared Courant numbers and fluxes in one launch (d_sw's w and pt)
      {"fv_tp_2d_pair",
       [](Dycore& dy, const std::vector<std::string>& f, const std::vector<double>& p) {
         need(f, 12, "fv_tp_2d_pair");
         Field& q = F(dy, f[0]);
         Field& q2 = F(dy, f[1]);
         if (q2.nk != q.nk) throw std::runtime_error("fv_tp_2d_pair: fields must share the level count");
         TpArgs a{};
         a.q = q.p; a.q2 = q2.p; a.nt = 1; a.nk = q.nk;
         a.crx = F(dy, f[2]).p; a.cry = F(dy, f[3]).p; a.xfx = F(dy, f[4]).p; a.yfx = F(dy, f[5]).p;
         a.mfx = f[6] == "-" ? nullptr : F(dy, f[6]).p;
         a.mfy = f[7] == "-" ? nullptr : F(dy, f[7]).p;
         a.fx = dy.field(f[8], q.nk).p; a.fy = dy.field(f[9], q.nk).p;
         a.fx_2 = dy.field(f[10], q.nk).p; a.fy_2 = dy.field(f[11], q.nk).p;
         a.ord = p.size() > 0 ? (int)p[0] : 6;
         fv_tp_2d(dy.ctx(), a);
       }},
      // c_sw(delp, pt, w, u, v | uc, vc, ua, va, ut, vt, delpc, ptc, wc) params: dt2
      {"c_sw",
       [](Dycore& dy, const std::vector<std::string>& f, const std::vector<double>& p) {
         need(f, 14, "c_sw");
         const int npz = F(dy, f[0]).nk;
         auto out = [&](int n) { return dy.field(f[n], npz).p; };
         CswArgs a{};
         a.npz = npz;
         a.dt2 = p.at(0);
         a.delp = F(dy, f[0]).p; a.pt = F(dy, f[1]).p; a.w = F(dy, f[2]).p; a.u = F(dy, f[3]).p; a.v = F(dy, f[4]).p;
         a.uc = out(5); a.vc = out(6); a.ua = out(7); a.va = out(8); a.ut = out(9); a.vt = out(10);
         a.delpc = out(11); a.ptc = out(12); a.wc = out(13);
         a.utmp = dy.field("_cs_utmp", npz).p; a.vtmp = dy.field("_cs_vtmp", npz).p;
         a.ke = dy.field("_cs_ke", npz).p; a.vort = dy.field("_cs_vort", npz).p;
         c_sw(dy.ctx(), a);
       }},
      // d_sw(delp, pt, w, u, v, uc, vc, ua, va | crx, cry, xfx, yfx, cx, cy, mfx, mfy, ke)
      // params: dt, dddmp, d2_bg, hord_mt, hord_vt, hord_tm, hord_dp[, fused thermo march]
      // (no sponge layers: d2_bg on every level, nord = 0, no other damping)
      {"d_sw",
       [](Dycore& dy, const std::vector<std::string>& f, const std::vector<double>& p) {
         need(f, 18, "d_sw");
         const int npz = F(dy, f[0]).nk;
         auto out = [&](int n) { return dy.field(f[n], npz).p; };
         auto scr = [&](const char* n) { return dy.field(n, npz).p; };
         DswArgs a{};
         a.npz = npz;
         a.dt = p.at(0); a.dddmp = p.at(1);
         {
           Namelist nl{};
           nl.npz = npz; nl.d2_bg = p.at(2); nl.n_sponge = -1;
           const std::vector<LevelDamp> col = column_damping(nl, dy.ctx().da_min, dy.ctx().da_min_c);
           a.lv = dy.level_table(col);
           a.hlv = dy.hlevel.data();
         }
         a.hord_mt = (int)p.at(3); a.hord_vt = (int)p.at(4); a.hord_tm = (int)p.at(5); a.hord_dp = (int)p.at(6);
         a.delp = F(dy, f[0]).p; a.pt = F(dy, f[1]).p; a.w = F(dy, f[2]).p; a.u = F(dy, f[3]).p; a.v = F(dy, f[4]).p;
         a.uc = F(dy, f[5]).p; a.vc = F(dy, f[6]).p; a.ua = F(dy, f[7]).p; a.va = F(dy, f[8]).p;
         a.crx = out(9); a.cry = out(10); a.xfx = out(11); a.yfx = out(12);
         a.cx = out(13); a.cy = out(14); a.mfx = out(15); a.mfy = out(16); a.ke = out(17);
         a.ut = scr("_ds_ut"); a.vt = scr("_ds_vt");
         a.fx = scr("_ds_fx"); a.fy = scr("_ds_fy"); a.gwx = scr("_ds_gwx"); a.gwy = scr("_ds_gwy");
         a.gtx = scr("_ds_gtx"); a.gty = scr("_ds_gty"); a.vort = scr("_ds_vort");
         a.gvx = scr("_ds_gvx"); a.gvy = scr("_ds_gvy");
         // params[7] (optional): 0 = the separate transport launches, ds_accum and ds_thermo;
         // else the fused thermo march (into scratch planes, copied back: in-place semantics)
         const bool fused = p.size() < 8 || p[7] != 0.0;
         if (fused) {
           a.delp_o = scr("_ds_delp_o"); a.w_o = scr("_ds_w_o"); a.pt_o = scr("_ds_pt_o");
           const long n = dy.field_elems(npz);  // halo points carried over as in place
           copy_levels(dy.ctx(), n, a.delp, a.delp_o);
           copy_levels(dy.ctx(), n, a.w, a.w_o);
           copy_levels(dy.ctx(), n, a.pt, a.pt_o);
         }
         d_sw(dy.ctx(), a);
         if (d_sw_thermo_fused(a)) {
           const long n = dy.field_elems(npz);
           copy_levels(dy.ctx(), n, a.delp_o, a.delp);
           copy_levels(dy.ctx(), n, a.w_o, a.w);
           copy_levels(dy.ctx(), n, a.pt_o, a.pt);
         }
       }},
      // divergence_corner(u, v, ua, va | divg): c_sw's corner divergence for nord > 0
      {"divergence_corner",
       [](Dycore& dy, const std::vector<std::string>& f, const std::vector<double>&) {
         need(f, 5, "divergence_corner");
         const int npz = F(dy, f[0]).nk;
         divergence_corner(dy.ctx(), npz, F(dy, f[0]).p, F(dy, f[1]).p, F(dy, f[2]).p, F(dy, f[3]).p,
                           dy.field(f[4], npz).p);
       }},
      // d_sw_damped(the 18 d_sw fields, divg, heat, diss): d_sw (fused thermo march unless
      // delp / pt take del-n damping) with the column of damping parameters of the namelist
      // below (damp.hip column_damping), then d_sw_post (d_con heat / diss += and the
      // vorticity-damping fluxes).  params: dt, dddmp, d2_bg, hord_mt, hord_vt, hord_tm, hord_dp,
      // nord, d4_bg, vtdm4, nord_v, d_con[, do_vort_damp (1), n_sponge (-1: none), d2_bg_k1,
      // d2_bg_k2, ke_bg]
      {"d_sw_damped",
       [](Dycore& dy, const std::vector<std::string>& f, const std::vector<double>& p) {
         need(f, 21, "d_sw_damped");
         if (p.size() < 12) throw std::runtime_error("d_sw_damped: 12 params");
         const int npz = F(dy, f[0]).nk;
         auto out = [&](int n) { return dy.field(f[n], npz).p; };
         auto scr = [&](const char* n) { return dy.field(n, npz).p; };
         DswArgs a{};
         a.npz = npz;
         a.dt = p[0]; a.dddmp = p[1];
         a.hord_mt = (int)p[3]; a.hord_vt = (int)p[4]; a.hord_tm = (int)p[5]; a.hord_dp = (int)p[6];
         Namelist nl{};
         nl.npz = npz;
         nl.d2_bg = p[2]; nl.nord = (int)p[7]; nl.d4_bg = p[8]; nl.vtdm4 = p[9]; nl.nord_v = (int)p[10];
         nl.d_con = p[11];
         nl.do_vort_damp = p.size() > 12 ? p[12] != 0.0 : true;
         nl.n_sponge = p.size() > 13 ? (int)p[13] : -1;
         nl.d2_bg_k1 = p.size() > 14 ? p[14] : 0.0;
         nl.d2_bg_k2 = p.size() > 15 ? p[15] : 0.0;
         nl.ke_bg = p.size() > 16 ? p[16] : 0.0;
         if (nl.nord < 0 || nl.nord > 3 || nl.nord_v < 0 || nl.nord_v > 2) throw std::runtime_error("d_sw_damped: nord");
         const std::vector<LevelDamp> col = column_damping(nl, dy.ctx().da_min, dy.ctx().da_min_c);
         a.lv = dy.level_table(col);
         a.hlv = dy.hlevel.data();
         a.nord = nl.nord; a.d4_bg = nl.d4_bg; a.d_con = nl.d_con;
         a.ke_dt = nl.ke_bg * std::fabs(a.dt);
         a.delp = F(dy, f[0]).p; a.pt = F(dy, f[1]).p; a.w = F(dy, f[2]).p; a.u = F(dy, f[3]).p; a.v = F(dy, f[4]).p;
         a.uc = F(dy, f[5]).p; a.vc = F(dy, f[6]).p; a.ua = F(dy, f[7]).p; a.va = F(dy, f[8]).p;
         a.crx = out(9); a.cry = out(10); a.xfx = out(11); a.yfx = out(12);
         a.cx = out(13); a.cy = out(14); a.mfx = out(15); a.mfy = out(16); a.ke = out(17);
         a.ut = scr("_ds_ut"); a.vt = scr("_ds_vt");
         a.fx = scr("_ds_fx"); a.fy = scr("_ds_fy"); a.gwx = scr("_ds_gwx"); a.gwy = scr("_ds_gwy");
         a.gtx = scr("_ds_gtx"); a.gty = scr("_ds_gty"); a.vort = scr("_ds_vort");
         a.gvx = scr("_ds_gvx"); a.gvy = scr("_ds_gvy");
         a.divg = a.nord > 0 ? F(dy, f[18]).p : nullptr;
         a.heat = out(19); a.diss = out(20);
         a.wk = scr("_dd_wk"); a.vd = scr("_dd_vd");
         a.dd = scr("_dd_dd"); a.dvcx = scr("_dd_vcx"); a.ducy = scr("_dd_ucy"); a.dvort = scr("_dd_vort");
         a.dqx = scr("_dd_qx"); a.dqy = scr("_dd_qy");
         a.d2 = scr("_dd_d2"); a.fx2 = scr("_dd_fx2"); a.fy2 = scr("_dd_fy2");
         a.td2 = scr("_dl_d2"); a.tfx2 = scr("_dl_fx2"); a.tfy2 = scr("_dl_fy2"); a.dw = scr("_dl_dw");
         a.hw = scr("_dl_hw");
         a.delp_o = scr("_ds_delp_o"); a.w_o = scr("_ds_w_o"); a.pt_o = scr("_ds_pt_o");
         const long n = dy.field_elems(npz);
         copy_levels(dy.ctx(), n, a.delp, a.delp_o);
         copy_levels(dy.ctx(), n, a.w, a.w_o);
         copy_levels(dy.ctx(), n, a.pt, a.pt_o);
         d_sw(dy.ctx(), a);
         if (d_sw_thermo_fused(a)) {
           copy_levels(dy.ctx(), n, a.delp_o, a.delp);
           copy_levels(dy.ctx(), n, a.w_o, a.w);
           copy_levels(dy.ctx(), n, a.pt_o, a.pt);
         }
         d_sw_post(dy.ctx(), a);
       }},
      // riem_solver_c(delpc, ptc, wc, phis, gz | pef): gz heights in (clamped to dz_min),
      // geopotential out.  params: dt2, ptop, p_fac, dz_min[, variant (0 blocked, 1 column)]
      {"riem_solver_c",
       [](Dycore& dy, const std::vector<std::string>& f, const std::vector<double>& p) {
         need(f, 6, "riem_solver_c");
         const int npz = F(dy, f[0]).nk;
         if (F(dy, f[4]).nk != npz + 1 || F(dy, f[3]).nk != 1) throw std::runtime_error("riem_solver_c: field shapes");
         NhScratch sc{};
         sc.s[5] = dy.field("_riem_gam", npz + 1).p;
         sc.s[6] = dy.field("_riem_pp", npz + 1).p;
         sc.s[13] = dy.field("_riem_w2", npz + 1).p;
         const int v0 = riem_variant();
         set_riem_variant(p.size() > 4 ? (int)p[4] : v0);
         riem_solver_c(dy.ctx(), npz, p.at(0), p.at(1), p.at(2), p.at(3), F(dy, f[0]).p, F(dy, f[1]).p,
                       F(dy, f[2]).p, F(dy, f[3]).p, F(dy, f[4]).p, dy.field(f[5], npz + 1).p, sc);
         set_riem_variant(v0);
       }},
      // riem_solver3(delp, pt, w, phis, zh | delz, ppe, pk3, pe, peln, pk, ws): w and zh in place.
      // params: dt, ptop, p_fac, dz_min, last_call[, variant]
      {"riem_solver3",
       [](Dycore& dy, const std::vector<std::string>& f, const std::vector<double>& p) {
         need(f, 12, "riem_solver3");
         const int npz = F(dy, f[0]).nk;
         if (F(dy, f[4]).nk != npz + 1 || F(dy, f[3]).nk != 1) throw std::runtime_error("riem_solver3: field shapes");
         NhScratch sc{};
         sc.s[5] = dy.field("_riem_gam", npz + 1).p;
         sc.s[6] = dy.field("_riem_pp", npz + 1).p;
         sc.s[13] = dy.field("_riem_w2", npz + 1).p;
         Riem3Args r{};
         r.npz = npz;
         r.dt = p.at(0); r.ptop = p.at(1); r.p_fac = p.at(2); r.dz_min = p.at(3); r.last_call = (int)p.at(4);
         r.delp = F(dy, f[0]).p; r.pt = F(dy, f[1]).p; r.w = F(dy, f[2]).p; r.phis = F(dy, f[3]).p;
         r.zh = F(dy, f[4]).p;
         r.delz = dy.field(f[5], npz).p; r.ppe = dy.field(f[6], npz + 1).p; r.pk3 = dy.field(f[7], npz + 1).p;
         r.pe = dy.field(f[8], npz + 1).p; r.peln = dy.field(f[9], npz + 1).p; r.pk = dy.field(f[10], npz + 1).p;
         r.ws = dy.field(f[11], 1).p;
         const int v0 = riem_variant();
         set_riem_variant(p.size() > 5 ? (int)p[5] : v0);
         riem_solver3(dy.ctx(), r, sc);
         set_riem_variant(v0);
       }},
      // K-column primitives (dsl_patterns KATs): column_top(in | out)
      {"column_top",
       [](Dycore& dy, const std::vector<std::string>& f, const std::vector<double>&) {
         need(f, 2, "column_top");
         Field& in = F(dy, f[0]);
         column_top(dy.ctx(), in.nk, in.p, dy.field(f[1], in.nk).p);
       }},
      // column_while_lt(in | out) params: thr
      {"column_while_lt",
       [](Dycore& dy, const std::vector<std::string>& f, const std::vector<double>& p) {
         need(f, 2, "column_while_lt");
         Field& in = F(dy, f[0]);
         column_while_lt(dy.ctx(), in.nk, p.at(0), in.p, dy.field(f[1], in.nk).p);
       }},
      // column_gather_k(data, kmask, kidx2d | out2d): out2d keeps its value where no level matches
      {"column_gather_k",
       [](Dycore& dy, const std::vector<std::string>& f, const std::vector<double>&) {
         need(f, 4, "column_gather_k");
         Field& data = F(dy, f[0]);
         Field& km = F(dy, f[1]);
         Field& kidx = F(dy, f[2]);
         if (km.nk != data.nk || kidx.nk != 1) throw std::runtime_error("column_gather_k: field shapes");
         column_gather_k(dy.ctx(), data.nk, data.p, km.p, kidx.p, dy.field(f[3], 1).p);
       }},
      // Lagrangian_to_Eulerian on the dycore's own state fields (pe, peln, pk, pkz, delp, delz,
      // pt, w, q, u, v, ps, ws; pt enters as virtual potential temperature) with the vertical
      // grid of set_vertical(); no field arguments.  params: fill
      {"lagrangian_to_eulerian",
       [](Dycore& dy, const std::vector<std::string>& f, const std::vector<double>& p) {
         need(f, 0, "lagrangian_to_eulerian");
         const int npz = dy.nl.npz, k1 = npz + 1, nq = dy.nl.nq;
         const double* vert = dy.vertical_dev();
         RemapState rs{dy.need("pe", k1).p, dy.need("peln", k1).p, dy.field("pk", k1).p, dy.field("pkz", npz).p,
                       dy.need("delp", npz).p, dy.need("delz", npz).p, dy.need("pt", npz).p, dy.need("w", npz).p,
                       dy.need("q", nq * npz).p, dy.need("u", npz).p, dy.need("v", npz).p, dy.field("ps", 1).p,
                       dy.field("ws", 1).p};
         RemapScratch rsc;
         for (int n = 0; n < 3; ++n) rsc.s[n] = dy.field("_rmj" + std::to_string(n), remap_scratch_slots(nq) * k1).p;
         lagrangian_to_eulerian(dy.ctx(), npz, nq, dy.ak.at(0), p.empty() || p[0] != 0.0, vert, vert + k1, rs, rsc,
                                p.size() > 1 ? (int)p[1] : 0);
       }},
      // edge_profile(crx, xfx, cry, yfx | crx_e, xfx_e, cry_e, yfx_e): update_dz_d's interface values
      // (npz+1 levels) with the reference thicknesses of set_vertical().  params: variant (0 by level
      // count, 1 the blocked edge_prof_k)
      {"edge_profile",
       [](Dycore& dy, const std::vector<std::string>& f, const std::vector<double>& p) {
         need(f, 8, "edge_profile");
         Field& cx = F(dy, f[0]);
         const int npz = cx.nk, k1 = npz + 1;
         if (npz != dy.nl.npz) throw std::runtime_error("edge_profile: fields must have npz levels");
         const double* vert = dy.vertical_dev();
         edge_profile(dy.ctx(), npz, vert + 2 * k1, cx.p, F(dy, f[1]).p, F(dy, f[2]).p, F(dy, f[3]).p,
                      dy.field(f[4], k1).p, dy.field(f[5], k1).p, dy.field(f[6], k1).p, dy.field(f[7], k1).p,
                      p.empty() ? 0 : (int)p[0]);
       }},
      // update_dz_d(zh, crx, cry, xfx, yfx): the interface heights zh (npz+1 levels) transported in
      // place with the interface-level Courant numbers and area fluxes (edge_profile + fv_tp_2d +
      // the flux-form update; FV3 update_dz_d before its dz_min clamp).  params: hord
      {"update_dz_d",
       [](Dycore& dy, const std::vector<std::string>& f, const std::vector<double>& p) {
         need(f, 5, "update_dz_d");
         Field& zh = F(dy, f[0]);
         const int npz = dy.nl.npz, k1 = npz + 1;
         if (zh.nk != k1 || F(dy, f[1]).nk != npz) throw std::runtime_error("update_dz_d: field shapes");
         const double* vert = dy.vertical_dev();
         UdzdArgs za{};
         za.npz = npz;
         za.hord = p.empty() ? 6 : (int)p[0];
         za.dp0 = vert + 2 * k1;
         za.crx = F(dy, f[1]).p; za.cry = F(dy, f[2]).p; za.xfx = F(dy, f[3]).p; za.yfx = F(dy, f[4]).p;
         za.crx_e = dy.field("_ud_crx", k1).p; za.cry_e = dy.field("_ud_cry", k1).p;
         za.xfx_e = dy.field("_ud_xfx", k1).p; za.yfx_e = dy.field("_ud_yfx", k1).p;
         za.zh = zh.p;
         Field& zo = dy.field("_ud_zh", k1);
         za.zh_out = zo.p;
         update_dz_d(dy.ctx(), za);
         // in place for the caller: the march writes the compute cells only, so the field's halo
         // ring goes onto the new planes first, then the planes back into the field
         copy_halo_ring(dy.ctx(), dy.d.nsub * k1, zh.p, zo.p);
         copy_levels(dy.ctx(), dy.field_elems(k1), zo.p, zh.p);
       }},
      // p_grad_c(delpc, pkc, gz | uc, vc): the C-grid pressure gradient of dyn_core (pkc, gz:
      // npz+1 interface levels with their first halo ring; uc, vc updated in place).  params: dt2
      {"p_grad_c",
       [](Dycore& dy, const std::vector<std::string>& f, const std::vector<double>& p) {
         need(f, 5, "p_grad_c");
         Field& dp = F(dy, f[0]);
         const int npz = dp.nk;
         if (F(dy, f[1]).nk != npz + 1 || F(dy, f[2]).nk != npz + 1 || F(dy, f[3]).nk != npz ||
             F(dy, f[4]).nk != npz)
           throw std::runtime_error("p_grad_c: field shapes");
         p_grad_c(dy.ctx(), npz, p.at(0), dp.p, F(dy, f[1]).p, F(dy, f[2]).p, F(dy, f[3]).p, F(dy, f[4]).p);
       }},
      // nh_p_grad(pp, pk3, gz, delp | u, v): the D-grid pressure gradient (a2b_ord4 of pp, pk3, gz
      // and delp to the corners, then u, v += the gradient terms, times rdx / rdy: the winds leave
      // d_sw as u dx, v dy).  pp, pk3, gz: npz+1 levels with halos; the top interface's pp and
      // pk3 are the model-top constants 0 and ptop**kappa.  params: dt, ptop
      {"nh_p_grad",
       [](Dycore& dy, const std::vector<std::string>& f, const std::vector<double>& p) {
         need(f, 6, "nh_p_grad");
         Field& dp = F(dy, f[3]);
         const int npz = dp.nk, k1 = npz + 1;
         for (int n = 0; n < 3; ++n)
           if (F(dy, f[n]).nk != k1) throw std::runtime_error("nh_p_grad: pp, pk3, gz need npz+1 levels");
         if (F(dy, f[4]).nk != npz || F(dy, f[5]).nk != npz) throw std::runtime_error("nh_p_grad: u, v levels");
         NhPgArgs a{};
         a.npz = npz;
         a.dt = p.at(0);
         a.ptop = p.at(1);
         a.pp = F(dy, f[0]).p; a.pk3 = F(dy, f[1]).p; a.gz = F(dy, f[2]).p; a.delp = dp.p;
         a.ppb = dy.field("_pg_pp", k1).p; a.pkb = dy.field("_pg_pk", k1).p; a.gzb = dy.field("_pg_gz", k1).p;
         a.wk1 = dy.field("_pg_wk", npz).p; a.qx = dy.field("_pg_qx", k1).p; a.qy = dy.field("_pg_qy", k1).p;
         a.u = F(dy, f[4]).p; a.v = F(dy, f[5]).p;
         nh_p_grad(dy.ctx(), a);
       }},
      // a2b_ord4(q | qout): cell means -> cell corners (4th order, cubed-sphere edge forms)
      {"a2b_ord4",
       [](Dycore& dy, const std::vector<std::string>& f, const std::vector<double>&) {
         need(f, 2, "a2b_ord4");
         Field& q = F(dy, f[0]);
         a2b_ord4(dy.ctx(), q.nk, q.p, dy.field(f[1], q.nk).p, nullptr, nullptr);
       }},
      // moist column physics
      // moist_qsat(T, pm | qsw, qsi, dqsw)
      {"moist_qsat",
       [](Dycore& dy, const std::vector<std::string>& f, const std::vector<double>&) {
         need(f, 5, "moist_qsat");
         Field& t = F(dy, f[0]);
         moist_qsat(dy.ctx(), t.nk, t.p, F(dy, f[1]).p, dy.field(f[2], t.nk).p, dy.field(f[3], t.nk).p,
                    dy.field(f[4], t.nk).p);
       }},
      // fillq2zero(q, delp | fill2d): q in place
      {"fillq2zero",
       [](Dycore& dy, const std::vector<std::string>& f, const std::vector<double>&) {
         need(f, 3, "fillq2zero");
         Field& q = F(dy, f[0]);
         fillq2zero(dy.ctx(), q.nk, q.p, F(dy, f[1]).p, dy.field(f[2], 1).p);
       }},
      // gfdl_1m(T, qv, ql, qr, qi, qs, qg, delp, delz | prec_r, prec_s, prec_g, prec_i) params: dt[,
      // variant: 0 the level-block form where instantiated, 1 the column driver]; the GFDL cloud
      // microphysics; the first seven fields are updated in place
      {"gfdl_1m",
       [](Dycore& dy, const std::vector<std::string>& f, const std::vector<double>& p) {
         need(f, 13, "gfdl_1m");
         Field& t = F(dy, f[0]);
         Gfdl1mArgs a{};
         a.nk = t.nk;
         a.dt = p.at(0);
         a.T = t.p;
         a.qv = F(dy, f[1]).p; a.ql = F(dy, f[2]).p; a.qr = F(dy, f[3]).p; a.qi = F(dy, f[4]).p;
         a.qs = F(dy, f[5]).p; a.qg = F(dy, f[6]).p;
         a.dp = F(dy, f[7]).p; a.dz = F(dy, f[8]).p;
         for (int n = 1; n <= 8; ++n)
           if (F(dy, f[n]).nk != t.nk) throw std::runtime_error("gfdl_1m: fields must share the level count");
         a.scr = dy.field("_mp_scr", gfdl_mp_scratch_levels(t.nk)).p;
         a.pr = dy.field(f[9], 1).p; a.ps = dy.field(f[10], 1).p; a.pg = dy.field(f[11], 1).p;
         a.pi = dy.field(f[12], 1).p;
         a.variant = p.size() > 1 ? (int)p[1] : 0;
         gfdl_1m(dy.ctx(), a);
       }},
      // evap_subl_pdf(T, qv, qlls, qils, qlcn, qicn, clls, clcn, pl, nactl, nacti) params: dt;
      // the first eight fields are updated in place
      {"evap_subl_pdf",
       [](Dycore& dy, const std::vector<std::string>& f, const std::vector<double>& p) {
         need(f, 11, "evap_subl_pdf");
         Field& t = F(dy, f[0]);
         for (int n = 1; n <= 10; ++n)
           if (F(dy, f[n]).nk != t.nk) throw std::runtime_error("evap_subl_pdf: fields must share the level count");
         EvapSublArgs a{};
         a.nk = t.nk;
         a.dt = p.at(0);
         a.T = t.p;
         a.qv = F(dy, f[1]).p; a.qlls = F(dy, f[2]).p; a.qils = F(dy, f[3]).p; a.qlcn = F(dy, f[4]).p;
         a.qicn = F(dy, f[5]).p; a.clls = F(dy, f[6]).p; a.clcn = F(dy, f[7]).p;
         a.pl = F(dy, f[8]).p; a.nactl = F(dy, f[9]).p; a.nacti = F(dy, f[10]).p;
         evap_subl_pdf(dy.ctx(), a);
       }},
      // GEOS RADCOUPLE, fields in / out:
      // radcouple(T, pl, cf, af, qv, qlls, qils, qlcn, qicn, qr, qs, qg, nactl | rad_qv, rad_ql, rad_qi, rad_qr, rad_qs, rad_qg, rad_cf, rad_rl, rad_ri)
      {"radcouple",
       [](Dycore& dy, const std::vector<std::string>& f, const std::vector<double>&) {
         need(f, 22, "radcouple");
         Field& t = F(dy, f[0]);
         for (int n = 1; n <= 12; ++n)
           if (F(dy, f[n]).nk != t.nk) throw std::runtime_error("radcouple: fields must share the level count");
         RadcoupleArgs a{};
         a.nk = t.nk;
         a.T = t.p; a.pl = F(dy, f[1]).p; a.cf = F(dy, f[2]).p; a.af = F(dy, f[3]).p; a.qv = F(dy, f[4]).p;
         a.qlls = F(dy, f[5]).p; a.qils = F(dy, f[6]).p; a.qlcn = F(dy, f[7]).p; a.qicn = F(dy, f[8]).p;
         a.qr = F(dy, f[9]).p; a.qs = F(dy, f[10]).p; a.qg = F(dy, f[11]).p; a.nl = F(dy, f[12]).p;
         double** outs[9] = {&a.rqv, &a.rql, &a.rqi, &a.rqr, &a.rqs, &a.rqg, &a.rcf, &a.rrl, &a.rri};
         for (int n = 0; n < 9; ++n) *outs[n] = dy.field(f[13 + n], t.nk).p;
         radcouple(dy.ctx(), a);
       }},
      // aer_activation(pl, T, qv, zm, w | nactl, nacti, smax)
      {"aer_activation",
       [](Dycore& dy, const std::vector<std::string>& f, const std::vector<double>&) {
         need(f, 8, "aer_activation");
         Field& t = F(dy, f[1]);
         for (int n = 0; n <= 4; ++n)
           if (F(dy, f[n]).nk != t.nk) throw std::runtime_error("aer_activation: fields must share the level count");
         aer_activation(dy.ctx(), t.nk, 0, F(dy, f[0]).p, t.p, F(dy, f[2]).p, F(dy, f[3]).p, F(dy, f[4]).p,
                        dy.field(f[5], t.nk).p, dy.field(f[6], t.nk).p, dy.field(f[7], t.nk).p);
       }},
      // cup_gf_sh(T, qv, pl, zm, delp, kpbl, hfx, qlcn, qicn | cf, mb, k22, kbcon, ktop) params: dt; T, qv, qlcn, qicn in place
      {"cup_gf_sh",
       [](Dycore& dy, const std::vector<std::string>& f, const std::vector<double>& p) {
         need(f, 14, "cup_gf_sh");
         Field& t = F(dy, f[0]);
         for (int n : {1, 2, 3, 4, 7, 8})
           if (F(dy, f[n]).nk != t.nk) throw std::runtime_error("cup_gf_sh: fields must share the level count");
         GfShArgs a{};
         a.nk = t.nk;
         a.dt = p.at(0);
         a.T = t.p; a.qv = F(dy, f[1]).p; a.pl = F(dy, f[2]).p; a.zm = F(dy, f[3]).p; a.dp = F(dy, f[4]).p;
         a.kpbl = F(dy, f[5]).p; a.hfx = F(dy, f[6]).p; a.qlcn = F(dy, f[7]).p; a.qicn = F(dy, f[8]).p;
         a.cf = dy.field(f[9], t.nk).p;
         a.mb = dy.field(f[10], 1).p; a.k22 = dy.field(f[11], 1).p; a.kbcon = dy.field(f[12], 1).p;
         a.ktop = dy.field(f[13], 1).p;
         a.scr = dy.field("_gf_scr", gf_scratch_levels(t.nk)).p;
         cup_gf_sh(dy.ctx(), a);
       }},
      // moist_prep(pe, delz | pl, zm, kpbl): layer pressure, layer-mid heights, PBL-top level
      {"moist_prep",
       [](Dycore& dy, const std::vector<std::string>& f, const std::vector<double>&) {
         need(f, 5, "moist_prep");
         Field& dz = F(dy, f[1]);
         if (F(dy, f[0]).nk != dz.nk + 1) throw std::runtime_error("moist_prep: pe must have nk+1 levels");
         moist_prep(dy.ctx(), dz.nk, F(dy, f[0]).p, dz.p, dy.field(f[2], dz.nk).p, dy.field(f[3], dz.nk).p,
                    dy.field(f[4], 1).p);
       }},
      // buoyancy(T, qv, pm, zm | buoy, cape, cin, klcl)
      {"buoyancy",
       [](Dycore& dy, const std::vector<std::string>& f, const std::vector<double>&) {
         need(f, 8, "buoyancy");
         Field& t = F(dy, f[0]);
         buoyancy(dy.ctx(), t.nk, t.p, F(dy, f[1]).p, F(dy, f[2]).p, F(dy, f[3]).p, dy.field(f[4], t.nk).p,
                  dy.field(f[5], 1).p, dy.field(f[6], 1).p, dy.field(f[7], 1).p);
       }},
      // aquaplanet_physics: the moist column step on the dycore state (pt, q tracers 0..5, delp,
      // delz, pe); params: dt
      {"aquaplanet_physics",
       [](Dycore& dy, const std::vector<std::string>&, const std::vector<double>& p) {
         dy.moist_physics(p.at(0));
       }},
      // tracer_stats: global diagnostics of the state's q (FV3 prt_mass / g_sum) into the field
      // "tracer_stats" (first 4 * nq values: per tracer sum(q delp area), min, max, non-finite count)
      {"tracer_stats",
       [](Dycore& dy, const std::vector<std::string>& f, const std::vector<double>&) {
         need(f, 0, "tracer_stats");
         const int npz = dy.nl.npz, nq = dy.nl.nq;
         Field& q = dy.need("q", nq * npz);
         Field& dp = dy.need("delp", npz);
         const long npart = 4L * nq * dy.d.nsub * npz, per = (long)dy.d.nsub * dy.d.plane;
         if (4L * nq > per) throw std::runtime_error("tracer_stats: too many tracers for one plane set");
         double* part = dy.field("_tr_part", (int)((npart + per - 1) / per)).p;
         tracer_stats(dy.ctx(), npz, nq, q.p, dp.p, part, dy.field("tracer_stats", 1).p);
       }},
      // Held-Suarez forcing: held_suarez(pe, pt, u, v) in place, params: dt
      {"held_suarez",
       [](Dycore& dy, const std::vector<std::string>& f, const std::vector<double>& p) {
         need(f, 4, "held_suarez");
         Field& pt = F(dy, f[1]);
         if (F(dy, f[0]).nk != pt.nk + 1) throw std::runtime_error("held_suarez: pe must have npz+1 levels");
         held_suarez(dy.ctx(), pt.nk, p.at(0), F(dy, f[0]).p, pt.p, F(dy, f[2]).p, F(dy, f[3]).p);
       }},
      // tracer_2d_1l: uses state fields q, dp1, cx, cy, mfx, mfy. params: nq[, fused (1: the
      // update inside the march, 0: flux planes and the separate update)[, tracers per march
      // wave (1, 2, 3; 0 default)]]
      {"tracer_2d_1l",
       [](Dycore& dy, const std::vector<std::string>& f, const std::vector<double>& p) {
         (void)f;
         int nq = p.size() > 0 ? (int)p[0] : dy.nl.nq;
         dy.tracer_2d(nq, dy.nl.dt_atmos, p.size() > 1 ? (int)p[1] : -1, p.size() > 2 ? (int)p[2] : 0);
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
