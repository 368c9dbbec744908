// gtfv3.hpp — core types of the MI355X-native FV3 dycore path behind the
// geos_gtfv3 bridge (reference boundary: src/tcn/py_ftn_interface/
// example_def_dycore.yaml:1-71, rendered by templates/interface.c.jinja2:8-29).
//
// Memory layout (HBM): every 3-D field of one rank is ONE allocation
//   field[s][k][j][i]   s = local sub-domain, k = level (0 = model top),
//                       j = row (-NG .. ny+NG), i = column (-NG .. nx+NG, pitch-padded)
// i is fastest, exactly GEOS/Fortran (i,j,k) order, so the bridge needs no
// transpose.  All staggerings (cell, x-edge, y-edge, corner) share one padded
// (nx+2NG+1) x (ny+2NG+1) plane so one index formula serves every kernel.
// 2-D metric terms use the same plane layout, one plane per sub-domain.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace gtfv3 {

constexpr int NG = 3;  // FV3 halo width (n_halo)

// GEOS constants (PACE_CONSTANTS=GEOS, ci/pipeline/gtfv3_config.py:20); MAPL values.
struct Constants {
  static constexpr double pi = 3.14159265358979323846;
  static constexpr double radius = 6371.0e3;
  static constexpr double grav = 9.80665;
  static constexpr double runiv = 8314.47;
  static constexpr double rdgas = 8314.47 / 28.965;
  static constexpr double rvgas = 8314.47 / 18.015;
  static constexpr double cp_air = 3.5 * (8314.47 / 28.965);
  static constexpr double kappa = 1.0 / 3.5;  // rdgas / cp_air
  static constexpr double omega = 2.0 * 3.14159265358979323846 / 86164.0;
  static constexpr double zvir = (8314.47 / 18.015) / (8314.47 / 28.965) - 1.0;
};

// The fixed synthetic namelist of SURVEY.md §8(d) (the reference input.nml is external).
struct Namelist {
  int npx = 49, npy = 49, npz = 72;  // FV3 convention: npx = N+1
  int ntiles = 6;
  int nq = 4;                        // tracers (q(...,1) = specific humidity)
  int layout_x = 1, layout_y = 1;    // sub-domains per tile edge
  double dt_atmos = 900.0;           // bdt
  int k_split = 1, n_split = 6;
  int hord_mt = 6, hord_vt = 6, hord_tm = 6, hord_dp = 6, hord_tr = 6;
  int kord_mt = 9, kord_wz = 9, kord_tr = 9, kord_tm = -9;
  double dddmp = 0.2, d2_bg = 0.0;   // nord = 0 divergence damping (Smagorinsky + background)
  // d_sw damping beyond the Held-Suarez namelist (damp.hip): del-(2 nord + 2) divergence
  // damping with d4_bg; del-(2 nord_v + 2) vorticity damping vtdm4; d_con: the damped kinetic
  // energy into heat (limited to delt_max * bdt K per call) and diss_est
  // (GTFV3_CONFIG follows fv_core_nml: nord_v defaults to min(2, nord) and vtdm4 acts only
  // with do_vort_damp, capi.cpp parse_config)
  int nord = 0, nord_v = 0;
  double d4_bg = 0.0, vtdm4 = 0.0, d_con = 0.0, delt_max = 1.0;
  bool do_vort_damp = false;
  // sponge layers (FV3 dyn_core's k loop, damp.hip column_damping): with n_sponge >= 0 the top
  // level takes del-2 divergence damping d2_bg_k1 (and del-2 w damping, d_con 0), the next
  // two d2_bg_k2 / 0.2 d2_bg_k2 when d2_bg_k2 > 0.01 / 0.05.  FV3's own defaults (4, 2) are
  // placeholders its documentation says to set; these are the values of the GEOS / pyFV3
  // test namelists.  ke_bg: background heating of the w damping; convert_ke: heat on every level.
  int n_sponge = 1;
  double d2_bg_k1 = 0.20, d2_bg_k2 = 0.10, ke_bg = 0.0;
  bool convert_ke = false;
  double p_fac = 0.05;               // SIM1 solver pressure floor factor
  double dz_min = 2.0;
  bool fill = true;                  // fillz negative tracers after remap
  bool adiabatic = false;
  double ptop = 1.0;
  bool host_only = false;            // grid + tables only (CPU tests)
  int loopback = 0;                  // >0: in-process multi-rank group id (single-GPU tests)
  // one rank only: every same-rank halo point goes through the message path -- pack, RCCL
  // ncclSend / ncclRecv to itself on a size-1 communicator, unpack -- and the tracer Courant
  // maximum through ncclAllReduce, so the NcclTransport runs on a one-GPU box
  bool rccl_self = false;
  // several ranks per GPU (the reference's PER_DEVICE_PROCESS): the same-node IPC transport
  // (ipc.cpp) instead of RCCL, which takes one rank per device
  bool ipc = false;
};

// One sub-domain (tile piece) owned by this rank.
struct SubInfo {
  int tile;      // 0..5
  int ioff, joff;// tile-global index of local (0,0) cell
  int N;         // cells per tile edge (npx-1)
  int flags;     // bit0 W tile edge, bit1 E, bit2 S, bit3 N (this sub touches that tile edge)
  int gid;       // global sub-domain id
  int pad0, pad1;
};
enum : int { EDGE_W = 1, EDGE_E = 2, EDGE_S = 4, EDGE_N = 8 };

struct Dims {
  int nx, ny;     // compute cells of each sub-domain
  int pitch;      // doubles per row (>= nx+2NG+1, padded to 8)
  int nj;         // rows per plane (ny+2NG+1)
  long plane;     // pitch*nj
  int nsub;       // sub-domains on this rank
  int npz;
};

// staggerings
enum Stagger : int { CELL = 0, XEDGE = 1, YEDGE = 2, CORNER = 3 };
// halo kinds (scalar staggerings + vector pairs)
enum HaloKind : int {
  H_CELL = 0, H_CORNER = 1, H_DGRID = 2, H_CGRID = 3, H_AGRID = 4,
  // C-grid tile-edge synchronisation: uc on east and vc on north tile edges take the
  // neighbouring tile's values at the same points (FV3 mpp_get_boundary; see halo.hip)
  H_CSYNC = 5,
  // H_CSYNC then H_CGRID as ONE exchange: a C halo point whose source is a synchronised
  // tile-edge point reads that point's own source instead (signs and components composed),
  // so every value the exchange reads is one it does not write -- bit-identical to the two
  // updates in sequence, with one message round per sub-step fewer
  H_CSC = 6, H_NKIND = 7
};

// host-side sub-domain decomposition of the cubed sphere
struct Decomp {
  int N = 0, lx = 1, ly = 1, nranks = 1, rank = 0;
  int nsub_total() const { return 6 * lx * ly; }
  int nsub_per_rank() const { return nsub_total() / nranks; }
  int sub_nx() const { return N / lx; }
  int sub_ny() const { return N / ly; }
  SubInfo sub(int gid) const;
  int owner_rank(int gid) const { return gid / nsub_per_rank(); }
};

std::string last_error();
void set_error(const std::string& msg);

}  // namespace gtfv3
