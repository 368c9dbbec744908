// dycore.hpp — process-global dycore context behind geos_gtfv3_{init,run,finalize}
// (reference hook surface: templates/hook.py.jinja2:11-34; lifecycle of
// init once, run once per dycore step, finalize).
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <functional>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "comm.hpp"
#include "grid.hpp"
#include "halo.hpp"
#include "kernels.hpp"
#include "kernels_damp.hpp"

namespace gtfv3 {

struct Field {
  double* p = nullptr;
  int nk = 0;
  long elems() const;
};

class Dycore {
 public:
  Dycore(const Namelist& nl, int rank, int nranks, const void* nccl_id);
  ~Dycore();
  Dycore(const Dycore&) = delete;
  Dycore& operator=(const Dycore&) = delete;

  Namelist nl;
  Decomp dc;
  Dims d{};
  std::unique_ptr<CubedSphere> cs;
  HostMetrics hm;
  std::vector<SubInfo> hsubs;
  SubInfo* dsubs = nullptr;
  double* dmet = nullptr;
  double* dcornerw = nullptr;
  double* darea4 = nullptr;
  HaloExchanger halo;
  hipStream_t st = nullptr;
  // side streams of the acoustic sub-step: d_sw's wind stage and update_dz_d run beside
  // its thermodynamic transport (fork after the Courant numbers, join before riem_solver3)
  hipStream_t st_b = nullptr, st_c = nullptr;
  hipEvent_t ev_fork = nullptr, ev_b = nullptr, ev_c = nullptr;
  // the thermo march's tile-edge kernel beside its interior kernel (Ctx::side; GTFV3_EDGE_SIDE=0:
  // in series on the main stream)
  hipStream_t st_d = nullptr;
  hipEvent_t ev_df = nullptr, ev_dj = nullptr;
  // early d_sw winds (GTFV3_EARLY_WINDS: 0 off, 1 (default) the kinetic energy on stream b as
  // soon as ut / vt exist, beside ds_courant; the cell vorticity is formed by c_sw's cs_tmp):
  // ut / vt written
  hipEvent_t ev_ut = nullptr;
  int early_winds = 1;
  bool fork_substep = true;  // GTFV3_STREAMS=0: one stream
  std::unique_ptr<Transport> comm;  // null for one rank
  std::map<std::string, Field> fields;
  std::vector<double> ak, bk;  // npz+1
  int ks = 0;
  std::map<std::string, double> timers;  // accumulated ms per phase (events)
  // device time of every completed step (first to last kernel of fv_dynamics on the library
  // stream), oldest first; the bench's median step time (report.py:152-153)
  std::vector<double> step_ms;
  // phase events of the last two steps (the step does not wait for its own end: a step's
  // events are read two steps later, or when the timers are queried)
  hipEvent_t ev_ph[2][5] = {};
  bool ev_pending[2] = {false, false};
  int ev_slot = 0;
  bool vert_dirty = true;
  void flush_timers(int slot);  // accumulate a completed step's phase times
  void flush_all_timers();
  // tracer_2d: the reduced per-level Courant maxima come back to the host through pinned
  // memory after an event, while the first tracer sub-step already runs
  double* h_cmax = nullptr;
  hipEvent_t ev_cmax = nullptr;
  // when set, the step's tracer transport waits for this event (the bridge uploads tracers
  // 1.. beside the acoustic sub-steps)
  hipEvent_t tracer_wait = nullptr;
  // when set, the exit phase (fv_wrapup's omega) waits for this event (the bridge uploads
  // omga's halo beside the step)
  hipEvent_t exit_wait = nullptr;
  // when set, the step records mark[m] as the fields of StepMark m are final (the bridge
  // starts copying each group back while the rest of the step runs)
  enum StepMark {
    SM_CWINDS,      // uc, vc (after the last acoustic sub-step's C-grid exchange)
    SM_ACOUSTIC,    // diss_est, phis (after the acoustic sub-steps and the heating)
    SM_FLUXES,      // mfx, mfy, cx, cy (after tracer_2d's split scaling, on its stream)
    SM_REMAP,       // w, delz, delp, q, pe, peln, pk, pkz, ps (after the vertical remap)
    SM_WRAPUP,      // pt, omga
    SM_WINDS,       // u, v (after their final halo update)
    SM_COUNT
  };
  hipEvent_t* marks = nullptr;
  // called on the host right after mark m is recorded (the bridge queues that group's copies
  // back then, not after step() returns: the step's host thread waits mid-way, in tracer_2d)
  std::function<void(int)> on_mark;
  void record_mark(int m, hipStream_t s);
  // the acoustic sub-steps as one HIP graph (GTFV3_GRAPH, Dycore::step): captured on the
  // second step (the first allocates every field and table), replayed while the key (field
  // generation, state planes, step constants) is unchanged
  hipGraphExec_t ac_exec = nullptr;
  std::vector<double> ac_key;
  long field_gen = 0;  // bumped when a field is created or freed
  long nsteps = 0;

  Field& field(const std::string& name, int nk);  // get or create (zeroed)
  Field* find(const std::string& name);
  Field& need(const std::string& name, int nk);  // existing field, level count checked
  const double* vertical_dev();                  // ak | bk | dp_ref on device
  // a column of d_sw parameters on the device (uploaded when it differs from the last one;
  // the pointer stays valid until the next upload of a longer column)
  // (slot 0: d_sw's column, npz levels; slot 1: update_dz_d's, npz+1 interface levels)
  const LevelDamp* level_table(const std::vector<LevelDamp>& t, int slot = 0);
  std::vector<LevelDamp> hlevel, hlevel_zh;
  LevelDamp* dlevel = nullptr;
  LevelDamp* dlevel_zh = nullptr;
  size_t dlevel_cap = 0, dlevel_zh_cap = 0;
  Ctx ctx() const;
  long field_elems(int nk) const { return (long)d.nsub * nk * d.plane; }
  double* guard_hi(double* p, int nk) const;  // GTFV3_SYNC_LAUNCH=1: a field's high guard zone

  // host <-> device copies of a whole named field in the padded device layout
  void upload(const std::string& name, const double* host, int nk);
  void download(const std::string& name, double* host);
  // host (nsub, nk, plane) into levels [k0, k0+nk) of an existing field (large tracer sets
  // are uploaded tracer by tracer)
  void upload_levels(const std::string& name, const double* host, int k0, int nk);
  // levels [k0, k0+nk) of every sub-domain into host (nsub, nk, plane)
  void download_levels(const std::string& name, double* host, int k0, int nk);

  // halo update of named fields; kinds: 'c' cell, 'b' corner, 'd' D-grid pair, 'C' C-grid pair, 'a' A-grid pair,
  // 'S' C-grid pair tile-edge synchronisation (east / north edge values from the neighbour)
  void halo_update(const std::vector<std::pair<std::string, char>>& items);
  // the two halves of an exchange (HaloExchanger::exchange_begin / exchange_end), on st
  void halo_begin(const std::vector<std::pair<std::string, char>>& items);
  void halo_end();
  std::vector<HaloField> halo_fields(const std::vector<std::pair<std::string, char>>& items);
  // max-reduce across ranks (in place, device, n doubles)
  void allreduce_max(double* dev, int n);

  // algorithm blocks
  // fused: 1 update inside the march, 0 flux planes + separate update, -1 GTFV3_TRACER_FUSED
  // nf: tracers per march wave (1, 2, 3; 0: GTFV3_TRACER_NF, else 2 for even nq, 1 for odd)
  void tracer_2d(int nq, double dt, int fused = -1, int nf = 0);
  void set_vertical(const double* ak_, const double* bk_, int ks_);
  void step();  // one fv_dynamics call on device-resident state
  // Aquaplanet moist column step on the state (tracers 0..5 = qv ql qr qi qs qg, nq >= 6)
  void moist_physics(double dt);
};

}  // namespace gtfv3
