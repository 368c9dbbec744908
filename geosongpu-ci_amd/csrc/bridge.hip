// bridge.hip — process-global geos_gtfv3 context and Fortran <-> HBM conversion.
#include "bridge.hpp"

#include <dlfcn.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "dycore.hpp"
#include "hip_util.hpp"

namespace gtfv3 {

namespace {

std::unique_ptr<Dycore> g_dy;
int g_tiles_per_rank = 1;
int g_is = 0, g_js = 0;

int env_int(const char* const* names, int dflt) {
  for (const char* const* n = names; *n; ++n) {
    const char* v = std::getenv(*n);
    if (v && *v) return std::atoi(v);
  }
  return dflt;
}

// Fortran array section (tile-global Fortran bounds -> local 0-based)
struct FDesc {
  int ilo, ni, jlo, nj, nk;  // ilo/jlo: local index of the first element
  int order;                 // 0: (i,j,k)  1: (i,k,j)
};

// Host <-> HBM movement of one run call.  The Fortran arrays are page-locked and mapped once
// (hipHostRegister: GEOS keeps them for the whole run).  Two transfer forms, both through one
// kernel (fort_move) that converts layout and precision:
//  * zero-copy: the kernel reads / writes the mapped Fortran array itself over PCIe -- one
//    launch per array (or section), no staging buffer, no DMA;
//  * staged: the array (in pieces of at most the staging buffer) by DMA into an HBM staging
//    buffer and scattered from there, or gathered there and sent by DMA, in one stream's order.
// GTFV3_BRIDGE_ZC (bit mask) picks zero-copy for: 1 the uploads before the step, 2 the uploads
// beside it, 4 the copies back.  Default 1: a zero-copy transfer beside the step slows it (its
// PCIe traffic goes through the CUs' memory path: gathers held the remap's kernels up ~10x,
// 32-workgroup uploads the first acoustic sub-step by ~25 %), the DMA engine's does not; before
// the step nothing else runs and the kernel form saves the DMA queue's per-copy latency.
// Arrays that could not be mapped (or GTFV3_BRIDGE_PIN=0) always go staged.
// Ordering (bridge_run): the arrays the step reads first go up before it; tracers 1.. and
// omga's halo go up on the side stream beside the acoustic sub-steps (the step waits for them
// before tracer_2d / fv_wrapup); each output group comes back on the side stream as soon as
// the step marks it final (Dycore::StepMark), while the rest of the step runs.  The runtime
// maps streams onto a few hardware queues (GPU_MAX_HW_QUEUES, 4 by default) in creation order,
// and two streams sharing a queue run in enqueue order: the step's three streams plus the side
// stream fit, so side traffic queued ahead of the step never holds up a step kernel.
enum { ZC_CRIT = 1, ZC_SIDE = 2, ZC_DOWN = 4 };
int zc_mode() {
  const char* e = std::getenv("GTFV3_BRIDGE_ZC");
  return e && *e ? std::atoi(e) : ZC_CRIT;
}
// staging buffer bytes (GTFV3_BRIDGE_STAGE_KB; tests use a small one to cut arrays into many
// pieces): one C180 L72 array of four tracers fits the default
size_t stage_bytes() {
  const char* e = std::getenv("GTFV3_BRIDGE_STAGE_KB");
  const long kb = e ? std::atol(e) : 0;
  return kb > 0 ? (size_t)kb << 10 : size_t(512) << 20;
}
// workgroups of a zero-copy launch beside the acoustic sub-steps (GTFV3_BRIDGE_ZC_BLOCKS):
// enough lanes in flight to cover the PCIe round trip, few enough to leave the CUs to the step
int zc_blocks(const char* env, int dflt) {
  const char* e = std::getenv(env);
  const int b = e ? std::atoi(e) : 0;
  return b > 0 ? b : dflt;
}

struct BridgeIO {
  hipStream_t side = nullptr;
  void* stage = nullptr;  // staged form (reuse is ordered by the stream)
  size_t stage_cap = 0;
  hipEvent_t ev_t[4] = {};  // call start, state scattered, step done, last copy back
  hipEvent_t ev_tracers = nullptr, ev_exit = nullptr, ev_crit = nullptr;
  hipEvent_t marks[Dycore::SM_COUNT] = {};
  struct Pinned {
    size_t bytes;
    void* dev;  // mapped device address (null: page-locked only)
  };
  std::map<const void*, Pinned> pinned;  // registered Fortran arrays
  double ms[3] = {0, 0, 0};    // last call: upload before the step, step, copy-back tail
  double bytes[2] = {0, 0};    // last call: host bytes uploaded / downloaded

  void init() {
    if (side) return;
    HIP_CHECK(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
    for (auto& e : ev_t) HIP_CHECK(hipEventCreate(&e));
    for (hipEvent_t* e : {&ev_tracers, &ev_exit, &ev_crit}) HIP_CHECK(hipEventCreateWithFlags(e, hipEventDisableTiming));
    for (auto& e : marks) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  void* staging() {
    const size_t want = stage_bytes();
    if (stage && stage_cap != want) {
      // nothing queued may still use the old buffer
      HIP_CHECK(hipDeviceSynchronize());
      HIP_CHECK(hipFree(stage));
      stage = nullptr;
    }
    if (!stage) {
      HIP_CHECK(hipMalloc(&stage, want));
      stage_cap = want;
    }
    return stage;
  }
  void release() {
    if (!side) return;
    (void)hipStreamSynchronize(side);
    unpin_except({});
    if (stage) (void)hipFree(stage);
    stage = nullptr;
    for (auto& e : ev_t) (void)hipEventDestroy(e);
    for (hipEvent_t e : {ev_tracers, ev_exit, ev_crit}) (void)hipEventDestroy(e);
    for (auto& e : marks) (void)hipEventDestroy(e);
    (void)hipStreamDestroy(side);
    side = nullptr;
  }
  // page-lock this call's arrays; arrays of earlier calls that are not among them are
  // released first (a caller that reallocates between calls keeps only one set pinned)
  void unpin_except(const std::vector<std::pair<const void*, size_t>>& keep) {
    for (auto it = pinned.begin(); it != pinned.end();) {
      bool k = false;
      for (auto& p : keep) k = k || (p.first == it->first && p.second == it->second.bytes);
      if (!k) {
        (void)hipHostUnregister(const_cast<void*>(it->first));
        it = pinned.erase(it);
      } else {
        ++it;
      }
    }
  }
  void pin(const std::vector<std::pair<const void*, size_t>>& arrays) {
    const char* e = std::getenv("GTFV3_BRIDGE_PIN");
    if (e && e[0] == '0') {
      unpin_except({});
      return;
    }
    unpin_except(arrays);
    for (auto& p : arrays) {
      if (pinned.count(p.first)) continue;
      // a range another array already pinned (or memory HIP allocated) stays pageable here
      void* h = const_cast<void*>(p.first);
      if (hipHostRegister(h, p.second, hipHostRegisterMapped) != hipSuccess) {
        (void)hipGetLastError();
        continue;
      }
      void* dev = nullptr;
      if (hipHostGetDevicePointer(&dev, h, 0) != hipSuccess) {
        (void)hipGetLastError();
        dev = nullptr;
      }
      pinned[p.first] = Pinned{p.second, dev};
    }
  }
  // the mapped device address of a registered array when this kind of transfer (ZC_*) goes
  // zero-copy, else null
  void* mapped(const void* host, int kind) const {
    if (!(zc_mode() & kind)) return nullptr;
    auto it = pinned.find(host);
    return it == pinned.end() ? nullptr : it->second.dev;
  }
};

BridgeIO g_io;

// the device plane offset of element t (flat Fortran index within one tile's section)
__device__ __forceinline__ long fort_dev_index(const Dims& d, int s, int nk_dev, const FDesc& fd, long t) {
  const int i = (int)(t % fd.ni);
  int j, k;
  if (fd.order == 0) {
    j = (int)((t / fd.ni) % fd.nj);
    k = (int)(t / ((long)fd.ni * fd.nj));
  } else {
    k = (int)((t / fd.ni) % fd.nk);
    j = (int)(t / ((long)fd.ni * fd.nk));
  }
  return ((long)s * nk_dev + k) * d.plane + pidx(d, fd.ilo + i, fd.jlo + j);
}

// Elements [t_lo, t_lo + span) of tiles s0, s0 + 1, ... of one Fortran array (`total` = tiles
// x span) between the device field and `f`, where element t of tile s sits at
// f[(s - s_base) * stride + t - t_base]: the mapped Fortran array itself (zero-copy: s_base =
// t_base = 0, stride = the tile's element count) or a staging piece.  Consecutive lanes take
// consecutive Fortran elements (full PCIe packets); ZC_U elements per lane are in flight per
// iteration of the grid-stride loop (a PCIe round trip is microseconds long).
constexpr int ZC_U = 4;
template <typename T, bool UP>
__global__ void __launch_bounds__(256) fort_move(T* __restrict__ f, double* __restrict__ dev, Dims d, int s0,
                                                 int nk_dev, FDesc fd, int s_base, long stride, long t_base,
                                                 long t_lo, long span, long total) {
  const long step = (long)gridDim.x * blockDim.x;
  for (long e0 = (long)blockIdx.x * blockDim.x + threadIdx.x; e0 < total; e0 += step * ZC_U) {
    long hi[ZC_U], di[ZC_U];
#pragma unroll
    for (int u = 0; u < ZC_U; ++u) {
      const long e = e0 + u * step;
      const long ee = e < total ? e : 0;
      const int s = s0 + (int)(ee / span);
      const long t = t_lo + ee % span;
      hi[u] = (long)(s - s_base) * stride + t - t_base;
      di[u] = fort_dev_index(d, s, nk_dev, fd, t);
    }
    if constexpr (UP) {
      T v[ZC_U];
#pragma unroll
      for (int u = 0; u < ZC_U; ++u) v[u] = e0 + u * step < total ? f[hi[u]] : T(0);
#pragma unroll
      for (int u = 0; u < ZC_U; ++u)
        if (e0 + u * step < total) dev[di[u]] = (double)v[u];
    } else {
      double v[ZC_U];
#pragma unroll
      for (int u = 0; u < ZC_U; ++u) v[u] = e0 + u * step < total ? dev[di[u]] : 0.0;
#pragma unroll
      for (int u = 0; u < ZC_U; ++u)
        if (e0 + u * step < total) f[hi[u]] = (T)v[u];
    }
  }
}

template <typename T, bool UP>
void launch_move(T* f, double* dev, const Dims& d, int s_lo, int s_hi, int nk_dev, const FDesc& fd, int s_base,
                 long stride, long t_base, long t_lo, long t_hi, hipStream_t st, int max_blocks) {
  const long span = t_hi - t_lo, total = span * (s_hi - s_lo);
  if (total <= 0) return;
  const int blocks = (int)std::min<long>(max_blocks, cdiv(total, 256L * ZC_U));
  GT_LAUNCH((fort_move<T, UP>), dim3(blocks), dim3(256), 0, st, f, dev, d, s_lo, nk_dev, fd, s_base, stride, t_base,
            t_lo, span, total);
  HIP_LAUNCH_CHECK();
}

// the staged pieces of tiles [s_lo, s_hi) x elements [t_lo, t_hi): whole tiles together while
// they fit the staging buffer and the range is the whole tile (one contiguous host block),
// else one tile at a time, cut to the buffer
template <typename F>
void staged_pieces(int s_lo, int s_hi, long n, long t_lo, long t_hi, long cap, F&& fn) {
  if (t_lo == 0 && t_hi == n && n <= cap) {
    const int per = (int)std::max<long>(1, cap / n);
    for (int s = s_lo; s < s_hi; s += per) fn(s, std::min(s + per, s_hi), t_lo, t_hi);
    return;
  }
  for (int s = s_lo; s < s_hi; ++s)
    for (long t = t_lo; t < t_hi; t += cap) fn(s, s + 1, t, std::min(t + cap, t_hi));
}

// Fortran array (all local sub-domains, tile-major) -> device field: elements [t_lo, t_hi) of
// each tile in [s_lo, s_hi), on stream `st`; `kind` the transfer's ZC_* class
template <typename T>
double copy_in(Dycore& dy, const char* name, int nk_dev, const T* host, const FDesc& fd, hipStream_t st, int kind,
               int zc_grid, int s_lo = 0, int s_hi = -1, long t_lo = 0, long t_hi = -1) {
  Field& f = dy.field(name, nk_dev);
  const long n = (long)fd.ni * fd.nj * fd.nk;
  if (s_hi < 0) s_hi = g_tiles_per_rank;
  if (t_hi < 0) t_hi = n;
  const double bytes = sizeof(T) * (double)(t_hi - t_lo) * (s_hi - s_lo);
  if (void* m = g_io.mapped(host, kind)) {
    launch_move<T, true>((T*)m, f.p, dy.d, s_lo, s_hi, nk_dev, fd, 0, n, 0, t_lo, t_hi, st, zc_grid);
    return bytes;
  }
  T* buf = (T*)g_io.staging();
  const long cap = (long)(g_io.stage_cap / sizeof(T));
  staged_pieces(s_lo, s_hi, n, t_lo, t_hi, cap, [&](int a, int b, long ta, long tb) {
    const long m = (tb - ta) * (b - a);  // contiguous on the host (whole tiles, or one tile's range)
    HIP_CHECK(hipMemcpyAsync(buf, host + (size_t)a * n + ta, sizeof(T) * m, hipMemcpyHostToDevice, st));
    launch_move<T, true>(buf, f.p, dy.d, a, b, nk_dev, fd, a, tb - ta, ta, ta, tb, st, 1024);
  });
  return bytes;
}

// device field -> Fortran array, on stream `st` (which the caller has made wait for the
// field's last writer)
template <typename T>
double copy_out(Dycore& dy, const char* name, T* host, const FDesc& fd, hipStream_t st, int zc_grid) {
  Field* f = dy.find(name);
  if (!f) throw std::runtime_error(std::string("bridge: missing field ") + name);
  const long n = (long)fd.ni * fd.nj * fd.nk;
  const double bytes = sizeof(T) * (double)n * g_tiles_per_rank;
  if (void* m = g_io.mapped(host, ZC_DOWN)) {
    launch_move<T, false>((T*)m, f->p, dy.d, 0, g_tiles_per_rank, f->nk, fd, 0, n, 0, 0, n, st, zc_grid);
    return bytes;
  }
  T* buf = (T*)g_io.staging();
  const long cap = (long)(g_io.stage_cap / sizeof(T));
  staged_pieces(0, g_tiles_per_rank, n, 0, n, cap, [&](int a, int b, long ta, long tb) {
    const long m = (tb - ta) * (b - a);
    launch_move<T, false>(buf, f->p, dy.d, a, b, f->nk, fd, a, tb - ta, ta, ta, tb, st, 1024);
    HIP_CHECK(hipMemcpyAsync(host + (size_t)a * n + ta, buf, sizeof(T) * m, hipMemcpyDeviceToHost, st));
  });
  return bytes;
}

}  // namespace

Dycore* bridge_dycore() { return g_dy.get(); }

void bridge_fatal(const std::string& msg) {
  set_error(msg);
  std::fprintf(stderr, "[geos_gtfv3] fatal: %s\n", msg.c_str());
  const char* nf = std::getenv("GTFV3_NONFATAL");
  if (!(nf && std::atoi(nf) == 1)) std::abort();
}

// ---- ncclUniqueId bootstrap ----
// Under GEOS the caller hands its Fortran communicator handle by value in `comm`
// (argument.py:57-58,83-84; the reference's C shim does MPI_Comm_f2c on it, base.py:89-96)
// and the executable itself links MPI.  The bridge does not link MPI: it resolves
// MPI_Comm_f2c / MPI_Comm_rank / MPI_Comm_size / MPI_Bcast from the process at run time
// (dlsym(RTLD_DEFAULT)), so one library serves MPICH-ABI MPIs (MPICH, Cray, Intel: MPI_Comm
// an int, MPI_BYTE = 0x4c00010d) and Open MPI (handles are pointers, MPI_BYTE is
// &ompi_mpi_byte).  Without MPI in the process (standalone runs) the rank comes from the
// launcher's environment and the id travels through GTFV3_NCCL_ID_FILE, stamped with a
// job token so that a file left by an earlier job is never taken for this job's id.
namespace {
struct MpiSyms {
  intptr_t (*f2c)(intptr_t) = nullptr;
  int (*rank)(intptr_t, int*) = nullptr;
  int (*size)(intptr_t, int*) = nullptr;
  int (*bcast)(void*, int, intptr_t, int, intptr_t) = nullptr;
  int (*initialized)(int*) = nullptr;
  intptr_t byte = 0;
  // MPI present in the process and initialised (any handle value, Open MPI's world is 0)
  bool ok() const {
    int flag = 0;
    return f2c && rank && size && bcast && initialized && initialized(&flag) == 0 && flag;
  }
};

MpiSyms mpi_syms() {
  MpiSyms m;
  m.f2c = (intptr_t(*)(intptr_t))dlsym(RTLD_DEFAULT, "MPI_Comm_f2c");
  m.rank = (int (*)(intptr_t, int*))dlsym(RTLD_DEFAULT, "MPI_Comm_rank");
  m.size = (int (*)(intptr_t, int*))dlsym(RTLD_DEFAULT, "MPI_Comm_size");
  m.bcast = (int (*)(void*, int, intptr_t, int, intptr_t))dlsym(RTLD_DEFAULT, "MPI_Bcast");
  m.initialized = (int (*)(int*))dlsym(RTLD_DEFAULT, "MPI_Initialized");
  void* ompi_byte = dlsym(RTLD_DEFAULT, "ompi_mpi_byte");
  m.byte = ompi_byte ? (intptr_t)ompi_byte : (intptr_t)0x4c00010d;
  return m;
}

// the Fortran handle is an integer passed by value through a void* parameter
intptr_t fortran_handle(void* comm) { return (intptr_t)(int)(intptr_t)comm; }

std::string job_token() {
  const char* names[] = {"GTFV3_JOB_TOKEN", "SLURM_JOB_ID", "PBS_JOBID", "TORCHELASTIC_RUN_ID", "MASTER_PORT",
                         nullptr};
  std::string t;
  for (const char* const* n = names; *n; ++n) {
    const char* v = std::getenv(*n);
    if (v && *v) { t = std::string(*n) + "=" + v; break; }
  }
  const char* step = std::getenv("SLURM_STEP_ID");
  if (step) t += std::string(".") + step;
  return t;
}

std::string g_id_file;  // written by rank 0, removed at finalize
}  // namespace

void job_rank_size(void* comm, int* rank, int* nranks) {
  MpiSyms m = mpi_syms();
  if (m.ok()) {
    intptr_t c = m.f2c(fortran_handle(comm));
    if (m.rank(c, rank) != 0 || m.size(c, nranks) != 0) throw std::runtime_error("MPI_Comm_rank/size failed");
    return;
  }
  const char* rk[] = {"GTFV3_RANK", "OMPI_COMM_WORLD_RANK", "PMI_RANK", "SLURM_PROCID", "RANK", nullptr};
  const char* sz[] = {"GTFV3_WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", "PMI_SIZE", "SLURM_NTASKS", "WORLD_SIZE", nullptr};
  *rank = env_int(rk, 0);
  *nranks = env_int(sz, 1);
}

void share_unique_id(void* comm, int rank, int nranks, unsigned char* id) {
  if (nranks <= 1) return;
  MpiSyms m = mpi_syms();
  if (m.ok()) {
    intptr_t c = m.f2c(fortran_handle(comm));
    if (m.bcast(id, 128, m.byte, 0, c) != 0) throw std::runtime_error("MPI_Bcast of the ncclUniqueId failed");
    return;
  }
  const char* fn = std::getenv("GTFV3_NCCL_ID_FILE");
  if (!fn) throw std::runtime_error("multi-rank bridge without MPI needs GTFV3_NCCL_ID_FILE");
  const std::string token = job_token();
  if (token.empty())
    throw std::runtime_error("GTFV3_NCCL_ID_FILE needs a job token (GTFV3_JOB_TOKEN, SLURM_JOB_ID, ...)");
  // record: "GTFV3ID1" | token length (4 B) | token | 128-byte id
  if (rank == 0) {
    std::string rec = "GTFV3ID1";
    uint32_t n = (uint32_t)token.size();
    rec.append((const char*)&n, 4);
    rec += token;
    rec.append((const char*)id, 128);
    std::string tmp = std::string(fn) + ".tmp." + std::to_string((long)getpid());
    {
      std::ofstream out(tmp, std::ios::binary | std::ios::trunc);
      out.write(rec.data(), (std::streamsize)rec.size());
      if (!out) throw std::runtime_error("cannot write the ncclUniqueId file");
    }
    if (std::rename(tmp.c_str(), fn) != 0) throw std::runtime_error("cannot publish the ncclUniqueId file");
    g_id_file = fn;
    return;
  }
  for (int t = 0;; ++t) {
    std::ifstream in(fn, std::ios::binary);
    std::string rec((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
    if (rec.size() >= 12 && rec.compare(0, 8, "GTFV3ID1") == 0) {
      uint32_t n;
      std::memcpy(&n, rec.data() + 8, 4);
      if (rec.size() == 12 + n + 128 && rec.compare(12, n, token) == 0) {
        std::memcpy(id, rec.data() + 12 + n, 128);
        return;
      }
    }
    if (t >= 6000) throw std::runtime_error("timed out waiting for this job's ncclUniqueId file");
    std::this_thread::sleep_for(std::chrono::milliseconds(10));
  }
}

void bridge_init(void* comm, int npx, int npy, int npz, int ntiles, int is, int ie, int js, int je, int isd, int ied,
                 int jsd, int jed, float bdt, int nq_tot) {
  (void)comm;
  if (ntiles != 6) throw std::runtime_error("geos_gtfv3_init: ntiles must be 6");
  if (npx != npy) throw std::runtime_error("geos_gtfv3_init: npx != npy");
  if (isd != is - NG || ied != ie + NG || jsd != js - NG || jed != je + NG)
    throw std::runtime_error("geos_gtfv3_init: data domain must be the compute domain +/- 3 halo points");
  const char* tp[] = {"GTFV3_BRIDGE_TILES_PER_RANK", nullptr};
  int rank = 0, nranks = 1;
  job_rank_size(comm, &rank, &nranks);
  g_tiles_per_rank = env_int(tp, 1);
  int N = npx - 1, nx = ie - is + 1, ny = je - js + 1;
  Namelist nl;
  nl.npx = nl.npy = npx;
  nl.npz = npz;
  nl.nq = nq_tot;
  nl.layout_x = N / nx;
  nl.layout_y = N / ny;
  nl.dt_atmos = bdt;
  // fv_core_nml options (n_split, hord_*, kord_*, dddmp, nord, d4_bg, vtdm4, d_con, ...): the
  // reference's Python side reads them from input.nml; here GTFV3_CONFIG carries them
  if (const char* cfg = std::getenv("GTFV3_CONFIG")) {
    const Namelist given = parse_config(cfg, nl);
    if (given.npx != nl.npx || given.npz != nl.npz || given.nq != nl.nq || given.layout_x != nl.layout_x ||
        given.layout_y != nl.layout_y)
      throw std::runtime_error("GTFV3_CONFIG may not change the grid the init arguments define");
    nl = given;
  }
  if (g_tiles_per_rank == 6) {
    if (nranks != 1 || nx != N || ny != N) throw std::runtime_error("6 tiles per rank needs 1 rank and layout 1x1");
  } else if (g_tiles_per_rank != 1) {
    throw std::runtime_error("GTFV3_BRIDGE_TILES_PER_RANK must be 1 or 6");
  } else if (nranks != 6 * nl.layout_x * nl.layout_y) {
    throw std::runtime_error("geos_gtfv3_init: one sub-domain per rank expected (6*layout ranks)");
  }
  // GTFV3_BRIDGE_PROXY=1 (measurement and test aid, never a numerical path): this rank alone
  // on the null transport -- each cross-rank receive is answered with a copy of this rank's
  // own send to that peer (comm.cpp), so the pack / copy / unpack work of a real exchange runs
  // but the remote halo points hold the wrong rows -- so the one-sub-domain-per-rank array
  // layout runs on a single GPU (tests/test_gpu_bridge.py compares the region the reflected
  // messages cannot reach with the six-tile run)
  const char* const px[] = {"GTFV3_BRIDGE_PROXY", nullptr};
  const bool proxy = nranks > 1 && env_int(px, 0) == 1;
  if (proxy) nl.loopback = -1;
  // GTFV3_TRANSPORT=ipc: several ranks per GPU (the reference's PER_DEVICE_PROCESS, 12 GEOS
  // ranks on each GPU): the same-node IPC transport (ipc.cpp) instead of RCCL, which takes one
  // rank per device; the ncclUniqueId bytes shared below are then the job's key
  if (const char* tr = std::getenv("GTFV3_TRANSPORT")) {
    if (std::strcmp(tr, "ipc") == 0) {
      nl.ipc = true;
      // one hardware queue per rank process unless the job says otherwise (read by the HIP
      // runtime at its first call: effective when nothing in the process has touched HIP yet)
      setenv("GPU_MAX_HW_QUEUES", "1", 0);
    }
    else if (std::strcmp(tr, "rccl") != 0) throw std::runtime_error("GTFV3_TRANSPORT must be rccl or ipc");
  }
  std::vector<unsigned char> id(128, 0);
  if (nranks > 1 && !proxy) {
    if (rank == 0) {
      ncclUniqueId uid;
      if (ncclGetUniqueId(&uid) != ncclSuccess) throw std::runtime_error("ncclGetUniqueId failed");
      std::memcpy(id.data(), &uid, sizeof(uid));
    }
    share_unique_id(comm, rank, nranks, id.data());
  }
  g_dy = std::make_unique<Dycore>(nl, rank, nranks, nranks > 1 && !proxy ? id.data() : nullptr);
  // ncclCommInitRank is collective: every rank has read the id once the Dycore exists
  if (!g_id_file.empty()) {
    std::remove(g_id_file.c_str());
    g_id_file.clear();
  }
  if (g_tiles_per_rank == 1) {
    const SubInfo& s = g_dy->hsubs[0];
    if (s.ioff != is - 1 || s.joff != js - 1)
      throw std::runtime_error("geos_gtfv3_init: rank's (is,js) does not match the FV3 rank layout");
  }
  g_is = is;
  g_js = js;
}

template <typename T>
void bridge_run(const BridgeArgs<T>& a) {
  if (!g_dy) throw std::runtime_error("geos_gtfv3_run before geos_gtfv3_init");
  Dycore& dy = *g_dy;
  const int npz = a.npz, nq = a.nq_tot;
  if (npz != dy.nl.npz || nq != dy.nl.nq || a.npx != dy.nl.npx) throw std::runtime_error("run: dims differ from init");
  if (a.ng != NG) throw std::runtime_error("run: ng must be 3");
  dy.nl.adiabatic = a.adiabatic != 0;
  dy.nl.ptop = a.ptop;
  dy.nl.dt_atmos = a.bdt;
  std::vector<double> ak(npz + 1), bk(npz + 1);
  for (int k = 0; k <= npz; ++k) { ak[k] = (double)a.ak[k]; bk[k] = (double)a.bk[k]; }
  dy.set_vertical(ak.data(), bk.data(), a.ks);
  const int nx = a.ie - a.is + 1, ny = a.je - a.js + 1;
  // local index of Fortran bound x is x - is (compute start = 0)
  auto D3 = [&](int ilo, int ihi, int jlo, int jhi, int nk, int order = 0) {
    return FDesc{ilo - a.is, ihi - ilo + 1, jlo - a.js, jhi - jlo + 1, nk, order};
  };
  const int is = a.is, ie = a.ie, js = a.js, je = a.je, isd = a.isd, ied = a.ied, jsd = a.jsd, jed = a.jed;
  (void)nx; (void)ny;
  struct Item {
    const char* name;
    T* p;
    FDesc fd;
    int nk_dev;
  };
  std::vector<Item> items = {
      {"u", a.u, D3(isd, ied, jsd, jed + 1, npz), npz},
      {"v", a.v, D3(isd, ied + 1, jsd, jed, npz), npz},
      {"w", a.w, D3(isd, ied, jsd, jed, npz), npz},
      {"delz", a.delz, D3(isd, ied, jsd, jed, npz), npz},
      {"pt", a.pt, D3(isd, ied, jsd, jed, npz), npz},
      {"delp", a.delp, D3(isd, ied, jsd, jed, npz), npz},
      {"q", a.q, D3(isd, ied, jsd, jed, npz * nq), npz * nq},
      {"ps", a.ps, D3(isd, ied, jsd, jed, 1), 1},
      {"pe", a.pe, D3(is - 1, ie + 1, js - 1, je + 1, npz + 1, 1), npz + 1},
      {"pk", a.pk, D3(is, ie, js, je, npz + 1), npz + 1},
      {"peln", a.peln, D3(is, ie, js, je, npz + 1, 1), npz + 1},
      {"pkz", a.pkz, D3(is, ie, js, je, npz), npz},
      {"phis", a.phis, D3(isd, ied, jsd, jed, 1), 1},
      {"q_con", a.q_con, D3(isd, ied, jsd, jed, npz), npz},
      {"omga", a.omga, D3(isd, ied, jsd, jed, npz), npz},
      {"ua", a.ua, D3(isd, ied, jsd, jed, npz), npz},
      {"va", a.va, D3(isd, ied, jsd, jed, npz), npz},
      {"uc", a.uc, D3(isd, ied + 1, jsd, jed, npz), npz},
      {"vc", a.vc, D3(isd, ied, jsd, jed + 1, npz), npz},
      {"mfx", a.mfx, D3(is, ie + 1, js, je, npz), npz},
      {"mfy", a.mfy, D3(is, ie, js, je + 1, npz), npz},
      {"cx", a.cx, D3(is, ie + 1, jsd, jed, npz), npz},
      {"cy", a.cy, D3(isd, ied, js, je + 1, npz), npz},
      {"diss_est", a.diss_est, D3(isd, ied, jsd, jed, npz), npz},
  };
  // What a call has to move.  Up: an inout the step overwrites over the whole Fortran extent
  // before reading it needs no upload -- mfx, mfy, cx, cy (zeroed at the step's start), pkz
  // (fv_prep writes the compute domain first), ua, va, uc, vc (d2a2c_vect writes the whole
  // data domain each sub-step), pe, peln, pk (riem_solver3's last call writes every level of
  // the compute domain and pk3_pe_halo pe's ring of one), diss_est (zeroed with d_con, else
  // untouched) -- and q_con, which the step never touches, moves neither way (its Fortran
  // values stay as they were, as after a copy round trip).  Down: diss_est only with d_con
  // (phis comes back: the step fills its halo).  GTFV3_BRIDGE_SKIP=0 moves every array both
  // ways, all of them before / after the step.
  const char* skip_env = std::getenv("GTFV3_BRIDGE_SKIP");
  const bool skip = !(skip_env && skip_env[0] == '0');
  const bool dcon = dy.nl.d_con > 1e-5;
  auto up = [&](const std::string& n) {
    if (!skip) return true;
    for (const char* x : {"mfx", "mfy", "cx", "cy", "pkz", "q_con", "ua", "va", "uc", "vc", "pe", "peln", "pk",
                          "diss_est"})
      if (n == x) return false;
    return true;
  };
  auto down = [&](const std::string& n) {
    if (!skip) return true;
    if (n == "q_con") return false;
    if (n == "diss_est") return dcon;
    return true;
  };
  g_io.init();
  std::vector<std::pair<const void*, size_t>> arrays;
  for (auto& it : items)
    arrays.push_back({it.p, sizeof(T) * (size_t)it.fd.ni * it.fd.nj * it.fd.nk * g_tiles_per_rank});
  g_io.pin(arrays);
  const int up_blocks = zc_blocks("GTFV3_BRIDGE_ZC_BLOCKS", 32);
  const int down_blocks = zc_blocks("GTFV3_BRIDGE_ZC_DOWN_BLOCKS", 1024);
  HIP_CHECK(hipEventRecord(g_io.ev_t[0], dy.st));
  double up_bytes = 0, down_bytes = 0;
  // the state the step reads first goes up before it (small arrays first); tracers 1.. are
  // first read by tracer_2d, after the acoustic sub-steps, and omga only by fv_wrapup (its
  // compute domain is overwritten there, the halo must come back as it went), so those go up
  // beside the step on the side stream and the step waits for them only there
  const long q0 = (long)(ied - isd + 1) * (jed - jsd + 1) * npz;  // tracer 0's share of a tile
  const bool defer = skip;
  auto find = [&](const char* n) -> Item& {
    for (auto& it : items)
      if (std::string(it.name) == n) return it;
    throw std::runtime_error(std::string("bridge: no item ") + n);
  };
  const char* first[] = {"ps", "phis", "delp", "delz", "pt", "q", "u", "v", "w"};
  for (const char* n : first) {
    Item& it = find(n);
    const bool qpart = defer && std::string(n) == "q";
    up_bytes += copy_in<T>(dy, it.name, it.nk_dev, it.p, it.fd, dy.st, ZC_CRIT, 1024, 0, -1, 0, qpart ? q0 : -1);
  }
  for (auto& it : items) {
    bool listed = false;
    for (const char* n : first) listed = listed || std::string(it.name) == n;
    if (listed || !up(it.name) || (defer && std::string(it.name) == "omga")) continue;
    up_bytes += copy_in<T>(dy, it.name, it.nk_dev, it.p, it.fd, dy.st, ZC_CRIT, 1024);
  }
  HIP_CHECK(hipEventRecord(g_io.ev_t[1], dy.st));
  dy.tracer_wait = dy.exit_wait = nullptr;
  if (defer) {
    // the deferred scatters write into q and omga, which the first call allocates and zeroes
    // on dy.st: the side stream starts behind everything queued there so far (the step itself
    // starts at ev_t[1] as well, so this costs no overlap)
    HIP_CHECK(hipEventRecord(g_io.ev_crit, dy.st));
    HIP_CHECK(hipStreamWaitEvent(g_io.side, g_io.ev_crit, 0));
    if (nq > 1) {
      Item& it = find("q");
      up_bytes += copy_in<T>(dy, it.name, it.nk_dev, it.p, it.fd, g_io.side, ZC_SIDE, up_blocks, 0, -1, q0, -1);
      HIP_CHECK(hipEventRecord(g_io.ev_tracers, g_io.side));
      dy.tracer_wait = g_io.ev_tracers;
    }
    Item& om = find("omga");
    up_bytes += copy_in<T>(dy, om.name, om.nk_dev, om.p, om.fd, g_io.side, ZC_SIDE, up_blocks);
    HIP_CHECK(hipEventRecord(g_io.ev_exit, g_io.side));
    dy.exit_wait = g_io.ev_exit;
    dy.marks = g_io.marks;
  }
  // copy back: each group once the step has marked it final (Dycore::StepMark), queued on the
  // side stream as the step records the mark (the step's host thread waits mid-way, in
  // tracer_2d, so groups queued after step() returns would start late), the rest after the step
  struct Group {
    int mark;  // Dycore::StepMark, or -1: after the step
    std::vector<const char*> names;
    bool queued;
  };
  std::vector<Group> groups;
  if (defer) {
    groups = {{Dycore::SM_CWINDS, {"uc", "vc"}, false},
              {Dycore::SM_ACOUSTIC, {"phis", "diss_est"}, false},
              {Dycore::SM_FLUXES, {"mfx", "mfy", "cx", "cy"}, false},
              {Dycore::SM_REMAP, {"w", "delz", "delp", "q", "pe", "peln", "pk", "pkz", "ps"}, false},
              {Dycore::SM_WRAPUP, {"pt", "omga"}, false},
              {Dycore::SM_WINDS, {"u", "v"}, false},
              {-1, {"ua", "va"}, false}};
  } else {
    groups = {{-1, {}, false}};
    for (auto& it : items) groups[0].names.push_back(it.name);
  }
  int ncopied = 0;
  auto queue = [&](Group& g, hipEvent_t ev) {
    HIP_CHECK(hipStreamWaitEvent(g_io.side, ev, 0));
    for (const char* n : g.names) {
      Item& it = find(n);
      if (!down(it.name)) continue;
      down_bytes += copy_out<T>(dy, it.name, it.p, it.fd, g_io.side, down_blocks);
      ++ncopied;
    }
    g.queued = true;
  };
  struct Unhook {  // the hooks reference this frame: cleared however step() ends
    Dycore& d;
    ~Unhook() {
      d.on_mark = nullptr;
      d.marks = nullptr;
      d.tracer_wait = d.exit_wait = nullptr;
    }
  } unhook{dy};
  if (defer)
    dy.on_mark = [&](int m) {
      for (auto& g : groups)
        if (g.mark == m && !g.queued) queue(g, g_io.marks[m]);
    };
  dy.step();
  HIP_CHECK(hipEventRecord(g_io.ev_t[2], dy.st));
  for (auto& g : groups)
    if (!g.queued) queue(g, g_io.ev_t[2]);
  if (ncopied != (int)std::count_if(items.begin(), items.end(), [&](const Item& it) { return down(it.name); }))
    throw std::runtime_error("bridge: copy-back groups do not cover the outputs");
  HIP_CHECK(hipEventRecord(g_io.ev_t[3], g_io.side));
  HIP_CHECK(hipStreamSynchronize(g_io.side));
  HIP_CHECK(hipStreamSynchronize(dy.st));
  for (int n = 0; n < 3; ++n) {
    float ms = 0;
    HIP_CHECK(hipEventElapsedTime(&ms, g_io.ev_t[n], g_io.ev_t[n + 1]));
    g_io.ms[n] = ms;
  }
  g_io.bytes[0] = up_bytes;
  g_io.bytes[1] = down_bytes;
  const char* lg = std::getenv("GTFV3_LOG");
  if (lg && std::atoi(lg) == 1) {
    std::printf(" 0 , geos_gtfv3 %.6f\n", 1e-3 * g_io.ms[1]);
    std::fflush(stdout);
  }
}

void bridge_stats(double* out) {
  for (int n = 0; n < 3; ++n) out[n] = g_io.ms[n];
  out[3] = g_io.bytes[0];
  out[4] = g_io.bytes[1];
  out[5] = (double)g_io.pinned.size();
}

template void bridge_run<float>(const BridgeArgs<float>&);
template void bridge_run<double>(const BridgeArgs<double>&);

void bridge_remove_id_file() {
  if (!g_id_file.empty()) {
    std::remove(g_id_file.c_str());
    g_id_file.clear();
  }
}

void bridge_finalize() {
  g_io.release();
  g_dy.reset();
  bridge_remove_id_file();
}

}  // namespace gtfv3
