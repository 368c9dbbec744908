// bridge.hip — process-global geos_gtfv3 context and Fortran <-> HBM conversion.
#include "bridge.hpp"

#include <dlfcn.h>
#include <unistd.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
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
void* g_stage = nullptr;
size_t g_stage_bytes = 0;

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

template <typename T>
__global__ void fort_to_dev(const T* __restrict__ f, double* __restrict__ dev, Dims d, int s, int nk_dev, FDesc fd,
                            long n) {
  long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  int i = (int)(t % fd.ni), j, k;
  if (fd.order == 0) {
    j = (int)((t / fd.ni) % fd.nj);
    k = (int)(t / ((long)fd.ni * fd.nj));
  } else {
    k = (int)((t / fd.ni) % fd.nk);
    j = (int)(t / ((long)fd.ni * fd.nk));
  }
  dev[((long)s * nk_dev + k) * d.plane + pidx(d, fd.ilo + i, fd.jlo + j)] = (double)f[t];
}

template <typename T>
__global__ void dev_to_fort(T* __restrict__ f, const double* __restrict__ dev, Dims d, int s, int nk_dev, FDesc fd,
                            long n) {
  long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  int i = (int)(t % fd.ni), j, k;
  if (fd.order == 0) {
    j = (int)((t / fd.ni) % fd.nj);
    k = (int)(t / ((long)fd.ni * fd.nj));
  } else {
    k = (int)((t / fd.ni) % fd.nk);
    j = (int)(t / ((long)fd.ni * fd.nk));
  }
  f[t] = (T)dev[((long)s * nk_dev + k) * d.plane + pidx(d, fd.ilo + i, fd.jlo + j)];
}

void* stage(size_t bytes) {
  if (bytes > g_stage_bytes) {
    if (g_stage) HIP_CHECK(hipFree(g_stage));
    HIP_CHECK(hipMalloc(&g_stage, bytes));
    g_stage_bytes = bytes;
  }
  return g_stage;
}

template <typename T>
void copy_in(Dycore& dy, const char* name, int nk_dev, const T* host, const FDesc& fd) {
  Field& f = dy.field(name, nk_dev);
  long n = (long)fd.ni * fd.nj * fd.nk;
  for (int s = 0; s < g_tiles_per_rank; ++s) {
    T* st = (T*)stage(sizeof(T) * n);
    HIP_CHECK(hipMemcpyAsync(st, host + (size_t)s * n, sizeof(T) * n, hipMemcpyHostToDevice, dy.st));
    GT_LAUNCH(fort_to_dev<T>, dim3(cdiv(n, 256)), dim3(256), 0, dy.st, st, f.p, dy.d, s, nk_dev, fd, n);
    HIP_LAUNCH_CHECK();
  }
}

template <typename T>
void copy_out(Dycore& dy, const char* name, T* host, const FDesc& fd) {
  Field* f = dy.find(name);
  if (!f) throw std::runtime_error(std::string("bridge: missing field ") + name);
  long n = (long)fd.ni * fd.nj * fd.nk;
  for (int s = 0; s < g_tiles_per_rank; ++s) {
    T* st = (T*)stage(sizeof(T) * n);
    GT_LAUNCH(dev_to_fort<T>, dim3(cdiv(n, 256)), dim3(256), 0, dy.st, st, f->p, dy.d, s, f->nk, fd, n);
    HIP_LAUNCH_CHECK();
    HIP_CHECK(hipMemcpyAsync(host + (size_t)s * n, st, sizeof(T) * n, hipMemcpyDeviceToHost, dy.st));
    HIP_CHECK(hipStreamSynchronize(dy.st));
  }
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
  std::vector<unsigned char> id(128, 0);
  if (nranks > 1) {
    if (rank == 0) {
      ncclUniqueId uid;
      if (ncclGetUniqueId(&uid) != ncclSuccess) throw std::runtime_error("ncclGetUniqueId failed");
      std::memcpy(id.data(), &uid, sizeof(uid));
    }
    share_unique_id(comm, rank, nranks, id.data());
  }
  g_dy = std::make_unique<Dycore>(nl, rank, nranks, nranks > 1 ? id.data() : nullptr);
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
  for (auto& it : items) copy_in<T>(dy, it.name, it.nk_dev, it.p, it.fd);
  HIP_CHECK(hipStreamSynchronize(dy.st));
  auto t0 = std::chrono::steady_clock::now();
  dy.step();
  HIP_CHECK(hipStreamSynchronize(dy.st));
  auto t1 = std::chrono::steady_clock::now();
  for (auto& it : items) copy_out<T>(dy, it.name, it.p, it.fd);
  const char* lg = std::getenv("GTFV3_LOG");
  if (lg && std::atoi(lg) == 1) {
    double sec = std::chrono::duration<double>(t1 - t0).count();
    std::printf(" 0 , geos_gtfv3 %.6f\n", sec);
    std::fflush(stdout);
  }
}

template void bridge_run<float>(const BridgeArgs<float>&);
template void bridge_run<double>(const BridgeArgs<double>&);

void bridge_finalize() {
  g_dy.reset();
  if (!g_id_file.empty()) {
    std::remove(g_id_file.c_str());
    g_id_file.clear();
  }
  if (g_stage) {
    (void)hipFree(g_stage);
    g_stage = nullptr;
    g_stage_bytes = 0;
  }
}

}  // namespace gtfv3
