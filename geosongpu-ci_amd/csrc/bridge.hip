// bridge.hip — process-global geos_gtfv3 context and Fortran <-> HBM conversion.
#include "bridge.hpp"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
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

void bridge_init(void* comm, int npx, int npy, int npz, int ntiles, int is, int ie, int js, int je, int isd, int ied,
                 int jsd, int jed, float bdt, int nq_tot) {
  (void)comm;
  if (ntiles != 6) throw std::runtime_error("geos_gtfv3_init: ntiles must be 6");
  if (npx != npy) throw std::runtime_error("geos_gtfv3_init: npx != npy");
  if (isd != is - NG || ied != ie + NG || jsd != js - NG || jed != je + NG)
    throw std::runtime_error("geos_gtfv3_init: data domain must be the compute domain +/- 3 halo points");
  const char* rk[] = {"GTFV3_RANK", "OMPI_COMM_WORLD_RANK", "PMI_RANK", "SLURM_PROCID", "RANK", nullptr};
  const char* sz[] = {"GTFV3_WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", "PMI_SIZE", "SLURM_NTASKS", "WORLD_SIZE", nullptr};
  const char* tp[] = {"GTFV3_BRIDGE_TILES_PER_RANK", nullptr};
  int rank = env_int(rk, 0), nranks = env_int(sz, 1);
  g_tiles_per_rank = env_int(tp, 1);
  int N = npx - 1, nx = ie - is + 1, ny = je - js + 1;
  Namelist nl;
  nl.npx = nl.npy = npx;
  nl.npz = npz;
  nl.nq = nq_tot;
  nl.layout_x = N / nx;
  nl.layout_y = N / ny;
  nl.dt_atmos = bdt;
  if (g_tiles_per_rank == 6) {
    if (nranks != 1 || nx != N || ny != N) throw std::runtime_error("6 tiles per rank needs 1 rank and layout 1x1");
  } else if (g_tiles_per_rank != 1) {
    throw std::runtime_error("GTFV3_BRIDGE_TILES_PER_RANK must be 1 or 6");
  } else if (nranks != 6 * nl.layout_x * nl.layout_y) {
    throw std::runtime_error("geos_gtfv3_init: one sub-domain per rank expected (6*layout ranks)");
  }
  std::vector<unsigned char> id(128, 0);
  if (nranks > 1) {
    // GEOS path: rank 0's ncclUniqueId would be broadcast over the communicator
    // handed in as `comm` (MPI_Comm_f2c, base.py:89-96).  MPI is not linked
    // here, so the id goes through a shared file named by GTFV3_NCCL_ID_FILE.
    const char* fn = std::getenv("GTFV3_NCCL_ID_FILE");
    if (!fn) throw std::runtime_error("multi-rank bridge needs GTFV3_NCCL_ID_FILE");
    std::string tmp = std::string(fn) + ".tmp";
    if (rank == 0) {
      ncclUniqueId uid;
      if (ncclGetUniqueId(&uid) != ncclSuccess) throw std::runtime_error("ncclGetUniqueId failed");
      std::memcpy(id.data(), &uid, sizeof(uid));
      std::ofstream(tmp, std::ios::binary).write((const char*)id.data(), 128);
      std::rename(tmp.c_str(), fn);
    } else {
      for (int t = 0; t < 6000; ++t) {
        std::ifstream in(fn, std::ios::binary);
        if (in && in.read((char*)id.data(), 128)) break;
        std::this_thread::sleep_for(std::chrono::milliseconds(10));
        if (t == 5999) throw std::runtime_error("timed out waiting for the ncclUniqueId file");
      }
    }
  }
  g_dy = std::make_unique<Dycore>(nl, rank, nranks, nranks > 1 ? id.data() : nullptr);
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
  if (g_stage) {
    (void)hipFree(g_stage);
    g_stage = nullptr;
    g_stage_bytes = 0;
  }
}

}  // namespace gtfv3
