// ipc.cpp — the same-node multi-process transport: several ranks (processes) per GPU, as the
// reference runs GEOS (PER_DEVICE_PROCESS = 12: 96 ranks on 8 GPUs,
// /root/reference/src/tcn/ci/pipeline/gtfv3_config.py:22), where RCCL allows one rank per
// device.  Each rank's halo send buffer is exported once as a HIP IPC memory handle; per
// exchange a rank posts (buffer, offset, length) for every message into a POSIX shared-memory
// control block, and each receiver copies its messages device-to-device straight out of the
// peers' send buffers (opened once through hipIpcOpenMemHandle) into its own receive buffer.
// Host barriers in the control block order the steps (packed -> posted -> copied -> reusable),
// as the in-process loopback transport does with a condition variable: a host-synchronous
// exchange (not graph-capturable), correct for any number of ranks on the node's GPUs.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "comm.hpp"
#include "hip_util.hpp"

namespace gtfv3 {
namespace {

constexpr int kMaxRanks = 32;   // ranks sharing one control block (one node)
constexpr int kMaxBases = 4;    // exported send allocations per rank
constexpr int kMaxPosts = 48;   // messages from one rank to one peer in one exchange
constexpr int kMaxRed = 1024;   // values of one allreduce

struct IpcPost {
  int base;
  int pad;
  uint64_t off;  // bytes from the exported base
  uint64_t n;    // doubles
};

struct IpcRank {
  std::atomic<int> nbase;
  int pad;
  hipIpcMemHandle_t handle[kMaxBases];
  uint64_t bytes[kMaxBases];
  int npost[kMaxRanks];  // messages to each destination in the current exchange
  IpcPost post[kMaxRanks][kMaxPosts];
  double red[kMaxRed];
};

struct IpcShared {
  std::atomic<int> ready;
  int nranks;
  std::atomic<int> arrived;
  int pad;
  std::atomic<long> generation;
  std::atomic<int> attached;
  IpcRank rank[kMaxRanks];
};

static_assert(std::atomic<int>::is_always_lock_free && std::atomic<long>::is_always_lock_free,
              "the control block's atomics are shared between processes");

std::string shm_name(const unsigned char* key) {
  char hex[33];
  for (int i = 0; i < 16; ++i) std::snprintf(hex + 2 * i, 3, "%02x", key[i]);
  return std::string("/gtfv3_ipc_") + hex;
}

class IpcTransport : public Transport {
 public:
  IpcTransport(int nranks, int rank, const void* key) : n_(nranks), me_(rank) {
    if (nranks < 2 || nranks > kMaxRanks) throw std::runtime_error("ipc transport: 2 .. 32 ranks per node");
    if (!key) throw std::runtime_error("ipc transport: the job key (the 128-byte id) is required");
    name_ = shm_name((const unsigned char*)key);
    const size_t bytes = sizeof(IpcShared);
    int fd = -1;
    if (rank == 0) {
      (void)shm_unlink(name_.c_str());  // a stale block of a killed job with the same key
      fd = shm_open(name_.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
      if (fd < 0) throw std::runtime_error("ipc transport: shm_open (create) failed");
      if (ftruncate(fd, (off_t)bytes) != 0) {
        close(fd);
        throw std::runtime_error("ipc transport: ftruncate failed");
      }
    } else {
      for (int t = 0;; ++t) {
        fd = shm_open(name_.c_str(), O_RDWR, 0600);
        if (fd >= 0) {
          struct stat sb;
          if (fstat(fd, &sb) == 0 && (size_t)sb.st_size == bytes) break;
          close(fd);
          fd = -1;
        }
        if (t >= 12000) throw std::runtime_error("ipc transport: timed out waiting for rank 0's control block");
        std::this_thread::sleep_for(std::chrono::milliseconds(5));
      }
    }
    void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) throw std::runtime_error("ipc transport: mmap failed");
    sh_ = (IpcShared*)p;
    if (rank == 0) {
      sh_->nranks = nranks;  // (ftruncate zero-filled the rest)
      sh_->ready.store(1, std::memory_order_release);
    } else {
      wait_for([&] { return sh_->ready.load(std::memory_order_acquire) == 1; }, "rank 0's control block");
      if (sh_->nranks != nranks) throw std::runtime_error("ipc transport: rank count differs from rank 0's");
    }
    sh_->attached.fetch_add(1, std::memory_order_acq_rel);
    barrier();
    if (rank == 0) (void)shm_unlink(name_.c_str());  // every rank holds its mapping: no name left behind
  }

  ~IpcTransport() override {
    if (std::getenv("GTFV3_IPC_TRACE"))
      std::fprintf(stderr, "ipc rank %d: %ld exchanges; host ms: pack wait %.1f, posted barrier %.1f, copies %.1f, "
                   "copy wait %.1f, done barrier %.1f\n", me_, nex_, t_[0], t_[1], t_[2], t_[3], t_[4]);
    for (auto& kv : opened_) (void)hipIpcCloseMemHandle(kv.second);
    if (sh_) munmap(sh_, sizeof(IpcShared));
  }

  void group_start() override {
    sends_.clear();
    recvs_.clear();
  }
  void send(const double* buf, size_t n, int peer, hipStream_t) override { sends_.push_back(make(peer, buf, n)); }
  void recv(double* buf, size_t n, int peer, hipStream_t) override { recvs_.push_back(make(peer, buf, n)); }

  void group_end(hipStream_t st) override {
    using clk = std::chrono::steady_clock;
    auto lap = [&](int i, clk::time_point& t) {
      const clk::time_point n = clk::now();
      t_[i] += std::chrono::duration<double, std::milli>(n - t).count();
      t = n;
    };
    clk::time_point t = clk::now();
    ++nex_;
    HIP_CHECK(hipStreamSynchronize(st));  // this rank's packed messages are in its send buffer
    lap(0, t);
    IpcRank& mine = sh_->rank[me_];
    for (int p = 0; p < n_; ++p) mine.npost[p] = 0;
    for (const Pending& s : sends_) {
      if (s.peer < 0 || s.peer >= n_) throw std::runtime_error("ipc transport: peer out of range");
      int& np = mine.npost[s.peer];
      if (np >= kMaxPosts) throw std::runtime_error("ipc transport: too many messages to one peer");
      uint64_t off = 0;
      const int b = export_base(s.p, s.n, &off);
      mine.post[s.peer][np++] = IpcPost{b, 0, off, (uint64_t)s.n};
    }
    barrier();  // every rank's posts (and exported handles) are visible
    lap(1, t);
    std::vector<int> taken(n_, 0);
    for (const Pending& r : recvs_) {
      const IpcRank& src = sh_->rank[r.peer];
      if (taken[r.peer] >= src.npost[me_]) throw std::runtime_error("ipc transport: unmatched receive");
      const IpcPost& m = src.post[me_][taken[r.peer]++];
      if (m.n != r.n) throw std::runtime_error("ipc transport: message size mismatch");
      if (m.base < 0 || m.base >= src.nbase.load(std::memory_order_acquire) ||
          m.off + 8 * m.n > src.bytes[m.base])
        throw std::runtime_error("ipc transport: message outside the peer's exported buffer");
      const char* base = (const char*)peer_base(r.peer, m.base);
      if (r.n) HIP_CHECK(hipMemcpyAsync(r.p, base + m.off, 8 * r.n, hipMemcpyDeviceToDevice, st));
    }
    lap(2, t);
    HIP_CHECK(hipStreamSynchronize(st));
    lap(3, t);
    barrier();  // every receiver has copied: the senders may pack again
    lap(4, t);
  }

  void allreduce_max(double* dev, int n, hipStream_t st) override {
    if (n > kMaxRed) throw std::runtime_error("ipc transport: allreduce too long");
    std::vector<double> h(n);
    HIP_CHECK(hipMemcpyAsync(h.data(), dev, sizeof(double) * n, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    std::memcpy(sh_->rank[me_].red, h.data(), sizeof(double) * n);
    barrier();
    for (int r = 0; r < n_; ++r)
      for (int i = 0; i < n; ++i) h[i] = std::max(h[i], sh_->rank[r].red[i]);
    barrier();  // every rank has read the values before any writes the next ones
    HIP_CHECK(hipMemcpyAsync(dev, h.data(), sizeof(double) * n, hipMemcpyHostToDevice, st));
    HIP_CHECK(hipStreamSynchronize(st));
  }

 private:
  struct Pending {
    int peer;
    double* p;
    size_t n;
  };
  Pending make(int peer, const double* p, size_t n) { return {peer, const_cast<double*>(p), n}; }

  template <class F>
  void wait_for(F done, const char* what) {
    const auto t0 = std::chrono::steady_clock::now();
    for (long spin = 0; !done(); ++spin) {
      if (spin > 64) std::this_thread::yield();
      if ((spin & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(120))
        throw std::runtime_error(std::string("ipc transport: timed out waiting for ") + what);
    }
  }

  // sense by generation: the last rank to arrive resets the count and advances the generation
  void barrier() {
    const long gen = sh_->generation.load(std::memory_order_acquire);
    if (sh_->arrived.fetch_add(1, std::memory_order_acq_rel) + 1 == n_) {
      sh_->arrived.store(0, std::memory_order_relaxed);
      sh_->generation.fetch_add(1, std::memory_order_acq_rel);
    } else {
      wait_for([&] { return sh_->generation.load(std::memory_order_acquire) != gen; }, "the other ranks");
    }
  }

  // the exported allocation holding [p, p + n): its index in this rank's table (exported on
  // first use) and p's byte offset in it
  int export_base(const double* p, size_t n, uint64_t* off) {
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    HIP_CHECK(hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)p));
    const char* b = (const char*)base;
    if ((const char*)p + 8 * n > b + size) throw std::runtime_error("ipc transport: message past its allocation");
    *off = (uint64_t)((const char*)p - b);
    IpcRank& mine = sh_->rank[me_];
    for (int i = 0; i < (int)bases_.size(); ++i)
      if (bases_[i] == b) return i;
    const int i = (int)bases_.size();
    if (i >= kMaxBases) throw std::runtime_error("ipc transport: too many send allocations");
    HIP_CHECK(hipIpcGetMemHandle(&mine.handle[i], (void*)b));
    mine.bytes[i] = size;
    bases_.push_back(b);
    mine.nbase.store(i + 1, std::memory_order_release);
    return i;
  }

  void* peer_base(int peer, int b) {
    const long key = (long)peer * kMaxBases + b;
    auto it = opened_.find(key);
    if (it != opened_.end()) return it->second;
    void* p = nullptr;
    HIP_CHECK(hipIpcOpenMemHandle(&p, sh_->rank[peer].handle[b], hipIpcMemLazyEnablePeerAccess));
    opened_[key] = p;
    return p;
  }

  int n_, me_;
  long nex_ = 0;
  double t_[5] = {0, 0, 0, 0, 0};
  std::string name_;
  IpcShared* sh_ = nullptr;
  std::vector<const char*> bases_;
  std::map<long, void*> opened_;
  std::vector<Pending> sends_, recvs_;
};

}  // namespace

std::unique_ptr<Transport> make_ipc_transport(int nranks, int rank, const void* key) {
  return std::make_unique<IpcTransport>(nranks, rank, key);
}

}  // namespace gtfv3
