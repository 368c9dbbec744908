// comm.hpp — rank-to-rank transport behind the halo exchange and the single
// reduction of a dycore step (the tracer Courant maximum).
//  * NcclTransport: RCCL point-to-point send/recv (grouped) and allreduce(max) on the
//    dycore stream — the production path, one process per GPU over xGMI.
//  * LoopbackTransport: several ranks of one process on one device; messages are
//    device-to-device copies through a shared mailbox with host barriers.  It runs the
//    exact same tables and pack / unpack kernels, so multi-rank steps can be verified
//    on a single GPU (tests/test_gpu_multirank.py).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <memory>

namespace gtfv3 {

class Transport {
 public:
  virtual ~Transport() = default;
  virtual void group_start() = 0;
  virtual void send(const double* buf, size_t n, int peer, hipStream_t st) = 0;
  virtual void recv(double* buf, size_t n, int peer, hipStream_t st) = 0;
  virtual void group_end(hipStream_t st) = 0;
  virtual void allreduce_max(double* dev, int n, hipStream_t st) = 0;
  // its enqueue makes no host wait, so a HIP graph can capture it (Dycore::step)
  virtual bool capturable() const { return false; }
};

// every device-to-device copy of one message group in one launch (halo.hip), as RCCL moves a
// grouped set of point-to-point messages in one kernel
struct CopyMsg {
  double* dst;
  const double* src;
  size_t n;
};
void batched_copy(const CopyMsg* msgs, int nmsg, hipStream_t st);

std::unique_ptr<Transport> make_nccl_transport(int nranks, int rank, const void* nccl_id);
// several ranks (processes) on one node's GPUs (ipc.cpp): HIP IPC handles of the send buffers
// and a shared-memory control block named by the 128-byte key every rank was given
std::unique_ptr<Transport> make_ipc_transport(int nranks, int rank, const void* key);
// group < 0: the null transport (one rank alone, each receive answered by its own send to
// that peer: measurement only)
std::unique_ptr<Transport> make_loopback_transport(int group, int nranks, int rank);

}  // namespace gtfv3
