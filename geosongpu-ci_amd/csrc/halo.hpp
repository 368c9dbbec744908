// halo.hpp — cubed-sphere halo update (replaces the NDSL/mpp halo updater the
// reference's external dycore uses over CUDA-aware MPI; the only comm touchpoint
// in the reference is the communicator hand-off, py_ftn_interface/base.py:72-96).
//
// Every halo point of every local sub-domain is resolved ONCE on the host to
// (owner rank, owner sub-domain, plane offset, component, sign): vector fields
// across rotated cube edges swap u<->v and flip sign by the lattice rotation
// between the two tiles.  Cube-corner regions (three tiles meet) are zero-filled;
// the stencils fill them on the fly (copy_corners / fill_4corners).
//  * same-rank sources: one gather kernel (tile edges on one GPU are device copies)
//  * other ranks: pack -> ncclSend/ncclRecv grouped per neighbour -> unpack,
//    point-to-point over xGMI (never a ring collective).
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <vector>

#include "comm.hpp"
#include "grid.hpp"

namespace gtfv3 {

struct HaloEntry {
  int dst_sub, dst_off, src_sub, src_off;  // src_sub < 0: zero-fill
  int comp;                                 // bit0: dst component, bit1: src component
  int sign;
};
struct PackEntry {
  int sub, off, comp, sign;  // sign 0 unused for unpack
  int pstart, pcount;        // peer segment start/length (entries)
};

struct HaloField {
  double* p[2];  // component pointers (p[1] == nullptr for scalars)
  int nk;
  int kind;      // HaloKind
};

class HaloExchanger {
 public:
  HaloExchanger() = default;
  ~HaloExchanger();
  void build(const CubedSphere& cs, const Decomp& dc, const Dims& d, int max_nk, int max_fields, bool device = true);
  void set_transport(Transport* t) { tr_ = t; }
  // before build(): one rank, its same-rank halo points as messages to itself (Namelist::rccl_self)
  void set_self_messages(bool on) { self_msgs_ = on; }
  // fill halos of all listed fields (enqueued on `stream`)
  void exchange(const HaloField* fields, int nf, hipStream_t stream);
  // the same exchange in two halves, for the interior / boundary split: begin enqueues the
  // pack and same-rank gather on `stream` and the messages on the exchange's communication
  // stream; whatever the caller enqueues on `stream` before end() runs beside the messages (it
  // must read no halo point and write no point the pack reads); end() makes `stream` wait for
  // the messages and unpacks.  One exchange at a time.  Without messages (one rank, no self
  // messages) begin is the whole exchange and end does nothing.
  void exchange_begin(const HaloField* fields, int nf, hipStream_t stream);
  void exchange_end(hipStream_t stream);
  bool remote() const { return remote_; }
  // host copies of tables for tests
  const std::vector<HaloEntry>& local_table(int kind) const { return h_local_[kind]; }
  // remote tables (dir 0: send/pack, 1: recv/unpack) as (sub, off, comp, sign, pos_in_peer_segment, peer)
  std::vector<int> remote_table(int kind, int dir) const;
  int nranks() const { return nranks_; }
  // an exchange enqueues without host waits (one rank, or a capturable transport)
  bool capturable() const { return !remote_ || !tr_ || tr_->capturable(); }

 private:
  Dims d_{};
  int rank_ = 0, nranks_ = 1;
  bool self_msgs_ = false;
  bool remote_ = false;  // the exchange runs the message path (several ranks, or self messages)
  Transport* tr_ = nullptr;
  std::vector<HaloEntry> h_local_[H_NKIND];
  std::vector<PackEntry> h_send_[H_NKIND], h_recv_[H_NKIND];
  HaloEntry* d_local_[H_NKIND] = {};
  int n_local_[H_NKIND] = {};
  // remote: per kind, concatenated over peers
  std::vector<int> send_peer_start_[H_NKIND], send_peer_count_[H_NKIND];
  std::vector<int> recv_peer_start_[H_NKIND], recv_peer_count_[H_NKIND];
  PackEntry* d_send_[H_NKIND] = {};
  PackEntry* d_recv_[H_NKIND] = {};
  int n_send_[H_NKIND] = {}, n_recv_[H_NKIND] = {};
  double* sendbuf_ = nullptr;
  double* recvbuf_ = nullptr;
  size_t buf_elems_ = 0;
  // multi-rank: the point-to-point messages run on their own stream, so the same-rank
  // gather (and whatever precedes the unpack) overlaps them
  hipStream_t comm_st_ = nullptr;
  hipEvent_t ev_packed_ = nullptr, ev_recvd_ = nullptr;
  // one stage of an exchange (0 same-rank gather, 1 pack, 2 unpack, 3 pack + gather) for the
  // fields and their pack-buffer offsets
  void launch_stage(int stage, const HaloField* fields, int nf, const std::vector<size_t>& foff, hipStream_t stream);
  std::vector<size_t> buffer_offsets(const HaloField* fields, int nf) const;
  void post_messages(const HaloField* fields, int nf, const std::vector<size_t>& foff, hipStream_t mst);
  std::vector<HaloField> pending_;  // an exchange begun and not yet ended
  std::vector<size_t> pending_off_;
  bool pending_open_ = false;
};

}  // namespace gtfv3
