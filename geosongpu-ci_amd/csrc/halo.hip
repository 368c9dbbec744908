// halo.hip — table construction (host) and halo gather / pack / unpack kernels.
#include <cstdlib>
#include <algorithm>
#include <stdexcept>

#include "halo.hpp"
#include "hip_util.hpp"

namespace gtfv3 {

namespace {

inline void rot_dir(int rot, int dx, int dy, int& ox, int& oy) {
  switch (rot & 3) {
    case 0: ox = dx; oy = dy; break;
    case 1: ox = -dy; oy = dx; break;
    case 2: ox = -dx; oy = -dy; break;
    default: ox = dy; oy = -dx; break;
  }
}

// staggering of component c of halo kind k
inline int comp_stagger(int kind, int c) {
  switch (kind) {
    case H_CELL: return CELL;
    case H_CORNER: return CORNER;
    case H_DGRID: return c == 0 ? XEDGE : YEDGE;   // u along x-edges, v along y-edges
    case H_CGRID:
    case H_CSYNC:
    case H_CSC: return c == 0 ? YEDGE : XEDGE;     // uc normal to y-edges, vc to x-edges
    default: return CELL;                           // A-grid pair
  }
}
inline int ncomp(int kind) { return (kind == H_CELL || kind == H_CORNER) ? 1 : 2; }

struct Src {
  int rank, lsub, off, comp, sign;
  bool zero;
  int gsub, li, lj;  // global owner sub-domain and local point (for the H_CSC redirect)
};

}  // namespace

HaloExchanger::~HaloExchanger() {
  for (int k = 0; k < H_NKIND; ++k) {
    debug_canary_drop(d_local_[k]);
    debug_canary_drop(d_send_[k]);
    debug_canary_drop(d_recv_[k]);
    if (d_local_[k]) (void)hipFree(d_local_[k]);
    if (d_send_[k]) (void)hipFree(d_send_[k]);
    if (d_recv_[k]) (void)hipFree(d_recv_[k]);
  }
  if (sendbuf_) (void)hipFree(sendbuf_);
  if (recvbuf_) (void)hipFree(recvbuf_);
  if (ev_packed_) (void)hipEventDestroy(ev_packed_);
  if (ev_recvd_) (void)hipEventDestroy(ev_recvd_);
  if (comm_st_) (void)hipStreamDestroy(comm_st_);
}

void HaloExchanger::build(const CubedSphere& cs, const Decomp& dc, const Dims& d, int max_nk,
                          int max_fields, bool device) {
  d_ = d;
  rank_ = dc.rank;
  nranks_ = dc.nranks;
  if (self_msgs_ && nranks_ != 1) throw std::runtime_error("halo: self messages need a one-rank layout");
  remote_ = nranks_ > 1 || self_msgs_;
  // a same-rank source point: gathered locally, or (self messages) packed, sent to this
  // rank and unpacked -- the send and receive entries are pushed at the same point in the
  // same walk, so their orders match as a peer's do
  const bool local_gather = !self_msgs_;
  const int nper = dc.nsub_per_rank();
  const int nx = d.nx, ny = d.ny;

  // resolve the source of one halo point of (global sub g, component c, staggering st)
  auto resolve = [&](int g, int kind, int c, int i, int j) -> Src {
    SubInfo si = dc.sub(g);
    int st = comp_stagger(kind, c);
    int x2 = 2 * (i + si.ioff) + ((st == CELL || st == XEDGE) ? 1 : 0);
    int y2 = 2 * (j + si.joff) + ((st == CELL || st == YEDGE) ? 1 : 0);
    Mapped m = cs.map(si.tile, x2, y2, false);
    Src s{};
    if (!m.valid) { s.zero = true; return s; }
    // owning sub-domain in tile m.t
    int found = -1, li = 0, lj = 0;
    for (int py = 0; py < dc.ly && found < 0; ++py)
      for (int px = 0; px < dc.lx && found < 0; ++px) {
        int ioff = px * nx, joff = py * ny;
        int ii = (m.x2 - (m.x2 & 1)) / 2 - ioff;
        int jj = (m.y2 - (m.y2 & 1)) / 2 - joff;
        int imax = (m.x2 & 1) ? nx - 1 : nx;
        int jmax = (m.y2 & 1) ? ny - 1 : ny;
        if (ii >= 0 && ii <= imax && jj >= 0 && jj <= jmax) {
          found = m.t * dc.lx * dc.ly + py * dc.lx + px;
          li = ii; lj = jj;
        }
      }
    if (found < 0) throw std::runtime_error("halo: no owner sub-domain");
    s.gsub = found; s.li = li; s.lj = lj;
    s.rank = dc.owner_rank(found);
    s.lsub = found % nper;
    s.off = (int)pidx(d, li, lj);
    if (ncomp(kind) == 1) { s.comp = 0; s.sign = 1; }
    else {
      int dx = c == 0 ? 1 : 0, dy = c == 0 ? 0 : 1, ox, oy;
      rot_dir(m.rot, dx, dy, ox, oy);
      s.comp = ox != 0 ? 0 : 1;
      s.sign = ox + oy;
    }
    s.zero = false;
    return s;
  };
  // a point ON the east (edge 1) / north (edge 3) tile edge, as the neighbouring tile holds
  // it (its west or south edge: the FV3 cube joins every east / north edge to one of those)
  auto resolve_edge = [&](int g, int kind, int c, int i, int j, int edge) -> Src {
    SubInfo si = dc.sub(g);
    int st = comp_stagger(kind, c);
    int x2 = 2 * (i + si.ioff) + ((st == CELL || st == XEDGE) ? 1 : 0);
    int y2 = 2 * (j + si.joff) + ((st == CELL || st == YEDGE) ? 1 : 0);
    Mapped m = cs.map_across(si.tile, edge, x2, y2);
    if (!(m.x2 == 0 || m.y2 == 0)) throw std::runtime_error("halo: an east / north edge must meet a west / south edge");
    int found = -1, li = 0, lj = 0;
    for (int py = 0; py < dc.ly && found < 0; ++py)
      for (int px = 0; px < dc.lx && found < 0; ++px) {
        int ii = (m.x2 - (m.x2 & 1)) / 2 - px * nx, jj = (m.y2 - (m.y2 & 1)) / 2 - py * ny;
        int imax = (m.x2 & 1) ? nx - 1 : nx, jmax = (m.y2 & 1) ? ny - 1 : ny;
        if (ii >= 0 && ii <= imax && jj >= 0 && jj <= jmax) {
          found = m.t * dc.lx * dc.ly + py * dc.lx + px;
          li = ii; lj = jj;
        }
      }
    if (found < 0) throw std::runtime_error("halo: no owner sub-domain of a shared edge point");
    Src s{};
    s.rank = dc.owner_rank(found);
    s.lsub = found % nper;
    s.off = (int)pidx(d, li, lj);
    int dx = c == 0 ? 1 : 0, dy = c == 0 ? 0 : 1, ox, oy;
    rot_dir(m.rot, dx, dy, ox, oy);
    s.comp = ox != 0 ? 0 : 1;
    s.sign = ox + oy;
    s.zero = false;
    return s;
  };

  // H_CSC: a C halo source that is itself a synchronised tile-edge point (uc on an east,
  // vc on a north tile edge) is replaced by that point's synchronisation source
  auto csc_redirect = [&](int kind, Src s) -> Src {
    if (kind != H_CSC || s.zero) return s;
    const SubInfo so = dc.sub(s.gsub);
    const bool east = s.comp == 0 && so.ioff + nx == so.N && s.li == nx && s.lj >= 0 && s.lj < ny;
    const bool north = s.comp == 1 && so.joff + ny == so.N && s.lj == ny && s.li >= 0 && s.li < nx;
    if (!east && !north) return s;
    Src t = resolve_edge(s.gsub, H_CSYNC, s.comp, s.li, s.lj, east ? 1 : 3);
    t.sign *= s.sign;
    return t;
  };
  for (int kind = 0; kind < H_NKIND; ++kind) {
    h_local_[kind].clear();
    std::vector<std::vector<PackEntry>> send(nranks_), recv(nranks_);
    for (int q = 0; q < nranks_; ++q) {
      for (int ls = 0; ls < nper; ++ls) {
        int g = q * nper + ls;
        for (int c = 0; c < ncomp(kind); ++c) {
          int st = comp_stagger(kind, c);
          int sx = (st == YEDGE || st == CORNER) ? 1 : 0;
          int sy = (st == XEDGE || st == CORNER) ? 1 : 0;
          if (kind == H_CSYNC || kind == H_CSC) {
            // targets: uc on the east tile edge, vc on the north tile edge of this sub-domain
            const SubInfo si = dc.sub(g);
            const bool east = c == 0 && si.ioff + nx == si.N, north = c == 1 && si.joff + ny == si.N;
            const int n = east ? ny : (north ? nx : 0);
            for (int p = 0; p < n; ++p) {
              const int i = east ? nx : p, j = east ? p : ny;
              Src s = resolve_edge(g, H_CSYNC, c, i, j, east ? 1 : 3);
              if (q != rank_) {
                if (s.rank == rank_) send[q].push_back({s.lsub, s.off, s.comp, s.sign, 0, 0});
                continue;
              }
              int doff = (int)pidx(d, i, j);
              if (s.rank == rank_ && local_gather)
                h_local_[kind].push_back({ls, doff, s.lsub, s.off, c | (s.comp << 1), s.sign});
              else {
                if (s.rank == rank_) send[rank_].push_back({s.lsub, s.off, s.comp, s.sign, 0, 0});
                recv[s.rank].push_back({ls, doff, c, 0, 0, 0});
              }
            }
            if (kind == H_CSYNC) continue;
          }
          for (int j = -NG; j <= ny - 1 + NG + sy; ++j)
            for (int i = -NG; i <= nx - 1 + NG + sx; ++i) {
              bool inside = i >= 0 && i <= nx - 1 + sx && j >= 0 && j <= ny - 1 + sy;
              if (inside) continue;
              if (q != rank_) {
                // only needed when this rank is the owner of the source
                Src s = csc_redirect(kind, resolve(g, kind, c, i, j));
                if (!s.zero && s.rank == rank_) send[q].push_back({s.lsub, s.off, s.comp, s.sign, 0, 0});
                continue;
              }
              Src s = csc_redirect(kind, resolve(g, kind, c, i, j));
              int doff = (int)pidx(d, i, j);
              if (s.zero) h_local_[kind].push_back({ls, doff, -1, 0, c, 0});
              else if (s.rank == rank_ && local_gather)
                h_local_[kind].push_back({ls, doff, s.lsub, s.off, c | (s.comp << 1), s.sign});
              else {
                if (s.rank == rank_) send[rank_].push_back({s.lsub, s.off, s.comp, s.sign, 0, 0});
                recv[s.rank].push_back({ls, doff, c, 0, 0, 0});
              }
            }
        }
      }
    }
    // concatenate per peer
    std::vector<PackEntry> hs, hr;
    send_peer_start_[kind].assign(nranks_, 0); send_peer_count_[kind].assign(nranks_, 0);
    recv_peer_start_[kind].assign(nranks_, 0); recv_peer_count_[kind].assign(nranks_, 0);
    for (int p = 0; p < nranks_; ++p) {
      send_peer_start_[kind][p] = (int)hs.size();
      send_peer_count_[kind][p] = (int)send[p].size();
      for (auto e : send[p]) { e.pstart = send_peer_start_[kind][p]; e.pcount = (int)send[p].size(); hs.push_back(e); }
      recv_peer_start_[kind][p] = (int)hr.size();
      recv_peer_count_[kind][p] = (int)recv[p].size();
      for (auto e : recv[p]) { e.pstart = recv_peer_start_[kind][p]; e.pcount = (int)recv[p].size(); hr.push_back(e); }
    }
    n_local_[kind] = (int)h_local_[kind].size();
    n_send_[kind] = (int)hs.size();
    n_recv_[kind] = (int)hr.size();
    h_send_[kind] = hs;
    h_recv_[kind] = hr;
    if (!device) continue;
    if (n_local_[kind]) {
      HIP_CHECK(hipMalloc(&d_local_[kind], sizeof(HaloEntry) * n_local_[kind]));
      HIP_CHECK(hipMemcpy(d_local_[kind], h_local_[kind].data(), sizeof(HaloEntry) * n_local_[kind], hipMemcpyHostToDevice));
      debug_canary("halo d_local_", d_local_[kind], h_local_[kind].data(), sizeof(HaloEntry) * n_local_[kind]);
    }
    if (n_send_[kind]) {
      HIP_CHECK(hipMalloc(&d_send_[kind], sizeof(PackEntry) * n_send_[kind]));
      HIP_CHECK(hipMemcpy(d_send_[kind], hs.data(), sizeof(PackEntry) * n_send_[kind], hipMemcpyHostToDevice));
      debug_canary("halo d_send_", d_send_[kind], hs.data(), sizeof(PackEntry) * n_send_[kind]);
    }
    if (n_recv_[kind]) {
      HIP_CHECK(hipMalloc(&d_recv_[kind], sizeof(PackEntry) * n_recv_[kind]));
      HIP_CHECK(hipMemcpy(d_recv_[kind], hr.data(), sizeof(PackEntry) * n_recv_[kind], hipMemcpyHostToDevice));
      debug_canary("halo d_recv_", d_recv_[kind], hr.data(), sizeof(PackEntry) * n_recv_[kind]);
    }
  }
  if (!device) return;
  size_t maxe = 0;
  for (int k = 0; k < H_NKIND; ++k) maxe = std::max<size_t>(maxe, std::max(n_send_[k], n_recv_[k]));
  buf_elems_ = maxe * (size_t)max_nk * max_fields;
  if (buf_elems_) {
    HIP_CHECK(hipMalloc(&sendbuf_, sizeof(double) * buf_elems_));
    HIP_CHECK(hipMalloc(&recvbuf_, sizeof(double) * buf_elems_));
    // zeroed (deterministic contents before the first message)
    HIP_CHECK(hipMemset(sendbuf_, 0, sizeof(double) * buf_elems_));
    HIP_CHECK(hipMemset(recvbuf_, 0, sizeof(double) * buf_elems_));
  }
  if (remote_) {
    HIP_CHECK(hipStreamCreateWithFlags(&comm_st_, hipStreamNonBlocking));
    HIP_CHECK(hipEventCreateWithFlags(&ev_packed_, hipEventDisableTiming));
    HIP_CHECK(hipEventCreateWithFlags(&ev_recvd_, hipEventDisableTiming));
  }
}

std::vector<int> HaloExchanger::remote_table(int kind, int dir) const {
  const auto& t = dir == 0 ? h_send_[kind] : h_recv_[kind];
  const auto& starts = dir == 0 ? send_peer_start_[kind] : recv_peer_start_[kind];
  const auto& counts = dir == 0 ? send_peer_count_[kind] : recv_peer_count_[kind];
  std::vector<int> out;
  for (int p = 0; p < (int)starts.size(); ++p)
    for (int e = starts[p]; e < starts[p] + counts[p]; ++e) {
      const PackEntry& h = t[e];
      out.insert(out.end(), {h.sub, h.off, h.comp, h.sign, e - starts[p], p});
    }
  return out;
}

namespace {

// All fields of one exchange in one launch per stage (grid z = field, y = level):
// up to HB fields; the per-field table, extent and pointers are picked by a uniform
// compare chain (no dynamically indexed kernel-argument array, no scratch).
constexpr int HB = 8;
struct HaloBatch {
  const void* tab[HB];
  int n[HB], nk[HB];
  double* p0[HB];
  double* p1[HB];
  long boff[HB];  // field offset in the pack buffers
};
struct HaloSel {
  const void* tab;
  int n, nk;
  double *p0, *p1;
  long boff;
};
__device__ __forceinline__ HaloSel halo_sel(const HaloBatch b, int f) {  // by value: no reference to the kernel argument
  HaloSel r{b.tab[0], b.n[0], b.nk[0], b.p0[0], b.p1[0], b.boff[0]};
#pragma unroll
  for (int q = 1; q < HB; ++q)
    if (f == q) r = HaloSel{b.tab[q], b.n[q], b.nk[q], b.p0[q], b.p1[q], b.boff[q]};
  return r;
}

// Each thread moves one halo point for HK consecutive levels: the table entry is read once
// per HK levels instead of once per level, and the HK loads are issued together.  HK = 8
// where the exchange has work enough to fill the chip that way (one rank holding whole
// tiles: C180 halo_local 0.93 -> 0.90 ms/step); HK = 1 for the smaller per-rank exchanges
// (8-rank share: pack / unpack 0.29 -> 0.34-0.36 ms/step with HK = 8, too few threads).
template <int HK>
__device__ __forceinline__ void halo_local_body(const HaloSel& F, long plane) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const int k0 = blockIdx.y * HK;
  if (e >= F.n || k0 >= F.nk) return;
  const HaloEntry h = static_cast<const HaloEntry*>(F.tab)[e];
  const double* src = (h.comp & 2) ? F.p1 : F.p0;
  double* dst = (h.comp & 1) ? F.p1 : F.p0;
  double v[HK];
#pragma unroll
  for (int u = 0; u < HK; ++u) {
    const int k = k0 + u;
    v[u] = (h.src_sub >= 0 && k < F.nk) ? h.sign * src[((long)h.src_sub * F.nk + k) * plane + h.src_off] : 0.0;
  }
#pragma unroll
  for (int u = 0; u < HK; ++u) {
    const int k = k0 + u;
    if (k < F.nk) dst[((long)h.dst_sub * F.nk + k) * plane + h.dst_off] = v[u];
  }
}

template <int HK>
__device__ __forceinline__ void halo_pack_body(const HaloSel& F, long plane, double* __restrict__ buf) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const int k0 = blockIdx.y * HK;
  if (e >= F.n || k0 >= F.nk) return;
  const PackEntry h = static_cast<const PackEntry*>(F.tab)[e];
  const double* src = h.comp ? F.p1 : F.p0;
#pragma unroll
  for (int u = 0; u < HK; ++u) {
    const int k = k0 + u;
    if (k < F.nk)
      buf[F.boff + (long)h.pstart * F.nk + (long)k * h.pcount + (e - h.pstart)] =
          h.sign * src[((long)h.sub * F.nk + k) * plane + h.off];
  }
}

template <int HK>
__global__ void halo_local_kernel(HaloBatch b, long plane) {
  halo_local_body<HK>(halo_sel(b, blockIdx.z), plane);
}

template <int HK>
__global__ void halo_pack_kernel(HaloBatch b, long plane, double* __restrict__ buf) {
  halo_pack_body<HK>(halo_sel(b, blockIdx.z), plane, buf);
}

// a remote exchange's pack and same-rank gather in one launch (grid z: the np packed fields,
// then the local ones): the gather writes halo points only, the pack reads owned points only
template <int HK>
__global__ void halo_pack_local_kernel(HaloBatch pk, int np, HaloBatch lc, long plane, double* __restrict__ buf) {
  const int z = blockIdx.z;
  if (z < np) halo_pack_body<HK>(halo_sel(pk, z), plane, buf);
  else halo_local_body<HK>(halo_sel(lc, z - np), plane);
}

template <int HK>
__global__ void halo_unpack_kernel(HaloBatch b, long plane, const double* __restrict__ buf) {
  const HaloSel F = halo_sel(b, blockIdx.z);
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const int k0 = blockIdx.y * HK;
  if (e >= F.n || k0 >= F.nk) return;
  const PackEntry h = static_cast<const PackEntry*>(F.tab)[e];
  double* dst = h.comp ? F.p1 : F.p0;
#pragma unroll
  for (int u = 0; u < HK; ++u) {
    const int k = k0 + u;
    if (k < F.nk)
      dst[((long)h.sub * F.nk + k) * plane + h.off] =
          buf[F.boff + (long)h.pstart * F.nk + (long)k * h.pcount + (e - h.pstart)];
  }
}

}  // namespace

namespace {
// up to CB_MAX messages per launch (kernel-argument table); block y = message
constexpr int CB_MAX = 96;
struct CopyBatch {
  CopyMsg m[CB_MAX];
};
__global__ void __launch_bounds__(256) batched_copy_k(CopyBatch b) {
  const CopyMsg m = b.m[blockIdx.y];
  for (size_t t = (size_t)blockIdx.x * 256 + threadIdx.x; t < m.n; t += (size_t)gridDim.x * 256) m.dst[t] = m.src[t];
}
}  // namespace

void batched_copy(const CopyMsg* msgs, int nmsg, hipStream_t st) {
  for (int m0 = 0; m0 < nmsg; m0 += CB_MAX) {
    CopyBatch b{};
    const int nb = std::min(CB_MAX, nmsg - m0);
    size_t maxn = 0;
    for (int q = 0; q < nb; ++q) {
      b.m[q] = msgs[m0 + q];
      maxn = std::max(maxn, msgs[m0 + q].n);
    }
    const unsigned gx = (unsigned)std::min<size_t>(cdiv((long)maxn, 256L), 64);
    GT_LAUNCH(batched_copy_k, dim3(gx, nb), dim3(256), 0, st, b);
    HIP_LAUNCH_CHECK();
  }
}

std::vector<size_t> HaloExchanger::buffer_offsets(const HaloField* fields, int nf) const {
  std::vector<size_t> foff(nf, 0);
  if (!remote_) return foff;
  size_t off = 0;
  for (int f = 0; f < nf; ++f) {
    foff[f] = off;
    off += (size_t)std::max(n_send_[fields[f].kind], n_recv_[fields[f].kind]) * fields[f].nk;
  }
  if (off > buf_elems_) throw std::runtime_error("halo: exchange buffer too small");
  if (!tr_) throw std::runtime_error("halo: multi-rank exchange without a transport");
  return foff;
}

// one launch per stage for (up to HB) fields; stage 0 local gather, 1 pack, 2 unpack,
// 3 pack + local gather together
void HaloExchanger::launch_stage(int stage, const HaloField* fields, int nf, const std::vector<size_t>& foff,
                                 hipStream_t stream) {
  auto batch = [&](int stg, int f0, HaloBatch& b, int& maxn, int& maxk) {
    b = HaloBatch{};
    int nb = 0;
    for (int f = f0; f < nf && f < f0 + HB; ++f) {
      const HaloField& F = fields[f];
      const int n = stg == 0 ? n_local_[F.kind] : (stg == 1 ? n_send_[F.kind] : n_recv_[F.kind]);
      if (!n) continue;
      b.tab[nb] = stg == 0 ? (const void*)d_local_[F.kind]
                           : (stg == 1 ? (const void*)d_send_[F.kind] : (const void*)d_recv_[F.kind]);
      b.n[nb] = n;
      b.nk[nb] = F.nk;
      b.p0[nb] = F.p[0];
      b.p1[nb] = F.p[1] ? F.p[1] : F.p[0];
      b.boff[nb] = stg ? (long)foff[f] : 0;
      maxn = std::max(maxn, n);
      maxk = std::max(maxk, F.nk);
      ++nb;
    }
    return nb;
  };
  for (int f0 = 0; f0 < nf; f0 += HB) {
    HaloBatch b{}, bl{};
    int maxn = 0, maxk = 0;
    const int nb = batch(stage == 3 ? 1 : stage, f0, b, maxn, maxk);
    const int nl = stage == 3 ? batch(0, f0, bl, maxn, maxk) : 0;
    if (!nb && !nl) continue;
    if ((long)cdiv(maxn, 256) * cdiv(maxk, 8) * (nb + nl) >= 2048) {  // >= 8 workgroups per CU at HK = 8
      const dim3 g(cdiv(maxn, 256), cdiv(maxk, 8), nb + nl);
      if (stage == 0) GT_LAUNCH_N("halo_local_kernel", halo_local_kernel<8>, g, dim3(256), 0, stream, b, d_.plane);
      else if (stage == 1) GT_LAUNCH_N("halo_pack_kernel", halo_pack_kernel<8>, g, dim3(256), 0, stream, b, d_.plane, sendbuf_);
      else if (stage == 2) GT_LAUNCH_N("halo_unpack_kernel", halo_unpack_kernel<8>, g, dim3(256), 0, stream, b, d_.plane, recvbuf_);
      else GT_LAUNCH_N("halo_pack_local_kernel", halo_pack_local_kernel<8>, g, dim3(256), 0, stream, b, nb, bl, d_.plane, sendbuf_);
    } else {
      const dim3 g(cdiv(maxn, 256), maxk, nb + nl);
      if (stage == 0) GT_LAUNCH_N("halo_local_kernel", halo_local_kernel<1>, g, dim3(256), 0, stream, b, d_.plane);
      else if (stage == 1) GT_LAUNCH_N("halo_pack_kernel", halo_pack_kernel<1>, g, dim3(256), 0, stream, b, d_.plane, sendbuf_);
      else if (stage == 2) GT_LAUNCH_N("halo_unpack_kernel", halo_unpack_kernel<1>, g, dim3(256), 0, stream, b, d_.plane, recvbuf_);
      else GT_LAUNCH_N("halo_pack_local_kernel", halo_pack_local_kernel<1>, g, dim3(256), 0, stream, b, nb, bl, d_.plane, sendbuf_);
    }
    HIP_LAUNCH_CHECK();
    // every halo point of every level: one value read, one written
    double pts = 0.0;
    for (int q = 0; q < nb; ++q) pts += (double)b.n[q] * b.nk[q];
    for (int q = 0; q < nl; ++q) pts += (double)bl.n[q] * bl.nk[q];
    ktimer_bytes(16.0 * pts);
  }
}

// the messages of an exchange, one NCCL group, on stream mst
void HaloExchanger::post_messages(const HaloField* fields, int nf, const std::vector<size_t>& foff, hipStream_t mst) {
  tr_->group_start();
  for (int f = 0; f < nf; ++f) {
    const HaloField& F = fields[f];
    for (int p = 0; p < nranks_; ++p) {
      int ns = send_peer_count_[F.kind][p], nr = recv_peer_count_[F.kind][p];
      if (ns) tr_->send(sendbuf_ + foff[f] + (size_t)send_peer_start_[F.kind][p] * F.nk, (size_t)ns * F.nk, p, mst);
      if (nr) tr_->recv(recvbuf_ + foff[f] + (size_t)recv_peer_start_[F.kind][p] * F.nk, (size_t)nr * F.nk, p, mst);
    }
  }
  tr_->group_end(mst);
}

void HaloExchanger::exchange(const HaloField* fields, int nf, hipStream_t stream) {
  if (pending_open_) throw std::runtime_error("halo: an exchange is still open (exchange_end missing)");
  if (!remote_) {
    launch_stage(0, fields, nf, {}, stream);
    return;
  }
  const std::vector<size_t> foff = buffer_offsets(fields, nf);
  // Default (GTFV3_HALO_FUSE=1): the pack and the same-rank gather in one launch, the
  // messages and the unpack after it, all on the exchange's own stream -- with nothing left
  // to overlap the messages with, a separate communication stream only added two cross-queue
  // hand-offs per exchange (pack -> messages -> unpack: ~13 us each in an 8-rank trace, 0.5 ms
  // per step).  GTFV3_HALO_FUSE=0: the round-4 form -- the pack, then the messages on the
  // communication stream while the gather runs on the compute stream, then the unpack.
  // Either way the next exchange's pack follows this unpack in stream order, so the pack
  // buffers are never rewritten while a send may still read them.
  static const bool fuse = [] {
    const char* e = std::getenv("GTFV3_HALO_FUSE");
    return !(e && e[0] == '0');
  }();
  hipStream_t mst = fuse ? stream : comm_st_;
  if (fuse) {
    launch_stage(3, fields, nf, foff, stream);
  } else {
    launch_stage(1, fields, nf, foff, stream);
    HIP_CHECK(hipEventRecord(ev_packed_, stream));
    launch_stage(0, fields, nf, foff, stream);
    HIP_CHECK(hipStreamWaitEvent(comm_st_, ev_packed_, 0));
  }
  post_messages(fields, nf, foff, mst);
  if (!fuse) {
    HIP_CHECK(hipEventRecord(ev_recvd_, comm_st_));
    HIP_CHECK(hipStreamWaitEvent(stream, ev_recvd_, 0));
  }
  launch_stage(2, fields, nf, foff, stream);
}

void HaloExchanger::exchange_begin(const HaloField* fields, int nf, hipStream_t stream) {
  if (pending_open_) throw std::runtime_error("halo: an exchange is still open (exchange_end missing)");
  if (!remote_) {
    launch_stage(0, fields, nf, {}, stream);
    return;
  }
  pending_.assign(fields, fields + nf);
  pending_off_ = buffer_offsets(fields, nf);
  pending_open_ = true;
  // the pack and the same-rank gather on the caller's stream, the messages on the
  // communication stream once the pack is done; the unpack waits for them in exchange_end
  launch_stage(3, fields, nf, pending_off_, stream);
  HIP_CHECK(hipEventRecord(ev_packed_, stream));
  HIP_CHECK(hipStreamWaitEvent(comm_st_, ev_packed_, 0));
  post_messages(fields, nf, pending_off_, comm_st_);
  HIP_CHECK(hipEventRecord(ev_recvd_, comm_st_));
}

void HaloExchanger::exchange_end(hipStream_t stream) {
  if (!pending_open_) return;
  HIP_CHECK(hipStreamWaitEvent(stream, ev_recvd_, 0));
  launch_stage(2, pending_.data(), (int)pending_.size(), pending_off_, stream);
  pending_open_ = false;
  pending_.clear();
}

}  // namespace gtfv3
