// grid.hpp — gnomonic equiangular cubed sphere, tile connectivity and FV3
// metric terms (Putman & Lin 2007; FV3 fv_grid_tools / fv_grid_utils
// restated).  Host code, run once at geos_gtfv3_init (the reference's init
// gets only npx/npy/npz/ntiles and the index bounds:
// example_def_dycore.yaml:4-20, so the dycore must build its own grid).
#pragma once
#include <array>
#include <vector>
#include "gtfv3.hpp"

namespace gtfv3 {

struct V3 {
  double x, y, z;
};

// Metric-term identifiers; the device holds them as [NMETRIC][nsub][plane].
enum Metric : int {
  M_AREA, M_RAREA, M_AREA_C, M_RAREA_C,
  M_DX, M_DY, M_DXA, M_DYA, M_DXC, M_DYC,
  M_RDX, M_RDY, M_RDXA, M_RDYA, M_RDXC, M_RDYC,
  M_SIN1, M_SIN2, M_SIN3, M_SIN4, M_SIN5, M_SIN6, M_SIN7, M_SIN8, M_SIN9,
  M_COS1, M_COS2, M_COS3, M_COS4, M_COS5, M_COS6, M_COS7, M_COS8, M_COS9,
  M_COSA_U, M_SINA_U, M_RSIN_U, M_COSA_V, M_SINA_V, M_RSIN_V,
  M_COSA_S, M_RSIN2, M_COSA, M_RSINA,
  M_FC, M_F0, M_A11, M_A12, M_A21, M_A22,
  M_LAT, M_LON,
  NMETRIC
};
extern const char* const kMetricNames[NMETRIC];

// Result of mapping a (doubled) lattice coordinate of one tile into the tile
// that owns it.  rot = number of +90 degree turns taking this tile's lattice
// directions to the owner's (vector components rotate with it).
struct Mapped {
  int t, x2, y2, rot;
  bool valid;  // false inside a cube-corner halo region (three tiles meet)
};

class CubedSphere {
 public:
  explicit CubedSphere(int N);
  int N;
  // own-tile corner point, 0 <= I,J <= N
  V3 tile_point(int t, int I, int J) const;
  // any lattice point; cube-corner regions use the copy_corners(XDir) rotation
  V3 point(int t, int I, int J) const;
  Mapped map(int t, int x2, int y2, bool geometry) const;
  // the point in the coordinates of the neighbour across `edge` (W,E,S,N = 0..3) even when it
  // lies on the edge itself (a shared edge point: its position in the neighbouring tile)
  Mapped map_across(int t, int edge, int x2, int y2) const;
  int neighbor(int t, int edge) const { return xf_[t][edge].nt; }
  int edge_rot(int t, int edge) const { return xf_[t][edge].rot; }

 private:
  struct Xf {
    int nt, rot, tx, ty;
  };
  Xf xf_[6][4];  // edge order W,E,S,N
  std::vector<double> tan_;
};

struct HostMetrics {
  Dims dims;
  // [NMETRIC][nsub][plane]
  std::vector<double> m;
  // cube-corner extrapolation weights for a2b_ord4: [nsub][4 corners][3]
  std::vector<double> corner_w;
  // corner points (x,y,z) per sub over i,j in [-NG-1, n+NG+1]: [nsub][(ny+2NG+3)][(nx+2NG+3)][3]
  std::vector<double> xyz;
  double da_min = 0, da_min_c = 0;
  double* at(int metric, int s) { return &m[((size_t)metric * dims.nsub + s) * dims.plane]; }
  const double* at(int metric, int s) const { return &m[((size_t)metric * dims.nsub + s) * dims.plane]; }
};

Dims make_dims(const Decomp& dc, int npz);
void build_metrics(const CubedSphere& cs, const Decomp& dc, const std::vector<SubInfo>& subs,
                   HostMetrics& out);

}  // namespace gtfv3
