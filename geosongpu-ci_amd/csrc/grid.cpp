// grid.cpp — cubed-sphere geometry and FV3 metric terms (host, init-time).
// Restated from the published FV3 grid construction (Putman & Lin 2007,
// "Finite-volume transport on various cubed-sphere grids"): equiangular
// gnomonic faces, great-circle edge lengths, spherical-excess areas, the
// nine-position sin/cos of the local grid angle (FV3 fv_grid_utils layout
//   9---4---8
//   |       |
//   1   5   3
//   |       |
//   6---2---7 ), and the C/D-grid non-orthogonality factors derived from them.
// Tile numbering/connectivity follows FV3 (odd tiles: E aligned, N rotated;
// even tiles: E rotated, N aligned); it is *derived* here by matching shared
// edge points, then checked.
#include "grid.hpp"

#include <algorithm>
#include <array>
#include <cmath>
#include <map>
#include <stdexcept>
#include <tuple>

namespace gtfv3 {

const char* const kMetricNames[NMETRIC] = {
    "area", "rarea", "area_c", "rarea_c", "dx", "dy", "dxa", "dya", "dxc", "dyc",
    "rdx", "rdy", "rdxa", "rdya", "rdxc", "rdyc",
    "sin_sg1", "sin_sg2", "sin_sg3", "sin_sg4", "sin_sg5", "sin_sg6", "sin_sg7", "sin_sg8", "sin_sg9",
    "cos_sg1", "cos_sg2", "cos_sg3", "cos_sg4", "cos_sg5", "cos_sg6", "cos_sg7", "cos_sg8", "cos_sg9",
    "cosa_u", "sina_u", "rsin_u", "cosa_v", "sina_v", "rsin_v",
    "cosa_s", "rsin2", "cosa", "rsina",
    "fC", "f0", "a11", "a12", "a21", "a22", "lat", "lon"};

namespace {
inline V3 add(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 scl(double s, V3 a) { return {s * a.x, s * a.y, s * a.z}; }
inline double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline V3 cross(V3 a, V3 b) {
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
inline double norm(V3 a) { return std::sqrt(dot(a, a)); }
inline V3 unit(V3 a) { return scl(1.0 / norm(a), a); }
// great-circle angle between unit vectors
inline double gc(V3 a, V3 b) { return std::atan2(norm(cross(a, b)), dot(a, b)); }
// spherical excess of triangle (unit sphere)
inline double tri(V3 a, V3 b, V3 c) {
  double num = std::fabs(dot(a, cross(b, c)));
  double den = 1.0 + dot(a, b) + dot(b, c) + dot(c, a);
  return 2.0 * std::atan2(num, den);
}
// unit tangent at p of the great circle through p towards q
inline V3 tangent(V3 p, V3 q) { return unit(sub(q, scl(dot(p, q), p))); }

struct Face {
  V3 c, ex, ey;
};
const Face kFaces[6] = {
    {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}},    {{0, 1, 0}, {-1, 0, 0}, {0, 0, 1}},
    {{0, 0, 1}, {-1, 0, 0}, {0, -1, 0}},  {{-1, 0, 0}, {0, 0, -1}, {0, -1, 0}},
    {{0, -1, 0}, {0, 0, -1}, {1, 0, 0}},  {{0, 0, -1}, {0, 1, 0}, {1, 0, 0}},
};

inline void rot_apply(int rot, int dx, int dy, int& ox, int& oy) {
  switch (rot & 3) {
    case 0: ox = dx; oy = dy; break;
    case 1: ox = -dy; oy = dx; break;
    case 2: ox = -dx; oy = -dy; break;
    default: ox = dy; oy = -dx; break;
  }
}
using Key = std::tuple<long, long, long>;
inline Key key_of(V3 p) {
  return Key(std::lround(p.x * 1e9), std::lround(p.y * 1e9), std::lround(p.z * 1e9));
}
}  // namespace

CubedSphere::CubedSphere(int N_) : N(N_) {
  if (N < 4) throw std::runtime_error("cubed sphere needs N >= 4");
  tan_.resize(N + 1);
  for (int i = 0; i <= N; ++i) {
    long m = 2L * i - N;  // alpha_i = m*pi/(4N): exactly antisymmetric
    double t = std::tan(std::fabs((double)m) * Constants::pi / (4.0 * N));
    tan_[i] = m < 0 ? -t : t;
  }
  std::map<Key, std::vector<std::array<int, 3>>> bmap;
  for (int t = 0; t < 6; ++t)
    for (int J = 0; J <= N; ++J)
      for (int I = 0; I <= N; ++I)
        if (I == 0 || J == 0 || I == N || J == N) bmap[key_of(tile_point(t, I, J))].push_back({t, I, J});
  const int ends[4][4] = {{0, 0, 0, N}, {N, 0, N, N}, {0, 0, N, 0}, {0, N, N, N}};
  for (int t = 0; t < 6; ++t) {
    for (int e = 0; e < 4; ++e) {
      int ax = ends[e][0], ay = ends[e][1], bx = ends[e][2], by = ends[e][3];
      const auto& la = bmap.at(key_of(tile_point(t, ax, ay)));
      const auto& lb = bmap.at(key_of(tile_point(t, bx, by)));
      int found = 0;
      for (const auto& a : la) {
        if (a[0] == t) continue;
        for (const auto& b : lb) {
          if (b[0] != a[0]) continue;
          int dx = (bx - ax) / N, dy = (by - ay) / N;
          int dxn = (b[1] - a[1]) / N, dyn = (b[2] - a[2]) / N;
          for (int r = 0; r < 4; ++r) {
            int ox, oy;
            rot_apply(r, dx, dy, ox, oy);
            if (ox == dxn && oy == dyn) {
              int rx, ry;
              rot_apply(r, 2 * ax, 2 * ay, rx, ry);
              xf_[t][e] = {a[0], r, 2 * a[1] - rx, 2 * a[2] - ry};
              ++found;
            }
          }
        }
      }
      if (found != 1) throw std::runtime_error("cubed-sphere connectivity: edge match failed");
    }
  }
  // check: every outward halo cell centre lands strictly inside the neighbour
  for (int t = 0; t < 6; ++t) {
    for (int k = 0; k < N; ++k) {
      int pts[4][2] = {{-1, 2 * k + 1}, {2 * N + 1, 2 * k + 1}, {2 * k + 1, -1}, {2 * k + 1, 2 * N + 1}};
      for (auto& p : pts) {
        Mapped m = map(t, p[0], p[1], false);
        if (!m.valid || m.x2 <= 0 || m.y2 <= 0 || m.x2 >= 2 * N || m.y2 >= 2 * N)
          throw std::runtime_error("cubed-sphere connectivity: halo does not map inside neighbour");
      }
    }
  }
}

V3 CubedSphere::tile_point(int t, int I, int J) const {
  const Face& f = kFaces[t];
  return unit(add(f.c, add(scl(tan_[I], f.ex), scl(tan_[J], f.ey))));
}

Mapped CubedSphere::map(int t, int x2, int y2, bool geometry) const {
  const int N2 = 2 * N;
  bool inx = x2 >= 0 && x2 <= N2, iny = y2 >= 0 && y2 <= N2;
  if (inx && iny) return {t, x2, y2, 0, true};
  if (!inx && !iny) {
    if (!geometry) return {t, x2, y2, 0, false};
    // rotate the cube-corner region about the corner into the x-side halo
    // (the XDir rule of FV3 copy_corners); geometry only.
    int nx2, ny2;
    if (x2 < 0 && y2 < 0) { nx2 = y2; ny2 = -x2; }
    else if (x2 > N2 && y2 < 0) { nx2 = N2 - y2; ny2 = x2 - N2; }
    else if (x2 > N2 && y2 > N2) { nx2 = y2; ny2 = 2 * N2 - x2; }
    else { nx2 = N2 - y2; ny2 = N2 + x2; }
    Mapped m = map(t, nx2, ny2, true);
    m.valid = false;
    return m;
  }
  int e = x2 < 0 ? 0 : (x2 > N2 ? 1 : (y2 < 0 ? 2 : 3));
  const Xf& xf = xf_[t][e];
  int rx, ry;
  rot_apply(xf.rot, x2, y2, rx, ry);
  Mapped m{xf.nt, rx + xf.tx, ry + xf.ty, xf.rot, true};
  if (m.x2 < 0 || m.y2 < 0 || m.x2 > N2 || m.y2 > N2)
    throw std::runtime_error("cubed-sphere map: halo deeper than a neighbour tile");
  return m;
}

Mapped CubedSphere::map_across(int t, int edge, int x2, int y2) const {
  const Xf& xf = xf_[t][edge];
  int rx, ry;
  rot_apply(xf.rot, x2, y2, rx, ry);
  return Mapped{xf.nt, rx + xf.tx, ry + xf.ty, xf.rot, true};
}

V3 CubedSphere::point(int t, int I, int J) const {
  Mapped m = map(t, 2 * I, 2 * J, true);
  return tile_point(m.t, m.x2 / 2, m.y2 / 2);
}

SubInfo Decomp::sub(int gid) const {
  SubInfo s{};
  int per_tile = lx * ly;
  s.tile = gid / per_tile;
  int r = gid % per_tile;
  int px = r % lx, py = r / lx;
  s.ioff = px * sub_nx();
  s.joff = py * sub_ny();
  s.N = N;
  s.flags = (px == 0 ? EDGE_W : 0) | (px == lx - 1 ? EDGE_E : 0) | (py == 0 ? EDGE_S : 0) |
            (py == ly - 1 ? EDGE_N : 0);
  s.gid = gid;
  return s;
}

Dims make_dims(const Decomp& dc, int npz) {
  Dims d{};
  d.nx = dc.sub_nx();
  d.ny = dc.sub_ny();
  int ni = d.nx + 2 * NG + 1;
  d.pitch = (ni + 7) / 8 * 8;
  d.nj = d.ny + 2 * NG + 1;
  d.plane = (long)d.pitch * d.nj;
  d.nsub = dc.nsub_per_rank();
  d.npz = npz;
  return d;
}

void build_metrics(const CubedSphere& cs, const Decomp& dc, const std::vector<SubInfo>& subs,
                   HostMetrics& out) {
  const double R = Constants::radius;
  const double tiny = 1.0e-14;
  const int N = cs.N;
  Dims d = out.dims;
  out.m.assign((size_t)NMETRIC * d.nsub * d.plane, 0.0);
  out.corner_w.assign((size_t)d.nsub * 12, 0.0);
  const int H = NG + 1;
  const int wx = d.nx + 2 * H + 1, wy = d.ny + 2 * H + 1;
  out.xyz.assign((size_t)d.nsub * wx * wy * 3, 0.0);

  for (int s = 0; s < d.nsub; ++s) {
    const SubInfo& si = subs[s];
    std::vector<V3> P((size_t)wx * wy), A((size_t)wx * wy);
    auto PI = [&](int i, int j) -> V3& { return P[(size_t)(j + H) * wx + (i + H)]; };
    auto AI = [&](int i, int j) -> V3& { return A[(size_t)(j + H) * wx + (i + H)]; };
    for (int j = -H; j <= d.ny + H; ++j)
      for (int i = -H; i <= d.nx + H; ++i) {
        V3 p = cs.point(si.tile, i + si.ioff, j + si.joff);
        PI(i, j) = p;
        double* x = &out.xyz[(((size_t)s * wy + (j + H)) * wx + (i + H)) * 3];
        x[0] = p.x; x[1] = p.y; x[2] = p.z;
      }
    for (int j = -H; j < d.ny + H; ++j)
      for (int i = -H; i < d.nx + H; ++i)
        AI(i, j) = unit(add(add(PI(i, j), PI(i + 1, j)), add(PI(i, j + 1), PI(i + 1, j + 1))));

    auto cube_corner_cell = [&](int i, int j) {
      int I = i + si.ioff, J = j + si.joff;
      return (I < 0 || I >= N) && (J < 0 || J >= N);
    };
    auto M = [&](int metric, int i, int j) -> double& {
      return out.at(metric, s)[(size_t)(j + NG) * d.pitch + (i + NG)];
    };
    // per-cell angle terms (needed before the averaged factors)
    for (int j = -NG; j <= d.ny + NG; ++j)
      for (int i = -NG; i <= d.nx + NG; ++i) {
        V3 p00 = PI(i, j), p10 = PI(i + 1, j), p01 = PI(i, j + 1), p11 = PI(i + 1, j + 1);
        V3 w = unit(add(p00, p01)), e = unit(add(p10, p11));
        V3 so = unit(add(p00, p10)), no = unit(add(p01, p11));
        V3 c = AI(i, j);
        double cs_[9];
        cs_[0] = dot(tangent(w, e), tangent(w, p01));                       // 1 W
        cs_[1] = dot(tangent(so, p10), tangent(so, no));                    // 2 S
        cs_[2] = dot(scl(-1.0, tangent(e, w)), tangent(e, p11));            // 3 E
        cs_[3] = dot(tangent(no, p11), scl(-1.0, tangent(no, so)));         // 4 N
        V3 ex = unit(sub(tangent(c, e), tangent(c, w)));
        V3 ey = unit(sub(tangent(c, no), tangent(c, so)));
        cs_[4] = dot(ex, ey);                                               // 5 C
        cs_[5] = dot(tangent(p00, p10), tangent(p00, p01));                 // 6 SW
        cs_[6] = dot(scl(-1.0, tangent(p10, p00)), tangent(p10, p11));      // 7 SE
        cs_[7] = dot(scl(-1.0, tangent(p11, p01)), scl(-1.0, tangent(p11, p10)));  // 8 NE
        cs_[8] = dot(tangent(p01, p11), scl(-1.0, tangent(p01, p00)));      // 9 NW
        for (int q = 0; q < 9; ++q) {
          M(M_COS1 + q, i, j) = cs_[q];
          M(M_SIN1 + q, i, j) = std::min(1.0, std::sqrt(std::max(0.0, 1.0 - cs_[q] * cs_[q])));
        }
        // lengths
        M(M_DX, i, j) = R * gc(p00, p10);
        M(M_DY, i, j) = R * gc(p00, p01);
        M(M_DXA, i, j) = R * gc(w, e);
        M(M_DYA, i, j) = R * gc(so, no);
        M(M_DXC, i, j) = R * gc(AI(i - 1, j), c);
        M(M_DYC, i, j) = R * gc(AI(i, j - 1), c);
        M(M_AREA, i, j) = R * R * (tri(p00, p10, p11) + tri(p00, p11, p01));
        M(M_AREA_C, i, j) = R * R * (tri(AI(i - 1, j - 1), AI(i, j - 1), c) + tri(AI(i - 1, j - 1), c, AI(i - 1, j)));
        M(M_FC, i, j) = 2.0 * Constants::omega * p00.z;
        M(M_F0, i, j) = 2.0 * Constants::omega * c.z;
        M(M_LAT, i, j) = std::asin(std::max(-1.0, std::min(1.0, c.z)));
        M(M_LON, i, j) = std::atan2(c.y, c.x);
        // covariant (along grid lines) -> (east, north), scaled by 1/2 for c2l_ord4
        V3 zhat{0, 0, 1};
        V3 ce = cross(zhat, c);
        V3 eE = norm(ce) < 1e-12 ? V3{0, 1, 0} : unit(ce);
        V3 eN = cross(c, eE);
        double m11 = dot(ex, eE), m12 = dot(ex, eN), m21 = dot(ey, eE), m22 = dot(ey, eN);
        double det = m11 * m22 - m12 * m21;
        M(M_A11, i, j) = 0.5 * m22 / det;
        M(M_A12, i, j) = -0.5 * m12 / det;
        M(M_A21, i, j) = -0.5 * m21 / det;
        M(M_A22, i, j) = 0.5 * m11 / det;
      }
    // cube-corner dual cells are triangles of the three cells meeting there
    const int cc[4][2] = {{0, 0}, {N, 0}, {N, N}, {0, N}};
    for (int q = 0; q < 4; ++q) {
      int i = cc[q][0] - si.ioff, j = cc[q][1] - si.joff;
      if (i < -NG || i > d.nx + NG || j < -NG || j > d.ny + NG) continue;
      V3 a, b, c;
      if (q == 0) { a = AI(0 + i, 0 + j); b = AI(i - 1, j); c = AI(i, j - 1); }
      else if (q == 1) { a = AI(i - 1, j); b = AI(i, j); c = AI(i - 1, j - 1); }
      else if (q == 2) { a = AI(i - 1, j - 1); b = AI(i, j - 1); c = AI(i - 1, j); }
      else { a = AI(i, j - 1); b = AI(i - 1, j - 1); c = AI(i, j); }
      M(M_AREA_C, i, j) = R * R * tri(a, b, c);
    }
    // averaged non-orthogonality factors (ignore cube-corner-region cells)
    for (int j = -NG; j <= d.ny + NG; ++j)
      for (int i = -NG; i <= d.nx + NG; ++i) {
        auto avg = [&](int m1, int i1, int j1, int m2, int i2, int j2) {
          bool ok1 = i1 >= -NG && j1 >= -NG && !cube_corner_cell(i1, j1);
          bool ok2 = !cube_corner_cell(i2, j2);
          if (ok1 && ok2) return 0.5 * (M(m1, i1, j1) + M(m2, i2, j2));
          if (ok1) return M(m1, i1, j1);
          return M(m2, i2, j2);
        };
        M(M_COSA_U, i, j) = avg(M_COS3, i - 1, j, M_COS1, i, j);
        M(M_SINA_U, i, j) = avg(M_SIN3, i - 1, j, M_SIN1, i, j);
        M(M_RSIN_U, i, j) = 1.0 / std::max(tiny, M(M_SINA_U, i, j) * M(M_SINA_U, i, j));
        M(M_COSA_V, i, j) = avg(M_COS4, i, j - 1, M_COS2, i, j);
        M(M_SINA_V, i, j) = avg(M_SIN4, i, j - 1, M_SIN2, i, j);
        M(M_RSIN_V, i, j) = 1.0 / std::max(tiny, M(M_SINA_V, i, j) * M(M_SINA_V, i, j));
        M(M_COSA_S, i, j) = M(M_COS5, i, j);
        M(M_RSIN2, i, j) = 1.0 / std::max(tiny, M(M_SIN5, i, j) * M(M_SIN5, i, j));
        double ca = avg(M_COS8, i - 1, j - 1, M_COS6, i, j);
        M(M_COSA, i, j) = ca;
        M(M_RSINA, i, j) = 1.0 / std::max(tiny, 1.0 - ca * ca);
        M(M_RAREA, i, j) = 1.0 / M(M_AREA, i, j);
        M(M_RAREA_C, i, j) = 1.0 / M(M_AREA_C, i, j);
        M(M_RDX, i, j) = 1.0 / M(M_DX, i, j);
        M(M_RDY, i, j) = 1.0 / M(M_DY, i, j);
        M(M_RDXA, i, j) = 1.0 / M(M_DXA, i, j);
        M(M_RDYA, i, j) = 1.0 / M(M_DYA, i, j);
        M(M_RDXC, i, j) = 1.0 / M(M_DXC, i, j);
        M(M_RDYC, i, j) = 1.0 / M(M_DYC, i, j);
      }
    // a2b_ord4 cube-corner extrapolation weights (extrap_corner: q1 + x1/(x2-x1)*(q1-q2))
    const int pairs[4][3][4] = {
        {{0, 0, 1, 1}, {-1, 0, -2, 1}, {0, -1, 1, -2}},
        {{N - 1, 0, N - 2, 1}, {N - 1, -1, N - 2, -2}, {N, 0, N + 1, 1}},
        {{N - 1, N - 1, N - 2, N - 2}, {N, N - 1, N + 1, N - 2}, {N - 1, N, N - 2, N + 1}},
        {{0, N - 1, 1, N - 2}, {-1, N - 1, -2, N - 2}, {0, N, 1, N + 1}}};
    for (int q = 0; q < 4; ++q) {
      int i0 = cc[q][0] - si.ioff, j0 = cc[q][1] - si.joff;
      bool has = (i0 >= 0 && i0 <= d.nx && j0 >= 0 && j0 <= d.ny);
      if (!has) continue;
      V3 p0 = PI(i0, j0);
      for (int r = 0; r < 3; ++r) {
        V3 p1 = AI(pairs[q][r][0] - si.ioff, pairs[q][r][1] - si.joff);
        V3 p2 = AI(pairs[q][r][2] - si.ioff, pairs[q][r][3] - si.joff);
        double x1 = gc(p1, p0), x2 = gc(p2, p0);
        out.corner_w[(size_t)s * 12 + q * 3 + r] = x1 / (x2 - x1);
      }
    }
  }
  // global minimum cell / dual-cell areas (da_min, da_min_c) over all 6 tiles
  double amin = 1e300, acmin = 1e300;
  for (int t = 0; t < 6; ++t) {
    std::vector<V3> P((size_t)(N + 3) * (N + 3));
    auto PP = [&](int I, int J) -> V3& { return P[(size_t)(J + 1) * (N + 3) + (I + 1)]; };
    for (int J = -1; J <= N + 1; ++J)
      for (int I = -1; I <= N + 1; ++I) PP(I, J) = cs.point(t, I, J);
    std::vector<V3> C((size_t)(N + 2) * (N + 2));
    auto CC = [&](int I, int J) -> V3& { return C[(size_t)(J + 1) * (N + 2) + (I + 1)]; };
    for (int J = -1; J <= N; ++J)
      for (int I = -1; I <= N; ++I)
        CC(I, J) = unit(add(add(PP(I, J), PP(I + 1, J)), add(PP(I, J + 1), PP(I + 1, J + 1))));
    for (int J = 0; J < N; ++J)
      for (int I = 0; I < N; ++I)
        amin = std::min(amin, R * R * (tri(PP(I, J), PP(I + 1, J), PP(I + 1, J + 1)) +
                                       tri(PP(I, J), PP(I + 1, J + 1), PP(I, J + 1))));
    for (int J = 1; J < N; ++J)
      for (int I = 1; I < N; ++I)
        acmin = std::min(acmin, R * R * (tri(CC(I - 1, J - 1), CC(I, J - 1), CC(I, J)) +
                                         tri(CC(I - 1, J - 1), CC(I, J), CC(I - 1, J))));
  }
  out.da_min = amin;
  out.da_min_c = acmin;
  (void)dc;
}

}  // namespace gtfv3
