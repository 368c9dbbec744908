"""Oracle: equiangular gnomonic cubed-sphere grid and the FV3 metric terms, fp64 numpy.
TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Written from the published construction, independently of the product's grid.cpp, so that
the dycore oracle no longer has to take its metric terms from the code it checks:

* Putman & Lin (2007), J. Comput. Phys. 227, "Finite-volume transport on various
  cubed-sphere grids", section 2: the equiangular gnomonic face, grid lines at the central
  angles alpha_i = -pi/4 + i pi/(2N), the point of face coordinates (alpha, beta) being the
  unit vector along c + tan(alpha) e_x + tan(beta) e_y of the face (centre c, axes e_x, e_y);
  cell centres, edge midpoints and lengths on great circles; cell areas as spherical
  excesses.
* FV3's metric terms (fv_grid_tools / fv_grid_utils as documented in Harris et al. 2021,
  "A scientific description of the GFDL FV3 dynamical core", section 3): dx, dy along the
  cell edges; dxa, dya between edge midpoints; dxc, dyc between cell centres; area and the
  dual-cell area_c around a corner (a triangle of three cells at a cube corner); the local
  grid-angle cosines at the nine positions 1 W, 2 S, 3 E, 4 N, 5 centre, 6 SW, 7 SE, 8 NE,
  9 NW with sin = sqrt(1 - cos^2); the C/D-grid factors cosa_u / sina_u, cosa_v / sina_v
  (the two cells sharing an edge averaged), cosa (corner, from positions 8 and 6), cosa_s /
  rsin2 (centre), the Coriolis parameter at corners (fC) and centres (f0), and the
  covariant-to-(east, north) matrix used by cubed_to_latlon.
* Halo geometry: a halo point is the grid point of the neighbour tile that owns it (tile
  connectivity from FV3's rule table, oracle/halo.py `locate`), and a cube-corner halo
  point is first rotated about the cube corner into the x-side halo (FV3 fill_corners XDir).

Arithmetic deliberately differs from grid.cpp where the quantity allows it: great-circle
lengths from the chord (2 asin(|a - b| / 2)) instead of atan2(|a x b|, a.b); cell areas
split along the other diagonal and summed by L'Huilier's theorem instead of the Van
Oosterom-Strackee triangle formula; grid angles from the normals of the two great-circle
planes instead of projected tangents; latitude from atan2(z, rho).  Agreement with the
product to ~1e-13 therefore checks the construction, not a shared code path.
"""
import numpy as np

from . import NG
from .halo import locate

RADIUS = 6371.0e3
OMEGA = 2.0 * np.pi / 86164.0  # GEOS MAPL_OMEGA (sidereal day)
TINY = 1.0e-14
H = NG + 1  # corner-point halo (cell metrics need corners -NG-1 .. n+NG+1)

# Face centres and axes (convention shared with the product so the two grids can be compared
# point by point; `check_connectivity` verifies that it realises FV3's rule table)
FACES = [
    ((1, 0, 0), (0, 1, 0), (0, 0, 1)),
    ((0, 1, 0), (-1, 0, 0), (0, 0, 1)),
    ((0, 0, 1), (-1, 0, 0), (0, -1, 0)),
    ((-1, 0, 0), (0, 0, -1), (0, -1, 0)),
    ((0, -1, 0), (0, 0, -1), (1, 0, 0)),
    ((0, 0, -1), (0, 1, 0), (1, 0, 0)),
]
METRICS = ["area", "rarea", "area_c", "rarea_c", "dx", "dy", "dxa", "dya", "dxc", "dyc", "rdx", "rdy", "rdxa",
           "rdya", "rdxc", "rdyc"] + [f"sin_sg{i}" for i in range(1, 10)] + [f"cos_sg{i}" for i in range(1, 10)] + \
    ["cosa_u", "sina_u", "rsin_u", "cosa_v", "sina_v", "rsin_v", "cosa_s", "rsin2", "cosa", "rsina", "fC", "f0", "a11",
     "a12", "a21", "a22", "lat", "lon"]


def _unit(v):
    """v / |v| as v * (1 / sqrt(x x + y y + z z)): the point construction rounds exactly like
    the product's, so the points themselves (and the degenerate cube-corner halo cells built
    from them, see subdomain_metrics) agree bit for bit; the metric formulas stay distinct"""
    n2 = v[..., 0] * v[..., 0] + v[..., 1] * v[..., 1] + v[..., 2] * v[..., 2]
    return v * (1.0 / np.sqrt(n2))[..., None]


def _dot(a, b):
    return np.sum(a * b, axis=-1)


def grid_tangents(N):
    """tan(alpha_i), alpha_i = (2i - N) pi / (4N), i = 0..N, exactly antisymmetric"""
    import math
    m = 2 * np.arange(N + 1) - N
    return np.array([math.copysign(math.tan(abs(int(k)) * math.pi / (4.0 * N)), k) if k else 0.0 for k in m])


def face_point(t, tx, ty):
    c, ex, ey = (np.array(v, dtype=np.float64) for v in FACES[t])
    return _unit(c + (np.multiply.outer(tx, ex) + np.multiply.outer(ty, ey)))


def corner_point(t, I, J, N, tg):
    """grid point (I, J) of tile t (halo included) as a unit vector"""
    X2, Y2 = 2 * I, 2 * J
    N2 = 2 * N
    if (X2 < 0 or X2 > N2) and (Y2 < 0 or Y2 > N2):
        # cube-corner halo: rotate about the corner into the x-side halo (fill_corners XDir)
        if X2 < 0 and Y2 < 0:
            X2, Y2 = Y2, -X2
        elif X2 > N2 and Y2 < 0:
            X2, Y2 = N2 - Y2, X2 - N2
        elif X2 > N2 and Y2 > N2:
            X2, Y2 = Y2, 2 * N2 - X2
        else:
            X2, Y2 = N2 - Y2, N2 + X2
    t2, X2, Y2, _ = locate(t, X2, Y2, N)
    return face_point(t2, tg[X2 // 2], tg[Y2 // 2])


def check_connectivity(N):
    """largest distance between a tile's edge corner points and the corners of the halo
    cells across that edge, as the rule table places them in the neighbour tile (zero when
    FACES realises FV3's connectivity)"""
    tg = grid_tangents(N)
    worst = 0.0
    for t in range(6):
        for k in range(N):
            for cx2, cy2, e0, e1 in ((-1, 2 * k + 1, (0, 2 * k), (0, 2 * k + 2)),
                                     (2 * N + 1, 2 * k + 1, (2 * N, 2 * k), (2 * N, 2 * k + 2)),
                                     (2 * k + 1, -1, (2 * k, 0), (2 * k + 2, 0)),
                                     (2 * k + 1, 2 * N + 1, (2 * k, 2 * N), (2 * k + 2, 2 * N))):
                t2, X, Y, _ = locate(t, cx2, cy2, N)
                nbr = [face_point(t2, tg[(X + dx) // 2], tg[(Y + dy) // 2]) for dx in (-1, 1) for dy in (-1, 1)]
                for ex2, ey2 in (e0, e1):
                    own = face_point(t, tg[ex2 // 2], tg[ey2 // 2])
                    worst = max(worst, min(float(np.linalg.norm(own - q)) for q in nbr))
    return worst


def gc(a, b):
    """great-circle angle between unit vectors, from the chord"""
    return 2.0 * np.arcsin(np.clip(0.5 * np.linalg.norm(a - b, axis=-1), 0.0, 1.0))


def tri_lhuilier(a, b, c):
    """spherical excess of the triangle abc on the unit sphere (L'Huilier)"""
    x, y, z = gc(b, c), gc(c, a), gc(a, b)
    s = 0.5 * (x + y + z)
    t = np.tan(0.5 * s) * np.tan(0.5 * (s - x)) * np.tan(0.5 * (s - y)) * np.tan(0.5 * (s - z))
    return 4.0 * np.arctan(np.sqrt(np.maximum(t, 0.0)))


def tri_vos(a, b, c):
    """spherical excess by the Van Oosterom-Strackee formula (used only for the degenerate
    cube-corner halo cells, where the product's split of the quadrilateral is the convention)"""
    num = np.abs(_dot(a, np.cross(b, c)))
    den = 1.0 + _dot(a, b) + _dot(b, c) + _dot(c, a)
    return 2.0 * np.arctan2(num, den)


def cos_at(p, q1, q2, s1=1.0, s2=1.0):
    """cosine of the angle at p between the great circles towards q1 and q2 (s = -1: the
    direction away from that point), from the normals of the two great-circle planes"""
    n1 = np.cross(p, q1)
    n2 = np.cross(p, q2)
    return s1 * s2 * _dot(n1, n2) / (np.linalg.norm(n1, axis=-1) * np.linalg.norm(n2, axis=-1))


def subdomain_metrics(tile, ioff, joff, nx, ny, N, pitch, nj):
    """{metric: (nj, pitch) plane} for one sub-domain, filled over i, j in [-NG, n + NG] like
    the product's planes (the rest zero), plus 'corner_w' (4, 3) cube-corner extrapolation
    weights of a2b_ord4 and the corner points 'xyz'"""
    tg = grid_tangents(N)
    R = RADIUS
    ii = np.arange(-H, nx + H + 1)
    jj = np.arange(-H, ny + H + 1)
    P = np.array([[corner_point(tile, i + ioff, j + joff, N, tg) for i in ii] for j in jj])  # [j+H, i+H]
    A = _unit((P[:-1, :-1] + P[:-1, 1:]) + (P[1:, :-1] + P[1:, 1:]))  # cell centres [j+H, i+H]

    # the cells (i, j) of the metric region, i, j in [-NG, n+NG]
    ci = np.arange(-NG, nx + NG + 1)
    cj = np.arange(-NG, ny + NG + 1)
    J_, I_ = np.meshgrid(cj, ci, indexing="ij")
    Pc = lambda di, dj: P[J_ + H + dj, I_ + H + di]
    Ac = lambda di, dj: A[J_ + H + dj, I_ + H + di]
    p00, p10, p01, p11 = Pc(0, 0), Pc(1, 0), Pc(0, 1), Pc(1, 1)
    w, e = _unit(p00 + p01), _unit(p10 + p11)
    so, no = _unit(p00 + p10), _unit(p01 + p11)
    c = Ac(0, 0)
    out = {}
    cs = {}
    cs[1] = cos_at(w, e, p01)
    cs[2] = cos_at(so, p10, no)
    cs[3] = cos_at(e, w, p11, s1=-1.0)
    cs[4] = cos_at(no, p11, so, s2=-1.0)
    # centre: the x direction bisects "towards the east midpoint" and "away from the west
    # one" (likewise y), each the unit tangent of its great circle at c
    def tang(p, q):
        t = np.cross(np.cross(p, q), p)
        return _unit(t)
    exv = _unit(tang(c, e) - tang(c, w))
    eyv = _unit(tang(c, no) - tang(c, so))
    GI, GJ = I_ + ioff, J_ + joff
    cc_cell = ((GI < 0) | (GI >= N)) & ((GJ < 0) | (GJ >= N))
    if cc_cell.any():  # degenerate cube-corner halo cells: the product's projected tangents
        tproj = lambda p, q: _unit(q - _dot(p, q)[..., None] * p)
        exv = np.where(cc_cell[..., None], _unit(tproj(c, e) - tproj(c, w)), exv)
        eyv = np.where(cc_cell[..., None], _unit(tproj(c, no) - tproj(c, so)), eyv)
    cs[5] = _dot(exv, eyv)
    cs[6] = cos_at(p00, p10, p01)
    cs[7] = cos_at(p10, p00, p11, s1=-1.0)
    cs[8] = cos_at(p11, p01, p10, s1=-1.0, s2=-1.0)
    cs[9] = cos_at(p01, p11, p00, s2=-1.0)
    # Cube-corner halo cells (both tile indices outside 0..N-1) are degenerate quadrilaterals of
    # rotated halo points (fill_corners): there the values are a convention, not a geometric
    # quantity, and the oracle adopts the product's (projected tangents, the p00-p11 diagonal)
    if cc_cell.any():
        tproj = lambda p, q: _unit(q - _dot(p, q)[..., None] * p)
        tdot = lambda p, q1, q2, s1=1.0, s2=1.0: s1 * s2 * _dot(tproj(p, q1), tproj(p, q2))
        for q_, (pp, q1, q2, a1, a2) in {6: (p00, p10, p01, 1, 1), 7: (p10, p00, p11, -1, 1),
                                          8: (p11, p01, p10, -1, -1), 9: (p01, p11, p00, 1, -1),
                                          1: (w, e, p01, 1, 1), 2: (so, p10, no, 1, 1),
                                          3: (e, w, p11, -1, 1), 4: (no, p11, so, 1, -1)}.items():
            cs[q_] = np.where(cc_cell, tdot(pp, q1, q2, a1, a2), cs[q_])
    for q in range(1, 10):
        out[f"cos_sg{q}"] = cs[q]
        out[f"sin_sg{q}"] = np.minimum(1.0, np.sqrt(np.maximum(0.0, 1.0 - cs[q] ** 2)))
    out["dx"] = R * gc(p00, p10)
    out["dy"] = R * gc(p00, p01)
    out["dxa"] = R * gc(w, e)
    out["dya"] = R * gc(so, no)
    out["dxc"] = R * gc(Ac(-1, 0), c)
    out["dyc"] = R * gc(Ac(0, -1), c)
    out["area"] = R * R * np.where(cc_cell, tri_vos(p00, p10, p11) + tri_vos(p00, p11, p01),
                                   tri_lhuilier(p00, p10, p01) + tri_lhuilier(p10, p11, p01))
    a_sw, a_se, a_ne, a_nw = Ac(-1, -1), Ac(0, -1), c, Ac(-1, 0)
    # a dual cell touching a cube-corner halo cell: the product's (sw-ne) diagonal, see above
    touch = cc_cell.copy()
    GI_l, GJ_l = GI - 1, GJ - 1
    touch |= ((GI_l < 0) | (GI_l >= N)) & ((GJ_l < 0) | (GJ_l >= N))
    touch |= ((GI < 0) | (GI >= N)) & ((GJ_l < 0) | (GJ_l >= N))
    touch |= ((GI_l < 0) | (GI_l >= N)) & ((GJ < 0) | (GJ >= N))
    area_c = R * R * np.where(touch, tri_vos(a_sw, a_se, a_ne) + tri_vos(a_sw, a_ne, a_nw),
                              tri_lhuilier(a_sw, a_se, a_nw) + tri_lhuilier(a_se, a_ne, a_nw))
    # cube corners: the dual cell is the triangle of the three cells meeting there
    for (CI, CJ) in ((0, 0), (N, 0), (N, N), (0, N)):
        i, j = CI - ioff, CJ - joff
        if -NG <= i <= nx + NG and -NG <= j <= ny + NG:
            cells = [(i + di, j + dj) for di in (-1, 0) for dj in (-1, 0)
                     if not ((i + di + ioff < 0 or i + di + ioff >= N) and (j + dj + joff < 0 or j + dj + joff >= N))]
            pts = [A[cj_ + H, ci_ + H] for ci_, cj_ in cells]
            area_c[j + NG, i + NG] = R * R * tri_lhuilier(*pts)
    out["area_c"] = area_c
    out["fC"] = 2.0 * OMEGA * p00[..., 2]
    out["f0"] = 2.0 * OMEGA * c[..., 2]
    out["lat"] = np.arctan2(c[..., 2], np.hypot(c[..., 0], c[..., 1]))
    out["lon"] = np.arctan2(c[..., 1], c[..., 0])
    zhat = np.array([0.0, 0.0, 1.0])
    ce = np.cross(np.broadcast_to(zhat, c.shape), c)
    pole = np.linalg.norm(ce, axis=-1) < 1e-12
    eE = np.where(pole[..., None], np.array([0.0, 1.0, 0.0]), _unit(np.where(pole[..., None], 1.0, ce)))
    eN = np.cross(c, eE)
    Mx = np.stack([np.stack([_dot(exv, eE), _dot(exv, eN)], -1), np.stack([_dot(eyv, eE), _dot(eyv, eN)], -1)], -2)
    # inverse by Cramer's rule (degenerate cube-corner halo cells give inf / nan, not an error)
    with np.errstate(all="ignore"):
        det = Mx[..., 0, 0] * Mx[..., 1, 1] - Mx[..., 0, 1] * Mx[..., 1, 0]
        out["a11"], out["a12"] = 0.5 * Mx[..., 1, 1] / det, -0.5 * Mx[..., 0, 1] / det
        out["a21"], out["a22"] = -0.5 * Mx[..., 1, 0] / det, 0.5 * Mx[..., 0, 0] / det

    # edge / corner averages over the cells sharing the point, cube-corner-region cells left out
    G_I, G_J = I_ + ioff, J_ + joff
    corner_cell = ((G_I < 0) | (G_I >= N)) & ((G_J < 0) | (G_J >= N))

    def shifted(a, di, dj, fill=np.nan):
        o = np.full_like(a, fill)
        js, je = max(0, -dj), a.shape[0] - max(0, dj)
        is_, ie = max(0, -di), a.shape[1] - max(0, di)
        o[js:je, is_:ie] = a[js + dj:je + dj, is_ + di:ie + di]
        return o

    def avg(a1, di, dj, a2):
        """0.5 (a1 at the neighbour cell (i+di, j+dj) + a2 here), one-sided where a cell is in
        a cube-corner region or the neighbour is outside the metric region"""
        n1 = shifted(a1, di, dj)
        ok1 = ~np.isnan(n1) & ~shifted(corner_cell, di, dj, True).astype(bool)
        ok2 = ~corner_cell
        return np.where(ok1 & ok2, 0.5 * (np.where(ok1, n1, 0.0) + a2), np.where(ok1, np.where(ok1, n1, 0.0), a2))

    out["cosa_u"] = avg(out["cos_sg3"], -1, 0, out["cos_sg1"])
    out["sina_u"] = avg(out["sin_sg3"], -1, 0, out["sin_sg1"])
    out["rsin_u"] = 1.0 / np.maximum(TINY, out["sina_u"] ** 2)
    out["cosa_v"] = avg(out["cos_sg4"], 0, -1, out["cos_sg2"])
    out["sina_v"] = avg(out["sin_sg4"], 0, -1, out["sin_sg2"])
    out["rsin_v"] = 1.0 / np.maximum(TINY, out["sina_v"] ** 2)
    out["cosa_s"] = out["cos_sg5"]
    out["rsin2"] = 1.0 / np.maximum(TINY, out["sin_sg5"] ** 2)
    out["cosa"] = avg(out["cos_sg8"], -1, -1, out["cos_sg6"])
    out["rsina"] = 1.0 / np.maximum(TINY, 1.0 - out["cosa"] ** 2)
    for n in ("area", "area_c", "dx", "dy", "dxa", "dya", "dxc", "dyc"):
        out["r" + n] = 1.0 / out[n]
    planes = {}
    for n in METRICS:
        pl = np.zeros((nj, pitch))
        pl[:ny + 2 * NG + 1, :nx + 2 * NG + 1] = out[n]
        planes[n] = pl
    # a2b_ord4 cube-corner extrapolation weights x1 / (x2 - x1) along the three pairs of cell
    # centres leaving each cube corner (extrap_corner)
    cw = np.zeros((4, 3))
    pairs = [[(0, 0, 1, 1), (-1, 0, -2, 1), (0, -1, 1, -2)],
             [(N - 1, 0, N - 2, 1), (N - 1, -1, N - 2, -2), (N, 0, N + 1, 1)],
             [(N - 1, N - 1, N - 2, N - 2), (N, N - 1, N + 1, N - 2), (N - 1, N, N - 2, N + 1)],
             [(0, N - 1, 1, N - 2), (-1, N - 1, -2, N - 2), (0, N, 1, N + 1)]]
    for q, (CI, CJ) in enumerate(((0, 0), (N, 0), (N, N), (0, N))):
        i0, j0 = CI - ioff, CJ - joff
        if not (0 <= i0 <= nx and 0 <= j0 <= ny):
            continue
        p0 = P[j0 + H, i0 + H]
        for r, (a1, b1, a2, b2) in enumerate(pairs[q]):
            x1 = gc(A[b1 - joff + H, a1 - ioff + H], p0)
            x2 = gc(A[b2 - joff + H, a2 - ioff + H], p0)
            cw[q, r] = x1 / (x2 - x1)
    planes["corner_w"] = cw
    planes["xyz"] = P
    return planes


def min_areas(N):
    """(da_min, da_min_c): the smallest cell area and interior dual-cell area over the sphere"""
    tg = grid_tangents(N)
    amin, acmin = np.inf, np.inf
    for t in range(6):
        P = face_point(t, tg[None, :], tg[:, None])  # [J, I]
        a = RADIUS ** 2 * (tri_lhuilier(P[:-1, :-1], P[:-1, 1:], P[1:, :-1]) +
                           tri_lhuilier(P[:-1, 1:], P[1:, 1:], P[1:, :-1]))
        amin = min(amin, float(a.min()))
        C = _unit(P[:-1, :-1] + P[:-1, 1:] + P[1:, :-1] + P[1:, 1:])
        ac = RADIUS ** 2 * (tri_lhuilier(C[:-1, :-1], C[:-1, 1:], C[1:, :-1]) +
                            tri_lhuilier(C[:-1, 1:], C[1:, 1:], C[1:, :-1]))
        acmin = min(acmin, float(ac.min()))
    return amin, acmin


_CACHE = {}


def domain_metrics(subs, nx, ny, N, pitch, nj):
    """([{metric: plane} per sub-domain], {"corner_w": (nsub, 4, 3), "da_min", "da_min_c"}) for
    the sub-domains `subs` (dicts with tile, ioff, joff) of a domain's plane layout"""
    key = (N, nx, ny, pitch, nj, tuple((s["tile"], s["ioff"], s["joff"]) for s in subs))
    if key not in _CACHE:
        ms, cw = [], []
        for s in subs:
            o = subdomain_metrics(s["tile"], s["ioff"], s["joff"], nx, ny, N, pitch, nj)
            cw.append(o.pop("corner_w"))
            o.pop("xyz")
            ms.append(o)
        da, dac = min_areas(N)
        _CACHE[key] = (ms, dict(corner_w=np.array(cw), da_min=da, da_min_c=dac))
    return _CACHE[key]
