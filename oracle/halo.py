"""Oracle cubed-sphere halo fill (TEST INFRASTRUCTURE ONLY, see oracle/__init__.py).

Independent of the product's geometric edge matching: the tile connectivity is
the FV3 rule table (1-based tiles) —
    odd  tile t: E -> t+1 aligned, N -> t+2 rotated, W -> t-2 rotated, S -> t-1 aligned
    even tile t: E -> t+2 rotated, N -> t+1 aligned, W -> t-1 aligned, S -> t-2 rotated
written as affine maps of continuous lattice coordinates (corner points at
integers).  Vector components rotate with the map; cube-corner halo regions are
zero (the stencils fill them via copy_corners).
"""
import numpy as np

from . import NG

# staggering offsets (in half cells) of the stored point (i, j): (dx2, dy2)
STAGGER = {"cell": (1, 1), "xedge": (1, 0), "yedge": (0, 1), "corner": (0, 0)}
# vector kinds: staggering of (x comp, y comp)
VECTOR = {"dgrid": ("xedge", "yedge"), "cgrid": ("yedge", "xedge"), "agrid": ("cell", "cell")}


def _edge_map(t, edge, N):
    """Map for tile t (0-based) across `edge`: returns (nbr, f) with f((X2,Y2)) in doubled coords
    and rot (number of +90 turns applied to directions)."""
    T = t + 1
    odd = T % 2 == 1
    N2 = 2 * N

    def wrap(x):
        return (x - 1) % 6
    if odd:
        if edge == "E":
            return wrap(T + 1), (lambda X, Y: (X - N2, Y)), 0
        if edge == "S":
            return wrap(T - 1), (lambda X, Y: (X, Y + N2)), 0
        if edge == "N":
            return wrap(T + 2), (lambda X, Y: (Y - N2, N2 - X)), 3
        return wrap(T - 2), (lambda X, Y: (N2 - Y, N2 + X)), 1
    if edge == "N":
        return wrap(T + 1), (lambda X, Y: (X, Y - N2)), 0
    if edge == "W":
        return wrap(T - 1), (lambda X, Y: (X + N2, Y)), 0
    if edge == "E":
        return wrap(T + 2), (lambda X, Y: (N2 - Y, X - N2)), 1
    return wrap(T - 2), (lambda X, Y: (N2 + Y, N2 - X)), 3


def _rot(rot, dx, dy):
    for _ in range(rot % 4):
        dx, dy = -dy, dx
    return dx, dy


def locate(tile, X2, Y2, N):
    """(tile', X2', Y2', rot) owning doubled lattice point (X2, Y2) of `tile`; None in cube corners."""
    N2 = 2 * N
    inx, iny = 0 <= X2 <= N2, 0 <= Y2 <= N2
    if inx and iny:
        return tile, X2, Y2, 0
    if not inx and not iny:
        return None
    edge = "W" if X2 < 0 else "E" if X2 > N2 else "S" if Y2 < 0 else "N"
    nb, f, rot = _edge_map(tile, edge, N)
    X, Y = f(X2, Y2)
    assert 0 <= X <= N2 and 0 <= Y <= N2
    return nb, X, Y, rot


class Layout:
    """Sub-domain decomposition identical in meaning to the product's Decomp."""

    def __init__(self, N, lx=1, ly=1):
        self.N, self.lx, self.ly = N, lx, ly
        self.nx, self.ny = N // lx, N // ly

    def subs(self):
        out = []
        for t in range(6):
            for py in range(self.ly):
                for px in range(self.lx):
                    out.append(dict(tile=t, ioff=px * self.nx, joff=py * self.ny, N=self.N))
        return out

    def owner(self, tile, X2, Y2):
        for py in range(self.ly):
            for px in range(self.lx):
                ioff, joff = px * self.nx, py * self.ny
                ii = (X2 - (X2 & 1)) // 2 - ioff
                jj = (Y2 - (Y2 & 1)) // 2 - joff
                imax = self.nx - 1 if X2 & 1 else self.nx
                jmax = self.ny - 1 if Y2 & 1 else self.ny
                if 0 <= ii <= imax and 0 <= jj <= jmax:
                    return tile * self.lx * self.ly + py * self.lx + px, ii, jj
        raise AssertionError("no owner")


def _scalar_table(layout, stagger):
    """(dst g, j, i), (src g, j, i) slot lists for one stagger; src g = -1 -> zero-fill"""
    key = ("s", layout.N, layout.lx, layout.ly, stagger)
    if key in _TABLES:
        return _TABLES[key]
    dx2, dy2 = STAGGER[stagger]
    sx = 1 if stagger in ("yedge", "corner") else 0
    sy = 1 if stagger in ("xedge", "corner") else 0
    nx, ny = layout.nx, layout.ny
    dst, src = [], []
    for g, sd in enumerate(layout.subs()):
        for j in range(-NG, ny + NG + sy):
            for i in range(-NG, nx + NG + sx):
                if 0 <= i <= nx - 1 + sx and 0 <= j <= ny - 1 + sy:
                    continue
                loc = locate(sd["tile"], 2 * (i + sd["ioff"]) + dx2, 2 * (j + sd["joff"]) + dy2, layout.N)
                dst.append((g, j + NG, i + NG))
                if loc is None:
                    src.append((-1, 0, 0))
                    continue
                gs, ii, jj = layout.owner(loc[0], loc[1], loc[2])
                src.append((gs, jj + NG, ii + NG))
    t = (np.array(dst).T, np.array(src).T)
    _TABLES[key] = t
    return t


_TABLES = {}


def fill_scalar(fields, layout, stagger="cell"):
    """fields: array (nsub_total, nk, nj, pitch) in HBM layout; halos overwritten in place."""
    (dg, dj, di), (sg, sj, si) = _scalar_table(layout, stagger)
    vals = fields[sg, :, sj, si]
    vals[sg < 0] = 0.0
    fields[dg, :, dj, di] = vals
    return fields


def _vector_table(layout, kind):
    key = ("v", layout.N, layout.lx, layout.ly, kind)
    if key in _TABLES:
        return _TABLES[key]
    out = []
    nx, ny = layout.nx, layout.ny
    for c, st in enumerate(VECTOR[kind]):
        dx2, dy2 = STAGGER[st]
        sx = 1 if st in ("yedge", "corner") else 0
        sy = 1 if st in ("xedge", "corner") else 0
        dst, src = [], []
        for g, sd in enumerate(layout.subs()):
            for j in range(-NG, ny + NG + sy):
                for i in range(-NG, nx + NG + sx):
                    if 0 <= i <= nx - 1 + sx and 0 <= j <= ny - 1 + sy:
                        continue
                    loc = locate(sd["tile"], 2 * (i + sd["ioff"]) + dx2, 2 * (j + sd["joff"]) + dy2, layout.N)
                    dst.append((g, j + NG, i + NG))
                    if loc is None:
                        src.append((-1, 0, 0, 0, 0))
                        continue
                    dxd, dyd = (1, 0) if c == 0 else (0, 1)
                    ox, oy = _rot(loc[3], dxd, dyd)
                    gs, ii, jj = layout.owner(loc[0], loc[1], loc[2])
                    src.append((gs, jj + NG, ii + NG, 0 if ox != 0 else 1, ox + oy))
        out.append((np.array(dst).T, np.array(src).T))
    _TABLES[key] = out
    return out


def fill_vector(fx, fy, layout, kind="dgrid"):
    """Vector pair halo fill with rotation of components across rotated tile edges."""
    srcs = (fx.copy(), fy.copy())
    dsts = (fx, fy)
    for c, ((dg, dj, di), (sg, sj, si, sc, sign)) in enumerate(_vector_table(layout, kind)):
        vals = np.where(sc[:, None] == 0, srcs[0][sg, :, sj, si], srcs[1][sg, :, sj, si]) * sign[:, None]
        vals[sg < 0] = 0.0
        dsts[c][dg, :, dj, di] = vals
    return fx, fy


def _sync_table(layout, kind):
    """Tile-edge synchronisation (FV3's mpp_get_boundary use in dyn_core): the vector
    components stored ON the east / north tile edges of a sub-domain take the values the
    neighbouring tile holds at the same points (its west / south edge; the FV3 connectivity
    always joins an east or north edge to a west or south one), so both tiles carry one
    value per shared edge point.  C grid: uc on east edges, vc on north edges; D grid: v on
    east edges, u on north edges."""
    key = ("e", layout.N, layout.lx, layout.ly, kind)
    if key in _TABLES:
        return _TABLES[key]
    out = []
    nx, ny, N = layout.nx, layout.ny, layout.N
    for c, st in enumerate(VECTOR[kind]):
        dx2, dy2 = STAGGER[st]
        dst, src = [], []
        for g, sd in enumerate(layout.subs()):
            pts = []
            if st == "yedge" and sd["ioff"] + nx == N:      # east tile edge, x-normal point
                pts = [(nx, j, "E") for j in range(ny)]
            elif st == "xedge" and sd["joff"] + ny == N:    # north tile edge, y-normal point
                pts = [(i, ny, "N") for i in range(nx)]
            for i, j, edge in pts:
                nb, f, rot = _edge_map(sd["tile"], edge, N)
                X, Y = f(2 * (i + sd["ioff"]) + dx2, 2 * (j + sd["joff"]) + dy2)
                assert X == 0 or Y == 0, "an east / north edge must meet a west / south edge"
                dxd, dyd = (1, 0) if c == 0 else (0, 1)
                ox, oy = _rot(rot, dxd, dyd)
                gs, ii, jj = layout.owner(nb, X, Y)
                dst.append((g, j + NG, i + NG))
                src.append((gs, jj + NG, ii + NG, 0 if ox != 0 else 1, ox + oy))
        out.append((np.array(dst, dtype=int).reshape(-1, 3).T, np.array(src, dtype=int).reshape(-1, 5).T))
    _TABLES[key] = out
    return out


def sync_edges(fx, fy, layout, kind="cgrid"):
    srcs = (fx.copy(), fy.copy())
    dsts = (fx, fy)
    for c, ((dg, dj, di), (sg, sj, si, sc, sign)) in enumerate(_sync_table(layout, kind)):
        if dg.size == 0:
            continue
        vals = np.where(sc[:, None] == 0, srcs[0][sg, :, sj, si], srcs[1][sg, :, sj, si]) * sign[:, None]
        dsts[c][dg, :, dj, di] = vals
    return fx, fy
