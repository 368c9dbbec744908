"""Host logic (CPU): cubed-sphere metric terms and the halo index tables of the
product, checked against geometric identities and against the oracle halo fill
(whose tile connectivity comes from FV3's rule table, not from geometry)."""
import ctypes

import numpy as np
import pytest

from conftest import rng
from oracle import NG
from oracle import halo as ohalo

R = 6371.0e3


def host_domain(pkg, npx=13, lx=1, ly=1):
    return pkg.Domain(npx=npx, npz=3, nq=1, layout_x=lx, layout_y=ly, host_only=1)


def interior(a, d):
    return a[..., NG:NG + d.ny, NG:NG + d.nx]


@pytest.mark.parametrize("npx", [13, 49])
def test_sphere_area_and_symmetry(pkg, npx):
    d = host_domain(pkg, npx)
    area = d.metric("area")
    assert abs(interior(area, d).sum() / (4 * np.pi * R * R) - 1) < 1e-13
    # all six faces are congruent
    a = interior(area, d)
    for t in range(1, 6):
        np.testing.assert_allclose(a[t], a[0], rtol=1e-12)
    sc = d.scalars()
    assert sc["da_min"] == pytest.approx(a.min(), rel=1e-12)
    # the equiangular face is symmetric about both face axes
    np.testing.assert_allclose(a[0], a[0][::-1, :], rtol=1e-12)
    np.testing.assert_allclose(a[0], a[0][:, ::-1], rtol=1e-12)


def test_dual_areas_and_lengths(pkg):
    d = host_domain(pkg, 25)
    N = d.N
    ac = d.metric("area_c")[:, NG:NG + N + 1, NG:NG + N + 1]
    # dual cells around corner points tile the sphere: interior points counted once, edges twice
    # (shared by two tiles), cube corners three times
    w = np.ones((N + 1, N + 1))
    w[0, :] = w[-1, :] = w[:, 0] = w[:, -1] = 0.5
    for c in [(0, 0), (0, -1), (-1, 0), (-1, -1)]:
        w[c] = 1.0 / 3.0
    tot = (ac * w).sum()
    assert abs(tot / (4 * np.pi * R * R) - 1) < 1e-12
    dx = d.metric("dx")
    dxa = d.metric("dxa")
    assert np.all(interior(dx, d) > 0) and np.all(interior(dxa, d) > 0)
    s = d.metric("sin_sg5")
    assert np.all((interior(s, d) > 0.85) & (interior(s, d) <= 1.0))
    # grid angle at the cube corner cells is 60 deg -> sin(60) at the corner point itself
    s6 = d.metric("sin_sg6")
    assert s6[0, NG, NG] == pytest.approx(np.sin(np.pi / 3), abs=1e-12)


def test_tile_edge_continuity(pkg):
    """dx along a tile edge seen from both tiles is the same great-circle arc."""
    d = host_domain(pkg, 13)
    dy = d.metric("dy")
    N = d.N
    # tile 0 east edge (y-edges i=N) == tile 1 west edge (i=0): aligned neighbours
    np.testing.assert_allclose(dy[0, NG:NG + N, NG + N], dy[1, NG:NG + N, NG + 0], rtol=1e-13)


def _apply_table(pkg, d, kind, comps):
    lib = pkg.lib()
    n = lib.gtfv3_halo_table(d.h, kind, None, 0)
    buf = (ctypes.c_int * (6 * n))()
    assert lib.gtfv3_halo_table(d.h, kind, buf, 6 * n) == n
    t = np.frombuffer(buf, dtype=np.int32).reshape(n, 6)
    flat = [c.reshape(c.shape[0], c.shape[1], -1) for c in comps]
    src = [f.copy() for f in flat]
    for dst_sub, dst_off, src_sub, src_off, comp, sign in t:
        dc, sc = comp & 1, (comp >> 1) & 1
        if src_sub < 0:
            flat[dc][dst_sub, :, dst_off] = 0.0
        else:
            flat[dc][dst_sub, :, dst_off] = sign * src[sc][src_sub, :, src_off]


@pytest.mark.parametrize("layout", [(1, 1), (2, 2), (1, 2)])
def test_halo_tables_match_oracle(pkg, layout):
    lx, ly = layout
    d = host_domain(pkg, 13, lx, ly)
    lay = ohalo.Layout(d.N, lx, ly)
    r = rng(7)
    shape = (d.nsub, 2, d.nj, d.pitch)
    # scalars
    for kind, st in ((0, "cell"), (1, "corner")):
        a = r.standard_normal(shape)
        b = a.copy()
        _apply_table(pkg, d, kind, [a])
        ohalo.fill_scalar(b, lay, st)
        np.testing.assert_array_equal(a, b)
    # vectors
    for kind, vk in ((2, "dgrid"), (3, "cgrid"), (4, "agrid")):
        u = r.standard_normal(shape)
        v = r.standard_normal(shape)
        u2, v2 = u.copy(), v.copy()
        _apply_table(pkg, d, kind, [u, v])
        ohalo.fill_vector(u2, v2, lay, vk)
        np.testing.assert_array_equal(u, u2)
        np.testing.assert_array_equal(v, v2)
    # C-grid tile-edge synchronisation (kind 5): east / north edge points from the neighbour
    u = r.standard_normal(shape)
    v = r.standard_normal(shape)
    u2, v2 = u.copy(), v.copy()
    _apply_table(pkg, d, 5, [u, v])
    ohalo.sync_edges(u2, v2, lay, "cgrid")
    np.testing.assert_array_equal(u, u2)
    np.testing.assert_array_equal(v, v2)
    assert not np.array_equal(u, r.standard_normal(shape))


@pytest.mark.parametrize("layout", [(1, 1), (2, 2), (1, 2)])
def test_merged_sync_and_cgrid_halo(pkg, layout):
    """Kind 6 (H_CSC, the step's single exchange of uc / vc per sub-step) equals the tile-edge
    synchronisation (kind 5) followed by the C-grid halo (kind 3), bit for bit, and so the
    oracle's sync_edges + fill_vector("cgrid")."""
    lx, ly = layout
    d = host_domain(pkg, 13, lx, ly)
    lay = ohalo.Layout(d.N, lx, ly)
    r = rng(11)
    shape = (d.nsub, 2, d.nj, d.pitch)
    u = r.standard_normal(shape)
    v = r.standard_normal(shape)
    u2, v2, u3, v3 = u.copy(), v.copy(), u.copy(), v.copy()
    _apply_table(pkg, d, 6, [u, v])
    _apply_table(pkg, d, 5, [u2, v2])
    _apply_table(pkg, d, 3, [u2, v2])
    np.testing.assert_array_equal(u, u2)
    np.testing.assert_array_equal(v, v2)
    ohalo.sync_edges(u3, v3, lay, "cgrid")
    ohalo.fill_vector(u3, v3, lay, "cgrid")
    np.testing.assert_array_equal(u, u3)
    np.testing.assert_array_equal(v, v3)
