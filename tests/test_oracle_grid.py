"""The product's cubed-sphere grid and FV3 metric terms (csrc/grid.cpp, read through the
library's host-only domain: no GPU) against the independent oracle restatement
oracle/grid.py (Putman & Lin 2007 construction, FV3 metric definitions, different
arithmetic), so that the dycore oracle's metric inputs are pinned by something other than
the code under test.

Compared on every plane slot the product fills, i, j in [-NG, n + NG], at C12 (1x1, 2x2),
C24 (1x4 bands) and C48: <= 1e-13 relative to the field's largest magnitude (a12 / a21: to the
matrix' diagonal), equal infinities / NaNs allowed.  The cube-corner halo cells (both tile
indices outside 0..N-1) are degenerate quadrilaterals of rotated halo points (FV3
fill_corners): there the oracle adopts the product's convention (oracle/grid.py) and, the
points being built with the same rounding, agrees with it bit for bit.
"""
import numpy as np
import pytest

from oracle import NG
from oracle import grid as og


def _masks(sub, d):
    li = np.arange(d.pitch) - NG
    lj = np.arange(d.nj) - NG
    I = li[None, :] + sub["ioff"]
    J = lj[:, None] + sub["joff"]
    N = d.N
    out_i = (I < 0) | (I >= N)
    out_j = (J < 0) | (J >= N)
    cell_cc = out_i & out_j
    # corner points whose four surrounding cells include a cube-corner-region cell (the four
    # cube corners themselves are triangles of three real cells and are compared)
    cor = np.zeros_like(cell_cc)
    for di in (-1, 0):
        for dj in (-1, 0):
            Ic, Jc = I + di, J + dj
            cor |= ((Ic < 0) | (Ic >= N)) & ((Jc < 0) | (Jc >= N))
    cube_corner = ((I == 0) | (I == N)) & ((J == 0) | (J == N))
    return cell_cc, cor & ~cube_corner


CORNER_BASED = {"area_c", "rarea_c", "cosa", "rsina", "fC", "sin_sg6", "sin_sg7", "sin_sg8", "sin_sg9",
                "cos_sg6", "cos_sg7", "cos_sg8", "cos_sg9"}


def test_oracle_faces_realise_fv3_connectivity():
    for N in (4, 12, 48):
        assert og.check_connectivity(N) < 1e-15


@pytest.mark.parametrize("npx,layout", [(13, (1, 1)), (13, (2, 2)), (25, (1, 4)), (49, (1, 1))])
def test_product_metrics_match_oracle(pkg, npx, layout):
    d = pkg.Domain(npx=npx, npz=2, nq=1, layout_x=layout[0], layout_y=layout[1], host_only=1)
    try:
        prod = {n: d.metric(n) for n in og.METRICS}
        xyz = d.corner_xyz()
        sc = d.scalars()
        worst = {}
        for s, sub in enumerate(d.subs):
            o = og.subdomain_metrics(sub["tile"], sub["ioff"], sub["joff"], d.nx, d.ny, d.N, d.pitch, d.nj)
            region = np.zeros((d.nj, d.pitch), bool)
            region[:d.ny + 2 * NG + 1, :d.nx + 2 * NG + 1] = True
            for n in og.METRICS:
                a, b = prod[n][s], o[n]
                # the off-diagonal a12 / a21 vanish along the tile's symmetry lines: the
                # matrix' scale (its diagonal) is the reference there
                ref = o["a11"] if n in ("a12", "a21") else b
                fin = region & np.isfinite(ref)
                scale = np.abs(ref[fin]).max()
                with np.errstate(all="ignore"):
                    e = np.where(a == b, 0.0, np.abs(a - b) / scale)
                err = float(np.nan_to_num(e[region], nan=1.0).max())
                worst[n] = max(worst.get(n, 0.0), err)
            np.testing.assert_allclose(xyz[s], o["xyz"], rtol=0, atol=1e-15)
            np.testing.assert_allclose(sc["corner_w"][s], o["corner_w"], rtol=1e-12, atol=0)
        bad = {k: v for k, v in worst.items() if not v <= 1e-13}
        assert not bad, bad
        da, dac = og.min_areas(d.N)
        assert abs(sc["da_min"] - da) <= 1e-13 * da and abs(sc["da_min_c"] - dac) <= 1e-13 * dac
    finally:
        d.close()
