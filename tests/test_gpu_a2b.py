"""a2b_ord4 (FV3 a2b_edge, 4th-order cell -> corner interpolation with the cubed-sphere
edge and corner forms) on the device against the oracle (oracle/nh_core.py a2b_ord4),
to 1e-12 of the field's mean magnitude, on 1x1 and 2x2 sub-domain layouts and on a
tile size whose corner columns span three strips of the column-marching kernel (one
of them shifted to end at the tile edge) and three row segments."""
import numpy as np
import pytest

from conftest import metrics_of, oracle_scalars, rng
from oracle import NG
from oracle import fv_dynamics as fvd
from oracle import nh_core

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("npx,layout", [(25, (1, 1)), (49, (2, 2)), (126, (1, 1))])
def test_a2b_variants_and_oracle(pkg, require_gpu, npx, layout):
    nk = 3
    d = pkg.Domain(npx=npx, npz=nk, nq=1, layout_x=layout[0], layout_y=layout[1])
    try:
        q = 1000.0 + 50.0 * rng(11).standard_normal(d.shape(nk))
        d.upload("t_q", q)
        d.stencil("a2b_ord4", ["t_q", "t_qb"])
        out = d.download("t_qb")
        J, I = slice(NG, NG + d.ny + 1), slice(NG, NG + d.nx + 1)
        ms = metrics_of(d)
        sc = oracle_scalars(d)
        g = fvd.Grid(d.N, layout[0], layout[1], ms, sc["corner_w"], sc["da_min_c"], d.nj, d.pitch)
        for s in range(d.nsub):
            ref = nh_core.a2b_ord4(q[s], g.P[s], ms[s], sc["corner_w"][s])
            a, b = out[s][:, J, I], ref[:, J, I]
            assert np.abs(a - b).max() <= 1e-12 * np.abs(b).mean(), s
    finally:
        d.close()
