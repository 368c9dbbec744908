"""K-column known-answer tests from the reference's DSL pattern programs
(dsl_patterns/Do__get_top_of_the_column.py:58-68, Do__while_in_gt_functions.py:54-62,
WIP__hybrid_index_2dout.py:68-90): the oracle (CPU) reproduces their asserts, and the
HIP column kernels, called through the NDSL-style surface (geosongpu-ci_amd/stencils.py),
equal the oracle bit for bit (index/mask semantics: exact)."""
import importlib

import numpy as np
import pytest

from oracle import column as oc

DOMAIN = (3, 3, 4)


def kat_input():
    a = np.ones(DOMAIN)
    a[:, :, DOMAIN[2] - 1] = 42
    return a


def gather_case(shape, seed):
    r = np.random.default_rng(seed)
    kmask = np.broadcast_to(np.arange(shape[2], dtype=np.float64), shape).copy()
    kidx = r.integers(0, shape[2], size=shape[:2]).astype(np.float64)
    data = r.integers(800, 900, size=shape).astype(np.float64)
    return data, kmask, kidx


def test_oracle_top_of_column_kat():
    assert np.all(oc.column_top(kat_input()) == 42)


def test_oracle_while_kat():
    out = oc.column_while_lt(kat_input(), 4.0)
    assert (out[0, 0, :] == [3.0, 2.0, 1.0, 0.0]).all()


def test_oracle_gather_kat():
    data, kmask, kidx = gather_case(DOMAIN, 0)
    out = oc.column_gather_k(data, kmask, kidx, np.zeros(DOMAIN[:2]))
    ii, jj = np.meshgrid(range(DOMAIN[0]), range(DOMAIN[1]), indexing="ij")
    np.testing.assert_array_equal(out, data[ii, jj, kidx.astype(int)])


@pytest.fixture(scope="module")
def ndsl(pkg):
    return importlib.import_module(pkg.__name__ + ".stencils")


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [DOMAIN, (37, 29, 72)])
def test_hip_column_kernels_match_oracle(pkg, require_gpu, ndsl, shape):
    sf, qf = ndsl.get_factories_single_tile(*shape, 0)
    dims3 = [ndsl.X_DIM, ndsl.Y_DIM, ndsl.Z_DIM]
    try:
        r = np.random.default_rng(7)
        inp = kat_input() if shape == DOMAIN else np.where(r.random(shape) < 0.1, 42.0, 1.0)
        # KAT-1: top of the column
        top = sf.from_dims_halo(func=ndsl.column_top, compute_dims=dims3)
        out = qf.zeros(dims3, "n/a")
        top(inp, out)
        np.testing.assert_array_equal(out.view[:], oc.column_top(inp))
        if shape == DOMAIN:
            assert np.all(out.view[:] == 42)
        # KAT-2: while loop with K-relative offsets
        wl = sf.from_dims_halo(func=ndsl.column_while_lt, compute_dims=dims3)
        o2 = np.zeros(shape)
        wl(inp, o2, thr=4.0)
        np.testing.assert_array_equal(o2, oc.column_while_lt(inp, 4.0))
        if shape == DOMAIN:
            assert (o2[0, 0, :] == [3.0, 2.0, 1.0, 0.0]).all()
        # KAT-3: gather data[i, j, kidx[i, j]] into a 2-D field
        data, kmask, kidx = gather_case(shape, 3)
        g = sf.from_dims_halo(func=ndsl.column_gather_k, compute_dims=dims3)
        o3 = qf.zeros([ndsl.X_DIM, ndsl.Y_DIM], "n/a")
        g(data, kmask, kidx, o3)
        np.testing.assert_array_equal(o3.view[:], oc.column_gather_k(data, kmask, kidx, np.zeros(shape[:2])))
    finally:
        sf.close()
