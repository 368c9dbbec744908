"""GPU parity of the vertical remap (Lagrangian_to_Eulerian).

The remap kernels (remap_prep_k, remap_blk_k / remap_job_k, remap_finish_k) against the oracle
(oracle/fv_mapz.py lagrangian_to_eulerian, one sub-domain at a time):
|hip - oracle| <= 1e-11 * mean|oracle| per state field the remap writes (exp / log from
ocml on the device and glibc on the host).
The source state is the JW06 state on Lagrangian surfaces displaced from the hybrid
levels (delp scaled by 1 +- 6 %), with negative tracer values in a scatter of cells so
that fillz runs, and a nonzero surface w; L72, L137 and L10.
"""
import importlib
import types

import numpy as np
import pytest

from conftest import rng
from oracle import NG
from oracle import fv_mapz

pytestmark = pytest.mark.gpu

FIELDS = ("pt", "delz", "w", "u", "v", "q", "pe", "peln", "pk", "pkz", "delp", "ps")


def lagrangian_state(pkg, d, npz, nq, r):
    state = importlib.import_module(pkg.__name__ + ".state")
    ak, bk, ks = state.hybrid_levels(npz)
    st = state.jablonowski_williamson(d, ak, bk)
    sh = d.shape(npz)
    st["delp"] = st["delp"] * (1.0 + 0.06 * (2.0 * r.random(sh) - 1.0))
    ptop = ak[0]
    pe = ptop + np.concatenate([np.zeros(sh[:1] + (1,) + sh[2:]), np.cumsum(st["delp"], axis=1)], axis=1)
    st["pe"] = pe
    st["peln"] = np.log(pe)
    st["w"] = 2.0 * r.standard_normal(sh)
    st["ws"] = 0.1 * r.standard_normal((sh[0], 1) + sh[2:])
    q = st["q"]
    neg = r.random(q.shape) < 0.02
    q[neg] = -1e-3 * r.random(int(neg.sum()))
    st["q"] = q
    for k in ("pk", "pkz", "ps"):
        st[k] = np.zeros(d.shape(npz + 1 if k == "pk" else (npz if k == "pkz" else 1)))
    return st, ak, bk, ks


@pytest.mark.parametrize("variant", [0, 1])
@pytest.mark.parametrize("npz,nq", [(72, 4), (137, 2), (10, 3), (137, 11), (137, 19), (72, 11), (20, 2)])
def test_remap_vs_oracle(pkg, require_gpu, npz, nq, variant):
    """variant 0: the level-block form (remap_blk_k, default), 1: the scratch-column job form"""
    d = pkg.Domain(npx=13, npz=npz, nq=nq)
    r = rng(300 + npz)
    st, ak, bk, ks = lagrangian_state(pkg, d, npz, nq, r)
    d.set_vertical(ak, bk, ks)
    for k, v in st.items():
        d.upload(k, v)
    d.stencil("lagrangian_to_eulerian", [], [1, variant])
    got = {k: d.download(k) for k in FIELDS}
    P = types.SimpleNamespace(nx=d.nx, ny=d.ny)
    ny, nx = d.ny, d.nx
    for s in range(d.nsub):
        sub = {k: st[k][s].copy() for k in FIELDS if k in st}
        sub["ws"] = st["ws"][s, 0]
        o = fv_mapz.lagrangian_to_eulerian(sub, ak, bk, ak[0], nq, 1, P)
        for k in FIELDS:
            if k == "u":
                sl = (slice(None), slice(NG, NG + ny + 1), slice(NG, NG + nx))
            elif k == "v":
                sl = (slice(None), slice(NG, NG + ny), slice(NG, NG + nx + 1))
            else:
                sl = (slice(None), slice(NG, NG + ny), slice(NG, NG + nx))
            a, b = got[k][s][sl], o[k][sl]
            scale = np.abs(b).mean() + 1e-300
            worst = np.abs(a - b).max() / scale
            assert worst <= 1e-11, f"sub{s} {k}: max scaled error {worst:.3e}"


@pytest.mark.parametrize("npz,nq", [(72, 11), (137, 5), (10, 3)])
def test_remap_shared_tracer_pivots_bitwise(pkg, require_gpu, npz, nq):
    """The tracer jobs with the pressure part shared by four tracers per wave (remap_blkq_k,
    variant 0; nq = 11 and 5 leave a partial last group) give bit for bit the one-tracer-per-
    wave level-block form (remap_blk_k, variant 3)."""
    outs = []
    for variant in (0, 3):
        d = pkg.Domain(npx=13, npz=npz, nq=nq)
        r = rng(900 + npz)
        st, ak, bk, ks = lagrangian_state(pkg, d, npz, nq, r)
        d.set_vertical(ak, bk, ks)
        for k, v in st.items():
            d.upload(k, v)
        d.stencil("lagrangian_to_eulerian", [], [1, variant])
        outs.append(d.download("q"))
        d.close()
    assert np.array_equal(outs[0], outs[1]), "shared-pivot tracer remap differs from the per-tracer form"
