"""The NDSL-style surface of the dycore stencils (geosongpu-ci_amd/stencils.py): the
reference's idiom (dsl_patterns/Do__get_top_of_the_column.py:28-55:
stencil_factory.from_dims_halo(func, compute_dims) then self.stencil(fields...)) over
device-resident quantities on the whole cubed sphere.

CPU: every StencilDef's argument count matches the signature comment of its registry entry
(csrc/stencils_registry.cpp).  GPU: c_sw, d_sw and fv_tp_2d called through the surface give
bit for bit what Domain.stencil gives on the same inputs."""
import importlib
import os
import re

import numpy as np
import pytest

from conftest import ROOT, rng


@pytest.fixture(scope="module")
def ndsl(pkg):
    return importlib.import_module(pkg.__name__ + ".stencils")


def test_stencil_defs_match_registry_signatures(ndsl):
    src = open(os.path.join(ROOT, "geosongpu-ci_amd", "csrc", "stencils_registry.cpp")).read()
    sigs = {}
    for line in src.splitlines():
        if not line.strip().startswith("//"):
            continue
        for m in re.finditer(r"(\w+)\(([^)]*)\)", line):
            args = [a.strip() for a in m.group(2).replace("|-", "").replace("|", ",").split(",") if a.strip()]
            sigs.setdefault(m.group(1), len(args))
    defs = {v.name: v for v in vars(ndsl).values() if isinstance(v, ndsl.StencilDef)}
    assert {"c_sw", "d_sw", "fv_tp_2d", "riem_solver_c", "riem_solver3", "update_dz_d", "a2b_ord4"} <= set(defs)
    for name, sd in defs.items():
        assert name in sigs, f"{name}: no signature comment in the registry"
        assert sigs[name] == sd.nargs, f"{name}: StencilDef has {sd.nargs} fields, registry {sigs[name]}"
        assert all(0 <= o < sd.nargs for o in sd.outputs)


@pytest.mark.gpu
def test_dycore_stencils_through_ndsl_surface(pkg, require_gpu, ndsl):
    X, Y, Z = ndsl.X_DIM, ndsl.Y_DIM, ndsl.Z_DIM
    npz = 3
    sf, qf = ndsl.get_factories_cubed_sphere(npx=25, npz=npz, nq=1)
    d = sf.domain
    r = rng(5)
    sh = d.shape(npz)
    host = dict(delp=1000.0 + 100.0 * r.random(sh), pt=300.0 + 10.0 * r.standard_normal(sh),
                w=r.standard_normal(sh), u=20.0 * r.standard_normal(sh), v=20.0 * r.standard_normal(sh))
    q = {n: qf.zeros([X, Y, Z], n) for n in host}
    for n, a in host.items():
        q[n].view[...] = a
    outs_c = ["uc", "vc", "ua", "va", "ut", "vt", "delpc", "ptc", "wc"]
    for n in outs_c:
        q[n] = qf.zeros([X, Y, Z], n)
    c_sw = sf.from_dims_halo(func=ndsl.c_sw, compute_dims=[X, Y, Z])
    c_sw(q["delp"], q["pt"], q["w"], q["u"], q["v"], *[q[n] for n in outs_c], dt2=300.0)
    # the same through the registry directly
    for n, a in host.items():
        d.upload("r_" + n, a)
    d.stencil("c_sw", ["r_" + n for n in ["delp", "pt", "w", "u", "v"] + outs_c], [300.0])
    for n in outs_c:
        assert np.array_equal(q[n].view, d.download("r_" + n)), f"c_sw {n}"
    # d_sw on the c_sw outputs
    outs_d = ["crx", "cry", "xfx", "yfx", "cx", "cy", "mfx", "mfy", "ke"]
    for n in outs_d:
        q[n] = qf.zeros([X, Y, Z], n)
    d_sw = sf.from_dims_halo(func=ndsl.d_sw, compute_dims=[X, Y, Z])
    d_sw(q["delp"], q["pt"], q["w"], q["u"], q["v"], q["uc"], q["vc"], q["ua"], q["va"], *[q[n] for n in outs_d],
         dt=600.0, dddmp=0.2, d2_bg=0.0, hord_mt=6, hord_vt=6, hord_tm=6, hord_dp=6)
    for n in outs_d:
        d.upload("r_" + n, np.zeros(sh))
    d.stencil("d_sw", ["r_" + n for n in ["delp", "pt", "w", "u", "v", "uc", "vc", "ua", "va"] + outs_d],
              [600.0, 0.2, 0.0, 6, 6, 6, 6])
    for n in ["delp", "pt", "w", "u", "v"] + outs_d:
        assert np.array_equal(q[n].view, d.download("r_" + n)), f"d_sw {n}"
    # fv_tp_2d without mass fluxes (optional arguments as None)
    fx, fy = qf.zeros([X, Y, Z], "fx"), qf.zeros([X, Y, Z], "fy")
    tp = sf.from_dims_halo(func=ndsl.fv_tp_2d, compute_dims=[X, Y, Z])
    tp(q["pt"], q["crx"], q["cry"], q["xfx"], q["yfx"], None, None, None, None, fx, fy, ord=6, nt=1)
    d.upload("r_fx", np.zeros(sh))
    d.upload("r_fy", np.zeros(sh))
    d.stencil("fv_tp_2d", ["r_pt", "r_crx", "r_cry", "r_xfx", "r_yfx", "-", "-", "-", "-", "r_fx", "r_fy"], [6, 1])
    assert np.array_equal(fx.view, d.download("r_fx")) and np.array_equal(fy.view, d.download("r_fy"))
    sf.close()
