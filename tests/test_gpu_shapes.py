"""GPU parity at the shapes the benchmark runs (VERDICT r01 "parity at the shapes that run").

* fv_tp_2d at C180 (npx = 181, one GPU, layout 1x1 and the 8-GPU band layout 1x4): four
  64-column strips per sub-domain, so the interior-strip instantiation (EX = false), the
  strip seams and multi-segment marches all run; single fields, pairs, MF on and off,
  hord 5 and 6, against oracle/tp_core.py fv_tp_2d (bar 1e-12 relative, the SURVEY §8c
  adopted tolerance) and pairs bit for bit against single launches.
* update_dz_d at L72 and L137 (register-column edge profiles edge_prof_reg_k<80> / <144>, and
  the blocked edge_prof_k) against oracle/nh_core.py (edge_profile, then the zh transport),
  and the register form bit for bit against the blocked form on the same inputs.
"""
import importlib

import numpy as np
import pytest

from conftest import metrics_of, rng
from oracle import NG
from oracle import nh_core, tp_core

pytestmark = pytest.mark.gpu
RTOL = 1e-12


def relerr(a, b):
    scale = max(np.abs(b).max(), 1e-300)
    return np.abs(a - b).max() / scale


def tp_inputs(d, npz, r, cmax=0.45):
    area = d.metric("area")[:, None]
    sh = d.shape(npz)
    q = 1.0 + 0.3 * r.standard_normal(sh)
    crx = r.uniform(-cmax, cmax, sh)
    cry = r.uniform(-cmax, cmax, sh)
    xfx = 0.3 * r.uniform(-1, 1, sh) * area
    yfx = 0.3 * r.uniform(-1, 1, sh) * area
    ra_x = area + xfx - np.roll(xfx, -1, axis=-1)
    ra_y = area + yfx - np.roll(yfx, -1, axis=-2)
    mfx = 800.0 * xfx
    mfy = 800.0 * yfx
    return dict(q=q, crx=crx, cry=cry, xfx=xfx, yfx=yfx, ra_x=ra_x, ra_y=ra_y, mfx=mfx, mfy=mfy)


def check_fluxes(d, inp, q, gfx, gfy, ord_, mf, ms, subs=None):
    nx, ny = d.nx, d.ny
    for s in (range(d.nsub) if subs is None else subs):
        fx, fy = tp_core.fv_tp_2d(q[s], inp["crx"][s], inp["cry"][s], inp["xfx"][s], inp["yfx"][s],
                                  inp["ra_x"][s], inp["ra_y"][s], d.subs[s], ms[s], nx, ny, ord_,
                                  inp["mfx"][s] if mf else None, inp["mfy"][s] if mf else None)
        ax, bx = gfx[s][:, NG:NG + ny, NG:NG + nx + 1], fx[:, NG:NG + ny, NG:NG + nx + 1]
        ay, by = gfy[s][:, NG:NG + ny + 1, NG:NG + nx], fy[:, NG:NG + ny + 1, NG:NG + nx]
        assert relerr(ax, bx) <= RTOL, (s, "fx", relerr(ax, bx))
        assert relerr(ay, by) <= RTOL, (s, "fy", relerr(ay, by))


@pytest.fixture(scope="module")
def c180(pkg):
    d = pkg.Domain(npx=181, npz=2, nq=1)
    yield d
    d.close()


@pytest.mark.parametrize("ord_,mf", [(6, False), (6, True), (5, True), (5, False)])
def test_fv_tp_2d_c180_single(c180, require_gpu, ord_, mf):
    d = c180
    assert d.nx == 180 and d.nsub == 6
    npz = 2
    r = rng(181 + ord_ + 10 * mf)
    inp = tp_inputs(d, npz, r)
    for k, v in inp.items():
        d.upload("s_" + k, v)
    m = ("s_mfx", "s_mfy") if mf else ("-", "-")
    d.stencil("fv_tp_2d", ["s_q", "s_crx", "s_cry", "s_xfx", "s_yfx", "s_ra_x", "s_ra_y", *m, "s_fx", "s_fy"],
              [ord_, 1])
    ms = metrics_of(d)
    check_fluxes(d, inp, inp["q"], d.download("s_fx"), d.download("s_fy"), ord_, mf, ms)


@pytest.mark.parametrize("ord_,mf", [(6, True), (5, False)])
def test_fv_tp_2d_c180_pairs(c180, require_gpu, ord_, mf):
    """Two fields per wave (d_sw's w + pt; tracer pairs) at C180: bit for bit the single-field
    launches, and the single launches against the oracle on two sub-domains."""
    d = c180
    npz = 2
    r = rng(2181 + ord_)
    inp = tp_inputs(d, npz, r, cmax=0.6)
    for k, v in inp.items():
        if k != "q":
            d.upload("p_" + k, v)
    qs = [inp["q"], 1.0 + 0.2 * r.standard_normal(d.shape(npz))]
    m = ("p_mfx", "p_mfy") if mf else ("-", "-")
    args = ["p_crx", "p_cry", "p_xfx", "p_yfx", "p_ra_x", "p_ra_y", *m]
    single = []
    for n, q in enumerate(qs):
        d.upload(f"p_q{n}", q)
        d.stencil("fv_tp_2d", [f"p_q{n}"] + args + [f"p_fx{n}", f"p_fy{n}"], [ord_, 1])
        single.append((d.download(f"p_fx{n}"), d.download(f"p_fy{n}")))
    d.stencil("fv_tp_2d_pair", ["p_q0", "p_q1", "p_crx", "p_cry", "p_xfx", "p_yfx", *m, "p_ax", "p_ay", "p_bx",
                                "p_by"], [ord_])
    assert np.array_equal(d.download("p_ax"), single[0][0])
    assert np.array_equal(d.download("p_ay"), single[0][1])
    assert np.array_equal(d.download("p_bx"), single[1][0])
    assert np.array_equal(d.download("p_by"), single[1][1])
    # two tracers in one array
    d.upload("p_q2", np.concatenate(qs, axis=1))
    d.stencil("fv_tp_2d", ["p_q2"] + args + ["p_fx2", "p_fy2"], [ord_, 2])
    gx, gy = d.download("p_fx2"), d.download("p_fy2")
    for n in range(2):
        assert np.array_equal(gx[:, n * npz:(n + 1) * npz], single[n][0])
        assert np.array_equal(gy[:, n * npz:(n + 1) * npz], single[n][1])
    ms = metrics_of(d)
    check_fluxes(d, inp, qs[1], single[1][0], single[1][1], ord_, mf, ms, subs=(0, 4))


def test_fv_tp_2d_c180_bands(pkg, require_gpu):
    """The 8-GPU band layout (1x4: 180 x 45 sub-domains, shorter segments) on one GPU."""
    d = pkg.Domain(npx=181, npz=1, nq=1, layout_x=1, layout_y=4)
    try:
        assert d.nx == 180 and d.ny == 45 and d.nsub == 24
        r = rng(4181)
        inp = tp_inputs(d, 1, r)
        for k, v in inp.items():
            d.upload("b_" + k, v)
        d.stencil("fv_tp_2d", ["b_q", "b_crx", "b_cry", "b_xfx", "b_yfx", "b_ra_x", "b_ra_y", "b_mfx", "b_mfy",
                               "b_fx", "b_fy"], [6, 1])
        ms = metrics_of(d)
        check_fluxes(d, inp, inp["q"], d.download("b_fx"), d.download("b_fy"), 6, True, ms,
                     subs=(0, 1, 5, 9, 14, 23))
    finally:
        d.close()


@pytest.mark.parametrize("npz", [72, 137])
def test_update_dz_d_levels(pkg, require_gpu, npz):
    """update_dz_d at the benchmark level counts: the register-column edge profile
    (edge_prof_reg_k<80> at L72, edge_prof_reg_k<144> at L137 -- its column in 256 VGPRs + 98
    AGPRs) against the oracle, and against the blocked edge_prof_k bit for bit."""
    state = importlib.import_module(pkg.__name__ + ".state")
    d = pkg.Domain(npx=25, npz=npz, nq=1)
    try:
        ak, bk, ks = state.hybrid_levels(npz)
        d.set_vertical(ak, bk, ks)
        r = rng(500 + npz)
        inp = tp_inputs(d, npz, r, cmax=0.4)
        zh = np.cumsum(50.0 + 10.0 * r.random(d.shape(npz + 1)), axis=1)[:, ::-1].copy()
        for k in ("crx", "cry", "xfx", "yfx"):
            d.upload("u_" + k, inp[k])
        dp0 = nh_core.dp_ref(ak, bk)
        outs = {}
        for variant in (0, 1):
            d.stencil("edge_profile", ["u_crx", "u_xfx", "u_cry", "u_yfx", "e_crx", "e_xfx", "e_cry", "e_yfx"],
                      [variant])
            outs[variant] = {k: d.download("e_" + k) for k in ("crx", "xfx", "cry", "yfx")}
        nx, ny = d.nx, d.ny
        for k in outs[0]:
            if k in ("crx", "xfx"):  # x faces: i in [0, nx], j in [-3, ny+2]
                sl = (slice(None), slice(0, ny + 2 * NG), slice(NG, NG + nx + 1))
            else:                    # y faces: j in [0, ny], i in [-3, nx+2]
                sl = (slice(None), slice(NG, NG + ny + 1), slice(0, nx + 2 * NG))
            for s in range(d.nsub):
                assert np.array_equal(outs[0][k][s][sl], outs[1][k][s][sl]), f"{k}: register form != blocked form"
                ref = nh_core.edge_profile(inp[k][s], dp0)
                assert relerr(outs[0][k][s][sl], ref[sl]) <= 1e-12, (k, s, relerr(outs[0][k][s][sl], ref[sl]))
        d.upload("u_zh", zh)
        d.stencil("update_dz_d", ["u_zh", "u_crx", "u_cry", "u_xfx", "u_yfx"], [6])
        got = d.download("u_zh")
        ms = metrics_of(d)
        for s in range(d.nsub):
            ref = nh_core.update_dz_d_transport(zh[s], inp["crx"][s], inp["cry"][s], inp["xfx"][s], inp["yfx"][s],
                                                d.subs[s], ms[s], nx, ny, dp0, 6)
            a = got[s][:, NG:NG + ny, NG:NG + nx]
            b = ref[:, NG:NG + ny, NG:NG + nx]
            # (the oracle's metric terms are its own grid's, within 1e-13 of the product's:
            # random Courant numbers carry that difference into the transported heights)
            assert relerr(a, b) <= 1e-11, (s, relerr(a, b))
    finally:
        d.close()
