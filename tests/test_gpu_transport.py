"""GPU parity: halo exchange, fv_tp_2d and tracer_2d_1l HIP kernels vs the oracle.

Bar: fp64, max relative difference <= 1e-12 (SURVEY.md §8c adopted tolerance;
kernels are built with -ffp-contract=off and keep the Fortran operation order,
so most points are bit-identical)."""
import numpy as np
import pytest

from conftest import metrics_of, rng
from oracle import NG
from oracle import halo as ohalo
from oracle import tp_core

pytestmark = pytest.mark.gpu
RTOL = 1e-12


def relerr(a, b):
    scale = max(np.abs(b).max(), 1e-300)
    return np.abs(a - b).max() / scale


def make_dom(pkg, npx=13, npz=5, nq=1, lx=1, ly=1):
    return pkg.Domain(npx=npx, npz=npz, nq=nq, layout_x=lx, layout_y=ly)


@pytest.mark.parametrize("layout", [(1, 1), (2, 2)])
def test_halo_exchange_gpu(pkg, require_gpu, layout):
    d = make_dom(pkg, 13, 4, 1, *layout)
    lay = ohalo.Layout(d.N, *layout)
    r = rng(3)
    for kind, spec in (("cell", "c"), ("corner", "b")):
        a = r.standard_normal(d.shape(4))
        d.upload("h_a", a)
        d.halo_update(f"h_a:{spec}")
        got = d.download("h_a")
        ohalo.fill_scalar(a, lay, kind)
        np.testing.assert_array_equal(got, a)
    for vk, spec in (("dgrid", "d"), ("cgrid", "C"), ("agrid", "a")):
        u = r.standard_normal(d.shape(4))
        v = r.standard_normal(d.shape(4))
        d.upload("h_u", u)
        d.upload("h_v", v)
        d.halo_update(f"h_u:{spec},h_v:{spec}")
        gu, gv = d.download("h_u"), d.download("h_v")
        ohalo.fill_vector(u, v, lay, vk)
        np.testing.assert_array_equal(gu, u)
        np.testing.assert_array_equal(gv, v)


def tp_inputs(d, npz, r):
    area = d.metric("area")[:, None]
    sh = d.shape(npz)
    q = 1.0 + 0.3 * r.standard_normal(sh)
    crx = r.uniform(-0.45, 0.45, sh)
    cry = r.uniform(-0.45, 0.45, sh)
    xfx = 0.3 * r.uniform(-1, 1, sh) * area
    yfx = 0.3 * r.uniform(-1, 1, sh) * area
    ra_x = area + xfx - np.roll(xfx, -1, axis=-1)
    ra_y = area + yfx - np.roll(yfx, -1, axis=-2)
    mfx = 800.0 * xfx
    mfy = 800.0 * yfx
    return dict(q=q, crx=crx, cry=cry, xfx=xfx, yfx=yfx, ra_x=ra_x, ra_y=ra_y, mfx=mfx, mfy=mfy)


@pytest.mark.parametrize("ord_", [5, 6])
@pytest.mark.parametrize("layout", [(1, 1), (2, 2)])
def test_fv_tp_2d_parity(pkg, require_gpu, ord_, layout):
    npz = 3
    d = make_dom(pkg, 13, npz, 1, *layout)
    r = rng(11)
    inp = tp_inputs(d, npz, r)
    for k, v in inp.items():
        d.upload("t_" + k, v)
    d.stencil("fv_tp_2d", ["t_q", "t_crx", "t_cry", "t_xfx", "t_yfx", "t_ra_x", "t_ra_y", "t_mfx", "t_mfy",
                           "t_fx", "t_fy"], [ord_, 1])
    gfx, gfy = d.download("t_fx"), d.download("t_fy")
    ms = metrics_of(d)
    nx, ny = d.nx, d.ny
    for s in range(d.nsub):
        fx, fy = tp_core.fv_tp_2d(inp["q"][s], inp["crx"][s], inp["cry"][s], inp["xfx"][s], inp["yfx"][s],
                                  inp["ra_x"][s], inp["ra_y"][s], d.subs[s], ms[s], nx, ny, ord_,
                                  inp["mfx"][s], inp["mfy"][s])
        ax = gfx[s][:, NG:NG + ny, NG:NG + nx + 1]
        bx = fx[:, NG:NG + ny, NG:NG + nx + 1]
        ay = gfy[s][:, NG:NG + ny + 1, NG:NG + nx]
        by = fy[:, NG:NG + ny + 1, NG:NG + nx]
        assert relerr(ax, bx) <= RTOL, (s, relerr(ax, bx))
        assert relerr(ay, by) <= RTOL, (s, relerr(ay, by))


@pytest.mark.parametrize("cmax_amp", [0.35, 1.2])
def test_tracer_2d_1l_parity(pkg, require_gpu, cmax_amp):
    npz, nq = 6, 3
    d = make_dom(pkg, 13, npz, nq)
    lay = ohalo.Layout(d.N)
    r = rng(5)
    area = d.metric("area")[:, None]
    sh = d.shape(npz)
    q = np.abs(1e-3 * (1.0 + 0.5 * r.standard_normal(d.shape(nq * npz))))
    dp1 = 500.0 + 100.0 * r.random(sh)
    cx = r.uniform(-cmax_amp, cmax_amp, sh)
    cy = r.uniform(-cmax_amp, cmax_amp, sh)
    mfx = 0.02 * r.uniform(-1, 1, sh) * area * 500.0
    mfy = 0.02 * r.uniform(-1, 1, sh) * area * 500.0
    for name, v in (("q", q), ("dp1", dp1), ("cx", cx), ("cy", cy), ("mfx", mfx), ("mfy", mfy)):
        d.upload(name, v)
    d.stencil("tracer_2d_1l", [], [nq])
    got = d.download("q")
    ms = metrics_of(d)
    ref, nsplt = tp_core.tracer_2d_1l(q, dp1, mfx, mfy, cx, cy, d.subs, ms, d.nx, d.ny, npz, nq, 6,
                                      lambda a: ohalo.fill_scalar(a, lay, "cell"))
    if cmax_amp > 1:
        assert nsplt.max() >= 2
    a = got[:, :, NG:NG + d.ny, NG:NG + d.nx]
    b = ref[:, :, NG:NG + d.ny, NG:NG + d.nx]
    assert relerr(a, b) <= RTOL, relerr(a, b)


@pytest.mark.parametrize("ord_,mf,layout", [(6, True, (1, 1)), (6, False, (2, 2)), (5, True, (2, 2))])
def test_fv_tp_2d_field_pairs_bitwise(pkg, require_gpu, ord_, mf, layout):
    """Field pairs in one wave (shared Courant / flux loads): nt = 4 tracers (two pairs) and a
    pair of separate arrays (d_sw's w, pt) give bit for bit the fluxes of one launch per field."""
    npz = 3
    d = make_dom(pkg, 13, npz, 1, *layout)
    r = rng(17)
    inp = tp_inputs(d, npz, r)
    for k, v in inp.items():
        if k != "q":
            d.upload("p_" + k, v)
    qs = [1.0 + 0.3 * r.standard_normal(d.shape(npz)) for _ in range(4)]
    mfx, mfy = ("p_mfx", "p_mfy") if mf else ("-", "-")
    args = ["p_crx", "p_cry", "p_xfx", "p_yfx", "p_ra_x", "p_ra_y", mfx, mfy]
    single = []
    for n, q in enumerate(qs):
        d.upload(f"p_q{n}", q)
        d.stencil("fv_tp_2d", [f"p_q{n}"] + args + [f"p_fx{n}", f"p_fy{n}"], [ord_, 1])
        single.append((d.download(f"p_fx{n}"), d.download(f"p_fy{n}")))
    # four tracers in one array [sub][t][k]: two pairs
    d.upload("p_q4", np.concatenate(qs, axis=1))
    d.stencil("fv_tp_2d", ["p_q4"] + args + ["p_fx4", "p_fy4"], [ord_, 4])
    gx, gy = d.download("p_fx4"), d.download("p_fy4")
    for n in range(4):
        assert np.array_equal(gx[:, n * npz:(n + 1) * npz], single[n][0]), f"tracer {n} fx"
        assert np.array_equal(gy[:, n * npz:(n + 1) * npz], single[n][1]), f"tracer {n} fy"
    # two separate arrays
    d.stencil("fv_tp_2d_pair", ["p_q0", "p_q1", "p_crx", "p_cry", "p_xfx", "p_yfx", mfx, mfy, "p_ax", "p_ay",
                                "p_bx", "p_by"], [ord_])
    assert np.array_equal(d.download("p_ax"), single[0][0])
    assert np.array_equal(d.download("p_ay"), single[0][1])
    assert np.array_equal(d.download("p_bx"), single[1][0])
    assert np.array_equal(d.download("p_by"), single[1][1])


def _tracer_inputs(d, npz, nq, cmax_amp, seed):
    r = rng(seed)
    area = d.metric("area")[:, None]
    sh = d.shape(npz)
    return dict(q=np.abs(1e-3 * (1.0 + 0.5 * r.standard_normal(d.shape(nq * npz)))), dp1=500.0 + 100.0 * r.random(sh),
                cx=r.uniform(-cmax_amp, cmax_amp, sh), cy=r.uniform(-cmax_amp, cmax_amp, sh),
                mfx=0.02 * r.uniform(-1, 1, sh) * area * 500.0, mfy=0.02 * r.uniform(-1, 1, sh) * area * 500.0)


@pytest.mark.parametrize("npx,npz,nq,cmax_amp", [(13, 6, 3, 1.2), (13, 6, 4, 0.35), (181, 2, 4, 0.45),
                                                 (181, 2, 3, 1.3)])
def test_tracer_update_in_march_matches_separate_update(pkg, require_gpu, npx, npz, nq, cmax_amp):
    """tracer_2d_1l with the update inside the march (dp2 and the flux-form update from the
    mass fluxes and tracer fluxes held in registers, ping-pong tracer planes) against the
    flux planes + tracer_dp2 + tracer_update, bit for bit: single tracers (nq odd) and pairs,
    one and several sub-steps (nsplt >= 2 where cmax > 1: the finished levels carry over),
    at C12 and C180 (interior strips, seams, segments)."""
    d = make_dom(pkg, npx, npz, nq)
    inp = _tracer_inputs(d, npz, nq, cmax_amp, 17)
    out = []
    for fused in (1, 0):
        for name, v in inp.items():
            d.upload(name, v)
        d.stencil("tracer_2d_1l", [], [nq, fused])
        out.append(d.download("q")[:, :, NG:NG + d.ny, NG:NG + d.nx])
    assert np.array_equal(out[0], out[1])
    d.close()


@pytest.mark.parametrize("npx,npz,nq,cmax_amp", [(181, 2, 9, 0.45), (181, 3, 6, 1.3), (13, 6, 3, 1.2)])
def test_tracer_march_three_fields_per_wave(pkg, require_gpu, npx, npz, nq, cmax_amp):
    """The fused tracer march with three tracers per wave (every TpM field slot below NF set,
    the updated tracer f written to its own slot) bit for bit against one tracer per wave and,
    for even nq, two: C180 with an odd tracer count (nq = 9), C180 with sub-steps, C12."""
    d = make_dom(pkg, npx, npz, nq)
    inp = _tracer_inputs(d, npz, nq, cmax_amp, 23)
    out = {}
    for nf in (3, 1) + ((2,) if nq % 2 == 0 else ()):
        for name, v in inp.items():
            d.upload(name, v)
        d.stencil("tracer_2d_1l", [], [nq, 1, nf])
        out[nf] = d.download("q")[:, :, NG:NG + d.ny, NG:NG + d.nx]
    for nf, v in out.items():
        assert np.array_equal(v, out[1]), f"nf = {nf} differs from one tracer per wave"
    with pytest.raises(Exception, match="nf must"):
        d.stencil("tracer_2d_1l", [], [nq, 1, 4])
    d.close()
