"""GPU parity of the shallow-water core (c_sw with d2a2c_vect, d_sw) vs the oracle.

Random but physically-scaled inputs fill every plane point (halos included), so
both implementations read identical data everywhere; outputs are compared on the
regions FV3 defines them.  Bar: fp64, |hip - oracle| <= 1e-12 * |oracle| + 1e-12 * mean|oracle|.
"""
import numpy as np
import pytest

from conftest import checked_metrics, metrics_of, oracle_scalars, rng
from oracle import NG
from oracle import sw_core

pytestmark = pytest.mark.gpu


def close(a, b, what, rtol=1e-12, skip=None):
    if skip is not None:  # cube-corner halo cells: degenerate geometry (see cube_corner_cells)
        a, b = a[..., ~skip], b[..., ~skip]
    assert np.all(np.isfinite(b)), f"{what}: oracle not finite (stencil reads outside the halo)"
    scale = np.abs(b).mean() + 1e-300
    err = np.abs(a - b) - rtol * np.abs(b)
    worst = err.max() / scale
    assert worst <= rtol, f"{what}: max scaled error {worst:.3e}"


def cube_corner_cells(sub, i0, i1, j0, j1):
    """mask over a reg() region of the cells inside a cube-corner halo region (both tile
    indices outside 0..N-1).  Their areas are those of degenerate quadrilaterals of rotated
    halo points (FV3 fill_corners): the oracle's grid (oracle/grid.py) and the product's agree
    there only to the conditioning of a near-zero area, so c_sw's halo-ring outputs (delpc,
    ptc, wc on the ring) are compared outside them; no compute-domain value reads them."""
    I = np.arange(i0, i1 + 1)[None, :] + sub["ioff"]
    J = np.arange(j0, j1 + 1)[:, None] + sub["joff"]
    N = sub["N"]
    return ((I < 0) | (I >= N)) & ((J < 0) | (J >= N))


def reg(a, i0, i1, j0, j1):
    return a[..., j0 + NG:j1 + NG + 1, i0 + NG:i1 + NG + 1]


def sw_inputs(d, npz, r):
    sh = d.shape(npz)
    return dict(
        delp=1000.0 + 100.0 * r.random(sh),
        pt=300.0 + 10.0 * r.standard_normal(sh),
        w=r.standard_normal(sh),
        u=20.0 * r.standard_normal(sh),
        v=20.0 * r.standard_normal(sh),
    )


@pytest.mark.parametrize("layout", [(1, 1), (2, 2)])
def test_c_sw_parity(pkg, require_gpu, layout):
    npz = 3
    d = pkg.Domain(npx=13, npz=npz, nq=1, layout_x=layout[0], layout_y=layout[1])
    r = rng(21)
    inp = sw_inputs(d, npz, r)
    for k, v in inp.items():
        d.upload("c_" + k, v)
    dt2 = 0.5 * 600.0
    outs = ["uc", "vc", "ua", "va", "ut", "vt", "delpc", "ptc", "wc"]
    d.stencil("c_sw", ["c_delp", "c_pt", "c_w", "c_u", "c_v"] + ["c_" + o for o in outs], [dt2])
    got = {o: d.download("c_" + o) for o in outs}
    ms = metrics_of(d)
    nx, ny = d.nx, d.ny
    for s in range(d.nsub):
        ref = sw_core.c_sw(inp["delp"][s], inp["pt"][s], inp["u"][s], inp["v"][s], inp["w"][s], d.subs[s], ms[s],
                           nx, ny, dt2)
        for o, (i0, i1, j0, j1) in dict(delpc=(-1, nx, -1, ny), ptc=(-1, nx, -1, ny), wc=(-1, nx, -1, ny),
                                         uc=(-1, nx + 1, -1, ny), vc=(-1, nx, -1, ny + 1), ua=(-2, nx + 1, -2, ny + 1),
                                         va=(-2, nx + 1, -2, ny + 1), ut=(-1, nx + 1, -1, ny),
                                         vt=(-1, nx, -1, ny + 1)).items():
            close(reg(got[o][s], i0, i1, j0, j1), reg(ref[o], i0, i1, j0, j1), f"sub{s} {o}",
                  skip=cube_corner_cells(d.subs[s], i0, i1, j0, j1))


C_OUTS = ["uc", "vc", "ua", "va", "ut", "vt", "delpc", "ptc", "wc"]


@pytest.mark.parametrize("layout", [(1, 1), (2, 2)])
def test_d_sw_parity(pkg, require_gpu, layout):
    npz = 3
    d = pkg.Domain(npx=13, npz=npz, nq=1, layout_x=layout[0], layout_y=layout[1])
    r = rng(33)
    inp = sw_inputs(d, npz, r)
    sh = d.shape(npz)
    inp.update(uc=15.0 * r.standard_normal(sh), vc=15.0 * r.standard_normal(sh),
               ua=15.0 * r.standard_normal(sh), va=15.0 * r.standard_normal(sh))
    for k, v in inp.items():
        d.upload("d_" + k, v)
    for k in ("cx", "cy", "mfx", "mfy"):
        d.upload("d_" + k, np.zeros(sh))
    dt, dddmp, d2_bg = 600.0, 0.2, 0.0075
    ords = (6, 6, 6, 6)
    names = ["delp", "pt", "w", "u", "v", "uc", "vc", "ua", "va", "crx", "cry", "xfx", "yfx", "cx", "cy", "mfx",
             "mfy", "ke"]
    d.stencil("d_sw", ["d_" + n for n in names], [dt, dddmp, d2_bg, *ords])
    got = {n: d.download("d_" + n) for n in names}
    ms = metrics_of(d)
    nx, ny = d.nx, d.ny
    dmc = oracle_scalars(d)["da_min_c"]
    for s in range(d.nsub):
        ref = sw_core.d_sw(inp["delp"][s], inp["pt"][s], inp["u"][s], inp["v"][s], inp["w"][s], inp["uc"][s],
                           inp["vc"][s], inp["ua"][s], inp["va"][s], d.subs[s], ms[s], nx, ny, dt, ords, dddmp,
                           d2_bg, dmc)
        ref["cx"], ref["cy"], ref["mfx"], ref["mfy"] = ref["crx"], ref["cry"], ref["fx"], ref["fy"]
        for o, (i0, i1, j0, j1) in dict(
                delp=(0, nx - 1, 0, ny - 1), pt=(0, nx - 1, 0, ny - 1), w=(0, nx - 1, 0, ny - 1),
                crx=(0, nx, -NG, ny + NG - 1), xfx=(0, nx, -NG, ny + NG - 1), cry=(-NG, nx + NG - 1, 0, ny),
                yfx=(-NG, nx + NG - 1, 0, ny), cx=(0, nx, -NG, ny + NG - 1), cy=(-NG, nx + NG - 1, 0, ny),
                mfx=(0, nx, 0, ny - 1), mfy=(0, nx - 1, 0, ny), ke=(0, nx, 0, ny),
                u=(0, nx - 1, 0, ny), v=(0, nx, 0, ny - 1)).items():
            close(reg(got[o][s], i0, i1, j0, j1), reg(ref[o], i0, i1, j0, j1), f"sub{s} {o}")


D_NAMES = ["delp", "pt", "w", "u", "v", "uc", "vc", "ua", "va", "crx", "cry", "xfx", "yfx", "cx", "cy", "mfx", "mfy",
           "ke"]


def _d_sw_run(d, inp, npz, fused, ords=(6, 6, 6, 6), tag="f"):
    sh = d.shape(npz)
    for k, v in inp.items():
        d.upload(tag + k, v)
    for k in ("cx", "cy", "mfx", "mfy"):
        d.upload(tag + k, 0.5 * np.ones(sh))  # accumulators start non-zero: the += is checked
    d.stencil("d_sw", [tag + n for n in D_NAMES], [600.0, 0.2, 0.0075, *ords, 1.0 if fused else 0.0])
    return {n: d.download(tag + n) for n in D_NAMES}


@pytest.mark.parametrize("npx,layout", [(13, (1, 1)), (181, (1, 1)), (181, (1, 4))])
def test_d_sw_thermo_march_matches_separate_launches(pkg, require_gpu, npx, layout):
    """The fused thermo march (delp / w / pt transport with in-register mass fluxes, the
    flux accumulation and the ds_thermo update in one launch) against the separate
    fv_tp_2d launches + ds_accum + ds_thermo, bit for bit on every output, at C12 and at
    C180 (interior strips, strip seams, multi-segment marches; band layout 1x4)."""
    npz = 2
    d = pkg.Domain(npx=npx, npz=npz, nq=1, layout_x=layout[0], layout_y=layout[1])
    r = rng(77)
    inp = sw_inputs(d, npz, r)
    sh = d.shape(npz)
    inp.update(uc=15.0 * r.standard_normal(sh), vc=15.0 * r.standard_normal(sh),
               ua=15.0 * r.standard_normal(sh), va=15.0 * r.standard_normal(sh))
    a = _d_sw_run(d, inp, npz, True, tag="f_")
    b = _d_sw_run(d, inp, npz, False, tag="s_")
    nx, ny = d.nx, d.ny
    for n in ("delp", "pt", "w", "mfx", "mfy", "cx", "cy", "u", "v"):
        ga = a[n][..., NG:NG + ny + 1, NG:NG + nx + 1]
        gb = b[n][..., NG:NG + ny + 1, NG:NG + nx + 1]
        assert np.array_equal(ga, gb), f"{n}: fused thermo march differs from the separate launches"
    d.close()


def test_paired_last_strip_bitwise(pkg, require_gpu, monkeypatch):
    """At C180 the last strip of a march row has 7 outputs (181 edges = 3 x 58 + 7), so one
    wave runs it for two levels (lanes 0-31 level k, 32-63 level k+1).  d_sw -- the split
    thermo march and the single-kernel vorticity / delp marches -- with and without the
    pairing, bit for bit, on an odd level count (the last level unpaired)."""
    npz = 3
    d = pkg.Domain(npx=181, npz=npz, nq=1)
    r = rng(79)
    inp = sw_inputs(d, npz, r)
    sh = d.shape(npz)
    inp.update(uc=15.0 * r.standard_normal(sh), vc=15.0 * r.standard_normal(sh),
               ua=15.0 * r.standard_normal(sh), va=15.0 * r.standard_normal(sh))
    monkeypatch.setenv("GTFV3_TP_NOPAIR", "1")
    b = _d_sw_run(d, inp, npz, True, tag="n_")
    monkeypatch.delenv("GTFV3_TP_NOPAIR")
    a = _d_sw_run(d, inp, npz, True, tag="p_")
    nx, ny = d.nx, d.ny
    for n in ("delp", "pt", "w", "mfx", "mfy", "cx", "cy", "u", "v"):
        ga = a[n][..., NG:NG + ny + 1, NG:NG + nx + 1]
        gb = b[n][..., NG:NG + ny + 1, NG:NG + nx + 1]
        assert np.array_equal(ga, gb), f"{n}: paired last strip differs from one level per wave"
    d.close()


def test_d_sw_parity_c180(pkg, require_gpu):
    """d_sw (fused thermo march) against the oracle at C180 on two levels, on the product's
    grid checked against the oracle grid (conftest.checked_metrics).  Bar 1e-12."""
    npz = 2
    d = pkg.Domain(npx=181, npz=npz, nq=1)
    r = rng(78)
    inp = sw_inputs(d, npz, r)
    sh = d.shape(npz)
    inp.update(uc=15.0 * r.standard_normal(sh), vc=15.0 * r.standard_normal(sh),
               ua=15.0 * r.standard_normal(sh), va=15.0 * r.standard_normal(sh))
    got = _d_sw_run(d, inp, npz, True, tag="o_")
    nx, ny = d.nx, d.ny
    for s in (0, 3, 5):
        m, sc = checked_metrics(d, s)
        ref = sw_core.d_sw(inp["delp"][s], inp["pt"][s], inp["u"][s], inp["v"][s], inp["w"][s], inp["uc"][s],
                           inp["vc"][s], inp["ua"][s], inp["va"][s], d.subs[s], m, nx, ny, 600.0, (6, 6, 6, 6),
                           0.2, 0.0075, sc["da_min_c"])
        ref["mfx"], ref["mfy"] = 0.5 + ref["fx"], 0.5 + ref["fy"]
        for o, (i0, i1, j0, j1) in dict(delp=(0, nx - 1, 0, ny - 1), pt=(0, nx - 1, 0, ny - 1),
                                        w=(0, nx - 1, 0, ny - 1), mfx=(0, nx, 0, ny - 1), mfy=(0, nx - 1, 0, ny),
                                        u=(0, nx - 1, 0, ny), v=(0, nx, 0, ny - 1)).items():
            close(reg(got[o][s], i0, i1, j0, j1), reg(ref[o], i0, i1, j0, j1), f"sub{s} {o}", rtol=1e-12)
    d.close()
