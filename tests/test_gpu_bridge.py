"""The drop-in boundary end to end: Fortran-layout buffers through the reference
ABI (geos_gtfv3_init_c / geos_gtfv3_run_f64_c, via the Python hook mirror) must give
exactly what the device API gives for the same state (same kernels), with every
array updated in place in its Fortran shape.

Fortran <-> numpy layout follows the reference's own rule, restated:
  fortran_to_python:  flat.reshape(reversed(dim)).transpose()   (data_conversion.py:141)
  python_to_fortran:  arr.flatten(order="F")                     (data_conversion.py:184)
so a Fortran array of bounds (ni, nj, nk) is a Fortran-ordered numpy array.
"""
import importlib
import os

import numpy as np
import pytest

from oracle import NG

pytestmark = pytest.mark.gpu


def to_fortran(dev, lo_i, hi_i, lo_j, hi_j, kj=False):
    """device-layout (nsub, nk, nj, pitch) -> Fortran (i, j, k, tile) [or (i, k, j, tile)]"""
    a = dev[:, :, lo_j + NG:hi_j + NG + 1, lo_i + NG:hi_i + NG + 1]      # (s, k, j, i)
    a = np.transpose(a, (3, 1, 2, 0) if kj else (3, 2, 1, 0))           # (i, k, j, s) / (i, j, k, s)
    return np.asfortranarray(a)


def from_fortran(f, nsub, nk, nj, pitch, lo_i, hi_i, lo_j, hi_j, kj=False):
    out = np.zeros((nsub, nk, nj, pitch))
    a = np.transpose(f, (3, 1, 2, 0) if kj else (3, 2, 1, 0))
    out[:, :, lo_j + NG:hi_j + NG + 1, lo_i + NG:hi_i + NG + 1] = a
    return out


def _shapes(N, npz, nq):
    """Fortran bounds of the 24 run arrays (example_def_dycore.yaml:21-70) as
    local 0-based (lo_i, hi_i, lo_j, hi_j, nk, k-in-the-middle)."""
    is_, ie, js, je = 1, N, 1, N
    isd, ied, jsd, jed = is_ - NG, ie + NG, js - NG, je + NG
    L = lambda x: x - 1  # noqa: E731
    return {
        "u": (L(isd), L(ied), L(jsd), L(jed + 1), npz, False),
        "v": (L(isd), L(ied + 1), L(jsd), L(jed), npz, False),
        "w": (L(isd), L(ied), L(jsd), L(jed), npz, False),
        "delz": (L(isd), L(ied), L(jsd), L(jed), npz, False),
        "pt": (L(isd), L(ied), L(jsd), L(jed), npz, False),
        "delp": (L(isd), L(ied), L(jsd), L(jed), npz, False),
        "q": (L(isd), L(ied), L(jsd), L(jed), npz * nq, False),
        "ps": (L(isd), L(ied), L(jsd), L(jed), 1, False),
        "pe": (L(is_ - 1), L(ie + 1), L(js - 1), L(je + 1), npz + 1, True),
        "pk": (L(is_), L(ie), L(js), L(je), npz + 1, False),
        "peln": (L(is_), L(ie), L(js), L(je), npz + 1, True),
        "pkz": (L(is_), L(ie), L(js), L(je), npz, False),
        "phis": (L(isd), L(ied), L(jsd), L(jed), 1, False),
        "q_con": (L(isd), L(ied), L(jsd), L(jed), npz, False),
        "omga": (L(isd), L(ied), L(jsd), L(jed), npz, False),
        "ua": (L(isd), L(ied), L(jsd), L(jed), npz, False),
        "va": (L(isd), L(ied), L(jsd), L(jed), npz, False),
        "uc": (L(isd), L(ied + 1), L(jsd), L(jed), npz, False),
        "vc": (L(isd), L(ied), L(jsd), L(jed + 1), npz, False),
        "mfx": (L(is_), L(ie + 1), L(js), L(je), npz, False),
        "mfy": (L(is_), L(ie), L(js), L(je + 1), npz, False),
        "cx": (L(is_), L(ie + 1), L(jsd), L(jed), npz, False),
        "cy": (L(isd), L(ied), L(js), L(je + 1), npz, False),
        "diss_est": (L(isd), L(ied), L(jsd), L(jed), npz, False),
    }


def _setup(pkg, npx, npz, nq, **cfg):
    state = importlib.import_module(pkg.__name__ + ".state")
    d = pkg.Domain(npx=npx, npz=npz, nq=nq, **cfg)
    ak, bk, ks = state.hybrid_levels(npz)
    st = state.jablonowski_williamson(d, ak, bk)
    d.set_vertical(ak, bk, ks)
    return d, st, ak, bk, ks


def _bridge_call(pkg, st, d, ak, bk, ks, npx, npz, nq, dtype=np.float64, adiabatic=0):
    """One geos_gtfv3 init/run/finalize over Fortran-layout copies of `st`; returns the
    updated Fortran arrays and the shape table."""
    os.environ["GTFV3_BRIDGE_TILES_PER_RANK"] = "6"
    os.environ["GTFV3_NONFATAL"] = "1"
    hook = importlib.import_module(pkg.__name__ + ".hook").geos_gtfv3
    N = npx - 1
    shapes = _shapes(N, npz, nq)
    zeros = lambda nk: np.zeros((d.nsub, nk, d.nj, d.pitch))  # noqa: E731
    fort = {}
    for name, (li, hi, lj, hj, nk, kj) in shapes.items():
        src = st[name] if name in st else zeros(nk)
        fort[name] = np.asfortranarray(to_fortran(src, li, hi, lj, hj, kj).astype(dtype))
    addr = {k: v.ctypes.data for k, v in fort.items()}
    scal = dict(comm=0, npx=npx, npy=npx, npz=npz, ntiles=6, is_=1, ie=N, js=1, je=N, isd=1 - NG, ied=N + NG,
                jsd=1 - NG, jed=N + NG, bdt=900.0, nq_tot=nq)
    hook.init(**scal)
    hook.run(**scal, ng=NG, ptop=float(ak[0]), ks=ks, layout_1=1, layout_2=1, adiabatic=adiabatic,
             ak=np.asfortranarray(ak.astype(dtype)), bk=np.asfortranarray(bk.astype(dtype)), **fort)
    hook.finalize()
    for k in fort:
        assert fort[k].ctypes.data == addr[k], "buffers must be updated in place"
    return fort, shapes


OUT = ("u", "v", "w", "delz", "pt", "delp", "q", "ps", "pe", "peln", "pk", "pkz", "ua", "va", "omga")


def test_bridge_run_matches_device_api(pkg, require_gpu):
    npx, npz, nq = 13, 10, 2
    N = npx - 1
    d, st, ak, bk, ks = _setup(pkg, npx, npz, nq)
    for k, v in st.items():
        d.upload(k, v)
    d.step(1)
    want = {k: d.download(k) for k in OUT}
    nsub, nj, pitch = d.nsub, d.nj, d.pitch
    fort, shapes = _bridge_call(pkg, st, d, ak, bk, ks, npx, npz, nq)
    d.close()
    for name in want:
        li, hi, lj, hj, nk, kj = shapes[name]
        got = from_fortran(fort[name], nsub, nk, nj, pitch, li, hi, lj, hj, kj)
        a = got[..., NG:NG + N, NG:NG + N]
        b = want[name][..., NG:NG + N, NG:NG + N]
        assert np.array_equal(a, b), f"{name}: bridge result differs from the device API"


def test_bridge_fp32_abi_matches_fp64(pkg, require_gpu):
    """geos_gtfv3_run_c (the CI's PACE_FLOAT_PRECISION=32 ABI, float* arrays) against the
    fp64 twin on the same fp32-representable state, with the reference hook's own bar
    np.isclose(rtol=1e-5, atol=1e-8) (hook.py.jinja2:58,69)."""
    npx, npz, nq = 13, 10, 2
    d, st, ak, bk, ks = _setup(pkg, npx, npz, nq)
    st = {k: v.astype(np.float32).astype(np.float64) for k, v in st.items()}
    ak = ak.astype(np.float32).astype(np.float64)
    bk = bk.astype(np.float32).astype(np.float64)
    f64, shapes = _bridge_call(pkg, st, d, ak, bk, ks, npx, npz, nq, np.float64)
    f32, _ = _bridge_call(pkg, st, d, ak, bk, ks, npx, npz, nq, np.float32)
    d.close()
    for name in OUT:
        a, b = f32[name].astype(np.float64), f64[name]
        assert f32[name].dtype == np.float32
        ok = np.isclose(a, b, rtol=1e-5, atol=1e-8)
        assert ok.all(), f"{name}: fp32 ABI differs from fp64 at {np.argwhere(~ok)[:3].tolist()}"
        # the fp32 result is the fp64 result rounded once (same device arithmetic in fp64)
        assert np.array_equal(f32[name], b.astype(np.float32)), f"{name}: fp32 ABI is not the rounded fp64 result"


def test_bridge_adiabatic_is_dry_dynamics(pkg, require_gpu):
    """adiabatic=1 through the ABI = the oracle step with zvir = 0 (no moisture in the
    virtual temperature); adiabatic=0 differs from it wherever q != 0."""
    from conftest import metrics_of, oracle_scalars
    from oracle import fv_dynamics as fvd
    npx, npz, nq = 13, 10, 2
    N = npx - 1
    d, st, ak, bk, ks = _setup(pkg, npx, npz, nq)
    ms = metrics_of(d)
    sc = oracle_scalars(d)
    g = fvd.Grid(d.N, 1, 1, ms, sc["corner_w"], sc["da_min_c"], d.nj, d.pitch)
    nsub, nj, pitch = d.nsub, d.nj, d.pitch
    fort, shapes = _bridge_call(pkg, st, d, ak, bk, ks, npx, npz, nq, adiabatic=1)
    moist, _ = _bridge_call(pkg, st, d, ak, bk, ks, npx, npz, nq, adiabatic=0)
    d.close()
    nl = dict(n_split=6, dt_atmos=900.0, hord_mt=6, hord_vt=6, hord_tm=6, hord_dp=6, hord_tr=6, dddmp=0.2,
              d2_bg=0.0, p_fac=0.05, dz_min=2.0, fill=1, nq=nq, adiabatic=1)
    ref = fvd.fv_dynamics(st, ak, bk, g, nl)
    for name in ("pt", "delp", "u", "v", "ps"):
        li, hi, lj, hj, nk, kj = shapes[name]
        got = from_fortran(fort[name], nsub, nk, nj, pitch, li, hi, lj, hj, kj)[..., NG:NG + N, NG:NG + N]
        b = ref[name][..., NG:NG + N, NG:NG + N]
        err = np.abs(got - b).max() / np.abs(b).mean()
        assert err <= 1e-9, f"{name}: adiabatic bridge step vs oracle {err:.2e}"
    assert not np.array_equal(fort["pt"], moist["pt"]), "adiabatic must change the virtual-temperature step"


# inouts the bridge does not upload (the step overwrites them over their whole Fortran
# extent before reading them) and q_con, which moves neither way (bridge.hip bridge_run)
SKIPPED_UP = ("mfx", "mfy", "cx", "cy", "pkz", "ua", "va", "uc", "vc", "pe", "peln", "pk", "diss_est", "q_con")


def _garbage_call(pkg, d, st, ak, bk, ks, npx, npz, nq, env):
    """bridge call with random values in every array the step does not read; `env` sets the
    bridge's copy switches for this call"""
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        rng = np.random.default_rng(7)
        st = dict(st)
        shapes = _shapes(npx - 1, npz, nq)
        for name in SKIPPED_UP:
            st[name] = rng.standard_normal((d.nsub, shapes[name][4], d.nj, d.pitch))
        return _bridge_call(pkg, st, d, ak, bk, ks, npx, npz, nq)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def test_bridge_copy_pipeline_equivalent(pkg, require_gpu):
    """The overlapped copies (page-locked mapped arrays; tracers 1.. and omga's halo uploaded
    beside the acoustic sub-steps; each output group copied back once the step marks it final;
    inouts the step overwrites not uploaded) give bit for bit what moving every array both
    ways before / after the step gives, with garbage in those inouts, in both transfer forms:
    zero-copy kernels (GTFV3_BRIDGE_ZC=7, few workgroups so the grid-stride loops wrap),
    staged DMA (GTFV3_BRIDGE_ZC=0, a 4 KiB staging buffer cutting every array into many
    pieces) and the default mix (zero-copy before the step, staged beside and after it);
    q_con comes back untouched."""
    npx, npz, nq = 13, 10, 3
    d, st, ak, bk, ks = _setup(pkg, npx, npz, nq)
    full, shapes = _garbage_call(pkg, d, st, ak, bk, ks, npx, npz, nq,
                                 {"GTFV3_BRIDGE_SKIP": "0", "GTFV3_BRIDGE_PIN": "0"})
    dma, _ = _garbage_call(pkg, d, st, ak, bk, ks, npx, npz, nq,
                           {"GTFV3_BRIDGE_SKIP": "1", "GTFV3_BRIDGE_ZC": "0", "GTFV3_BRIDGE_STAGE_KB": "4"})
    zc, _ = _garbage_call(pkg, d, st, ak, bk, ks, npx, npz, nq,
                          {"GTFV3_BRIDGE_SKIP": "1", "GTFV3_BRIDGE_ZC": "7", "GTFV3_BRIDGE_ZC_BLOCKS": "3",
                           "GTFV3_BRIDGE_ZC_DOWN_BLOCKS": "5"})
    ref, _ = _garbage_call(pkg, d, st, ak, bk, ks, npx, npz, nq, {"GTFV3_BRIDGE_SKIP": "1"})
    d.close()
    for name in shapes:
        if name == "q_con":
            continue
        assert np.array_equal(full[name], dma[name]), f"{name}: staged DMA copies differ from full copies"
        assert np.array_equal(full[name], zc[name]), f"{name}: zero-copy (3 / 5 workgroups) differs from full copies"
        assert np.array_equal(full[name], ref[name]), f"{name}: default copies differ from full copies"
    # q_con never moves: the caller's values stay
    rng = np.random.default_rng(7)
    for name in SKIPPED_UP:
        g = rng.standard_normal((d.nsub, shapes[name][4], d.nj, d.pitch))
        if name == "q_con":
            li, hi, lj, hj, nk, kj = shapes[name]
            for got in (dma, zc):
                assert np.array_equal(got[name], to_fortran(g, li, hi, lj, hj, kj)), "q_con must stay untouched"
    # the bridge reports what it moved (the last call: default chunks)
    import ctypes
    out = (ctypes.c_double * 6)()
    assert pkg.lib().gtfv3_bridge_stats(out) == 0
    ms_up, ms_step, ms_down, up_b, down_b = out[0], out[1], out[2], out[3], out[4]
    assert min(ms_up, ms_step, ms_down) > 0
    total = sum(a.nbytes for a in ref.values())
    assert up_b < total and down_b < total and up_b < down_b


def _bridge_call_rank(pkg, st, ak, bk, ks, npx, npz, nq, rank):
    """geos_gtfv3 init/run/finalize in GEOS's own topology, one sub-domain (here one tile,
    layout 1x1) per rank with 2-D / 3-D Fortran arrays and no tile axis, as rank `rank` of 6
    alone on the null transport (GTFV3_BRIDGE_PROXY=1)"""
    env = dict(GTFV3_BRIDGE_TILES_PER_RANK="1", GTFV3_RANK=str(rank), GTFV3_WORLD_SIZE="6",
               GTFV3_BRIDGE_PROXY="1", GTFV3_NONFATAL="1")
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        hook = importlib.import_module(pkg.__name__ + ".hook").geos_gtfv3
        N = npx - 1
        shapes = _shapes(N, npz, nq)
        fort = {}
        for name, (li, hi, lj, hj, nk, kj) in shapes.items():
            src = st[name][rank:rank + 1] if name in st else np.zeros((1, nk) + st["delp"].shape[2:])
            fort[name] = np.asfortranarray(to_fortran(src, li, hi, lj, hj, kj)[..., 0])
        scal = dict(comm=0, npx=npx, npy=npx, npz=npz, ntiles=6, is_=1, ie=N, js=1, je=N, isd=1 - NG, ied=N + NG,
                    jsd=1 - NG, jed=N + NG, bdt=900.0, nq_tot=nq)
        hook.init(**scal)
        hook.run(**scal, ng=NG, ptop=float(ak[0]), ks=ks, layout_1=1, layout_2=1, adiabatic=0,
                 ak=np.asfortranarray(ak), bk=np.asfortranarray(bk), **fort)
        hook.finalize()
        return fort, shapes
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def test_bridge_one_subdomain_per_rank(pkg, require_gpu):
    """GEOS's rank topology through the ABI -- one sub-domain per rank (six ranks, one tile
    each), Fortran arrays without a tile axis, the rank's (is, js) checked against the FV3
    layout -- run as ranks 0 and 4 alone on one GPU with the null transport: the compute
    domain the missing cross-rank halo messages cannot reach in one step (the tile minus a
    band along its edges) equals the six-tile single-process bridge run bit for bit."""
    npx, npz, nq = 145, 10, 2
    N = npx - 1
    d, st, ak, bk, ks = _setup(pkg, npx, npz, nq)
    six, shapes = _bridge_call(pkg, st, d, ak, bk, ks, npx, npz, nq)
    d.close()
    band = 50  # cells along each tile edge reached by the missing messages in one step (measured 45)
    for rank in (0, 4):
        one, _ = _bridge_call_rank(pkg, st, ak, bk, ks, npx, npz, nq, rank)
        for name in ("u", "v", "w", "delz", "pt", "delp", "q", "ps", "pe", "peln", "pk", "pkz", "omga"):
            li, hi, lj, hj, nk, kj = shapes[name]
            a, b = one[name], six[name][..., rank]
            # Fortran index i -> array position i - (li + 1); the central window of the tile
            i0, i1 = band - li, N - band - li
            j0, j1 = band - lj, N - band - lj
            if kj:
                wa, wb = a[i0:i1, :, j0:j1], b[i0:i1, :, j0:j1]
            else:
                wa, wb = a[i0:i1, j0:j1], b[i0:i1, j0:j1]
            assert np.all(np.isfinite(wb)), f"{name}: six-tile run not finite"
            # reach of the missing messages: the deepest differing compute point from the edge
            ca = a[-li:N - li, :, -lj:N - lj] if kj else a[-li:N - li, -lj:N - lj]
            cb = b[-li:N - li, :, -lj:N - lj] if kj else b[-li:N - li, -lj:N - lj]
            diff = np.argwhere(ca != cb)
            if diff.size:
                ii, jj = diff[:, 0], diff[:, 2 if kj else 1]
                depth = np.minimum(np.minimum(ii, N - 1 - ii), np.minimum(jj, N - 1 - jj)).max()
                print(f"rank {rank} {name}: differences reach {depth} cells from the tile edge")
            bad = np.argwhere(wa != wb)
            assert bad.size == 0, (f"rank {rank} {name}: {len(bad)} points of the central window differ, "
                                   f"first at {bad[:3].tolist()}")
