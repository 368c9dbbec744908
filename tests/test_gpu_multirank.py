"""Multi-rank dycore steps on one GPU: N ranks of one process exchange halos through
the loopback transport (comm.cpp), which runs the same host tables and the same
pack / unpack kernels as the RCCL path, with device-to-device copies in place of
ncclSend / ncclRecv.  The sub-domain layouts are exactly bench.py's for the driver's
2, 4 and 8 GPU runs, plus config 3's one tile per rank on 6 ranks; every rank's state after a full fv_dynamics step must equal the
single-rank step of the same global state bit for bit."""
import importlib
import itertools
import threading

import numpy as np
import pytest

from oracle import NG

pytestmark = pytest.mark.gpu

FIELDS = ("u", "v", "w", "delz", "pt", "delp", "q", "ps", "pe", "ua", "va", "omga")
_gid = itertools.count(101)


def _run_ranks(pkg, nranks, layout, npx=13, npz=10, nq=2, **kw):
    state = importlib.import_module(pkg.__name__ + ".state")
    ak, bk, ks = state.hybrid_levels(npz)
    gid = next(_gid)
    doms = [pkg.Domain(r, nranks, None, npx=npx, npz=npz, nq=nq, layout_x=layout[0], layout_y=layout[1],
                       loopback=gid, **kw) for r in range(nranks)]
    for d in doms:
        st = state.jablonowski_williamson(d, ak, bk)
        d.set_vertical(ak, bk, ks)
        for k, v in st.items():
            d.upload(k, v)
    errors = []

    def work(d):
        try:
            d.step(1)
        except Exception as e:  # surfaced below
            errors.append(repr(e))

    threads = [threading.Thread(target=work, args=(d,), daemon=True) for d in doms]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=120)
    assert not errors, errors  # a rank that raised leaves the others waiting at a barrier
    assert not any(t.is_alive() for t in threads), "a rank did not finish (loopback barrier)"
    out = [{k: d.download(k) for k in FIELDS} for d in doms]
    return doms, out


@pytest.mark.parametrize("nranks,layout,npx,npz", [(2, (1, 1), 13, 10), (4, (1, 2), 13, 10), (6, (1, 1), 13, 10),
                                                      (6, (1, 1), 49, 10), (8, (2, 2), 13, 10), (8, (1, 4), 25, 10),
                                                      (6, (1, 1), 181, 72)])
def test_multirank_step_matches_single_rank(pkg, require_gpu, nranks, layout, npx, npz):
    """(6, 1x1, C180 L72): BASELINE.json config 3's layout (one tile per rank, held_suarez.py:149-151)
    at its own size"""
    _check_multirank(pkg, nranks, layout, npx, npz)


@pytest.mark.parametrize("nranks,layout,npx,npz", [(8, (1, 4), 25, 10), (6, (1, 1), 49, 10), (2, (1, 1), 13, 10)])
def test_multirank_split_exchange_matches_single_rank(pkg, require_gpu, monkeypatch, nranks, layout, npx, npz):
    """The interior / boundary split of the uc / vc and u / v exchanges forced on
    (GTFV3_HALO_SPLIT=1; by default it runs only where the messages cross GPUs): every rank's
    state after a step through the loopback transport equals the single-rank step bit for bit"""
    monkeypatch.setenv("GTFV3_HALO_SPLIT", "1")
    _check_multirank(pkg, nranks, layout, npx, npz)


def _check_multirank(pkg, nranks, layout, npx, npz, **kw):
    state = importlib.import_module(pkg.__name__ + ".state")
    ak, bk, ks = state.hybrid_levels(npz)
    ref = pkg.Domain(npx=npx, npz=npz, nq=2, layout_x=layout[0], layout_y=layout[1], **kw)
    st = state.jablonowski_williamson(ref, ak, bk)
    ref.set_vertical(ak, bk, ks)
    for k, v in st.items():
        ref.upload(k, v)
    ref.step(1)
    want = {k: ref.download(k) for k in FIELDS}
    nx, ny = ref.nx, ref.ny
    ref.close()
    doms, got = _run_ranks(pkg, nranks, layout, npx=npx, npz=npz, **kw)
    nper = doms[0].nsub
    for r, d in enumerate(doms):
        for k in FIELDS:
            a = got[r][k][..., NG:NG + ny, NG:NG + nx]
            b = want[k][r * nper:(r + 1) * nper, ..., NG:NG + ny, NG:NG + nx]
            assert np.array_equal(a, b), f"rank {r} field {k} differs from the single-rank step"


def test_multirank_c720_config5_layout(pkg, require_gpu, monkeypatch):
    """BASELINE.json config 5's decomposition (C720 on 8 GPUs: 1x4 bands, three 720 x 180
    sub-domains per rank) through the loopback transport with the interior / boundary split on,
    as the RCCL ranks run it: every rank's state after a full step equals the single-rank step
    bit for bit.  Reduced levels and tracers (L8, nq 2: config 5's L137 x 54 state is 0.2 TB);
    dt scaled to the resolution (450 s x 180 / 720)."""
    monkeypatch.setenv("GTFV3_HALO_SPLIT", "1")
    _check_multirank(pkg, 8, (1, 4), 721, 8, dt=112.5)


MOIST_FIELDS = FIELDS + ("clls", "clcn", "qlcn", "qicn", "prec_rain", "prec_snow", "prec_graupel", "prec_ice",
                         "rad_cf", "rad_rl", "rad_ri")


def test_multirank_aquaplanet_step_matches_single_rank(pkg, require_gpu):
    """Config 4's coupled step (aquaplanet.py:99-178: fv_dynamics, then GEOS's moist physics)
    on the 8-GPU layout bench.py runs -- 8 ranks of bands 1x4 (three sub-domains each) --
    through the loopback transport at C48 L72 with the six moist tracers: every rank's state,
    condensate, cloud fractions, precipitation and radiation inputs after one coupled step
    equal the single-rank step of the same global state bit for bit.  The global state is
    made once (aquaplanet_tracers draws its humidity noise per sub-domain) and each rank gets
    its three sub-domains of it."""
    state = importlib.import_module(pkg.__name__ + ".state")
    npx, npz, nq, dt, nranks, layout = 49, 72, 6, 450.0, 8, (1, 4)
    ak, bk, ks = state.hybrid_levels(npz)
    ref = pkg.Domain(npx=npx, npz=npz, nq=nq, layout_x=layout[0], layout_y=layout[1], dt=dt)
    st = state.jablonowski_williamson(ref, ak, bk)
    state.aquaplanet_tracers(ref, st, ak, bk)
    ref.set_vertical(ak, bk, ks)
    for k, v in st.items():
        ref.upload(k, v)
    ref.step(1)
    ref.stencil("aquaplanet_physics", [], [dt])
    want = {k: ref.download(k) for k in MOIST_FIELDS}
    nx, ny = ref.nx, ref.ny
    ref.close()
    gid = next(_gid)
    doms = [pkg.Domain(r, nranks, None, npx=npx, npz=npz, nq=nq, layout_x=layout[0], layout_y=layout[1], dt=dt,
                       loopback=gid) for r in range(nranks)]
    nper = doms[0].nsub
    assert nper * nranks == 6 * layout[0] * layout[1]
    for r, d in enumerate(doms):
        d.set_vertical(ak, bk, ks)
        for k, v in st.items():
            d.upload(k, np.ascontiguousarray(v[r * nper:(r + 1) * nper]))
    del st
    errors = []

    def work(d):
        try:
            d.step(1)
            d.stencil("aquaplanet_physics", [], [dt])
        except Exception as e:  # surfaced below
            errors.append(repr(e))

    threads = [threading.Thread(target=work, args=(d,), daemon=True) for d in doms]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=120)
    assert not errors, errors
    assert not any(t.is_alive() for t in threads), "a rank did not finish (loopback barrier)"
    try:
        for r, d in enumerate(doms):
            for k in MOIST_FIELDS:
                a = d.download(k)[..., NG:NG + ny, NG:NG + nx]
                b = want[k][r * nper:(r + 1) * nper, ..., NG:NG + ny, NG:NG + nx]
                assert np.all(np.isfinite(b)), f"{k}: single-rank step not finite"
                assert np.array_equal(a, b), f"rank {r} field {k} differs from the single-rank coupled step"
    finally:
        for d in doms:
            d.close()


@pytest.mark.parametrize("proxy,npx,layout", [(8, 181, (1, 4)), (2, 49, (1, 1))])
def test_halo_split_bitwise_on_rank_proxy(pkg, require_gpu, monkeypatch, proxy, npx, layout):
    """The interior / boundary split of the uc / vc and u / v exchanges (messages on the
    exchange's communication stream beside ds_utvt1's / cs_tmp's interior; GTFV3_HALO_SPLIT)
    against the whole exchanges, on rank 0 of the 8-rank bands (bench.py --rank-proxy 8) and of
    two ranks, null transport: two steps bit for bit (NaN equal to NaN: the proxy's reflected
    halos)"""
    state = importlib.import_module(pkg.__name__ + ".state")
    npz = 20
    ak, bk, ks = state.hybrid_levels(npz)
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("GTFV3_HALO_SPLIT", mode)
        d = pkg.Domain(0, proxy, None, npx=npx, npz=npz, nq=2, layout_x=layout[0], layout_y=layout[1], loopback=-1,
                       dt=450.0 * 180.0 / (npx - 1))
        st = state.jablonowski_williamson(d, ak, bk)
        d.set_vertical(ak, bk, ks)
        for k, v in st.items():
            d.upload(k, v)
        d.step(2)
        out[mode] = {k: d.download(k) for k in FIELDS}
        d.close()
    for k in FIELDS:
        assert np.array_equal(out["0"][k], out["1"][k], equal_nan=True), f"{k}: the split exchange differs"
