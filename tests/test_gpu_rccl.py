"""The RCCL transport (csrc/comm.cpp NcclTransport) executing on one GPU.

This pool gives one GPU per box and RCCL refuses two ranks on one device, so the production
transport runs here as ONE rank on a size-1 communicator (`rccl_self=1`, Namelist::rccl_self):
every halo point the one-rank layout would gather between its own sub-domains is packed,
sent with ncclSend to rank 0 (itself) and received with ncclRecv inside the exchange's NCCL
group, then unpacked; tracer_2d's per-level Courant maximum goes through ncclAllReduce(max).
The tables, pack / unpack kernels, message sizes and the stream discipline of the calls are
those of a multi-GPU run.  Bar: the step through RCCL equals the one-rank gather
step bit for bit (a halo value is a signed copy either way) -- C48 L72 (config 2's grid) and
C180 L72 (the benchmark grid), on the default three streams."""
import importlib
import time

import numpy as np
import pytest

FIELDS = ("u", "v", "w", "delz", "pt", "delp", "q", "ps", "pe", "peln", "pk", "pkz", "ua", "va", "uc", "vc",
          "omga", "mfx", "mfy", "cx", "cy")


def _domain(pkg, npx, npz, nq, **kw):
    state = importlib.import_module(pkg.__name__ + ".state")
    d = pkg.Domain(npx=npx, npz=npz, nq=nq, dt=450.0 * 180.0 / (npx - 1), **kw)
    ak, bk, ks = state.hybrid_levels(npz)
    st = state.jablonowski_williamson(d, ak, bk)
    d.set_vertical(ak, bk, ks)
    for k, v in st.items():
        d.upload(k, v)
    return d


@pytest.mark.gpu
@pytest.mark.parametrize("npx,npz,steps,split", [(49, 72, 2, "1"), (181, 72, 1, "1"), (49, 72, 2, "0")])
def test_rccl_self_step_matches_gather(pkg, require_gpu, monkeypatch, npx, npz, steps, split):
    """split "1" (the default with messages): the uc / vc and u / v exchanges begin, ds_utvt1's
    and cs_tmp's interiors run beside the RCCL messages on the exchange's communication stream,
    the exchanges end and the boundary frames follow (Dycore::step); "0": the whole exchange,
    then the stencil"""
    monkeypatch.setenv("GTFV3_HALO_SPLIT", split)
    nq = 4
    ref = _domain(pkg, npx, npz, nq)
    t0 = time.perf_counter()
    ref.step(steps)
    ref.sync()
    t_ref = time.perf_counter() - t0
    want = {k: ref.download(k) for k in FIELDS}
    ref.close()
    d = _domain(pkg, npx, npz, nq, rccl_self=1)
    try:
        t0 = time.perf_counter()
        d.step(steps)
        d.sync()
        t_msg = time.perf_counter() - t0
        for k in FIELDS:
            a = d.download(k)
            assert np.all(np.isfinite(a)), k
            assert np.array_equal(a, want[k]), f"{k}: the RCCL self-message step differs from the gather step"
    finally:
        d.close()
    print(f"C{npx - 1} L{npz}: {steps} step(s) gather {1e3 * t_ref:.1f} ms, RCCL self messages {1e3 * t_msg:.1f} ms "
          f"(first steps: allocation and communicator set-up included)")


@pytest.mark.parametrize("layout,npx", [((1, 1), 13), ((1, 4), 25)])
def test_rccl_self_tables_match_oracle(pkg, layout, npx):
    """(CPU, no GPU calls) the one-rank self-message tables: the same-rank gather keeps only
    the cube-corner zero fills, every other halo point is a message to rank 0 whose pack and
    unpack entries line up; applied on the host they give the oracle halo fill bit for bit,
    for every halo kind"""
    import sys

    from conftest import ROOT
    sys.path.insert(0, ROOT + "/tests")
    from oracle import halo as ohalo
    from test_multirank_cpu import KINDS, _table
    lib = pkg.lib()
    lx, ly = layout
    d = pkg.Domain(npx=npx, npz=2, nq=1, layout_x=lx, layout_y=ly, host_only=1, rccl_self=1)
    try:
        lay = ohalo.Layout(d.N, lx, ly)
        r = np.random.default_rng(23)
        nk, n = 2, d.nsub
        shape = (n, nk, d.nj, d.pitch)
        for kind, st, vk in KINDS:
            comps = [r.standard_normal(shape)] if st else [r.standard_normal(shape), r.standard_normal(shape)]
            ref = [c.copy() for c in comps]
            if st:
                ohalo.fill_scalar(ref[0], lay, st)
            elif vk in ("csync", "csc"):
                ohalo.sync_edges(ref[0], ref[1], lay, "cgrid")
                if vk == "csc":
                    ohalo.fill_vector(ref[0], ref[1], lay, "cgrid")
            else:
                ohalo.fill_vector(ref[0], ref[1], lay, vk)
            loc = [c.reshape(n, nk, -1).copy() for c in comps]
            src = [x.copy() for x in loc]
            lt = _table(lib, lib.gtfv3_halo_table, d.h, kind)
            assert np.all(lt[:, 2] < 0), f"kind {kind}: a same-rank gather entry left"
            for dst_sub, dst_off, _, _, comp, _ in lt:
                loc[comp & 1][dst_sub, :, dst_off] = 0.0
            snd = _table(lib, lib.gtfv3_halo_remote, d.h, kind, 0)
            rcv = _table(lib, lib.gtfv3_halo_remote, d.h, kind, 1)
            assert len(snd) == len(rcv) > 0 and np.all(snd[:, 5] == 0) and np.all(rcv[:, 5] == 0)
            buf = np.zeros((len(snd), nk))
            for sub, off, comp, sign, pos, _ in snd:
                buf[pos] = sign * src[comp][sub, :, off]
            for sub, off, comp, _, pos, _ in rcv:
                loc[comp][sub, :, off] = buf[pos]
            for c in range(len(comps)):
                assert np.array_equal(loc[c], ref[c].reshape(n, nk, -1)), f"kind {kind} comp {c}"
    finally:
        d.close()
