"""Multi-rank decomposition on CPU (gloo, world_size 2 and 4): each rank builds the
product's host-side halo tables (local gather + cross-rank pack/unpack, the exact
tables the RCCL send/recv path executes on the GPU) and exchanges real buffers
over torch.distributed/gloo.  The result on every rank must equal the single-rank
oracle halo fill of the global field, bit for bit, for scalar, corner and vector
(D/C/A-grid) kinds."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

KINDS = ((0, "cell", None), (1, "corner", None), (2, None, "dgrid"), (3, None, "cgrid"), (4, None, "agrid"),
         (5, None, "csync"), (6, None, "csc"))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _table(lib, fn, *args):
    import ctypes
    n = fn(*args, None, 0)
    assert n >= 0
    buf = (ctypes.c_int * max(6 * n, 1))()
    assert fn(*args, buf, 6 * n) == n
    return np.frombuffer(buf, dtype=np.int32)[:6 * n].reshape(n, 6).copy()


def _worker(rank, world, port, layout, q, npx=13):
    try:
        sys.path.insert(0, ROOT)
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import ctypes

        import torch
        import torch.distributed as dist

        import gtfv3_pkg
        from oracle import halo as ohalo
        pkg = gtfv3_pkg.load()
        lib = pkg.lib()
        dist.init_process_group("gloo", rank=rank, world_size=world)
        lx, ly = layout
        d = pkg.Domain(rank, world, None, npx=npx, npz=2, nq=1, layout_x=lx, layout_y=ly, host_only=1)
        nper = d.nsub
        ntot = 6 * lx * ly
        lay = ohalo.Layout(d.N, lx, ly)
        r = np.random.default_rng(11)
        nk = 2
        shape = (ntot, nk, d.nj, d.pitch)
        fails = []
        for kind, st, vk in KINDS:
            comps = [r.standard_normal(shape)] if st else [r.standard_normal(shape), r.standard_normal(shape)]
            ref = [c.copy() for c in comps]
            if st:
                ohalo.fill_scalar(ref[0], lay, st)
            elif vk == "csync":
                ohalo.sync_edges(ref[0], ref[1], lay, "cgrid")
            elif vk == "csc":  # the sync and the C halo as one exchange
                ohalo.sync_edges(ref[0], ref[1], lay, "cgrid")
                ohalo.fill_vector(ref[0], ref[1], lay, "cgrid")
            else:
                ohalo.fill_vector(ref[0], ref[1], lay, vk)
            loc = [c[rank * nper:(rank + 1) * nper].reshape(nper, nk, -1).copy() for c in comps]
            src = [x.copy() for x in loc]
            # same-rank gather
            lt = _table(lib, lib.gtfv3_halo_table, d.h, kind)
            for dst_sub, dst_off, src_sub, src_off, comp, sign in lt:
                dc, sc = comp & 1, (comp >> 1) & 1
                loc[dc][dst_sub, :, dst_off] = 0.0 if src_sub < 0 else sign * src[sc][src_sub, :, src_off]
            # cross-rank: pack per peer, exchange over gloo, unpack
            snd = _table(lib, lib.gtfv3_halo_remote, d.h, kind, 0)
            rcv = _table(lib, lib.gtfv3_halo_remote, d.h, kind, 1)
            reqs, rbufs = [], {}
            for p in range(world):
                if p == rank:
                    continue
                s = snd[snd[:, 5] == p]
                buf = np.zeros((len(s), nk))
                for sub, off, comp, sign, pos, _ in s:
                    buf[pos] = sign * src[comp][sub, :, off]
                rr = rcv[rcv[:, 5] == p]
                rb = torch.zeros((len(rr), nk), dtype=torch.float64)
                rbufs[p] = (rr, rb)
                if len(s):
                    reqs.append(dist.isend(torch.from_numpy(buf), p))
                if len(rr):
                    reqs.append(dist.irecv(rb, p))
            for rq in reqs:
                rq.wait()
            for p, (rr, rb) in rbufs.items():
                rb = rb.numpy()
                for sub, off, comp, sign, pos, _ in rr:
                    loc[comp][sub, :, off] = rb[pos]
            for c in range(len(comps)):
                want = ref[c][rank * nper:(rank + 1) * nper].reshape(nper, nk, -1)
                if not np.array_equal(loc[c], want):
                    fails.append(f"kind {kind} comp {c}: {np.sum(loc[c] != want)} mismatches")
        d.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, fails))
    except Exception as e:  # report to the parent instead of hanging it
        q.put((rank, [repr(e)]))


@pytest.mark.parametrize("world,layout,npx", [(2, (1, 1), 13), (2, (2, 2), 13), (4, (1, 2), 13), (4, (1, 4), 25)])
def test_gloo_halo_exchange_matches_oracle(world, layout, npx):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, layout, q, npx)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert res[r] == [], f"rank {r}: {res[r]}"


def test_bench_layouts_cover_driver_rank_counts():
    sys.path.insert(0, ROOT)
    import bench
    for n in (1, 2, 4, 8):
        lx, ly = bench.layout_for(n)
        assert (6 * lx * ly) % n == 0 and 180 % lx == 0 and 180 % ly == 0
