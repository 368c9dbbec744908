"""GEOS's rank topology through the drop-in ABI with several ranks on one GPU: each rank a
process calling geos_gtfv3 init / run / finalize (the Python hook over the C ABI) on its own
sub-domain's Fortran arrays (no tile axis), the ranks found from GTFV3_RANK / GTFV3_WORLD_SIZE,
the bootstrap id through the job-stamped id file, the halos through the same-node IPC
transport (GTFV3_TRANSPORT=ipc; csrc/ipc.cpp) -- the reference's PER_DEVICE_PROCESS ranks
sharing a GPU (/root/reference/src/tcn/ci/pipeline/gtfv3_config.py:22).  Every rank's
updated arrays must equal the single-process step of the same global state (device API,
which the bridge equals bit for bit: test_gpu_bridge.py) on its section, bit for bit.
Layouts: six ranks of one tile, and twelve ranks of half tiles (1x2)."""
import importlib
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NG = 3
OUT = ("u", "v", "w", "delz", "pt", "delp", "q", "ps", "pe", "peln", "pk", "pkz", "ua", "va", "omga")


def _shapes(nx, ny, npz, nq):
    """Fortran bounds of the run arrays of a section of nx x ny compute cells, as local 0-based
    (lo_i, hi_i, lo_j, hi_j, nk, k-in-the-middle) -- test_gpu_bridge._shapes for a section"""
    d = lambda: (-NG, nx - 1 + NG, -NG, ny - 1 + NG)  # noqa: E731
    lo_i, hi_i, lo_j, hi_j = d()
    c = (0, nx - 1, 0, ny - 1)
    return {
        "u": (lo_i, hi_i, lo_j, hi_j + 1, npz, False), "v": (lo_i, hi_i + 1, lo_j, hi_j, npz, False),
        "w": d() + (npz, False), "delz": d() + (npz, False), "pt": d() + (npz, False),
        "delp": d() + (npz, False), "q": d() + (npz * nq, False), "ps": d() + (1, False),
        "pe": (-1, nx, -1, ny, npz + 1, True), "pk": c + (npz + 1, False), "peln": c + (npz + 1, True),
        "pkz": c + (npz, False), "phis": d() + (1, False), "q_con": d() + (npz, False),
        "omga": d() + (npz, False), "ua": d() + (npz, False), "va": d() + (npz, False),
        "uc": (lo_i, hi_i + 1, lo_j, hi_j, npz, False), "vc": (lo_i, hi_i, lo_j, hi_j + 1, npz, False),
        "mfx": (0, nx, 0, ny - 1, npz, False), "mfy": (0, nx - 1, 0, ny, npz, False),
        "cx": (0, nx, lo_j, hi_j, npz, False), "cy": (lo_i, hi_i, 0, ny, npz, False),
        "diss_est": d() + (npz, False),
    }


def _to_fortran(dev, li, hi, lj, hj, kj):
    a = dev[0, :, lj + NG:hj + NG + 1, li + NG:hi + NG + 1]   # (k, j, i) of the one sub-domain
    return np.asfortranarray(np.transpose(a, (2, 0, 1) if kj else (2, 1, 0)))


def _from_fortran(f, nk, nj, pitch, li, hi, lj, hj, kj):
    out = np.zeros((1, nk, nj, pitch))
    out[0, :, lj + NG:hj + NG + 1, li + NG:hi + NG + 1] = np.transpose(f, (1, 2, 0) if kj else (2, 1, 0))
    return out


def _worker(argv):
    """one GEOS rank: NPX NPZ NQ LX LY OUT (rank, size, transport from the environment)"""
    npx, npz, nq, lx, ly = (int(a) for a in argv[:5])
    out = argv[5]
    rank, nranks = int(os.environ["GTFV3_RANK"]), int(os.environ["GTFV3_WORLD_SIZE"])
    sys.path.insert(0, ROOT)
    pkg = importlib.import_module("geosongpu-ci_amd")
    state = importlib.import_module(pkg.__name__ + ".state")
    hook = importlib.import_module(pkg.__name__ + ".hook").geos_gtfv3
    h = pkg.Domain(rank, nranks, None, npx=npx, npz=npz, nq=nq, layout_x=lx, layout_y=ly, host_only=1)
    ak, bk, ks = state.hybrid_levels(npz)
    st = state.jablonowski_williamson(h, ak, bk)
    nx, ny, nj, pitch = h.nx, h.ny, h.nj, h.pitch
    sub = h.subs[0]
    h.close()
    shapes = _shapes(nx, ny, npz, nq)
    fort = {}
    for name, (li, hi, lj, hj, nk, kj) in shapes.items():
        src = st[name] if name in st else np.zeros((1, nk, nj, pitch))
        fort[name] = _to_fortran(src, li, hi, lj, hj, kj)
    is_, js = sub["ioff"] + 1, sub["joff"] + 1
    ie, je = is_ + nx - 1, js + ny - 1
    scal = dict(comm=0, npx=npx, npy=npx, npz=npz, ntiles=6, is_=is_, ie=ie, js=js, je=je, isd=is_ - NG,
                ied=ie + NG, jsd=js - NG, jed=je + NG, bdt=900.0, nq_tot=nq)
    hook.init(**scal)
    hook.run(**scal, ng=NG, ptop=float(ak[0]), ks=ks, layout_1=lx, layout_2=ly, adiabatic=0,
             ak=np.asfortranarray(ak), bk=np.asfortranarray(bk), **fort)
    hook.finalize()
    res = {}
    for name in OUT:
        li, hi, lj, hj, nk, kj = shapes[name]
        res[name] = _from_fortran(fort[name], nk, nj, pitch, li, hi, lj, hj, kj)
    np.savez(out, **res)


@pytest.mark.gpu
@pytest.mark.parametrize("nranks,layout", [(6, (1, 1)), (12, (1, 2))])
def test_bridge_ipc_ranks_match_single_process(pkg, require_gpu, tmp_path, nranks, layout):
    npx, npz, nq = 25, 10, 2
    state = importlib.import_module(pkg.__name__ + ".state")
    ref = pkg.Domain(npx=npx, npz=npz, nq=nq, layout_x=layout[0], layout_y=layout[1])
    ak, bk, ks = state.hybrid_levels(npz)
    st = state.jablonowski_williamson(ref, ak, bk)
    ref.set_vertical(ak, bk, ks)
    for k, v in st.items():
        ref.upload(k, v)
    ref.step(1)
    want = {k: ref.download(k) for k in OUT}
    nx, ny = ref.nx, ref.ny
    ref.close()
    token = os.urandom(8).hex()
    procs = []
    for r in range(nranks):
        env = dict(os.environ, GTFV3_RANK=str(r), GTFV3_WORLD_SIZE=str(nranks), GTFV3_BRIDGE_TILES_PER_RANK="1",
                   GTFV3_TRANSPORT="ipc", GTFV3_NCCL_ID_FILE=str(tmp_path / "id"), GTFV3_JOB_TOKEN=token,
                   GTFV3_NONFATAL="1")
        cmd = [sys.executable, os.path.abspath(__file__), str(npx), str(npz), str(nq), str(layout[0]),
               str(layout[1]), str(tmp_path / f"rank{r}.npz")]
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    logs = []
    try:
        for p in procs:
            o, _ = p.communicate(timeout=240)
            logs.append(o)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    for r, p in enumerate(procs):
        assert p.returncode == 0, f"rank {r} exited {p.returncode}:\n{logs[r][-3000:]}"
    assert not os.path.exists(tmp_path / "id"), "rank 0 removes the id file once every rank has it"
    for r in range(nranks):
        got = np.load(tmp_path / f"rank{r}.npz")
        for k in OUT:
            a = got[k][..., NG:NG + ny, NG:NG + nx]
            b = want[k][r:r + 1, ..., NG:NG + ny, NG:NG + nx]
            assert np.array_equal(a, b), f"rank {r} {k}: the bridge step over IPC differs from one process"


if __name__ == "__main__":
    _worker(sys.argv[1:])
