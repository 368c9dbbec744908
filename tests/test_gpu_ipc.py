"""Several ranks (processes) on one GPU through the same-node IPC transport (csrc/ipc.cpp):
the reference runs GEOS with PER_DEVICE_PROCESS = 12 ranks on each GPU
(/root/reference/src/tcn/ci/pipeline/gtfv3_config.py:22) and RCCL takes one rank per device,
so `ipc=1` (the bridge: GTFV3_TRANSPORT=ipc) moves the halo messages between the ranks' own
device buffers through HIP IPC handles and a shared-memory control block.  Each rank here is
its own process (this file run as a script), as a GEOS rank is; every rank's state after the
steps must equal the single-rank steps of the same global state bit for bit (a halo value is a
copy either way).  The layouts: 2 ranks of three tiles, 4 ranks of 1x2 bands, and GEOS's own
topology -- one sub-domain per rank -- with 12 ranks on the GPU (layout 1x2)."""
import importlib
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIELDS = ("u", "v", "w", "delz", "pt", "delp", "q", "ps", "pe", "ua", "va", "omga")
NG = 3


def _state(pkg, d, npz):
    state = importlib.import_module(pkg.__name__ + ".state")
    ak, bk, ks = state.hybrid_levels(npz)
    st = state.jablonowski_williamson(d, ak, bk)
    d.set_vertical(ak, bk, ks)
    for k, v in st.items():
        d.upload(k, v)


def _worker(argv):
    """one rank: RANK NRANKS KEY_HEX NPX NPZ LX LY STEPS OUT"""
    rank, nranks, key, npx, npz, lx, ly, steps, out = argv
    sys.path.insert(0, ROOT)
    pkg = importlib.import_module("geosongpu-ci_amd")
    d = pkg.Domain(int(rank), int(nranks), bytes.fromhex(key), npx=int(npx), npz=int(npz), nq=2, layout_x=int(lx),
                   layout_y=int(ly), ipc=1)
    _state(pkg, d, int(npz))
    d.step(int(steps))
    d.sync()
    np.savez(out, **{k: d.download(k) for k in FIELDS})
    d.close()


@pytest.mark.gpu
@pytest.mark.parametrize("nranks,layout,npx,npz,steps", [(2, (1, 1), 13, 10, 2), (4, (1, 2), 25, 10, 1),
                                                           (12, (1, 2), 25, 10, 1)])
def test_ipc_ranks_match_single_rank(pkg, require_gpu, tmp_path, nranks, layout, npx, npz, steps):
    ref = pkg.Domain(npx=npx, npz=npz, nq=2, layout_x=layout[0], layout_y=layout[1])
    _state(pkg, ref, npz)
    ref.step(steps)
    want = {k: ref.download(k) for k in FIELDS}
    nx, ny = ref.nx, ref.ny
    ref.close()
    key = os.urandom(128).hex()
    procs = []
    for r in range(nranks):
        out = tmp_path / f"rank{r}.npz"
        cmd = [sys.executable, os.path.abspath(__file__), str(r), str(nranks), key, str(npx), str(npz),
               str(layout[0]), str(layout[1]), str(steps), str(out)]
        procs.append(subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
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
    nper = 6 * layout[0] * layout[1] // nranks
    for r in range(nranks):
        got = np.load(tmp_path / f"rank{r}.npz")
        for k in FIELDS:
            a = got[k][..., NG:NG + ny, NG:NG + nx]
            b = want[k][r * nper:(r + 1) * nper, ..., NG:NG + ny, NG:NG + nx]
            assert np.array_equal(a, b), f"rank {r} field {k}: the IPC multi-process step differs from one rank"


if __name__ == "__main__":
    _worker(sys.argv[1:])
