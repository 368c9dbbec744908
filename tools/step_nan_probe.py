#!/usr/bin/env python3
"""Debug aid: one C12 fv_dynamics step per riem form (GTFV3_RIEM is read once per process,
so each form runs in its own child process) and the non-finite count of every state field.

    python tools/step_nan_probe.py [--npz 10] [--n-split 5]
"""
import argparse
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def one(npz, n_split):
    sys.path.insert(0, ROOT)
    import importlib
    import numpy as np
    import gtfv3_pkg
    pkg = gtfv3_pkg.load()
    state = importlib.import_module(pkg.__name__ + ".state")
    d = pkg.Domain(npx=13, npz=npz, nq=2, n_split=n_split)
    ak, bk, ks = state.hybrid_levels(npz)
    st = state.jablonowski_williamson(d, ak, bk)
    d.set_vertical(ak, bk, ks)
    for k, v in st.items():
        d.upload(k, v)
    d.step(1)
    out = {}
    for k in ("u", "v", "w", "delz", "pt", "delp", "pe", "pk", "peln", "ps"):
        a = d.download(k)[..., 3:3 + d.ny, 3:3 + d.nx]
        out[k] = int((~np.isfinite(a)).sum())
    print(os.environ.get("GTFV3_RIEM", "0"), out, flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--npz", type=int, default=10)
    ap.add_argument("--n-split", type=int, default=5)
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        one(a.npz, a.n_split)
    else:
        for v in ("1", "0"):
            env = dict(os.environ, GTFV3_RIEM=v)
            subprocess.run([sys.executable, __file__, "--child", "--npz", str(a.npz), "--n-split", str(a.n_split)],
                           env=env, check=False)
