#!/usr/bin/env python3
"""Debug aid: one fv_dynamics step of rank 0 of an N-rank layout alone on the GPU (the null
transport, as bench.py --rank-proxy) and, per state field, the non-finite count and where
the non-finite points lie (sub-domain, level range, distance from the sub-domain edge).

    python tools/proxy_probe.py [--npx 721] [--npz 137] [--nq 4] [--ranks 8] [--layout 1x4] [--dt 112.5]
    (--ranks 1: the whole layout on one rank)
"""
import argparse
import importlib
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
NG = 3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--npx", type=int, default=721)
    ap.add_argument("--npz", type=int, default=137)
    ap.add_argument("--nq", type=int, default=4)
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--layout", default="1x4")
    ap.add_argument("--dt", type=float, default=0.0)
    ap.add_argument("--steps", type=int, default=1)
    a = ap.parse_args()
    if a.dt <= 0:
        a.dt = 450.0 * 180.0 / (a.npx - 1)
    import gtfv3_pkg
    pkg = gtfv3_pkg.load()
    state = importlib.import_module(pkg.__name__ + ".state")
    lx, ly = (int(v) for v in a.layout.split("x"))
    t0 = time.time()
    if a.ranks > 1:
        d = pkg.Domain(0, a.ranks, None, npx=a.npx, npz=a.npz, nq=a.nq, layout_x=lx, layout_y=ly, dt=a.dt, loopback=-1)
    else:
        d = pkg.Domain(npx=a.npx, npz=a.npz, nq=a.nq, layout_x=lx, layout_y=ly, dt=a.dt)
    ak, bk, ks = state.hybrid_levels(a.npz)
    st = state.jablonowski_williamson(d, ak, bk)
    d.set_vertical(ak, bk, ks)
    for k, v in st.items():
        d.upload(k, v)
    del st
    print(f"set-up {time.time() - t0:.0f} s, subs {[(s['tile'], s['ioff'], s['joff']) for s in d.subs]}", flush=True)
    for it in range(a.steps):
        d.step(1)
        print(f"step {it + 1} done {time.time() - t0:.0f} s", flush=True)
        for k in ("u", "v", "w", "delz", "pt", "delp", "ps", "q"):
            x = d.download(k)[..., NG:NG + d.ny, NG:NG + d.nx]
            bad = ~np.isfinite(x)
            nb = int(bad.sum())
            line = f"  {k:5s} non-finite {nb}/{x.size}"
            if nb:
                idx = np.argwhere(bad)
                j, i = idx[:, -2], idx[:, -1]
                dist = np.minimum(np.minimum(i, d.nx - 1 - i), np.minimum(j, d.ny - 1 - j))
                line += (f" subs {sorted(set(idx[:, 0].tolist()))} levels {idx[:, 1].min()}..{idx[:, 1].max()}"
                         f" edge distance min {dist.min()} max {dist.max()}")
            else:
                fin = x[np.isfinite(x)]
                line += f" range {fin.min():.4g} .. {fin.max():.4g}"
            print(line, flush=True)
    d.close()


if __name__ == "__main__":
    main()
