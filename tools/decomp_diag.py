#!/usr/bin/env python3
"""Debug aid: one fv_dynamics step of the same global state on 1x1 and on LXxLY sub-domains
per tile; per field, how many compute-domain values differ, by how much, and where (level,
distance from the nearest sub-domain edge, first few points).

    python tools/decomp_diag.py [--npx 13] [--npz 10] [--layout 2x2] [--n-split 6]
"""
import argparse
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
NG = 3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--npx", type=int, default=13)
    ap.add_argument("--npz", type=int, default=10)
    ap.add_argument("--layout", default="2x2")
    ap.add_argument("--n-split", type=int, default=6)
    ap.add_argument("--nq", type=int, default=2)
    a = ap.parse_args()
    import gtfv3_pkg
    pkg = gtfv3_pkg.load()
    state = importlib.import_module(pkg.__name__ + ".state")
    lx, ly = (int(v) for v in a.layout.split("x"))
    ak, bk, ks = state.hybrid_levels(a.npz)
    names = ("u", "v", "w", "delz", "pt", "delp", "q", "ps", "pe", "omga", "ua", "va")
    outs = {}
    for lay in ((1, 1), (lx, ly)):
        d = pkg.Domain(npx=a.npx, npz=a.npz, nq=a.nq, layout_x=lay[0], layout_y=lay[1], n_split=a.n_split)
        st = state.jablonowski_williamson(d, ak, bk)
        d.set_vertical(ak, bk, ks)
        for k, v in st.items():
            d.upload(k, v)
        d.step(1)
        outs[lay] = (d, {k: d.download(k) for k in names})
    d1, o1 = outs[(1, 1)]
    d2, o2 = outs[(lx, ly)]
    for k in names:
        nd, worst, where = 0, 0.0, []
        hist = {}
        for s2, sub in enumerate(d2.subs):
            t, io, jo = sub["tile"], sub["ioff"], sub["joff"]
            a2 = o2[k][s2][..., NG:NG + d2.ny, NG:NG + d2.nx]
            b1 = o1[k][t][..., NG + jo:NG + jo + d2.ny, NG + io:NG + io + d2.nx]
            m = a2 != b1
            if not m.any():
                continue
            nd += int(m.sum())
            worst = max(worst, float(np.abs(a2 - b1)[m].max() / (np.abs(b1).mean() + 1e-300)))
            idx = np.argwhere(m)
            for p in idx:
                j, i = p[-2], p[-1]
                dist = int(min(i, j, d2.nx - 1 - i, d2.ny - 1 - j))
                hist[dist] = hist.get(dist, 0) + 1
            if len(where) < 6:
                where += [(s2, t, io, jo) + tuple(int(x) for x in p) for p in idx[:6 - len(where)]]
        total = sum(o2[k][s][..., NG:NG + d2.ny, NG:NG + d2.nx].size for s in range(len(d2.subs)))
        print(f"{k:5s} differ {nd:7d}/{total}  max scaled {worst:.2e}  by edge distance {dict(sorted(hist.items()))}"
              f"  first (sub, tile, ioff, joff, [k,] j, i): {where}", flush=True)


if __name__ == "__main__":
    main()
