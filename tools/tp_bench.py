#!/usr/bin/env python3
"""Time the fv_tp_2d kernel variants (stencil param cfg) at C180 L72 on one GPU,
checking each against the default variant bit for bit.

    python tools/tp_bench.py [--npx 181] [--npz 72] [--reps 10]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--npx", type=int, default=181)
    ap.add_argument("--npz", type=int, default=72)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--cfgs", default="-1,30,45,60,90")
    a = ap.parse_args()
    import torch
    import gtfv3_pkg
    torch.cuda.set_device(0)
    pkg = gtfv3_pkg.load()
    d = pkg.Domain(npx=a.npx, npz=a.npz, nq=1)
    r = np.random.default_rng(3)
    sh = d.shape(a.npz)
    area = d.metric("area")[:, None]
    inp = dict(q=1.0 + 0.2 * r.standard_normal(sh), crx=r.uniform(-0.4, 0.4, sh), cry=r.uniform(-0.4, 0.4, sh),
               xfx=0.2 * r.uniform(-1, 1, sh) * area, yfx=0.2 * r.uniform(-1, 1, sh) * area)
    inp["ra_x"] = area + inp["xfx"] - np.roll(inp["xfx"], -1, axis=-1)
    inp["ra_y"] = area + inp["yfx"] - np.roll(inp["yfx"], -1, axis=-2)
    for k, v in inp.items():
        d.upload("t_" + k, v)
    names = ["t_q", "t_crx", "t_cry", "t_xfx", "t_yfx", "t_ra_x", "t_ra_y", "-", "-", "t_fx", "t_fy"]
    ref = None
    for cfg in [int(x) for x in a.cfgs.split(",")]:
        d.stencil("fv_tp_2d", names, [6, 1, cfg])
        d.sync()
        got = (d.download("t_fx"), d.download("t_fy"))
        if ref is None:
            ref = got
        same = all(np.array_equal(x, y) for x, y in zip(got, ref))
        d.kernel_timing(True)
        for _ in range(a.reps):
            d.stencil("fv_tp_2d", names, [6, 1, cfg])
        st = d.kernel_stats()
        d.kernel_timing(False)
        ms = {k: v[0] / v[1] for k, v in st.items()}
        gb = {k: v[2] / (v[0] * 1e-3) / 1e9 for k, v in st.items()}
        cells = d.nsub * d.nx * d.ny * a.npz
        for k, v in ms.items():
            print(f"cfg {cfg:2d} {k[:40]:40s} {v:.4f} ms  {gb[k]:7.1f} GB/s algorithmic  identical={same}", flush=True)


if __name__ == "__main__":
    main()
