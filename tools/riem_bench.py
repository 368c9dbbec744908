#!/usr/bin/env python3
"""Time the SIM1 Riemann solver kernels (riem_solver_c / riem_solver3) at C180 L72 on one
GPU from near-hydrostatic synthetic columns (tests/test_gpu_riem.py), per variant.

    python tools/riem_bench.py [--npx 181] [--npz 72] [--reps 5] [--vars 0,1]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--npx", type=int, default=181)
    ap.add_argument("--npz", type=int, default=72)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--vars", default="0")
    a = ap.parse_args()
    import numpy as np
    import torch
    import gtfv3_pkg
    from conftest import rng
    from test_gpu_riem import DZ_MIN, P_FAC, PTOP, columns
    torch.cuda.set_device(0)
    pkg = gtfv3_pkg.load()
    d = pkg.Domain(npx=a.npx, npz=a.npz, nq=1)
    col = columns(d, a.npz, rng(7), True)
    for k in ("delp", "pt", "w", "phis"):
        d.upload("r_" + k, col[k])
    d.upload("r_zh0", col["zh"])
    for var in [int(x) for x in a.vars.split(",")]:
        for name, fields, params in (
                ("riem_solver_c", ["r_delp", "r_pt", "r_w", "r_phis", "r_gz", "r_pef"],
                 [225.0, PTOP, P_FAC, DZ_MIN, var]),
                ("riem_solver3", ["r_delp", "r_pt", "r_w3", "r_phis", "r_zh", "r_delz", "r_ppe", "r_pk3", "r_pe",
                                  "r_peln", "r_pk", "r_ws"], [450.0, PTOP, P_FAC, DZ_MIN, 0, var])):
            d.kernel_timing(True)
            for _ in range(a.reps):
                d.upload("r_gz", col["zh"])
                d.upload("r_zh", col["zh"])
                d.upload("r_w3", col["w"])
                d.stencil(name, fields, params)
            st = d.kernel_stats()
            d.kernel_timing(False)
            for k, v in st.items():
                if "riem" in k:
                    print(f"var {var} {name:14s} {k:32s} {v[0] / v[1]:.4f} ms  "
                          f"{(v[2] / (v[0] * 1e-3) / 1e9) if v[2] else 0:7.1f} GB/s algorithmic", flush=True)
    del np


if __name__ == "__main__":
    main()
