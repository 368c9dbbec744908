"""Per-level differences of the blocked Riemann kernel (dump mode) against the column
kernel's work planes (debug aid)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import gtfv3_pkg  # noqa: E402
from conftest import rng  # noqa: E402
from test_gpu_riem import DZ_MIN, P_FAC, PTOP, columns, region  # noqa: E402

pkg = gtfv3_pkg.load()
for npz, thin in ((12, False),):
    d = pkg.Domain(npx=13, npz=npz, nq=1)
    r = rng(100 + npz)
    col = columns(d, npz, r, thin)
    dt2 = 225.0
    for k in ("delp", "pt", "w", "phis"):
        d.upload("rc_" + k, col[k])
    got = {}
    for var in (1, 2):
        d.upload("rc_gz", col["zh"])
        d.stencil("riem_solver_c", ["rc_delp", "rc_pt", "rc_w", "rc_phis", "rc_gz", "rc_pef"],
                  [dt2, PTOP, P_FAC, DZ_MIN, var])
        got[var] = {k: region(d.download(k), 1, d.nx, d.ny)[0] for k in
                    ("rc_gz", "rc_pef", "_riem_w2", "_riem_gam", "_riem_pp")}
    print(f"npz={npz} thin={thin}")
    for k in got[1]:
        a, b = got[2][k], got[1][k]
        e = np.abs(a - b).max(axis=(1, 2)) / (np.abs(b).mean() + 1e-300)
        print(f"  {k:10s}: " + " ".join(f"{x:.1e}" for x in e))
    print("w2 col 0:", got[1]["_riem_w2"][:, 1, 1])
    print("w2 blk 0:", got[2]["_riem_w2"][:, 1, 1])
    print("gam col :", got[1]["_riem_gam"][:, 1, 1])
    print("gam blk :", got[2]["_riem_gam"][:, 1, 1])
    d.close()
