#!/usr/bin/env python3
"""Debug aid: replay the first C-grid Riemann solve of an oracle C12 step (inputs recorded at
the oracle's call site) through the scan kernel, and dump the intermediates of one column
(riem_solver_c's optional debug field) next to the numpy model of the kernel
(tests/test_blockscan_emul.py's tri_solve is the model of the solves).

    python tools/dbg_riem_replay.py [npz] [j i]

The dump needs a library built with the column dump compiled in:
    make -C geosongpu-ci_amd/csrc clean && make -C geosongpu-ci_amd/csrc CXXFLAGS+=-DGTFV3_RIEM_DEBUG
(without it the debug field stays NaN and only the non-finite column scan is meaningful).
"""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

import gtfv3_pkg  # noqa: E402
from conftest import metrics_of, oracle_scalars  # noqa: E402
from oracle import fv_dynamics as fvd, nh_core  # noqa: E402

NAMES = ["pem", "dz", "pm", "pl", "g", "pp", "aat", "w2", "pe", "p1v", "dz2", "gz", "-", "gl", "G", "dd", "rhs_w",
         "p1"]


def main():
    npz = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    jc, ic = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (9, 10)
    pkg = gtfv3_pkg.load()
    state = importlib.import_module(pkg.__name__ + ".state")
    d = pkg.Domain(npx=13, npz=npz, nq=2, n_split=6)
    ak, bk, ks = state.hybrid_levels(npz)
    st = state.jablonowski_williamson(d, ak, bk)
    sc = oracle_scalars(d)
    g = fvd.Grid(d.N, 1, 1, metrics_of(d), sc["corner_w"], sc["da_min_c"], d.nj, d.pitch)
    rec = []
    orig = nh_core.riem_solver_c

    def rc(*a):
        a = [np.copy(x) if isinstance(x, np.ndarray) else x for x in a]
        out = orig(*a)
        rec.append((a, out))
        return out

    nh_core.riem_solver_c = rc
    nl = dict(n_split=6, dt_atmos=900.0, hord_mt=6, hord_vt=6, hord_tm=6, hord_dp=6, hord_tr=6, dddmp=0.2,
              d2_bg=0.0, p_fac=0.05, dz_min=2.0, fill=1, nq=2)
    fvd.fv_dynamics(st, ak, bk, g, nl)
    cin = [rec[s][0] for s in range(d.nsub)]
    for k, i in (("delp", 1), ("pt", 2), ("w", 3), ("zh", 4)):
        d.upload("rs_" + k, np.stack([c[i] for c in cin]))
    d.upload("rs_phis", np.stack([c[5][None] for c in cin]))
    col = (jc + 1) * (d.nx + 2) + (ic + 1)
    if os.environ.get("COL_FIRST"):  # the column form first, on the same planes (as the test does)
        d.stencil("riem_solver_c", ["rs_delp", "rs_pt", "rs_w", "rs_phis", "rs_zh", "rs_pef"],
                  [cin[0][0], cin[0][7], 0.05, 2.0, 1])
        d.upload("rs_zh", np.stack([c[4] for c in cin]))
    d.upload("rs_dbg", np.full(d.shape(32), np.nan))
    d.stencil("riem_solver_c", ["rs_delp", "rs_pt", "rs_w", "rs_phis", "rs_zh", "rs_pef", "rs_dbg"],
              [cin[0][0], cin[0][7], 0.05, 2.0, 0, col])
    dbg = d.download("rs_dbg").ravel()
    allp = d.download("rs_pef")
    bad = [(s, j - 3, i - 3) for s in range(d.nsub) for j in range(2, d.ny + 4) for i in range(2, d.nx + 4)
           if np.isfinite(rec[s][1][0][:, j, i]).all() and not np.isfinite(allp[s][:, j, i]).all()]
    print("non-finite columns where the oracle is finite:", bad[:20])
    pef = allp[0][:, jc + 3, ic + 3]
    print("pef", pef)
    print("want", rec[0][1][0][:, jc + 3, ic + 3])
    M, NB = {10: (3, 4), 72: (9, 8)}.get(npz, (3, 4))
    for ph, nm in enumerate(NAMES):
        v = dbg[ph * NB * M:(ph + 1) * NB * M]
        print(f"{nm:6s}", np.array2string(v, precision=6, max_line_width=250))


if __name__ == "__main__":
    main()
