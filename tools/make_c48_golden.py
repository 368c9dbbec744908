#!/usr/bin/env python3
"""Golden fixture for BASELINE config 2 (Held-Suarez C48 L72, all 6 tiles on one GPU): one
oracle fv_dynamics step (oracle/fv_dynamics.py, numpy fp64) from the JW06 state, run HERE on
the CPU (~75 s; too slow to repeat inside a GPU test).  The fixture keeps, per state field,
the value at a fixed random sample of compute-domain points and the mean over the compute
domain of every (sub-domain, level) plane:

    python tools/make_c48_golden.py              ->  tests/golden/c48_l72_step.npz
    python tools/make_c48_golden.py --no-sponge  ->  tests/golden/c48_l72_step_nosponge.npz
                                                     (n_sponge = -1: the round-4 namelist)

tests/test_gpu_configs.py runs the HIP step on the same state and compares."""
import importlib
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import gtfv3_pkg  # noqa: E402
from conftest import metrics_of, oracle_scalars  # noqa: E402
from oracle import NG  # noqa: E402
from oracle import fv_dynamics as fvd  # noqa: E402

NPX, NPZ, NQ, DT = 49, 72, 4, 900.0
FIELDS = ("u", "v", "w", "delz", "pt", "delp", "q", "ua", "va", "omga", "pkz", "ps", "pe", "peln", "pk")
NSAMPLE = 1500
NL = dict(n_split=6, dt_atmos=DT, hord_mt=6, hord_vt=6, hord_tm=6, hord_dp=6, hord_tr=6, dddmp=0.2, d2_bg=0.0,
          p_fac=0.05, dz_min=2.0, fill=1, nq=NQ)


def main():
    nosponge = "--no-sponge" in sys.argv
    nl = dict(NL, n_sponge=-1) if nosponge else NL
    pkg = gtfv3_pkg.load()
    state = importlib.import_module(pkg.__name__ + ".state")
    d = pkg.Domain(npx=NPX, npz=NPZ, nq=NQ, host_only=1)
    ak, bk, ks = state.hybrid_levels(NPZ)
    st = state.jablonowski_williamson(d, ak, bk)
    ms = metrics_of(d)
    sc = oracle_scalars(d)
    g = fvd.Grid(d.N, 1, 1, ms, sc["corner_w"], sc["da_min_c"], d.nj, d.pitch)
    t0 = time.time()
    ref = fvd.fv_dynamics(st, ak, bk, g, nl)
    print(f"oracle step {time.time() - t0:.1f} s")
    n = d.N
    r = np.random.default_rng(4872)
    out = dict(npx=NPX, npz=NPZ, nq=NQ, dt=DT)
    for k in FIELDS:
        a = ref[k][..., NG:NG + n, NG:NG + n]  # (6, nk, n, n) compute domain
        idx = np.stack([r.integers(0, m, NSAMPLE) for m in a.shape], axis=1).astype(np.int16)
        out[f"{k}_idx"] = idx
        out[f"{k}_val"] = a[tuple(idx.T)]
        out[f"{k}_mean"] = a.mean(axis=(2, 3))
    np.savez_compressed(os.path.join(ROOT, "tests", "golden",
                                     "c48_l72_step_nosponge.npz" if nosponge else "c48_l72_step.npz"), **out)


if __name__ == "__main__":
    main()
