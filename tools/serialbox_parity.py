#!/usr/bin/env python3
"""Step a serialized FVDynamics-In savepoint (one archive prefix per tile, layout 1x1:
Generator_rank0..5) with this package's dycore and compare with FVDynamics-Out, field by
field, with the CI's own bar (relative 1e-4, physics_standalone.py:132-144) -- the route to
reference-numeric parity once a GEOS dump (geos_build/serialize) is available.

    python tools/serialbox_parity.py DATA_DIR [--engine hip|oracle] [--savepoint N]

Namelist and vertical grid come from the savepoint (ak, bk, ks, bdt, nq) and DATA_DIR/input.nml
(n_split, hord_*, dddmp, p_fac, dz_min).  `--engine oracle` runs oracle/fv_dynamics.py on the
CPU instead of the HIP step (test infrastructure)."""
import argparse
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def load(data, k):
    import gtfv3_pkg
    pkg = gtfv3_pkg.load()
    sb = importlib.import_module(pkg.__name__ + ".serialbox")
    readers = [sb.SerialboxReader(data, f"Generator_rank{r}") for r in range(6)]
    sp_in = [rd.get_savepoint("FVDynamics-In")[k] for rd in readers]
    r0 = readers[0]
    scal = {n: sb.read_serialized_data(r0, sp_in[0], n) for n in ("bdt", "ks", "nq", "ptop")
            if n in r0.fields_at_savepoint(sp_in[0])}
    ak = np.asarray(r0.read("ak", sp_in[0]), dtype=np.float64).ravel()
    bk = np.asarray(r0.read("bk", sp_in[0]), dtype=np.float64).ravel()
    npz = len(ak) - 1
    delp0 = r0.read("delp", sp_in[0])
    n = delp0.shape[0] - 6
    nq = int(scal.get("nq", 6))
    return pkg, sb, readers, sp_in, scal, ak, bk, npz, n, nq


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("data")
    p.add_argument("--engine", default="hip", choices=("hip", "oracle"))
    p.add_argument("--savepoint", type=int, default=0)
    p.add_argument("--rtol", type=float, default=1e-4)
    a = p.parse_args(argv)
    pkg, sb, readers, sp_in, scal, ak, bk, npz, n, nq = load(a.data, a.savepoint)
    nml = sb.read_namelist(os.path.join(a.data, "input.nml")).get("fv_core_nml", {}) \
        if os.path.exists(os.path.join(a.data, "input.nml")) else {}
    cfg = dict(n_split=int(nml.get("n_split", 6)), dt_atmos=float(scal.get("bdt", 900.0)),
               hord_mt=int(nml.get("hord_mt", 6)), hord_vt=int(nml.get("hord_vt", 6)),
               hord_tm=int(nml.get("hord_tm", 6)), hord_dp=int(nml.get("hord_dp", 6)),
               hord_tr=int(nml.get("hord_tr", 6)), dddmp=float(nml.get("dddmp", 0.2)),
               d2_bg=float(nml.get("d2_bg", 0.0)), p_fac=float(nml.get("p_fac", 0.05)),
               dz_min=float(nml.get("dz_min", 2.0)), fill=1, nq=nq)
    host = pkg.Domain(npx=n + 1, npz=npz, nq=nq, host_only=1)
    per = [sb.fv_dynamics_state(rd, sp, host) for rd, sp in zip(readers, sp_in)]
    st = {k: np.stack([ps[k] for ps in per]) for k in per[0]}
    ks = int(scal.get("ks", 0))
    if a.engine == "oracle":
        from conftest import metrics_of, oracle_scalars
        from oracle import fv_dynamics as fvd
        ms = metrics_of(host)
        sc = oracle_scalars(host)
        g = fvd.Grid(host.N, 1, 1, ms, sc["corner_w"], sc["da_min_c"], host.nj, host.pitch)
        out = fvd.fv_dynamics(st, ak, bk, g, cfg)
    else:
        d = pkg.Domain(npx=n + 1, npz=npz, nq=nq, dt=cfg["dt_atmos"], n_split=cfg["n_split"],
                       hord_mt=cfg["hord_mt"], hord_vt=cfg["hord_vt"], hord_tm=cfg["hord_tm"],
                       hord_dp=cfg["hord_dp"], hord_tr=cfg["hord_tr"], dddmp=cfg["dddmp"], d2_bg=cfg["d2_bg"],
                       p_fac=cfg["p_fac"])
        d.set_vertical(ak, bk, ks)
        for k, v in st.items():
            d.upload(k, v)
        d.step(1)
        out = {k: d.download(k) for k in st}
        d.close()
    worst = {}
    for r, rd in enumerate(readers):
        sp_out = rd.get_savepoint("FVDynamics-Out")[a.savepoint]
        got = sb.state_to_savepoint(out, r, n)
        for name in sorted(set(got) & set(rd.fields_at_savepoint(sp_out))):
            ref = np.asarray(sb.read_serialized_data(rd, sp_out, name), dtype=np.float64)
            g = got[name]
            if name in ("u", "v", "uc", "vc", "ua", "va", "delp", "pt", "delz", "w", "omga", "q_con") or \
                    name in sb.FV_DYNAMICS_TRACERS:
                g, ref = g[3:-3, 3:-3], ref[3:-3, 3:-3]  # compute domain (+ staggered edge)
            scale = max(np.abs(ref).max(), 1e-300)
            worst[name] = max(worst.get(name, 0.0), float(np.abs(g - ref).max() / scale))
    bad = {k: v for k, v in worst.items() if v > a.rtol}
    for k, v in sorted(worst.items()):
        print(f"{k:10s} max |diff| / max |ref| = {v:.2e}{'  FAIL' if k in bad else ''}")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
