#!/usr/bin/env python3
"""PCIe-inclusive time of the drop-in boundary: geos_gtfv3_run_f64_c (through the Python
hook mirror) on Fortran-layout host buffers, C180 L72 nq=4, all six tiles on one GPU.
Each call moves the state arrays host -> device (fused transpose), runs one fv_dynamics
step and copies them back in place, the uploads the step reads late and the copies back of
the groups it finishes early overlapped with it.  GTFV3_BRIDGE_ZC selects the
transfer forms (bridge.hip).  The device-resident step
alone is what bench.py reports.

    python tools/bridge_bench.py [--npx 181] [--npz 72] [--steps 3]
"""
import argparse
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--npx", type=int, default=181)
    ap.add_argument("--npz", type=int, default=72)
    ap.add_argument("--nq", type=int, default=4)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--dtype", choices=("f64", "f32"), default="f64",
                    help="f64: geos_gtfv3_run_f64_c; f32: geos_gtfv3_run_c (float* arrays)")
    a = ap.parse_args()
    os.environ["GTFV3_BRIDGE_TILES_PER_RANK"] = "6"
    import numpy as np
    import gtfv3_pkg
    from oracle import NG
    from test_gpu_bridge import to_fortran
    pkg = gtfv3_pkg.load()
    hook = importlib.import_module(pkg.__name__ + ".hook").geos_gtfv3
    state = importlib.import_module(pkg.__name__ + ".state")
    npx, npz, nq = a.npx, a.npz, a.nq
    dt = np.float64 if a.dtype == "f64" else np.float32
    N = npx - 1
    d = pkg.Domain(npx=npx, npz=npz, nq=nq)
    ak, bk, ks = state.hybrid_levels(npz)
    st = state.jablonowski_williamson(d, ak, bk)
    nsub, nj, pitch = d.nsub, d.nj, d.pitch
    d.close()
    is_, ie, js, je = 1, N, 1, N
    isd, ied, jsd, jed = is_ - NG, ie + NG, js - NG, je + NG
    L = lambda x: x - 1  # noqa: E731
    cell = (L(isd), L(ied), L(jsd), L(jed))
    shapes = {"u": (L(isd), L(ied), L(jsd), L(jed + 1), npz, False), "v": (L(isd), L(ied + 1), L(jsd), L(jed), npz, False),
              "w": cell + (npz, False), "delz": cell + (npz, False), "pt": cell + (npz, False), "delp": cell + (npz, False),
              "q": cell + (npz * nq, False), "ps": cell + (1, False),
              "pe": (L(is_ - 1), L(ie + 1), L(js - 1), L(je + 1), npz + 1, True),
              "pk": (L(is_), L(ie), L(js), L(je), npz + 1, False), "peln": (L(is_), L(ie), L(js), L(je), npz + 1, True),
              "pkz": (L(is_), L(ie), L(js), L(je), npz, False), "phis": cell + (1, False), "q_con": cell + (npz, False),
              "omga": cell + (npz, False), "ua": cell + (npz, False), "va": cell + (npz, False),
              "uc": (L(isd), L(ied + 1), L(jsd), L(jed), npz, False), "vc": (L(isd), L(ied), L(jsd), L(jed + 1), npz, False),
              "mfx": (L(is_), L(ie + 1), L(js), L(je), npz, False), "mfy": (L(is_), L(ie), L(js), L(je + 1), npz, False),
              "cx": (L(is_), L(ie + 1), L(jsd), L(jed), npz, False), "cy": (L(isd), L(ied), L(js), L(je + 1), npz, False),
              "diss_est": cell + (npz, False)}
    fort = {}
    for name, (li, hi, lj, hj, nk, kj) in shapes.items():
        src = st[name] if name in st else np.zeros((nsub, nk, nj, pitch))
        fort[name] = to_fortran(src, li, hi, lj, hj, kj).astype(dt)
    del st
    nbytes = sum(v.nbytes for v in fort.values())
    scal = dict(comm=0, npx=npx, npy=npx, npz=npz, ntiles=6, is_=is_, ie=ie, js=js, je=je, isd=isd, ied=ied,
                jsd=jsd, jed=jed, bdt=450.0, nq_tot=nq)
    run = dict(scal, ng=NG, ptop=float(ak[0]), ks=ks, layout_1=1, layout_2=1, adiabatic=1,
               ak=np.asfortranarray(ak.astype(dt)), bk=np.asfortranarray(bk.astype(dt)))
    hook.init(**scal)
    hook.run(**run, **fort)  # warm-up
    import ctypes
    st_out = (ctypes.c_double * 6)()
    phases = []
    t0 = time.perf_counter()
    for _ in range(a.steps):
        hook.run(**run, **fort)
        pkg.lib().gtfv3_bridge_stats(st_out)
        phases.append(list(st_out))
    el = (time.perf_counter() - t0) / a.steps
    hook.finalize()
    ph = np.median(np.array(phases), axis=0)
    cells = 6 * N * N * npz
    fn = "geos_gtfv3_run_f64_c" if a.dtype == "f64" else "geos_gtfv3_run_c"
    print(json.dumps({"what": f"{fn} incl. host<->device copies", "dtype": a.dtype, "npx": npx, "npz": npz,
                      "nq": nq, "ms_per_call": 1e3 * el, "cell_updates_per_s": cells / el,
                      "host_bytes_of_the_arrays": nbytes,
                      "transfer_zc_mask": int(os.environ.get("GTFV3_BRIDGE_ZC", "1")),
                      "median_phases_ms": {"upload_before_step": ph[0], "step_incl_waits": ph[1],
                                           "copy_back_after_step": ph[2]},
                      "bytes_up": ph[3], "bytes_down": ph[4], "arrays_pinned": int(ph[5])}))


if __name__ == "__main__":
    main()
