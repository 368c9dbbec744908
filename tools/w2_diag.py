"""Williamson 2 diagnostics on the GPU: where the h / u errors sit after n sub-steps."""
import sys
import numpy as np
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import importlib
pkg = importlib.import_module("geosongpu-ci_amd")
import test_gpu_williamson2 as w2
from oracle import NG

npx = int(sys.argv[1]) if len(sys.argv) > 1 else 49
dt = float(sys.argv[2]) if len(sys.argv) > 2 else 450.0
dddmp = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
d2 = float(sys.argv[4]) if len(sys.argv) > 4 else 0.0
d = pkg.Domain(npx=npx, npz=1, nq=1)
u, v, h = w2.setup_case(d)
for n, a in (("u", u), ("v", v), ("delp", h), ("pt", np.ones(d.shape(1))), ("w", d.zeros(1))):
    d.upload(n, a)
sw = w2.ShallowWater(d, dt, dddmp, d2)
area = d.metric("area")[:, None]
c = (Ellipsis, slice(NG, NG + d.ny), slice(NG, NG + d.nx))
cu = (Ellipsis, slice(NG, NG + d.ny + 1), slice(NG, NG + d.nx))
done = 0
for n in (1, 10, 100, int(5 * 86400 / dt)):
    while done < n:
        sw.substep()
        done += 1
    hh = d.download("delp")
    uu = d.download("u")
    r = w2.norms(hh, h, area, d)
    eh = np.abs(hh[c] - h[c])[:, 0]
    eu = np.abs(uu[cu] - u[cu])[:, 0]
    ih = np.unravel_index(np.argmax(eh), eh.shape)
    iu = np.unravel_index(np.argmax(eu), eu.shape)
    print(f"n={n}: l2 {r['l2']:.3e} linf {r['linf']:.3e} mass {r['mass']:.3e}; max|dh| {eh.max():.3e} at tile,j,i {ih};"
          f" max|du| {eu.max():.3e} at {iu}; median|du| {np.median(eu):.3e}", flush=True)
    if n == 10:
        # error by distance to the nearest cube corner / edge
        N = d.N
        jj, ii = np.meshgrid(np.arange(d.ny), np.arange(d.nx), indexing="ij")
        dist = np.minimum(np.minimum(ii, N - 1 - ii), np.minimum(jj, N - 1 - jj))
        for k in range(0, 6):
            m = dist == k
            print(f"   edge distance {k}: mean|dh| {eh[:, m].mean():.3e} mean|du| {eu[:, :-1][:, m].mean():.3e}")
        m = dist > 8
        print(f"   interior: mean|dh| {eh[:, m].mean():.3e} mean|du| {eu[:, :-1][:, m].mean():.3e}")
d.close()
