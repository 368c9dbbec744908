"""Williamson 2 at several resolutions: global and interior (edge distance > N/8) height errors
after 5 days, and the mass change."""
import sys
import importlib
import numpy as np
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
pkg = importlib.import_module("geosongpu-ci_amd")
import test_gpu_williamson2 as w2
from oracle import NG

for npx, dt in ((25, 900.0), (49, 450.0), (97, 225.0)):
    d = pkg.Domain(npx=npx, npz=1, nq=1)
    u, v, h = w2.setup_case(d)
    for n, a in (("u", u), ("v", v), ("delp", h), ("pt", np.ones(d.shape(1))), ("w", d.zeros(1))):
        d.upload(n, a)
    sw = w2.ShallowWater(d, dt)
    for _ in range(int(round(5 * 86400 / dt))):
        sw.substep()
    hh = d.download("delp")
    area = d.metric("area")[:, None]
    r = w2.norms(hh, h, area, d)
    c = (Ellipsis, slice(NG, NG + d.ny), slice(NG, NG + d.nx))
    N = d.N
    jj, ii = np.meshgrid(np.arange(d.ny), np.arange(d.nx), indexing="ij")
    dist = np.minimum(np.minimum(ii, N - 1 - ii), np.minimum(jj, N - 1 - jj))
    m = dist >= N // 8
    e = (hh[c] - h[c])[:, 0][:, m]
    w = area[c][:, 0][:, m]
    ref = h[c][:, 0][:, m]
    l2i = np.sqrt((e ** 2 * w).sum() / (ref ** 2 * w).sum())
    print(f"C{npx - 1}: {r}  interior l2 {l2i:.3e} linf {np.abs(e).max() / np.abs(ref).max():.3e}", flush=True)
    d.close()
