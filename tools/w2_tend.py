"""Williamson 2: the one-sub-step tendencies du/dt, dv/dt, dh/dt of the balanced state (small dt),
by resolution -- where the discrete balance is inconsistent (a tendency that does not shrink
with the grid spacing)."""
import sys
import importlib
import numpy as np
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
pkg = importlib.import_module("geosongpu-ci_amd")
import test_gpu_williamson2 as w2
from oracle import NG

dt = 10.0
for npx in (25, 49, 97):
    d = pkg.Domain(npx=npx, npz=1, nq=1)
    u, v, h = w2.setup_case(d)
    for n, a in (("u", u), ("v", v), ("delp", h), ("pt", np.ones(d.shape(1))), ("w", d.zeros(1))):
        d.upload(n, a)
    sw = w2.ShallowWater(d, dt)
    sw.substep()
    N = d.N
    out = []
    for name, ref, ex, ey in (("u", u, 0, 1), ("v", v, 1, 0), ("delp", h, 0, 0)):
        a = d.download(name)
        t = (a - ref)[:, 0, NG:NG + d.ny + ey, NG:NG + d.nx + ex] / dt
        jj, ii = np.meshgrid(np.arange(d.ny + ey), np.arange(d.nx + ex), indexing="ij")
        # distance to the nearest cube corner (in cells)
        dc = np.minimum.reduce([np.hypot(ii - ci, jj - cj) for ci in (0, N) for cj in (0, N)])
        de = np.minimum(np.minimum(ii, N - ii), np.minimum(jj, N - jj))
        at = np.abs(t)
        k = np.unravel_index(np.argmax(at), at.shape)
        s = [f"{name}: max|d/dt| {at.max():.3e} at tile,j,i {tuple(int(x) for x in k)}"]
        for lab, m in (("corner<2", dc < 2), ("corner 2-4", (dc >= 2) & (dc < 4)), ("edge (not corner)", (de == 0) & (dc >= 4)),
                       ("edge+1", (de == 1) & (dc >= 4)), ("interior", de >= N // 8)):
            s.append(f"{lab} {at[:, m].max():.2e}")
        out.append("; ".join(s))
    print(f"C{npx - 1}:\n  " + "\n  ".join(out), flush=True)
    d.close()
