"""Williamson et al. (1992) shallow-water test case 1 -- advection of a cosine bell by solid-body
rotation for 12 days (one revolution) -- run on the HIP tracer transport (tracer_2d_1l: the
fused fv_tp_2d column marches + the flux-form update, with the cubed-sphere halo exchange
between sub-steps), as Putman & Lin (2007, J. Comput. Phys. 227, section 5.1) ran it on the
FV3 transport scheme.  A published case that pins the transport independently of this
package's own oracle.

Set-up (Williamson 1992 section 3.1): bell h = (h0 / 2)(1 + cos(pi r / R)) for r < R = a / 3,
h0 = 1000 m, centred at (3 pi / 2, 0); rotation with u0 = 2 pi a / (12 days) about an axis
tilted by alpha.  The flow enters as area fluxes through the cell edges, differences of the
stream function psi = -a u0 (sin(lat) cos(alpha) - cos(lon) cos(lat) sin(alpha)) between the
edge's end points (exactly non-divergent up to round-off: dp2 stays 1), the Courant numbers
from those fluxes with tracer_2d's own upwind metric factors.

Checked (hord 6, alpha = pi / 4: the bell crosses two cube corners, and alpha = 0):
  * mass: the area integral of h.  The two tiles at a shared edge compute its flux each from
    their own halo: identical to round-off except on the two edges next to each cube corner,
    whose inner cross-sweep reads the tile's own copy_corners fill -- FV3's fv_tp_2d, shown on
    the oracle by tests/test_oracle_transport_corners.py.  So alpha = 0 (the bell away from
    the corners) conserves to 1.6e-10 over the revolution, and through the corners the HIP
    mass trajectory is pinned to the oracle's (test_williamson1_corner_mass_matches_oracle:
    same run, same fields to 1e-11, the same mass change, 8.8e-5 over the first 24 C24 steps);
  * accuracy after one revolution, normalised l1 / l2 / l_inf errors at C48 (1.875 deg):
    Putman & Lin (2007) report errors of a few 1e-2 for PPM at this resolution; the bar here
    is l2 <= 0.05 and l_inf <= 0.05 (measured on MI355X: alpha = pi/4 l1 0.027, l2 0.019,
    l_inf 0.026; alpha = 0 l1 0.029, l2 0.022, l_inf 0.029);
  * convergence from C24 to C48: l2 falls by at least 2.5x (measured 6.3x and 5.4x: order
    2.4-2.7; the scheme is formally 2nd-3rd order, limited by the bell's C1 edge).
"""
import numpy as np
import pytest

from oracle import NG

pytestmark = pytest.mark.gpu

A = 6371.0e3
DAY = 86400.0


def _bell(lat, lon):
    lc, tc = 1.5 * np.pi, 0.0
    r = A * np.arccos(np.clip(np.sin(tc) * np.sin(lat) + np.cos(tc) * np.cos(lat) * np.cos(lon - lc), -1.0, 1.0))
    return np.where(r < A / 3.0, 500.0 * (1.0 + np.cos(np.pi * r / (A / 3.0))), 0.0)


def setup_case(d, alpha, nsteps):
    """(q0, cx, cy, xfx, yfx, area) planes of a Domain (host-only suffices) for one revolution in
    `nsteps` steps about an axis tilted by alpha"""
    dt = 12.0 * DAY / nsteps
    u0 = 2.0 * np.pi * A / (12.0 * DAY)
    xyz = d.corner_xyz()  # (nsub, ny+2H+1, nx+2H+1, 3), corner (i, j) at [j+H, i+H]
    H = NG + 1
    lat_c = np.arcsin(np.clip(xyz[..., 2], -1, 1))
    lon_c = np.arctan2(xyz[..., 1], xyz[..., 0])
    psi = -A * u0 * (np.sin(lat_c) * np.cos(alpha) - np.cos(lon_c) * np.cos(lat_c) * np.sin(alpha))
    m = {n: d.metric(n) for n in ("dxa", "dya", "dx", "dy", "sin_sg1", "sin_sg2", "sin_sg3", "sin_sg4", "area",
                                  "lat", "lon")}
    sh = d.shape(1)
    xfx, yfx = np.zeros(sh), np.zeros(sh)
    # plane slot (j, i) holds corner (i - NG, j - NG), at xyz slot (j + H - NG, i + H - NG)
    o = H - NG
    P = psi[:, o:, o:]
    nj, pitch = sh[-2], sh[-1]
    # area flux through the y-edge (i, j) (corner (i, j) -> (i, j+1)) and the x-edge (i, j)
    jm, im = min(nj, P.shape[1] - 1), min(pitch, P.shape[2])
    xfx[:, 0, :jm, :im] = -(P[:, 1:jm + 1, :im] - P[:, :jm, :im]) * dt
    jm, im = min(nj, P.shape[1]), min(pitch, P.shape[2] - 1)
    yfx[:, 0, :jm, :im] = (P[:, :jm, 1:im + 1] - P[:, :jm, :im]) * dt
    # Courant numbers with tracer_2d's upwind metric factors (tracer_prep forms xfx back from them)
    sx = lambda a: np.roll(a, 1, axis=-1)   # a[i-1]
    sy = lambda a: np.roll(a, 1, axis=-2)   # a[j-1]
    with np.errstate(all="ignore"):
        up_x = (sx(m["dxa"]) * m["dy"] * sx(m["sin_sg3"]))[:, None]
        dn_x = (m["dxa"] * m["dy"] * m["sin_sg1"])[:, None]
        up_y = (sy(m["dya"]) * m["dx"] * sy(m["sin_sg4"]))[:, None]
        dn_y = (m["dya"] * m["dx"] * m["sin_sg2"])[:, None]
        cx = np.where(xfx > 0.0, xfx / up_x, xfx / dn_x)
        cy = np.where(yfx > 0.0, yfx / up_y, yfx / dn_y)
    # the sub-domain's own edges only: the halo values come from their owners by the C-grid
    # vector halo exchange, as the dycore's accumulated Courant numbers and mass fluxes do
    # (the cube-corner halo cells then stay zero)
    own_x = np.zeros(sh, bool)
    own_x[..., NG:NG + d.ny, NG:NG + d.nx + 1] = True
    own_y = np.zeros(sh, bool)
    own_y[..., NG:NG + d.ny + 1, NG:NG + d.nx] = True
    cx = np.where(own_x, np.nan_to_num(cx, nan=0.0, posinf=0.0, neginf=0.0), 0.0)
    xfx = np.where(own_x, xfx, 0.0)
    cy = np.where(own_y, np.nan_to_num(cy, nan=0.0, posinf=0.0, neginf=0.0), 0.0)
    yfx = np.where(own_y, yfx, 0.0)
    q0 = _bell(m["lat"], m["lon"])[:, None]
    return q0, cx, cy, xfx, yfx, m["area"][:, None]


def norms(q, q0, area, d):
    c = (Ellipsis, slice(NG, NG + d.ny), slice(NG, NG + d.nx))
    err, w, ref = q[c] - q0[c], area[c], q0[c]
    return dict(mass=abs((q[c] * w).sum() - (ref * w).sum()) / (ref * w).sum(),
                l1=(np.abs(err) * w).sum() / (np.abs(ref) * w).sum(),
                l2=np.sqrt((err ** 2 * w).sum() / (ref ** 2 * w).sum()),
                linf=np.abs(err).max() / np.abs(ref).max(), min=float(q[c].min()), max=float(q[c].max()),
                finite=bool(np.all(np.isfinite(q[c]))))


def _run(pkg, npx, alpha, nsteps):
    d = pkg.Domain(npx=npx, npz=1, nq=1)
    try:
        q0, cx, cy, xfx, yfx, area = setup_case(d, alpha, nsteps)
        d.upload("q", q0)
        ones = np.ones(d.shape(1))
        for _ in range(nsteps):
            # tracer_2d splits the Courant numbers / fluxes in place when a level sub-steps:
            # hand it the full-step values every step
            for n, v in (("cx", cx), ("cy", cy), ("mfx", xfx), ("mfy", yfx), ("dp1", ones)):
                d.upload(n, v)
            # the dycore's synchronised C-grid exchange ('X': a tile's east / north edge values
            # replaced by the neighbour's west / south ones, then the C halo), as uc / vc get
            d.halo_update("cx:X,cy:X,mfx:X,mfy:X")
            d.stencil("tracer_2d_1l", [], [1])
        return norms(d.download("q"), q0, area, d)
    finally:
        d.close()


@pytest.mark.parametrize("alpha", [np.pi / 4, 0.0])
def test_williamson1_cosine_bell(pkg, require_gpu, alpha):
    r48 = _run(pkg, 49, alpha, 288)
    r24 = _run(pkg, 25, alpha, 144)
    print(f"\nWilliamson 1, alpha = {alpha:.3f}: C48 {r48}\n  C24 {r24}")
    # mass: along the equator (alpha = 0) the bell's own values never reach a corner edge and
    # only its far undershoot ripples do (measured 1.6e-10 over the revolution at C48); through
    # two cube corners the corner edges move it by a few 1e-4 (measured 4.6e-4 at C48, 2.0e-3
    # at C24: FV3's copy_corners views, the HIP trajectory pinned to the oracle's in
    # test_williamson1_corner_mass_matches_oracle)
    mass_bar = 1e-9 if alpha == 0.0 else 1e-3
    assert r48["finite"] and r48["mass"] <= mass_bar, r48
    # C24 (3.75 deg): measured l2 0.12 at both angles -- the resolution Putman & Lin (2007) show
    # the bell still clipped and spread at (l2 of order 1e-1)
    assert r24["finite"] and r24["l2"] <= 0.2, r24
    assert r48["l2"] <= 0.05 and r48["linf"] <= 0.05, r48
    assert r24["l2"] / r48["l2"] >= 2.5, (r24["l2"], r48["l2"])


def test_williamson1_corner_mass_matches_oracle(pkg, require_gpu):
    """C24, alpha = pi / 4, the 24 steps in which the bell's edge reaches the first cube corner
    (the mass starts to move at step 10): the HIP transport and the oracle's (oracle/tp_core.py
    tracer_2d_1l, FV3's algorithm) give the same fields and the same mass change each step"""
    from oracle import tp_core
    from oracle.halo import Layout, fill_scalar, fill_vector, sync_edges
    from conftest import metrics_of
    npx, alpha, nsteps, nrun = 25, np.pi / 4, 144, 24
    d = pkg.Domain(npx=npx, npz=1, nq=1)
    try:
        q0, cx, cy, xfx, yfx, area = setup_case(d, alpha, nsteps)
        lay = Layout(d.N, 1, 1)
        ms = metrics_of(d)
        ocx, ocy, ox, oy = cx.copy(), cy.copy(), xfx.copy(), yfx.copy()
        for a, b in ((ocx, ocy), (ox, oy)):
            sync_edges(a, b, lay, "cgrid")
            fill_vector(a, b, lay, "cgrid")
        ones = np.ones(d.shape(1))
        c = (Ellipsis, slice(NG, NG + d.ny), slice(NG, NG + d.nx))
        mass = lambda q: float((q[c] * area[c]).sum())
        m0 = mass(q0)
        d.upload("q", q0)
        qo = q0.copy()
        moved = 0.0
        for it in range(nrun):
            for n, v in (("cx", cx), ("cy", cy), ("mfx", xfx), ("mfy", yfx), ("dp1", ones)):
                d.upload(n, v)
            d.halo_update("cx:X,cy:X,mfx:X,mfy:X")
            d.stencil("tracer_2d_1l", [], [1])
            qo, _ = tp_core.tracer_2d_1l(qo, ones, ox, oy, ocx, ocy, d.subs, ms, d.nx, d.ny, 1, 1, 6,
                                         lambda a: fill_scalar(a, lay, "cell"))
            qh = d.download("q")
            err = np.abs(qh[c] - qo[c]).max() / np.abs(qo[c]).max()
            assert err <= 1e-11, (it, err)
            dmh, dmo = (mass(qh) - m0) / m0, (mass(qo) - m0) / m0
            assert abs(dmh - dmo) <= 1e-13, (it, dmh, dmo)
            moved = max(moved, abs(dmo))
        print(f"\nC24 alpha = pi/4, {nrun} steps: mass change through the corner {moved:.2e} (HIP = oracle)")
        assert moved > 1e-10  # the corner was reached: the check above compared a real loss
    finally:
        d.close()
