"""GPU parity of the SIM1 Riemann solvers (riem_solver_c, riem_solver3).

Both kernel forms -- the level-block scan kernel (default: partitioned Thomas solves,
Kogge-Stone prefix sums, fastmath.hpp log / exp) and the column-sweep kernel (variant 1,
ocml log / exp) -- against the oracle (oracle/nh_core.py, after the dz_min clamp FV3
applies in update_dz_c / update_dz_d): |hip - oracle| <= 1e-11 * mean|oracle| (1e-9 for
ppe, a small difference of large pressures), including columns where the dz_min clamp is
active in several blocks (the blocked clamp is speculative).  The scan form associates its
sums and products differently, so the two forms agree to rounding, not bit for bit.
Inputs are near-hydrostatic columns (pt chosen so that the nonhydrostatic pressure is
the layer-mean pressure to 1e-3), so the perturbation pressures the solver forms are
well conditioned.
"""
import numpy as np
import pytest

from conftest import rng
from oracle import NG
from oracle import nh_core

pytestmark = pytest.mark.gpu

GRAV, RDGAS, KAPPA = nh_core.GRAV, nh_core.RDGAS, nh_core.KAPPA
PTOP, P_FAC, DZ_MIN = 300.0, 0.05, 2.0


def columns(d, npz, r, thin):
    """delp, pt, w, heights (npz+1), zs, phis on the whole plane of every sub-domain"""
    sh = d.shape(npz)
    delp = 800.0 + 1200.0 * r.random(sh)
    pem = PTOP + np.concatenate([np.zeros(sh[:1] + (1,) + sh[2:]), np.cumsum(delp, axis=1)], axis=1)
    T = 220.0 + 60.0 * r.random(sh)
    dz = -RDGAS * T / GRAV * np.log(pem[:, 1:] / pem[:, :-1])
    if thin:  # layers thinner than dz_min in a scatter of columns and levels
        m = r.random(sh) < 0.03
        dz = np.where(m, -0.5 * r.random(sh), dz)
    zs = 1500.0 * r.random((sh[0], 1) + sh[2:])
    zh = np.concatenate([np.zeros_like(pem[:, :-1]), zs], axis=1)
    for k in range(npz - 1, -1, -1):
        zh[:, k] = zh[:, k + 1] - dz[:, k]
    zh[:, npz] += 0.3 * r.standard_normal(zs.shape[:1] + zs.shape[2:])  # nonzero ws
    pm = delp / np.log(pem[:, 1:] / pem[:, :-1])
    dzc = np.minimum(dz, -1.0)
    pt = np.exp((1.0 - KAPPA) * np.log(pm)) * (-dzc) / (delp / GRAV * RDGAS)
    pt *= 1.0 + 1e-3 * r.standard_normal(sh)
    w = 0.5 * r.standard_normal(sh)
    return dict(delp=delp, pt=pt, w=w, zh=zh, zs=zs, phis=zs * GRAV)


def clamp(h):
    h = h.copy()
    for k in range(h.shape[0] - 2, -1, -1):
        h[k] = np.maximum(h[k], h[k + 1] + DZ_MIN)
    return h


def region(a, ring, nx, ny):
    return a[..., NG - ring:NG + ny + ring, NG - ring:NG + nx + ring]


def close(a, b, what, rtol=1e-11, atol=0.0):
    scale = np.abs(b).mean() + 1e-300
    worst = (np.abs(a - b).max() - atol) / scale
    assert worst <= rtol, f"{what}: max scaled error {worst:.3e}"


@pytest.mark.parametrize("npz,thin", [(12, True), (10, False), (72, True), (7, True), (8, False), (20, True), (70, True),
                                      (91, True), (137, True), (137, False)])
def test_riem_solver_c(pkg, require_gpu, npz, thin):
    d = pkg.Domain(npx=13, npz=npz, nq=1)
    r = rng(100 + npz)
    col = columns(d, npz, r, thin)
    dt2 = 225.0
    for k in ("delp", "pt", "w", "phis"):
        d.upload("rc_" + k, col[k])
    got = {}
    for var in (1, 0):
        d.upload("rc_gz", col["zh"])
        d.stencil("riem_solver_c", ["rc_delp", "rc_pt", "rc_w", "rc_phis", "rc_gz", "rc_pef"],
                  [dt2, PTOP, P_FAC, DZ_MIN, var])
        got[var] = {k: region(d.download(k), 1, d.nx, d.ny) for k in ("rc_gz", "rc_pef")}
    for s in range(d.nsub):
        gz = clamp(col["zh"][s])
        ws = (col["zs"][s, 0] - col["zh"][s, npz]) * (1.0 / dt2)
        reg = np.ones(gz.shape[1:], dtype=bool)
        pef, gzo = nh_core.riem_solver_c(dt2, col["delp"][s], col["pt"][s], col["w"][s], gz, col["phis"][s, 0], ws,
                                         PTOP, P_FAC, reg)
        for var in (0, 1):
            close(got[var]["rc_pef"][s], region(pef, 1, d.nx, d.ny), f"variant {var} sub{s} pef")
            close(got[var]["rc_gz"][s], region(gzo, 1, d.nx, d.ny), f"variant {var} sub{s} gz")


@pytest.mark.parametrize("npz,last", [(12, 1), (72, 0), (72, 1), (10, 1), (20, 1), (70, 0), (91, 1), (137, 1), (137, 0)])
def test_riem_solver3(pkg, require_gpu, npz, last):
    d = pkg.Domain(npx=13, npz=npz, nq=1)
    r = rng(200 + npz)
    col = columns(d, npz, r, True)
    dt = 450.0
    for k in ("delp", "pt", "phis"):
        d.upload("r3_" + k, col[k])
    outs = ["r3_w", "r3_zh", "r3_delz", "r3_ppe", "r3_pk3", "r3_pe", "r3_peln", "r3_pk", "r3_ws"]
    got = {}
    for var in (1, 0):
        d.upload("r3_w", col["w"])
        d.upload("r3_zh", col["zh"])
        for k in ("r3_pe", "r3_peln", "r3_pk"):
            d.upload(k, np.zeros(d.shape(npz + 1)))
        d.stencil("riem_solver3", ["r3_delp", "r3_pt", "r3_w", "r3_phis", "r3_zh", "r3_delz", "r3_ppe", "r3_pk3",
                                   "r3_pe", "r3_peln", "r3_pk", "r3_ws"], [dt, PTOP, P_FAC, DZ_MIN, last, var])
        got[var] = {k: region(d.download(k), 0, d.nx, d.ny) for k in outs}
    for s, var in ((s, var) for s in range(d.nsub) for var in (0, 1)):
        zh = clamp(col["zh"][s])
        ws = (col["zs"][s, 0] - col["zh"][s, npz]) * (1.0 / dt)
        reg = np.ones(zh.shape[1:], dtype=bool)
        o = nh_core.riem_solver3(dt, col["delp"][s], col["pt"][s], col["w"][s], zh, col["zs"][s, 0], ws, PTOP, P_FAC,
                                 reg, bool(last))
        g = {k[3:]: v[s] for k, v in got[var].items()}
        t = f"variant {var} sub{s}"
        close(g["ws"][0], region(ws, 0, d.nx, d.ny), f"{t} ws")
        close(g["w"], region(o["w"], 0, d.nx, d.ny), f"{t} w", atol=1e-12)
        for k in ("zh", "delz", "pk3"):
            close(g[k], region(o[k], 0, d.nx, d.ny), f"{t} {k}")
        close(g["ppe"], region(o["ppe"], 0, d.nx, d.ny), f"{t} ppe", rtol=1e-9)
        if last:
            for k in ("pe", "peln", "pk"):
                close(g[k], region(o[k], 0, d.nx, d.ny), f"{t} {k}")


@pytest.mark.parametrize("npz", [10, 20, 72, 137])
@pytest.mark.parametrize("cgrid", [True, False])
def test_riem_on_bench_state(pkg, require_gpu, npz, cgrid):
    """Both forms against the oracle on the columns of the bench's initial state (the
    Jablonowski-Williamson atmosphere on the analytic hybrid levels: ptop = 1 Pa, layers
    thinning towards the top, hydrostatic heights from delz), w a small random field"""
    import importlib
    state = importlib.import_module(pkg.__name__ + ".state")
    d = pkg.Domain(npx=13, npz=npz, nq=1)
    ak, bk, ks = state.hybrid_levels(npz)
    st = state.jablonowski_williamson(d, ak, bk)
    ptop = float(ak[0])
    zs = st["phis"][:, 0] / GRAV
    zh = np.zeros(d.shape(npz + 1))
    zh[:, npz] = zs
    for k in range(npz - 1, -1, -1):
        zh[:, k] = zh[:, k + 1] - st["delz"][:, k]
    w = 0.05 * rng(300 + npz).standard_normal(d.shape(npz))
    dt = 75.0
    ring = 1 if cgrid else 0
    got = {}
    for k, v in (("delp", st["delp"]), ("pt", st["pt"]), ("phis", st["phis"])):
        d.upload("rb_" + k, v)
    for var in (1, 0):
        d.upload("rb_w", w)
        d.upload("rb_zh", zh)
        if cgrid:
            d.stencil("riem_solver_c", ["rb_delp", "rb_pt", "rb_w", "rb_phis", "rb_zh", "rb_pef"],
                      [dt, ptop, P_FAC, DZ_MIN, var])
            got[var] = {k: region(d.download(k), 1, d.nx, d.ny) for k in ("rb_zh", "rb_pef")}
        else:
            for k in ("rb_pe", "rb_peln", "rb_pk"):
                d.upload(k, np.zeros(d.shape(npz + 1)))
            d.stencil("riem_solver3", ["rb_delp", "rb_pt", "rb_w", "rb_phis", "rb_zh", "rb_delz", "rb_ppe", "rb_pk3",
                                       "rb_pe", "rb_peln", "rb_pk", "rb_ws"], [dt, ptop, P_FAC, DZ_MIN, 1, var])
            got[var] = {k: region(d.download(k), 0, d.nx, d.ny)
                        for k in ("rb_w", "rb_zh", "rb_delz", "rb_ppe", "rb_pk3", "rb_pe")}
    for s, var in ((s, var) for s in range(d.nsub) for var in (1, 0)):
        g = {k[3:]: v[s] for k, v in got[var].items()}
        t = f"variant {var} sub{s}"
        h = clamp(zh[s])
        ws = (zs[s] - zh[s, npz]) * (1.0 / dt)
        reg = np.ones(h.shape[1:], dtype=bool)
        if cgrid:
            pef, gzo = nh_core.riem_solver_c(dt, st["delp"][s], st["pt"][s], w[s], h, st["phis"][s, 0], ws, ptop,
                                             P_FAC, reg)
            close(g["pef"], region(pef, 1, d.nx, d.ny), f"{t} pef")
            close(g["zh"], region(gzo, 1, d.nx, d.ny), f"{t} gz")
        else:
            o = nh_core.riem_solver3(dt, st["delp"][s], st["pt"][s], w[s], h, zs[s], ws, ptop, P_FAC, reg, True)
            close(g["w"], region(o["w"], 0, d.nx, d.ny), f"{t} w", atol=1e-12)
            for k in ("zh", "delz", "pk3", "pe"):
                close(g[k], region(o[k], 0, d.nx, d.ny), f"{t} {k}")
            close(g["ppe"], region(o["ppe"], 0, d.nx, d.ny), f"{t} ppe", rtol=1e-9)


@pytest.mark.parametrize("npz", [10, 20, 72, 137])
@pytest.mark.parametrize("cgrid", [True, False])
def test_riem_nan_column_stays_isolated(pkg, require_gpu, npz, cgrid):
    """A column of garbage (NaN delp: an unused cube-corner halo column in the step) must
    leave every other column bit-identical: the scan form hands values between the lanes of
    a column only, and the shifts that reach into the neighbouring columns' lanes are selected
    away (never multiplied by a zero coefficient) -- including in the rows past the bottom of a
    partial last block (L10, L20, L137)"""
    d = pkg.Domain(npx=13, npz=npz, nq=1)
    r = rng(400 + npz)
    col = columns(d, npz, r, True)
    bad = col["delp"].copy()
    spots = [(NG + 4, NG + 5), (NG + 7, NG + 0)]
    for jb, ib in spots:
        bad[0, :, jb, ib] = np.nan
    ring = 1 if cgrid else 0
    got = []
    for delp in (col["delp"], bad):
        for k, v in (("delp", delp), ("pt", col["pt"]), ("phis", col["phis"]), ("w", col["w"]), ("zh", col["zh"])):
            d.upload("rn_" + k, v)
        if cgrid:
            d.stencil("riem_solver_c", ["rn_delp", "rn_pt", "rn_w", "rn_phis", "rn_zh", "rn_pef"],
                      [225.0, PTOP, P_FAC, DZ_MIN, 0])
            outs = ("rn_zh", "rn_pef")
        else:
            for k in ("rn_pe", "rn_peln", "rn_pk"):
                d.upload(k, np.zeros(d.shape(npz + 1)))
            d.stencil("riem_solver3", ["rn_delp", "rn_pt", "rn_w", "rn_phis", "rn_zh", "rn_delz", "rn_ppe",
                                       "rn_pk3", "rn_pe", "rn_peln", "rn_pk", "rn_ws"],
                      [450.0, PTOP, P_FAC, DZ_MIN, 1, 0])
            outs = ("rn_w", "rn_zh", "rn_delz", "rn_ppe")
        got.append({k: region(d.download(k), ring, d.nx, d.ny) for k in outs})
    for k in got[0]:
        a, b = got[0][k].copy(), got[1][k].copy()
        for jb, ib in spots:
            a[0, :, jb - NG + ring, ib - NG + ring] = b[0, :, jb - NG + ring, ib - NG + ring] = 0.0
        assert np.array_equal(a, b), f"{k}: a NaN column changed other columns"


@pytest.mark.parametrize("npz,n_split", [(10, 5), (10, 6), (72, 6)])
def test_riem_on_step_inputs(pkg, require_gpu, monkeypatch, npz, n_split):
    """Replays the Riemann solves of an oracle fv_dynamics step (C12, JW06 state, hybrid
    levels with ptop = 1 Pa) -- the inputs recorded at the oracle's own call sites, first
    acoustic sub-step -- through both kernel forms, against the oracle's outputs"""
    import importlib
    from conftest import metrics_of, oracle_scalars
    from oracle import fv_dynamics as fvd
    state = importlib.import_module(pkg.__name__ + ".state")
    d = pkg.Domain(npx=13, npz=npz, nq=2, n_split=n_split)
    ak, bk, ks = state.hybrid_levels(npz)
    st = state.jablonowski_williamson(d, ak, bk)
    g = fvd.Grid(d.N, 1, 1, metrics_of(d), oracle_scalars(d)["corner_w"], oracle_scalars(d)["da_min_c"], d.nj, d.pitch)
    rec = {"c": [], "d": []}
    orig_c, orig_d = nh_core.riem_solver_c, nh_core.riem_solver3

    def snap(a):  # the oracle updates some of these arrays in place later in the step
        return [np.copy(x) if isinstance(x, np.ndarray) else x for x in a]

    def rc(*a):
        a = snap(a)
        out = orig_c(*a)
        rec["c"].append((a, out))
        return out

    def rd(*a):
        a = snap(a)
        out = orig_d(*a)
        rec["d"].append((a, out))
        return out

    monkeypatch.setattr(nh_core, "riem_solver_c", rc)
    monkeypatch.setattr(nh_core, "riem_solver3", rd)
    nl = dict(n_split=n_split, dt_atmos=900.0, hord_mt=6, hord_vt=6, hord_tm=6, hord_dp=6, hord_tr=6, dddmp=0.2,
              d2_bg=0.0, p_fac=0.05, dz_min=2.0, fill=1, nq=2)
    fvd.fv_dynamics(st, ak, bk, g, nl)
    ns = d.nsub
    cin = [rec["c"][s][0] for s in range(ns)]
    din = [rec["d"][s][0] for s in range(ns)]
    def closef(got, want, what, rtol=1e-11, atol=0.0):
        # the unused cube-corner columns of the C grid's ring hold garbage in the oracle too:
        # compare where the oracle is finite, and require HIP finite there
        ok = np.isfinite(want).all(axis=0)
        badc = ok & ~np.isfinite(got).all(axis=0)
        assert not badc.any(), f"{what}: non-finite where the oracle is finite at (j, i) {np.argwhere(badc)[:8].tolist()}"
        close(got[:, ok], want[:, ok], what, rtol, atol)

    for var in (1, 0):
        # C grid: (dt2, delpc, ptc, wc, gz, hs, ws, ptop, p_fac, reg)
        dt2, ptop = cin[0][0], cin[0][7]
        for k, i in (("delp", 1), ("pt", 2), ("w", 3), ("zh", 4)):
            d.upload("rs_" + k, np.stack([c[i] for c in cin]))
        d.upload("rs_phis", np.stack([c[5][None] for c in cin]))
        d.stencil("riem_solver_c", ["rs_delp", "rs_pt", "rs_w", "rs_phis", "rs_zh", "rs_pef"],
                  [dt2, ptop, P_FAC, DZ_MIN, var])
        pef, gz = d.download("rs_pef"), d.download("rs_zh")
        for s in range(ns):
            want_pef, want_gz = rec["c"][s][1]
            closef(region(pef[s], 1, d.nx, d.ny), region(want_pef, 1, d.nx, d.ny), f"C variant {var} sub{s} pef")
            closef(region(gz[s], 1, d.nx, d.ny), region(want_gz, 1, d.nx, d.ny), f"C variant {var} sub{s} gz")
        # D grid: (dt, delp, pt, w, zh, zs, ws, ptop, p_fac, reg, last)
        dt = din[0][0]
        for k, i in (("delp", 1), ("pt", 2), ("w", 3), ("zh", 4)):
            d.upload("rs_" + k, np.stack([a[i] for a in din]))
        d.upload("rs_phis", np.stack([a[5][None] * GRAV for a in din]))
        for k in ("rs_pe", "rs_peln", "rs_pk"):
            d.upload(k, np.zeros(d.shape(npz + 1)))
        last = int(din[0][10])
        d.stencil("riem_solver3", ["rs_delp", "rs_pt", "rs_w", "rs_phis", "rs_zh", "rs_delz", "rs_ppe", "rs_pk3",
                                   "rs_pe", "rs_peln", "rs_pk", "rs_ws"], [dt, ptop, P_FAC, DZ_MIN, last, var])
        got = {k: d.download("rs_" + k) for k in ("w", "zh", "delz", "ppe", "pk3")}
        for s in range(ns):
            o = rec["d"][s][1]
            t = f"D variant {var} sub{s}"
            closef(region(got["w"][s], 0, d.nx, d.ny), region(o["w"], 0, d.nx, d.ny), f"{t} w", atol=1e-12)
            for k in ("zh", "delz", "pk3"):
                closef(region(got[k][s], 0, d.nx, d.ny), region(o[k], 0, d.nx, d.ny), f"{t} {k}")
            # ppe on the first sub-step from w = 0 is a small difference of large pressures: the
            # column form (ocml exp / log against glibc) is 2.4e-9 from the oracle here
            closef(region(got["ppe"][s], 0, d.nx, d.ny), region(o["ppe"], 0, d.nx, d.ny), f"{t} ppe", rtol=1e-8)
    d.close()


@pytest.mark.parametrize("npz", [10, 72, 137])
@pytest.mark.parametrize("cgrid", [True, False])
@pytest.mark.parametrize("shift", [1, 5])
def test_riem_column_position_invariant(pkg, require_gpu, npz, cgrid, shift):
    """Each column's result depends on that column's data only, not on which lanes (or which
    neighbours in its wave) it lands on: the inputs rolled by `shift` columns along x give
    the outputs rolled by the same amount, bit for bit (the step's 1x1 vs 2x2 and 1x1 vs
    1x4 identity rests on this)"""
    d = pkg.Domain(npx=13, npz=npz, nq=1)
    col = columns(d, npz, rng(500 + npz), True)
    ring = 1 if cgrid else 0
    got = []
    for sh in (0, shift):
        for k in ("delp", "pt", "phis", "w", "zh"):
            d.upload("rp_" + k, np.roll(col[k], sh, axis=-1))
        if cgrid:
            d.stencil("riem_solver_c", ["rp_delp", "rp_pt", "rp_w", "rp_phis", "rp_zh", "rp_pef"],
                      [225.0, PTOP, P_FAC, DZ_MIN, 0])
            outs = ("rp_zh", "rp_pef")
        else:
            for k in ("rp_pe", "rp_peln", "rp_pk"):
                d.upload(k, np.zeros(d.shape(npz + 1)))
            d.stencil("riem_solver3", ["rp_delp", "rp_pt", "rp_w", "rp_phis", "rp_zh", "rp_delz", "rp_ppe",
                                       "rp_pk3", "rp_pe", "rp_peln", "rp_pk", "rp_ws"],
                      [450.0, PTOP, P_FAC, DZ_MIN, 1, 0])
            outs = ("rp_w", "rp_zh", "rp_delz", "rp_ppe", "rp_pk3")
        got.append({k: d.download(k) for k in outs})
    lo, hi = NG - ring, NG + d.nx + ring  # computed columns; compare where both runs computed
    for k in got[0]:
        a = got[0][k][..., NG - ring:NG + d.ny + ring, lo:hi - shift]
        b = got[1][k][..., NG - ring:NG + d.ny + ring, lo + shift:hi]
        nbad = int((a != b).sum())
        assert nbad == 0, f"{k}: {nbad} values depend on the column's position (max diff {np.abs(a - b).max():.3e})"
