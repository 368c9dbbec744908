"""CPU tests of d_sw's per-level damping parameters (no GPU): the product's column
(csrc/damp.hip column_damping, read back through gtfv3_level_damping) against the oracle's
restatement of FV3 dyn_core's k loop (oracle/sw_core.py column_namelist, heat_levels), for
the Held-Suarez namelist with its sponge layers and for damping namelists; the namelist keys
of the sponge and the kord guard of the config parser.

Parity unpinned against FV3 itself: the reference holds no fv_core_nml and no FV3 source
(SURVEY §8c); the rule restated is dyn_core's (as in pyFV3 get_column_namelist).
"""
import ctypes

import pytest

from oracle import sw_core
from oracle.fv_dynamics import SPONGE_DEFAULTS

HS = dict()  # the Held-Suarez namelist: the product defaults (sponge on)
CASES = {
    "held_suarez": HS,
    "hs_no_sponge": dict(n_sponge=-1),
    "hs_k2_small": dict(d2_bg_k2=0.03),
    "hs_k2_off": dict(d2_bg_k2=0.0),
    "vort_damp": dict(nord=2, d4_bg=0.15, vtdm4=0.05, do_vort_damp=1, d_con=1.0),
    "vtdm4_without_switch": dict(nord=1, d4_bg=0.12, vtdm4=0.05, d_con=0.5),
    "nord3_del2": dict(nord=3, d4_bg=0.12, d2_bg=0.005, vtdm4=0.02, do_vort_damp=1, nord_v=1),
    "strong_sponge": dict(d2_bg_k1=0.25, d2_bg_k2=0.12, ke_bg=3.0, do_vort_damp=1, vtdm4=0.0),
    "convert_ke": dict(convert_ke=1, d2_bg_k1=0.0),
    # deeper sponge: dyn_core's second / third overrides at levels max(2, n_sponge-1) and
    # max(3, n_sponge) (1-based), here 4 and 5
    "n_sponge5": dict(n_sponge=5),
    "n_sponge5_vort": dict(n_sponge=5, do_vort_damp=1, vtdm4=0.03),
}


def _oracle(nl, npz, da_min, da_min_c):
    sp = {k: nl.get(k, v) for k, v in SPONGE_DEFAULTS.items()}
    nord = nl.get("nord", 0)
    cols = sw_core.column_namelist(npz, nord=nord, d2_bg=nl.get("d2_bg", 0.0), vtdm4=nl.get("vtdm4", 0.0),
                                   do_vort_damp=bool(nl.get("do_vort_damp", 0)), nord_v=nl.get("nord_v"),
                                   d_con=nl.get("d_con", 0.0), **sp)
    out = []
    for c in cols:
        out.append(dict(
            d2_divg=c["d2_divg"],
            vt4=(c["damp_vt"] * da_min_c) ** (c["nord_v"] + 1) if c["damp_vt"] > 1e-5 else 0.0,
            dp4=(c["damp_vt"] * da_min) ** (c["nord_v"] + 1) if c["damp_vt"] > 1e-4 else 0.0,
            w4=(c["damp_w"] * da_min_c) ** (c["nord_w"] + 1) if c["damp_w"] > 1e-5 else 0.0,
            pt4=(c["damp_t"] * da_min) ** (c["nord_t"] + 1) if c["damp_t"] > 1e-4 else 0.0,
            d_con=c["d_con"], nord=c["nord"], nord_v=c["nord_v"], nord_w=c["nord_w"], nord_t=c["nord_t"]))
    n_con = min(npz, sw_core.heat_levels(npz, nl.get("vtdm4", 0.0), sp["d2_bg_k1"], sp["d2_bg_k2"],
                                         bool(nl.get("convert_ke", 0))))
    return out, n_con


@pytest.mark.parametrize("npz", [1, 2, 10])
@pytest.mark.parametrize("case", list(CASES))
def test_column_matches_oracle(pkg, case, npz):
    nl = CASES[case]
    d = pkg.Domain(npx=13, npz=npz, nq=1, host_only=1, **nl)
    try:
        got, n_con = d.level_damping()
        sc = d.scalars()
        ref, n_ref = _oracle(nl, npz, sc["da_min"], sc["da_min_c"])
    finally:
        d.close()
    assert n_con == n_ref
    for k, (g, r) in enumerate(zip(got, ref)):
        for key, rv in r.items():
            assert g[key] == rv, f"{case} level {k} {key}: {g[key]} != {rv}"


def test_held_suarez_sponge_levels(pkg):
    """the benchmark namelist's top levels: del-2 divergence damping 0.2 / 0.1 / 0.02, del-2 w
    damping with the same coefficients, the rest of the column undamped (nord 0, d2_bg 0)"""
    d = pkg.Domain(npx=13, npz=10, nq=1, host_only=1)
    try:
        col, n_con = d.level_damping()
        dac = d.scalars()["da_min_c"]
    finally:
        d.close()
    assert [c["d2_divg"] for c in col[:4]] == [0.2, 0.1, 0.2 * 0.1, 0.0]
    assert [c["w4"] for c in col[:4]] == [0.2 * dac, 0.1 * dac, 0.2 * 0.1 * dac, 0.0]
    assert all(c["vt4"] == 0.0 and c["dp4"] == 0.0 and c["pt4"] == 0.0 for c in col)
    assert n_con == 2


def test_deep_sponge_override_levels(pkg):
    """n_sponge = 5: the overrides land on levels 0, 3 and 4 (0-based), levels 1-2 ordinary"""
    d = pkg.Domain(npx=13, npz=10, nq=1, host_only=1, n_sponge=5)
    try:
        col, _ = d.level_damping()
    finally:
        d.close()
    assert [c["d2_divg"] for c in col[:6]] == [0.2, 0.0, 0.0, 0.1, 0.2 * 0.1, 0.0]


def test_height_damping_column(pkg):
    """update_dz_d's damping of the heights: with do_vort_damp the oracle's
    update_dz_d adds del6_vt_flux of the old heights, an effect far above the step's parity bar"""
    import numpy as np

    from oracle import nh_core
    from conftest import metrics_of
    d = pkg.Domain(npx=13, npz=4, nq=1, host_only=1)
    try:
        m = metrics_of(d)[0]
        sub, nx, ny = d.subs[0], d.nx, d.ny
        sh = d.shape(5)[1:]
        r = np.random.default_rng(5)
        zh = 1e4 - 2e3 * np.arange(5)[:, None, None] + 50.0 * r.standard_normal(sh)
        z4 = np.zeros(d.shape(4)[1:])
        dp0 = np.full(4, 2000.0)
        args = (zh, z4, z4, z4, z4, zh[4], sub, m, nx, ny, dp0, 75.0, 6, 2.0)
        plain, _ = nh_core.update_dz_d(*args)
        damp = [(0, 0.0), (0, 0.02 * 1e8), (1, 0.0), (1, 0.0), (1, 0.0)]
        damped, _ = nh_core.update_dz_d(*args, damp=damp)
    finally:
        d.close()
    c = (slice(None), slice(3, 3 + ny), slice(3, 3 + nx))
    diff = np.abs(damped - plain)[c]
    assert diff[1].max() > 1e-3 and diff[0].max() == 0.0 and diff[2:].max() == 0.0


def test_config_kord_and_sponge_keys(pkg, capfd):
    lib = pkg.lib()
    buf = ctypes.create_string_buffer(256)
    ok = lib.gtfv3_create(b"npx=13,npz=3,nq=1,host_only=1,n_sponge=3,d2_bg_k1=0.15,d2_bg_k2=0.02,ke_bg=1.5,"
                          b"convert_ke=0,kord_mt=9,kord_tm=-9", 0, 1, None)
    assert ok
    lib.gtfv3_destroy(ok)
    # only the implemented kord = 9 (kord_tm = -9) remap: anything else is refused, not run as 9
    for bad in (b"kord_mt=10", b"kord_wz=8", b"kord_tr=11", b"kord_tm=9", b"kord_tm=-10"):
        h = lib.gtfv3_create(b"npx=13,npz=3,nq=1,host_only=1," + bad, 0, 1, None)
        assert not h, bad
        assert lib.geos_gtfv3_last_error(buf, 256) > 0 and b"kord" in buf.value, buf.value
    # vtdm4 without do_vort_damp: FV3 semantics (no del-n damping, heat on every level), said
    capfd.readouterr()
    h = lib.gtfv3_create(b"npx=13,npz=3,nq=1,host_only=1,vtdm4=0.05,d_con=1", 0, 1, None)
    assert h
    lib.gtfv3_destroy(h)
    assert "without do_vort_damp" in capfd.readouterr().err
