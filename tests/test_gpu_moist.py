"""Moist column physics on the device against the
oracles (oracle/moist.py, oracle/gfdl_mp.py, oracle/geos_moist.py) on an aquaplanet-like
synthetic state (tests/moist_inputs.py), all sub-domains of a C24 cube on the device.
Bars: the table reads (qsat) and fillq2zero are bit-exact (same table, same arithmetic
order); the schemes with exp / log / pow (ocml vs glibc) are held to the reference's moist
bar, 0.01 % relative per value (physics_standalone.py:132-144), and, tighter, to 1e-9 of
each field's scale; the LCL level index is bit-exact.  The GFDL driver's oracle walks its
columns in Python, so it checks a sample of 2 x 3 rows of columns."""
import numpy as np
import pytest

from moist_inputs import moist_state
from oracle import NG
from oracle import geos_moist as gm
from oracle import gf_shallow as gf
from oracle import gfdl_mp as mp
from oracle import moist as om

pytestmark = pytest.mark.gpu
NK = 30


@pytest.fixture(scope="module")
def dom(pkg):
    d = pkg.Domain(npx=25, npz=NK, nq=1)
    yield d
    d.close()


def comp(d, a):
    return a[..., NG:NG + d.ny, NG:NG + d.nx]


def upload_state(d, st):
    for k, v in st.items():
        d.upload("m_" + k, v if v.ndim == 4 else v[:, None])


def rel(a, b):
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-300)


def test_qsat_bit_exact(dom, require_gpu):
    st = moist_state(dom.shape(NK))
    upload_state(dom, st)
    dom.stencil("moist_qsat", ["m_T", "m_pm", "m_qsw", "m_qsi", "m_dqsw"])
    qsw, dqsw = om.qsat(st["T"], st["pm"], ice=False)
    qsi, _ = om.qsat(st["T"], st["pm"], ice=True)
    for name, ref in (("m_qsw", qsw), ("m_qsi", qsi), ("m_dqsw", dqsw)):
        np.testing.assert_array_equal(comp(dom, dom.download(name)), comp(dom, ref))


def test_fillq2zero_bit_exact(dom, require_gpu):
    st = moist_state(dom.shape(NK), seed=9)
    upload_state(dom, st)
    dom.stencil("fillq2zero", ["m_ql", "m_delp", "m_fill"])
    got = dom.download("m_ql")
    fill = dom.download("m_fill")[:, 0]
    for s in range(dom.nsub):
        ref, rfill = om.fillq2zero(st["ql"][s], st["delp"][s])
        np.testing.assert_array_equal(comp(dom, got[s]), comp(dom, ref))
        np.testing.assert_array_equal(comp(dom, fill[s]), comp(dom, rfill))


SAMPLE = ((0, slice(0, 3)), (4, slice(10, 13)))   # (sub-domain, rows) checked against the column oracle


def cols_of(d, a, s, rows):
    """[k, ncol] columns of sub-domain s, compute rows `rows` (all i), from an HBM-layout array"""
    x = a[s][:, NG:NG + d.ny, NG:NG + d.nx][:, rows, :]
    return x.reshape(x.shape[0], -1)


def close(got, ref, what, floor=1e-300):
    """max |got - ref| within 1e-9 of the field's scale (max |ref|, at least `floor`), and the
    reference's 0.01 % per value above that"""
    scale = max(np.abs(ref).max(), floor)
    err = np.abs(got - ref).max()
    assert err <= 1e-9 * scale, (what, err / scale)
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-9 * scale, err_msg=what)


@pytest.mark.parametrize("variant", [0, 1])
def test_gfdl_mp_matches_oracle(dom, require_gpu, variant):
    """variant 0: the level-block form (mpdrv_blk_k<2, 16> at 30 levels), 1: the column driver"""
    st = moist_state(dom.shape(NK), seed=13)
    upload_state(dom, st)
    dt = 450.0
    names = ["m_T", "m_qv", "m_ql", "m_qr", "m_qi", "m_qs", "m_qg", "m_delp", "m_delz",
             "m_pr", "m_ps", "m_pg", "m_pi"]
    dom.stencil("gfdl_1m", names, [dt, variant])
    got = {n: dom.download(n) for n in names[:7] + names[9:]}
    for s, rows in SAMPLE:
        c = {k: cols_of(dom, st[k], s, rows) for k in ("T", "delp", "delz", "qv", "ql", "qr", "qi", "qs", "qg")}
        (T, qv, ql, qr, qi, qs, qg), prec = mp.mpdrv(c["T"], c["delp"], c["delz"], c["qv"], c["ql"], c["qr"],
                                                     c["qi"], c["qs"], c["qg"], dt)
        for n, ref in zip(names[:7], (T, qv, ql, qr, qi, qs, qg)):
            close(cols_of(dom, got[n], s, rows), ref, (n, s))
        # surface precipitation: a species that melts on the way down reaches the ground as
        # round-off (1e-17 kg m-2): the absolute bar is at least 1e-15 of the column water
        cw = (sum(c[k] for k in ("qv", "ql", "qr", "qi", "qs", "qg")) * c["delp"]).sum(0).max() / om.GRAV
        for n, ref in zip(names[9:], prec):
            close(cols_of(dom, got[n], s, rows)[0], ref, (n, s), floor=1e-6 * cw)
    # column water + surface precipitation is conserved on the device everywhere
    w0 = np.einsum("skji,skji->sji", sum(st[k] for k in ("qv", "ql", "qr", "qi", "qs", "qg")), st["delp"]) / om.GRAV
    w1 = np.einsum("skji,skji->sji", sum(got[n] for n in names[1:7]), st["delp"]) / om.GRAV + \
        sum(got[n][:, 0] for n in names[9:])
    assert rel(comp(dom, w1), comp(dom, w0)) <= 1e-13
    assert sum(comp(dom, got[n][:, 0]).sum() for n in names[9:]) > 0.0


def test_evap_subl_pdf_matches_oracle(dom, require_gpu):
    st = moist_state(dom.shape(NK), seed=21)
    r = np.random.default_rng(22)
    extra = dict(qlcn=0.3 * np.maximum(st["ql"], 0.0), qicn=0.3 * np.maximum(st["qi"], 0.0),
                 clls=0.3 * r.random(st["T"].shape), clcn=0.2 * r.random(st["T"].shape),
                 nactl=5.0e7 * (1.0 + r.random(st["T"].shape)), nacti=1.0e3 * r.random(st["T"].shape))
    upload_state(dom, dict(st, **extra))
    dt = 450.0
    names = ["m_T", "m_qv", "m_ql", "m_qi", "m_qlcn", "m_qicn", "m_clls", "m_clcn", "m_pm", "m_nactl", "m_nacti"]
    dom.stencil("evap_subl_pdf", names, [dt])
    ref = gm.evap_subl_pdf(dt, st["pm"], st["T"], st["qv"], st["ql"], st["qi"], extra["qlcn"], extra["qicn"],
                           extra["clls"], extra["clcn"], extra["nactl"], extra["nacti"])
    for n, k in zip(names[:8], ("t", "qv", "qlls", "qils", "qlcn", "qicn", "clls", "clcn")):
        close(comp(dom, dom.download(n)), comp(dom, ref[k]), n)


def test_radcouple_matches_oracle(dom, require_gpu):
    st = moist_state(dom.shape(NK), seed=23)
    r = np.random.default_rng(24)
    shp = st["T"].shape
    extra = dict(cf=0.8 * r.random(shp), af=0.3 * r.random(shp), qlcn=1e-4 * r.random(shp), qicn=1e-4 * r.random(shp),
                 nactl=5.0e7 * (1.0 + r.random(shp)))
    upload_state(dom, dict(st, **extra))
    ins = ["m_T", "m_pm", "m_cf", "m_af", "m_qv", "m_ql", "m_qi", "m_qlcn", "m_qicn", "m_qr", "m_qs", "m_qg", "m_nactl"]
    outs = ["m_rad_qv", "m_rad_ql", "m_rad_qi", "m_rad_qr", "m_rad_qs", "m_rad_qg", "m_rad_cf", "m_rad_rl", "m_rad_ri"]
    dom.stencil("radcouple", ins + outs)
    ref = gm.radcouple(st["T"], st["pm"], extra["cf"], extra["af"], st["qv"], st["ql"], st["qi"], extra["qlcn"],
                       extra["qicn"], st["qr"], st["qs"], st["qg"], extra["nactl"], None)
    for n in outs:
        close(comp(dom, dom.download(n)), comp(dom, ref[n[2:]]), n)


def test_aer_activation_matches_oracle(dom, require_gpu):
    st = moist_state(dom.shape(NK), seed=25)
    r = np.random.default_rng(26)
    w = 0.5 * r.standard_normal(st["T"].shape)
    upload_state(dom, dict(st, w=w))
    dom.stencil("aer_activation", ["m_pm", "m_T", "m_qv", "m_zm", "m_w", "m_nactl", "m_nacti", "m_smax"])
    na, ni, sm = gm.aer_activation(st["pm"], st["T"], st["qv"], st["zm"], w)
    close(comp(dom, dom.download("m_nactl")), comp(dom, na), "nactl")
    close(comp(dom, dom.download("m_nacti")), comp(dom, ni), "nacti")
    close(comp(dom, dom.download("m_smax")), comp(dom, sm), "smax")


def test_cup_gf_sh_matches_oracle(dom, require_gpu):
    """the shallow cumulus on the device against oracle/gf_shallow.py on a sample of columns:
    T, qv, the detrained condensate, the cloud fraction and the cloud-base mass flux within
    the bars; the source / cloud-base / cloud-top level indices bit-exact"""
    st = moist_state(dom.shape(NK), seed=31)
    sh = st["T"].shape
    r = np.random.default_rng(32)
    kpbl = np.zeros((sh[0], 1) + sh[2:])
    for s in range(sh[0]):   # PBL top: the highest level below 1 km
        z = st["zm"][s]
        kpbl[s, 0] = np.where(z < 1000.0, np.arange(NK)[:, None, None], NK - 1).min(axis=0)
    hfx = 5.0 + 30.0 * r.random((sh[0], 1) + sh[2:])
    z0 = np.zeros(sh)
    upload_state(dom, dict(st, kpbl=kpbl, hfx=hfx, qlcn=z0, qicn=z0))
    dt = 450.0
    names = ["m_T", "m_qv", "m_pm", "m_zm", "m_delp", "m_kpbl", "m_hfx", "m_qlcn", "m_qicn",
             "m_cf", "m_mb", "m_k22", "m_kbcon", "m_ktop"]
    dom.stencil("cup_gf_sh", names, [dt])
    got = {n: dom.download(n) for n in names}
    active = 0
    for s, rows in SAMPLE:
        c = {k: cols_of(dom, st[k], s, rows) for k in ("T", "qv", "pm", "zm", "delp")}
        kp = cols_of(dom, kpbl, s, rows)[0]
        hf = cols_of(dom, hfx, s, rows)[0]
        ref = gf.cup_gf_sh(dt, c["T"], c["qv"], c["pm"], c["zm"], c["delp"], kp, hf)
        for n, k in (("m_T", "t"), ("m_qv", "qv"), ("m_qlcn", "dqlcn"), ("m_qicn", "dqicn"), ("m_cf", "cf")):
            close(cols_of(dom, got[n], s, rows), ref[k], (n, s), floor=1e-30)
        close(cols_of(dom, got["m_mb"], s, rows)[0], ref["mb"], ("mb", s), floor=1e-30)
        for n, k in (("m_k22", "k22"), ("m_kbcon", "kbcon"), ("m_ktop", "ktop")):
            np.testing.assert_array_equal(cols_of(dom, got[n], s, rows)[0], ref[k], err_msg=n)
        active += int((ref["ktop"] >= 0).sum())
    assert active > 0, "no shallow convection in the sample"
    # column moist static energy and water are conserved on the device everywhere
    cp, lv = om.CP_AIR, om.HLV
    h0 = np.einsum("skji,skji->sji", cp * st["T"] + lv * st["qv"], st["delp"])
    h1 = np.einsum("skji,skji->sji", cp * got["m_T"] + lv * got["m_qv"], st["delp"])
    w0 = np.einsum("skji,skji->sji", st["qv"], st["delp"])
    w1 = np.einsum("skji,skji->sji", got["m_qv"] + got["m_qlcn"] + got["m_qicn"], st["delp"])
    assert rel(comp(dom, h1), comp(dom, h0)) <= 1e-14
    assert rel(comp(dom, w1), comp(dom, w0)) <= 1e-14


def test_buoyancy_matches_oracle(dom, require_gpu):
    st = moist_state(dom.shape(NK), seed=17)
    upload_state(dom, st)
    dom.stencil("buoyancy", ["m_T", "m_qv", "m_pm", "m_zm", "m_by", "m_cape", "m_cin", "m_klcl"])
    by = dom.download("m_by")
    cape, cin, klcl = (dom.download(n)[:, 0] for n in ("m_cape", "m_cin", "m_klcl"))
    for s in range(dom.nsub):
        rb, rc, ri, rk = om.buoyancy(st["T"][s], st["qv"][s], st["pm"][s], st["zm"][s])
        assert rel(comp(dom, by[s]), comp(dom, rb)) <= 1e-12
        assert rel(comp(dom, cape[s]), comp(dom, rc)) <= 1e-12
        assert rel(comp(dom, cin[s]), comp(dom, ri)) <= 1e-12
        np.testing.assert_array_equal(comp(dom, klcl[s]), comp(dom, rk))
