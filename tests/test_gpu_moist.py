"""Moist column physics on the device against oracle/moist.py on
an aquaplanet-like synthetic state (tests/moist_inputs.py), all sub-domains of a C24
cube.  Bars: the table reads (qsat) and fillq2zero are bit-exact (same table, same
arithmetic order); the GFDL-style step and buoyancy use exp/log (ocml vs glibc), so
they are held to 1e-12 relative, and the LCL level index is bit-exact."""
import numpy as np
import pytest

from moist_inputs import moist_state
from oracle import NG
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


def test_gfdl_1m_matches_oracle(dom, require_gpu):
    st = moist_state(dom.shape(NK), seed=13)
    upload_state(dom, st)
    dt = 450.0
    names = ["m_T", "m_qv", "m_ql", "m_qr", "m_qi", "m_qs", "m_qg", "m_delp", "m_delz", "m_pm",
             "m_pr", "m_ps", "m_pg", "m_pi"]
    dom.stencil("gfdl_1m", names, [dt])
    got = {n: dom.download(n) for n in names[:7] + names[10:]}
    for s in range(dom.nsub):
        args = [st[k][s] for k in ("T", "delp", "delz", "pm", "qv", "ql", "qr", "qi", "qs", "qg")]
        (T, qv, ql, qr, qi, qs, qg), prec = om.gfdl_1m(*args, dt)
        for n, ref in zip(names[:7], (T, qv, ql, qr, qi, qs, qg)):
            assert rel(comp(dom, got[n][s]), comp(dom, ref)) <= 1e-12, (n, s)
        for n, ref in zip(names[10:], prec):
            assert rel(comp(dom, got[n][s, 0]), comp(dom, ref)) <= 1e-12, (n, s)
    # column water + surface precipitation is conserved on the device too
    w0 = np.einsum("skji,skji->sji", sum(st[k] for k in ("qv", "ql", "qr", "qi", "qs", "qg")), st["delp"]) / om.GRAV
    w1 = np.einsum("skji,skji->sji", sum(got[n] for n in names[1:7]), st["delp"]) / om.GRAV + \
        sum(got[n][:, 0] for n in names[10:])
    assert rel(comp(dom, w1), comp(dom, w0)) <= 1e-12


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
