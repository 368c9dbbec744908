"""The drop-in boundary end to end: Fortran-layout buffers through the reference
ABI (geos_gtfv3_init_c / geos_gtfv3_run_f64_c, via the Python hook mirror) must give
exactly what the device API gives for the same state (same kernels), with every
array updated in place in its Fortran shape.

Fortran <-> numpy layout follows the reference's own rule, restated:
  fortran_to_python:  flat.reshape(reversed(dim)).transpose()   (data_conversion.py:141)
  python_to_fortran:  arr.flatten(order="F")                     (data_conversion.py:184)
so a Fortran array of bounds (ni, nj, nk) is a Fortran-ordered numpy array.
"""
import importlib
import os

import numpy as np
import pytest

from oracle import NG

pytestmark = pytest.mark.gpu


def to_fortran(dev, lo_i, hi_i, lo_j, hi_j, kj=False):
    """device-layout (nsub, nk, nj, pitch) -> Fortran (i, j, k, tile) [or (i, k, j, tile)]"""
    a = dev[:, :, lo_j + NG:hi_j + NG + 1, lo_i + NG:hi_i + NG + 1]      # (s, k, j, i)
    a = np.transpose(a, (3, 1, 2, 0) if kj else (3, 2, 1, 0))           # (i, k, j, s) / (i, j, k, s)
    return np.asfortranarray(a)


def from_fortran(f, nsub, nk, nj, pitch, lo_i, hi_i, lo_j, hi_j, kj=False):
    out = np.zeros((nsub, nk, nj, pitch))
    a = np.transpose(f, (3, 1, 2, 0) if kj else (3, 2, 1, 0))
    out[:, :, lo_j + NG:hi_j + NG + 1, lo_i + NG:hi_i + NG + 1] = a
    return out


def test_bridge_run_matches_device_api(pkg, require_gpu):
    os.environ["GTFV3_BRIDGE_TILES_PER_RANK"] = "6"
    os.environ["GTFV3_NONFATAL"] = "1"
    hook = importlib.import_module(pkg.__name__ + ".hook").geos_gtfv3
    state = importlib.import_module(pkg.__name__ + ".state")
    npx, npz, nq = 13, 10, 2
    N = npx - 1
    d = pkg.Domain(npx=npx, npz=npz, nq=nq)
    ak, bk, ks = state.hybrid_levels(npz)
    st = state.jablonowski_williamson(d, ak, bk)
    d.set_vertical(ak, bk, ks)
    for k, v in st.items():
        d.upload(k, v)
    d.step(1)
    want = {k: d.download(k) for k in ("u", "v", "w", "delz", "pt", "delp", "q", "ps", "pe", "peln", "pk", "pkz",
                                       "ua", "va", "omga")}
    nsub, nj, pitch = d.nsub, d.nj, d.pitch
    d.close()

    # Fortran bounds (1-based FV3 -> local 0-based: subtract is = 1)
    is_, ie, js, je = 1, N, 1, N
    isd, ied, jsd, jed = is_ - NG, ie + NG, js - NG, je + NG
    L = lambda x: x - 1  # noqa: E731
    shapes = {  # name: (lo_i, hi_i, lo_j, hi_j, nk, kj)
        "u": (L(isd), L(ied), L(jsd), L(jed + 1), npz, False),
        "v": (L(isd), L(ied + 1), L(jsd), L(jed), npz, False),
        "w": (L(isd), L(ied), L(jsd), L(jed), npz, False),
        "delz": (L(isd), L(ied), L(jsd), L(jed), npz, False),
        "pt": (L(isd), L(ied), L(jsd), L(jed), npz, False),
        "delp": (L(isd), L(ied), L(jsd), L(jed), npz, False),
        "q": (L(isd), L(ied), L(jsd), L(jed), npz * nq, False),
        "ps": (L(isd), L(ied), L(jsd), L(jed), 1, False),
        "pe": (L(is_ - 1), L(ie + 1), L(js - 1), L(je + 1), npz + 1, True),
        "pk": (L(is_), L(ie), L(js), L(je), npz + 1, False),
        "peln": (L(is_), L(ie), L(js), L(je), npz + 1, True),
        "pkz": (L(is_), L(ie), L(js), L(je), npz, False),
        "phis": (L(isd), L(ied), L(jsd), L(jed), 1, False),
        "q_con": (L(isd), L(ied), L(jsd), L(jed), npz, False),
        "omga": (L(isd), L(ied), L(jsd), L(jed), npz, False),
        "ua": (L(isd), L(ied), L(jsd), L(jed), npz, False),
        "va": (L(isd), L(ied), L(jsd), L(jed), npz, False),
        "uc": (L(isd), L(ied + 1), L(jsd), L(jed), npz, False),
        "vc": (L(isd), L(ied), L(jsd), L(jed + 1), npz, False),
        "mfx": (L(is_), L(ie + 1), L(js), L(je), npz, False),
        "mfy": (L(is_), L(ie), L(js), L(je + 1), npz, False),
        "cx": (L(is_), L(ie + 1), L(jsd), L(jed), npz, False),
        "cy": (L(isd), L(ied), L(js), L(je + 1), npz, False),
        "diss_est": (L(isd), L(ied), L(jsd), L(jed), npz, False),
    }
    zeros = lambda nk: np.zeros((nsub, nk, nj, pitch))  # noqa: E731
    fort = {}
    for name, (li, hi, lj, hj, nk, kj) in shapes.items():
        src = st[name] if name in st else zeros(nk)
        fort[name] = to_fortran(src, li, hi, lj, hj, kj)
    addr = {k: v.ctypes.data for k, v in fort.items()}
    scal = dict(comm=0, npx=npx, npy=npx, npz=npz, ntiles=6, is_=is_, ie=ie, js=js, je=je, isd=isd, ied=ied,
                jsd=jsd, jed=jed, bdt=900.0, nq_tot=nq)
    hook.init(**scal)
    hook.run(**scal, ng=NG, ptop=float(ak[0]), ks=ks, layout_1=1, layout_2=1, adiabatic=1,
             ak=np.asfortranarray(ak), bk=np.asfortranarray(bk), **fort)
    hook.finalize()
    for name in want:
        assert fort[name].ctypes.data == addr[name], "buffers must be updated in place"
        li, hi, lj, hj, nk, kj = shapes[name]
        got = from_fortran(fort[name], nsub, nk, nj, pitch, li, hi, lj, hj, kj)
        a = got[..., NG:NG + N, NG:NG + N]
        b = want[name][..., NG:NG + N, NG:NG + N]
        assert np.array_equal(a, b), f"{name}: bridge result differs from the device API"
