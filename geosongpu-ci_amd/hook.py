"""Python mirror of the generated `geos_gtfv3` hook (reference:
src/tcn/py_ftn_interface/templates/hook.py.jinja2:11-34,74), backed by the HIP
library instead of an embedded Python dycore.

    from geosongpu_ci_amd.hook import geos_gtfv3
    geos_gtfv3.init(comm=0, npx=181, npy=181, npz=72, ntiles=6, is_=1, ie=180, ...)
    geos_gtfv3.run(comm=0, ..., u=u, v=v, ...)     # arrays in Fortran layout, updated in place
    geos_gtfv3.finalize()

Arrays are what the reference hook receives from FortranPythonConversion.fortran_to_python
(data_conversion.py:134-148): zero-copy views of Fortran buffers with i fastest,
i.e. Fortran-ordered numpy arrays of the FV3 shapes listed in SURVEY.md §8(b)
(`pe` and `peln` are (i, k, j)).  With GTFV3_BRIDGE_TILES_PER_RANK=6 (all six tiles
on one GPU, one process) every array carries a trailing tile axis of length 6.

The keyword `is` of the reference argument list is spelled `is_` here (Python
keyword); `is` is also accepted through **kwargs.

The CI's two environment switches (ci/pipeline/gtfv3_config.py:11,19-21) are honoured:
  * PACE_FLOAT_PRECISION (32 | 64, unset: either): the precision of the state arrays the hook
    takes -- 32 routes float32 arrays through geos_gtfv3_run_c (the CI's benchmark mode,
    gtfv3_config.py:27), 64 float64 arrays through geos_gtfv3_run_f64_c; arrays of the other
    precision raise TypeError.  The stencils compute in fp64 either way: the
    arithmetic is never below the precision the switch names.
  * GTFV3_BACKEND: this build has one backend, the HIP kernels for gfx950.  Unset, "hip" or
    "hip:gfx950" select it; the reference's GPU backends ("dace:gpu", "gt:gpu", "cuda") are
    mapped to it; a CPU backend ("numpy", "gt:cpu_ifirst", "dace:cpu", ...) or "fortran" (the
    Fortran dycore: the hook is not called at all) raise ValueError.
"""
import ctypes
import os

import numpy as np

from ._lib import lib

INIT_ARGS = ("comm", "npx", "npy", "npz", "ntiles", "is", "ie", "js", "je", "isd", "ied", "jsd", "jed", "bdt",
             "nq_tot")
RUN_SCALARS = INIT_ARGS + ("ng", "ptop", "ks", "layout_1", "layout_2", "adiabatic")
RUN_ARRAYS = ("ak", "bk", "u", "v", "w", "delz", "pt", "delp", "q", "ps", "pe", "pk", "peln", "pkz", "phis",
              "q_con", "omga", "ua", "va", "uc", "vc", "mfx", "mfy", "cx", "cy", "diss_est")
FLOATS = ("bdt", "ptop")


def expected_sizes(kw):
    """Element count of every run array implied by the scalar arguments (FV3 declarations,
    SURVEY.md §8b); the bridge copies exactly this many elements in and out, so a smaller
    caller buffer would be read and written out of bounds."""
    i0, i1, j0, j1 = kw["is"], kw["ie"], kw["js"], kw["je"]
    ni_d, nj_d = kw["ied"] - kw["isd"] + 1, kw["jed"] - kw["jsd"] + 1
    ni, nj, npz, nq = i1 - i0 + 1, j1 - j0 + 1, kw["npz"], kw["nq_tot"]
    cell = ni_d * nj_d
    n = {
        "ak": npz + 1, "bk": npz + 1,
        "u": ni_d * (nj_d + 1) * npz, "v": (ni_d + 1) * nj_d * npz,
        "q": cell * npz * nq, "ps": cell, "phis": cell,
        "pe": (ni + 2) * (nj + 2) * (npz + 1), "pk": ni * nj * (npz + 1), "peln": ni * nj * (npz + 1),
        "pkz": ni * nj * npz, "uc": (ni_d + 1) * nj_d * npz, "vc": ni_d * (nj_d + 1) * npz,
        "mfx": (ni + 1) * nj * npz, "mfy": ni * (nj + 1) * npz,
        "cx": (ni + 1) * nj_d * npz, "cy": ni_d * (nj + 1) * npz,
    }
    for f in ("w", "delz", "pt", "delp", "q_con", "omga", "ua", "va", "diss_est"):
        n[f] = cell * npz
    tiles = int(os.environ.get("GTFV3_BRIDGE_TILES_PER_RANK", "1"))
    return {k: v * (tiles if k not in ("ak", "bk") else 1) for k, v in n.items()}


GPU_BACKENDS = ("hip", "hip:gfx950", "dace:gpu", "gt:gpu", "cuda", "gpu")


def check_environment():
    """(precision in bits or None, backend name) from PACE_FLOAT_PRECISION / GTFV3_BACKEND"""
    prec = os.environ.get("PACE_FLOAT_PRECISION", "").strip()
    if prec not in ("", "32", "64"):
        raise ValueError(f"PACE_FLOAT_PRECISION must be 32 or 64, not {prec!r}")
    backend = os.environ.get("GTFV3_BACKEND", "hip").strip() or "hip"
    if backend not in GPU_BACKENDS:
        raise ValueError(f"GTFV3_BACKEND={backend!r}: this build runs the HIP (gfx950) backend only; "
                         f"accepted: {', '.join(GPU_BACKENDS)}")
    return (int(prec) if prec else None), backend


def _norm(kwargs):
    if "is_" in kwargs:
        kwargs = dict(kwargs)
        kwargs["is"] = kwargs.pop("is_")
    return kwargs


def _scalar_args(kw, names):
    out = []
    for n in names:
        v = kw[n]
        if n == "comm":
            out.append(ctypes.c_void_p(int(v)))
        elif n in FLOATS:
            out.append(ctypes.c_float(float(v)))
        else:
            out.append(ctypes.c_int(int(v)))
    return out


class GEOS_GTFV3:
    """init / run / finalize with the reference hook's argument names and order."""

    def init(self, **kwargs):
        check_environment()
        kw = _norm(kwargs)
        lib().geos_gtfv3_init_c(*_scalar_args(kw, INIT_ARGS))

    def run(self, **kwargs):
        kw = _norm(kwargs)
        arrs = []
        dtype = np.asarray(kw["u"]).dtype
        if dtype not in (np.float32, np.float64):
            raise TypeError("geos_gtfv3.run: state arrays must be float32 or float64")
        prec, _ = check_environment()
        if prec is not None and dtype != (np.float32 if prec == 32 else np.float64):
            raise TypeError(f"geos_gtfv3.run: PACE_FLOAT_PRECISION={prec} but the state arrays are {dtype}")
        ct = ctypes.c_double if dtype == np.float64 else ctypes.c_float
        need = expected_sizes(kw)
        for n in RUN_ARRAYS:
            a = kw[n]
            if not (isinstance(a, np.ndarray) and a.dtype == dtype and (a.flags.f_contiguous or a.ndim == 1)):
                raise TypeError(f"geos_gtfv3.run: {n} must be a Fortran-contiguous {dtype} array "
                                "(in-place update of the caller's buffer)")
            if a.size != need[n]:
                raise ValueError(f"geos_gtfv3.run: {n} has {a.size} elements, the bounds imply {need[n]}")
            arrs.append(a.ctypes.data_as(ctypes.POINTER(ct)))
        fn = lib().geos_gtfv3_run_f64_c if dtype == np.float64 else lib().geos_gtfv3_run_c
        fn(*_scalar_args(kw, RUN_SCALARS), *arrs)

    def finalize(self):
        lib().geos_gtfv3_finalize_c()


geos_gtfv3 = GEOS_GTFV3()
