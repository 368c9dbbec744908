"""A Fortran program calls the library through the reference's generated binding
(interface.f90.jinja2:24-82 -> include/geos_gtfv3_interface_mod.f90), as GEOS does.
CPU: the program compiles with amdflang, links libgeos_gtfv3_interface.so and binds the
three reference symbols.  GPU: one init/run/finalize on C12 L10 from Fortran gives, bit
for bit, what the Python hook gives through geos_gtfv3_run_c on the same fp32 buffers
(the reference's own bridge check is a Fortran program too,
test/py_ftn_interface/data/fortran_program.f90:16-32)."""
import importlib
import os
import shutil
import subprocess

import numpy as np
import pytest

from conftest import ROOT

NATIVE = os.path.join(ROOT, "tests", "native")
DRIVER = os.path.join(NATIVE, "bin", "fortran_driver")


def _build():
    if not shutil.which("amdflang") and not os.path.exists("/opt/rocm/bin/amdflang"):
        pytest.skip("amdflang not in this image")
    subprocess.run(["make", "-C", NATIVE], check=True, capture_output=True)


def test_fortran_driver_builds_and_binds_reference_symbols(pkg):
    _build()
    nm = subprocess.run(["nm", "-D", "--undefined-only", DRIVER], check=True, capture_output=True, text=True).stdout
    for sym in ("geos_gtfv3_init_c", "geos_gtfv3_run_c", "geos_gtfv3_finalize_c"):
        assert sym in nm, sym
    ldd = subprocess.run(["ldd", DRIVER], check=True, capture_output=True, text=True).stdout
    assert "libgeos_gtfv3_interface.so" in ldd and "not found" not in ldd.split("libgeos_gtfv3_interface.so")[1].split("\n")[0]


@pytest.mark.gpu
def test_fortran_caller_matches_python_hook(pkg, require_gpu, tmp_path):
    from test_gpu_bridge import OUT, _bridge_call, _setup, _shapes, to_fortran
    assert os.path.exists(DRIVER), "build it first: python -c 'import __graft_entry__ as g; g.build()'"
    npx, npz, nq = 13, 10, 2
    d, st, ak, bk, ks = _setup(pkg, npx, npz, nq)
    hook = importlib.import_module(pkg.__name__ + ".hook")
    shapes = _shapes(npx - 1, npz, nq)
    # the Python hook through geos_gtfv3_run_c (fp32)
    want, _ = _bridge_call(pkg, st, d, ak, bk, ks, npx, npz, nq, np.float32)
    # the same fp32 buffers written for the Fortran program (column-major, tiles last)
    zeros = lambda nk: np.zeros((d.nsub, nk, d.nj, d.pitch))  # noqa: E731
    arrs = [ak.astype(np.float32), bk.astype(np.float32)]
    for name in hook.RUN_ARRAYS[2:]:
        li, hi, lj, hj, nk, kj = shapes[name]
        src = st[name] if name in st else zeros(nk)
        arrs.append(to_fortran(src, li, hi, lj, hj, kj).astype(np.float32))
    d.close()
    fin, fout = tmp_path / "in.bin", tmp_path / "out.bin"
    with open(fin, "wb") as f:
        np.array([npx, npz, nq, ks, 0], dtype=np.int32).tofile(f)
        np.array([ak[0], 900.0], dtype=np.float32).tofile(f)
        for a in arrs:
            a.ravel(order="F").tofile(f)
    env = dict(os.environ, GTFV3_BRIDGE_TILES_PER_RANK="6")
    r = subprocess.run([DRIVER, str(fin), str(fout)], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    flat = np.fromfile(fout, dtype=np.float32)
    off = 0
    for name, a in zip(hook.RUN_ARRAYS, arrs):
        got = flat[off:off + a.size].reshape(a.shape, order="F")
        off += a.size
        if name in OUT:
            assert np.array_equal(got, want[name]), f"{name}: Fortran caller differs from the Python hook"
    assert off == flat.size
