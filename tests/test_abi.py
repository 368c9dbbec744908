"""The C-ABI library loads and exports every symbol include/*.h declares (CPU)."""
import ctypes

import numpy as np
import os
import re

import pytest

from conftest import ROOT


def _declared():
    names = set()
    for h in ("geos_gtfv3_interface.h", "gtfv3_device.h"):
        txt = open(os.path.join(ROOT, "include", h)).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        for m in re.finditer(r"^\s*(?:void\s*\*?|int)\s+(\w+)\s*\(", txt, flags=re.M):
            names.add(m.group(1))
    return names


def test_library_exports_all_declared_symbols(pkg):
    lib = ctypes.CDLL(pkg.LIB_PATH)
    declared = _declared()
    assert {"geos_gtfv3_init_c", "geos_gtfv3_run_c", "geos_gtfv3_finalize_c"} <= declared
    for name in declared:
        assert hasattr(lib, name), name
    assert declared == set(pkg.BRIDGE_SYMBOLS) | set(pkg.DEVICE_SYMBOLS)


def test_reference_signature_order():
    """Argument order of geos_gtfv3_run_c == example_def_dycore.yaml:21-70 (inputs, then inouts)."""
    yaml_order = ["comm", "npx", "npy", "npz", "ntiles", "is", "ie", "js", "je", "isd", "ied", "jsd", "jed", "bdt",
                  "nq_tot", "ng", "ptop", "ks", "layout_1", "layout_2", "adiabatic", "ak", "bk", "u", "v", "w",
                  "delz", "pt", "delp", "q", "ps", "pe", "pk", "peln", "pkz", "phis", "q_con", "omga", "ua", "va",
                  "uc", "vc", "mfx", "mfy", "cx", "cy", "diss_est"]
    txt = open(os.path.join(ROOT, "include", "geos_gtfv3_interface.h")).read()
    m = re.search(r"void geos_gtfv3_run_c\((.*?)\);", txt, flags=re.S)
    args = [a.strip().split()[-1].lstrip("*") for a in m.group(1).split(",")]
    assert args == yaml_order
    types = [a.strip().rsplit(" ", 1)[0].replace(" ", "") for a in m.group(1).split(",")]
    # argument.py:54-86 type map: MPI->void*, int->int, float->float, array_float->float*
    assert types[0] == "void*"
    assert types[13] == "float" and types[16] == "float"
    assert all(t == "float*" for t in types[21:])


def test_last_error_channel(pkg):
    lib = pkg.lib()
    h = lib.gtfv3_create(b"npx=13;bogus_key=1", 0, 1, None)
    assert not h
    buf = ctypes.create_string_buffer(256)
    n = lib.geos_gtfv3_last_error(buf, 256)
    assert n > 0 and b"bogus_key" in buf.value


def test_layout_rule_matches_reference():
    """numpy restatement of data_conversion.py:141/184 == Fortran-ordered arrays"""
    dim = [5, 4, 3]
    flat = np.arange(np.prod(dim), dtype=np.float64)
    view = flat.reshape(tuple(reversed(dim))).transpose()
    assert view.shape == tuple(dim) and view.flags.f_contiguous
    assert view[1, 0, 0] == 1.0 and view[0, 1, 0] == dim[0] and view[0, 0, 1] == dim[0] * dim[1]
    np.testing.assert_array_equal(view.flatten(order="F"), flat)


def test_no_kernel_uses_scratch(pkg, tmp_path):
    """Every gfx950 kernel of the library runs without private (scratch) memory: a
    stack object or a register spill in scratch costs HBM round trips on the hot path.
    (The round-1 multi-rank loopback fault was traced to an out-of-plane read in
    a2b_march_k -- the prefetched J == 1 edge row below a segment, fixed in 27fdd8c --
    not to scratch.)  Reads .private_segment_fixed_size from the code-object metadata."""
    import shutil
    import subprocess
    llvm = "/opt/rocm/lib/llvm/bin"
    if not os.path.exists(os.path.join(llvm, "llvm-readelf")):
        pytest.skip("ROCm LLVM tools not installed")
    lib = tmp_path / "lib.so"
    shutil.copy(pkg.LIB_PATH, lib)
    subprocess.run([os.path.join(llvm, "llvm-objdump"), "--offloading", str(lib)], check=True, cwd=tmp_path,
                   capture_output=True)
    objs = [p for p in tmp_path.iterdir() if "amdgcn" in p.name and "gfx950" in p.name]
    assert objs, "no gfx950 code object in the library"
    bad, nkern = [], 0
    for obj in objs:
        notes = subprocess.run([os.path.join(llvm, "llvm-readelf"), "--notes", str(obj)], check=True,
                               capture_output=True, text=True).stdout
        name = None
        for line in notes.splitlines():
            line = line.strip()
            if line.startswith(".name:"):
                name = line.split(":", 1)[1].strip()
            elif line.startswith(".private_segment_fixed_size:"):
                nkern += 1
                if int(line.split(":")[1]) != 0:
                    bad.append(name)
    assert nkern > 20
    assert not bad, f"kernels using scratch memory: {bad}"


def test_config_separators_and_malformed_values(pkg):
    """GTFV3_CONFIG items split on ',' or ';' (INTEGRATION.md's comma form); a value that is
    not a whole number (or not an integer for an integer key) is an error, never truncated"""
    lib = pkg.lib()
    buf = ctypes.create_string_buffer(256)
    ok = lib.gtfv3_create(b"npx=13, npz=3; nq=1,host_only=1,n_split=5 ,hord_mt=5", 0, 1, None)
    assert ok
    lib.gtfv3_destroy(ok)
    for bad, what in ((b"npx=13,npz=3,nq=1,host_only=1,n_split=6x", b"n_split"),
                      (b"npx=13,npz=3,nq=1,host_only=1,n_split=6.5", b"n_split"),
                      (b"npx=13,npz=3,nq=1,host_only=1,d4_bg=", b"d4_bg"),
                      (b"npx=13,npz=3,nq=1,host_only=1,nord=2,d4_bg=0.15,vtdm4=0.05x", b"vtdm4")):
        h = lib.gtfv3_create(bad, 0, 1, None)
        assert not h, bad
        assert lib.geos_gtfv3_last_error(buf, 256) > 0 and what in buf.value, buf.value


def test_hook_environment_switches(pkg, monkeypatch):
    """The CI's PACE_FLOAT_PRECISION / GTFV3_BACKEND (ci/pipeline/gtfv3_config.py:11,19-21)
    are read by the hook: the precision names the state arrays' dtype (32: the fp32 entry
    point, the CI's benchmark mode), the backend must be a GPU one (this build: HIP gfx950)"""
    import importlib

    import numpy as np
    hook = importlib.import_module(pkg.__name__ + ".hook")
    monkeypatch.delenv("PACE_FLOAT_PRECISION", raising=False)
    monkeypatch.delenv("GTFV3_BACKEND", raising=False)
    assert hook.check_environment() == (None, "hip")
    monkeypatch.setenv("PACE_FLOAT_PRECISION", "32")
    monkeypatch.setenv("GTFV3_BACKEND", "dace:gpu")
    assert hook.check_environment() == (32, "dace:gpu")
    for bad in ("numpy", "gt:cpu_ifirst", "fortran"):
        monkeypatch.setenv("GTFV3_BACKEND", bad)
        with pytest.raises(ValueError):
            hook.check_environment()
    monkeypatch.setenv("GTFV3_BACKEND", "hip")
    monkeypatch.setenv("PACE_FLOAT_PRECISION", "16")
    with pytest.raises(ValueError):
        hook.check_environment()
    # a float64 state under PACE_FLOAT_PRECISION=32 is refused before any library call
    monkeypatch.setenv("PACE_FLOAT_PRECISION", "32")
    with pytest.raises(TypeError):
        hook.geos_gtfv3.run(u=np.zeros(4))
