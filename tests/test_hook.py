"""Host logic of the Python hook mirror (hook.py.jinja2:11-34): the array sizes implied by
the scalar bounds, and the refusal of a mis-sized buffer before any library call (the
bridge copies exactly those sizes in and out of the caller's memory)."""
import importlib

import numpy as np
import pytest

from test_gpu_bridge import _shapes


def _scal(N, npz, nq):
    return {"comm": 0, "npx": N + 1, "npy": N + 1, "npz": npz, "ntiles": 6, "is": 1, "ie": N, "js": 1, "je": N,
            "isd": -2, "ied": N + 3, "jsd": -2, "jed": N + 3, "bdt": 900.0, "nq_tot": nq}


@pytest.mark.parametrize("tiles", ["1", "6"])
def test_expected_sizes_match_fv3_bounds(pkg, monkeypatch, tiles):
    hook = importlib.import_module(pkg.__name__ + ".hook")
    monkeypatch.setenv("GTFV3_BRIDGE_TILES_PER_RANK", tiles)
    N, npz, nq = 12, 10, 3
    need = hook.expected_sizes(_scal(N, npz, nq))
    for name, (li, hi, lj, hj, nk, _) in _shapes(N, npz, nq).items():
        assert need[name] == (hi - li + 1) * (hj - lj + 1) * nk * int(tiles), name
    assert need["ak"] == need["bk"] == npz + 1
    assert set(need) == set(hook.RUN_ARRAYS)


def test_run_refuses_undersized_buffer(pkg, monkeypatch):
    hook = importlib.import_module(pkg.__name__ + ".hook")
    monkeypatch.setenv("GTFV3_BRIDGE_TILES_PER_RANK", "1")
    N, npz, nq = 12, 4, 2
    kw = _scal(N, npz, nq)
    need = hook.expected_sizes(kw)
    arrs = {n: np.zeros(need[n]) for n in hook.RUN_ARRAYS}
    arrs["q"] = np.zeros(need["q"] - need["w"])  # one tracer short
    with pytest.raises(ValueError, match="q has"):
        hook.geos_gtfv3.run(**kw, ng=3, ptop=1.0, ks=0, layout_1=1, layout_2=1, adiabatic=0, **arrs)
