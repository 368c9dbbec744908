import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import gtfv3_pkg  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


@pytest.fixture(scope="session")
def pkg():
    return gtfv3_pkg.load()


def gpu_available():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def require_gpu():
    if not gpu_available():
        pytest.fail("GPU test selected but no GPU is visible")


def metrics_of(dom, s=None):
    """dict name -> plane(s) of the FV3 metric terms for a Domain's sub-domains, from the
    independent oracle grid (oracle/grid.py; tests/test_oracle_grid.py compares it with the
    product's grid.cpp), so the oracle never consumes the product's metrics"""
    from oracle import grid as og
    ms, _ = og.domain_metrics(dom.subs, dom.nx, dom.ny, dom.N, dom.pitch, dom.nj)
    if s is None:
        return ms
    return ms[s]


def oracle_scalars(dom):
    """{"corner_w", "da_min", "da_min_c"} of the oracle grid (the product's: Domain.scalars())"""
    from oracle import grid as og
    return og.domain_metrics(dom.subs, dom.nx, dom.ny, dom.N, dom.pitch, dom.nj)[1]


def checked_metrics(dom, s, tol=1e-12):
    """(metrics, scalars) of sub-domain s for random-input stencil tests: the product's grid
    after checking it field by field against the independent oracle grid to `tol` of each
    field's magnitude.  Random inputs put PPM's limiter branches next to their switch points,
    so a metric differing in the last digits (the two grids compute areas by different
    formulas: <= 7e-13 at C180) flips a few branches; the stencil is then checked on exactly
    the inputs the kernel saw, and the grid by this comparison (and tests/test_oracle_grid.py)."""
    mo = metrics_of(dom, s)
    so = oracle_scalars(dom)
    mp = {}
    for k, a in mo.items():
        b = dom.metric(k)[s]
        fin = np.isfinite(a) & np.isfinite(b)
        scale = np.abs(a[fin]).max() + 1e-300
        err = np.abs(a[fin] - b[fin]).max() / scale if fin.any() else 0.0
        assert err <= tol, f"metric {k}: product vs oracle grid {err:.2e} > {tol:.0e}"
        mp[k] = b
    sp = dom.scalars()
    for k in ("da_min", "da_min_c"):
        assert abs(sp[k] - so[k]) <= tol * abs(so[k]), k
    assert np.allclose(sp["corner_w"], so["corner_w"], rtol=tol, atol=tol)
    return mp, dict(da_min=sp["da_min"], da_min_c=sp["da_min_c"], corner_w=sp["corner_w"][s])


def rng(seed=20250117):
    return np.random.default_rng(seed)
