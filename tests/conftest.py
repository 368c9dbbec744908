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


def rng(seed=20250117):
    return np.random.default_rng(seed)
