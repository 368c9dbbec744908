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
    """dict name -> plane(s) for all metrics of a Domain"""
    names = ["area", "rarea", "area_c", "rarea_c", "dx", "dy", "dxa", "dya", "dxc", "dyc", "rdx", "rdy",
             "rdxa", "rdya", "rdxc", "rdyc"] + [f"sin_sg{i}" for i in range(1, 10)] + \
        [f"cos_sg{i}" for i in range(1, 10)] + ["cosa_u", "sina_u", "rsin_u", "cosa_v", "sina_v", "rsin_v",
                                                "cosa_s", "rsin2", "cosa", "rsina", "fC", "f0",
                                                "a11", "a12", "a21", "a22", "lat", "lon"]
    allm = {n: dom.metric(n) for n in names}
    if s is None:
        return [{n: v[k] for n, v in allm.items()} for k in range(dom.nsub)]
    return {n: v[s] for n, v in allm.items()}


def rng(seed=20250117):
    return np.random.default_rng(seed)
