"""Profiler ranges of the hook's callers (profiler.py; reference cuda_profiler.py:22-75):
timings recorded per label, the reference's class names, roctx ranges that nest, and on the
GPU a range around a dycore step whose time covers the device work."""
import importlib
import time

import pytest


def _prof(pkg):
    return importlib.import_module(pkg.__name__ + ".profiler")


def test_timed_profiler_records_per_label(pkg):
    p = _prof(pkg)
    timings = {}
    for _ in range(2):
        with p.TimedHIPProfiler("step", timings):
            time.sleep(0.01)
    with p.TimedCUDAProfiler("other", timings):
        pass
    assert sorted(timings) == ["other", "step"]
    assert len(timings["step"]) == 2 and all(t >= 0.009 for t in timings["step"])
    assert len(timings["other"]) == 1
    assert p.CUDAProfiler is p.HIPProfiler and p.TimedCUDAProfiler is p.TimedHIPProfiler


def test_roctx_ranges_nest(pkg):
    p = _prof(pkg)
    lib = p.roctx()
    if lib is None:
        pytest.skip("no roctx library in this image")
    # roctxRangePushA returns the nesting level of the range it opens (or a negative error)
    a = lib.roctxRangePushA(b"outer")
    b = lib.roctxRangePushA(b"inner")
    assert lib.roctxRangePop() >= 0 and lib.roctxRangePop() >= 0
    assert a >= 0 and b == a + 1
    p.HIPProfiler.mark_cuda_profiler("mark")  # no-op without a GPU or an attached profiler


@pytest.mark.gpu
def test_range_covers_device_work(pkg, require_gpu):
    p = _prof(pkg)
    state = importlib.import_module(pkg.__name__ + ".state")
    assert p.gpu_available()
    d = pkg.Domain(npx=49, npz=30, nq=1)
    ak, bk, ks = state.hybrid_levels(30)
    for k, v in state.jablonowski_williamson(d, ak, bk).items():
        d.upload(k, v)
    d.set_vertical(ak, bk, ks)
    d.step(1)
    timings = {}
    p.HIPProfiler.stop_cuda_profiler()
    p.HIPProfiler.start_cuda_profiler()
    with p.TimedHIPProfiler("fv_dynamics", timings):
        d.step(1)
    t_range = timings["fv_dynamics"][0]
    # the same step timed by hand with a device synchronisation after it: the range (device
    # synchronised on both sides) measures the same thing
    t0 = time.perf_counter()
    d.step(1)
    p.HIPProfiler.sync_device()
    t_sync = time.perf_counter() - t0
    assert 0.5 * t_sync < t_range < 2.0 * t_sync + 0.05
    d.close()
