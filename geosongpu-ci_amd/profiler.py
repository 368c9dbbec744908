"""Profiler ranges for the hook's callers: the counterpart of the reference's generated
`cuda_profiler.py` (src/tcn/py_ftn_interface/templates/cuda_profiler.py:22-75), with roctx
ranges in place of NVTX and the HIP runtime's device synchronisation in place of cupy's.

    from geosongpu_ci_amd.profiler import TimedHIPProfiler
    timings = {}
    with TimedHIPProfiler("geos_gtfv3", timings):
        geos_gtfv3.run(...)
    # timings["geos_gtfv3"] == [seconds, ...]; under `rocprofv3 --marker-trace` the range
    # "geos_gtfv3" brackets the step's kernels

Semantics follow the reference class by class: entering / leaving a range synchronises the
device (so the range and the wall time cover the GPU work), `start_cuda_profiler` /
`stop_cuda_profiler` resume / pause the attached profiler's collection, `mark_cuda_profiler`
drops a marker, and everything is a no-op when no GPU is present (the reference's
GPU_AVAILABLE).  The reference's names are kept as aliases (CUDAProfiler,
TimedCUDAProfiler) so code written against it runs unchanged.

roctx: librocprofiler-sdk-roctx (the marker library rocprofv3 --marker-trace records);
without a profiler attached its calls return at once.  Neither library is required: a
missing one makes the ranges no-ops, like the reference without cupy.
"""
import ctypes
import time
from typing import Dict, List

_ROCTX_NAMES = ("librocprofiler-sdk-roctx.so.1", "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1",
                "libroctx64.so.4", "/opt/rocm/lib/libroctx64.so.4")
_HIP_NAMES = ("libamdhip64.so", "/opt/rocm/lib/libamdhip64.so")


def _load(names):
    for n in names:
        try:
            return ctypes.CDLL(n)
        except OSError:
            continue
    return None


_roctx = None
_hip = None
_gpu = None


def roctx():
    """the roctx library (or None), loaded once"""
    global _roctx
    if _roctx is None:
        _roctx = _load(_ROCTX_NAMES) or False
        if _roctx:
            _roctx.roctxRangePushA.argtypes = [ctypes.c_char_p]
            _roctx.roctxRangePushA.restype = ctypes.c_int
            _roctx.roctxRangePop.restype = ctypes.c_int
            _roctx.roctxMarkA.argtypes = [ctypes.c_char_p]
    return _roctx or None


def gpu_available():
    """whether a HIP device is present (the reference's GPU_AVAILABLE, probed on first use
    instead of at import so importing this module never initialises the GPU)"""
    global _hip, _gpu
    if _gpu is None:
        _hip = _load(_HIP_NAMES)
        n = ctypes.c_int(0)
        _gpu = bool(_hip) and _hip.hipGetDeviceCount(ctypes.byref(n)) == 0 and n.value > 0
    return _gpu


def _sync():
    if gpu_available():
        err = _hip.hipDeviceSynchronize()
        if err != 0:
            raise RuntimeError(f"hipDeviceSynchronize failed (hipError_t {err})")


class HIPProfiler:
    """A roctx range around a block, the device synchronised on entry and exit
    (cuda_profiler.py:22-36)."""

    def __init__(self, label: str) -> None:
        self.label = label

    def __enter__(self):
        _sync()
        lib = roctx()
        if lib:
            lib.roctxRangePushA(self.label.encode())

    def __exit__(self, _type, _val, _traceback):
        _sync()
        lib = roctx()
        if lib:
            lib.roctxRangePop()

    @classmethod
    def sync_device(cls):
        _sync()

    @classmethod
    def _tid(cls):
        lib = roctx()
        if not lib or not hasattr(lib, "roctxGetThreadId"):
            return None
        tid = ctypes.c_uint64(0)
        lib.roctxGetThreadId(ctypes.byref(tid))
        return tid

    @classmethod
    def start_cuda_profiler(cls):
        """resume the attached profiler's collection (cupy.cuda.profiler.start)"""
        tid = cls._tid()
        if gpu_available() and tid is not None:
            roctx().roctxProfilerResume(tid)

    @classmethod
    def stop_cuda_profiler(cls):
        """pause the attached profiler's collection (cupy.cuda.profiler.stop)"""
        tid = cls._tid()
        if gpu_available() and tid is not None:
            roctx().roctxProfilerPause(tid)

    @classmethod
    def mark_cuda_profiler(cls, message: str):
        lib = roctx()
        if gpu_available() and lib:
            lib.roctxMarkA(message.encode())


class TimedHIPProfiler(HIPProfiler):
    """HIPProfiler that appends the block's wall time (seconds, device work included) to
    timings[label] (cuda_profiler.py:59-75)."""

    def __init__(self, label: str, timings: Dict[str, List[float]]) -> None:
        super().__init__(label)
        self._start_time = 0.0
        self._timings = timings

    def __enter__(self):
        super().__enter__()
        self._start_time = time.perf_counter()

    def __exit__(self, _type, _val, _traceback):
        super().__exit__(_type, _val, _traceback)
        t = time.perf_counter() - self._start_time
        self._timings.setdefault(self.label, []).append(t)


# the reference's names
CUDAProfiler = HIPProfiler
TimedCUDAProfiler = TimedHIPProfiler
