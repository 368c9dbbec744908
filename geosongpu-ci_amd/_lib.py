"""ctypes binding of libgeos_gtfv3_interface.so (include/*.h).

The shared library is the product: every stencil runs as a HIP kernel in it.
There is no CPU fallback — if the library is missing this module raises.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libgeos_gtfv3_interface.so")

# every symbol declared in include/geos_gtfv3_interface.h and include/gtfv3_device.h
BRIDGE_SYMBOLS = [
    "geos_gtfv3_init_c",
    "geos_gtfv3_run_c",
    "geos_gtfv3_finalize_c",
    "geos_gtfv3_run_f64_c",
    "geos_gtfv3_last_error",
]
DEVICE_SYMBOLS = [
    "gtfv3_bridge_stats",
    "gtfv3_create",
    "gtfv3_destroy",
    "gtfv3_get_unique_id",
    "gtfv3_bootstrap_id",
    "gtfv3_bootstrap_done",
    "gtfv3_dims",
    "gtfv3_sub_info",
    "gtfv3_field_create",
    "gtfv3_field_nk",
    "gtfv3_field_upload",
    "gtfv3_field_download",
    "gtfv3_field_upload_levels",
    "gtfv3_field_download_levels",
    "gtfv3_field_ptr",
    "gtfv3_get_metric",
    "gtfv3_get_xyz",
    "gtfv3_get_scalars",
    "gtfv3_level_damping",
    "gtfv3_halo_table",
    "gtfv3_halo_update",
    "gtfv3_stencil",
    "gtfv3_set_vertical",
    "gtfv3_step",
    "gtfv3_sync",
    "gtfv3_stream",
    "gtfv3_timers",
    "gtfv3_step_times",
    "gtfv3_halo_remote",
    "gtfv3_kernel_timing",
    "gtfv3_kernel_timing_filter",
    "gtfv3_set_streams",
    "gtfv3_kernel_stats",
]

_lib = None


class GTFV3Error(RuntimeError):
    pass


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise GTFV3Error(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
        )
    L = ctypes.CDLL(LIB_PATH)
    P = ctypes.c_void_p
    I = ctypes.c_int
    S = ctypes.c_char_p
    DP = ctypes.POINTER(ctypes.c_double)
    IP = ctypes.POINTER(ctypes.c_int)
    sig = {
        "geos_gtfv3_last_error": (I, [ctypes.c_char_p, I]),
        "gtfv3_create": (P, [S, I, I, P]),
        "gtfv3_destroy": (None, [P]),
        "gtfv3_get_unique_id": (I, [P]),
        "gtfv3_bootstrap_id": (I, [P, ctypes.c_char_p, IP, IP]),
        "gtfv3_bootstrap_done": (I, []),
        "gtfv3_bridge_stats": (I, [DP]),
        "gtfv3_dims": (I, [P, IP]),
        "gtfv3_sub_info": (I, [P, I, IP]),
        "gtfv3_field_create": (I, [P, S, I]),
        "gtfv3_field_nk": (I, [P, S]),
        "gtfv3_field_upload": (I, [P, S, I, DP]),
        "gtfv3_field_download": (I, [P, S, DP]),
        "gtfv3_field_upload_levels": (I, [P, S, I, I, DP]),
        "gtfv3_field_download_levels": (I, [P, S, I, I, DP]),
        "gtfv3_field_ptr": (P, [P, S]),
        "gtfv3_get_metric": (I, [P, S, DP]),
        "gtfv3_get_xyz": (I, [P, DP]),
        "gtfv3_get_scalars": (I, [P, DP]),
        "gtfv3_level_damping": (I, [P, DP, I]),
        "gtfv3_halo_table": (I, [P, I, IP, I]),
        "gtfv3_halo_update": (I, [P, S]),
        "gtfv3_stencil": (I, [P, S, S, DP, I]),
        "gtfv3_set_vertical": (I, [P, DP, DP, I]),
        "gtfv3_step": (I, [P, I]),
        "gtfv3_sync": (I, [P]),
        "gtfv3_stream": (P, [P]),
        "gtfv3_timers": (I, [P, ctypes.c_char_p, I]),
        "gtfv3_step_times": (I, [P, DP, I, I]),
        "gtfv3_halo_remote": (I, [P, I, I, IP, I]),
        "gtfv3_kernel_timing": (I, [P, I]),
        "gtfv3_kernel_timing_filter": (I, [P, ctypes.c_char_p]),
        "gtfv3_set_streams": (I, [P, I]),
        "gtfv3_kernel_stats": (I, [P, ctypes.c_char_p, I]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def last_error():
    buf = ctypes.create_string_buffer(4096)
    lib().geos_gtfv3_last_error(buf, 4096)
    return buf.value.decode(errors="replace")


def check(rc):
    if rc != 0:
        raise GTFV3Error(last_error())
    return rc


def dptr(a: np.ndarray):
    assert a.dtype == np.float64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
