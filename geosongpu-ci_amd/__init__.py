"""geosongpu-ci_amd — MI355X-native FV3 dycore path behind the geos_gtfv3 bridge.

Product code: libgeos_gtfv3_interface.so (HIP kernels for gfx950 + C ABI) and the
Python host surface mirroring the reference's bridge/hook.
Imported as `geosongpu_ci_amd` through gtfv3_pkg.load().
"""
from ._lib import BRIDGE_SYMBOLS, DEVICE_SYMBOLS, LIB_PATH, GTFV3Error, lib  # noqa: F401
from .domain import NG, Domain, unique_id  # noqa: F401
