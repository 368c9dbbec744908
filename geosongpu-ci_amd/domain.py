"""Python handle on a device-resident dycore domain (libgeos_gtfv3_interface.so).

Arrays crossing this boundary use the HBM layout of DESIGN.md, fp64:
    field[s, k, j + NG, i + NG]      shape (nsub, nk, nj, pitch)
with s the local sub-domain, i,j local indices (compute cells 0..nx-1 / 0..ny-1,
halo down to -NG), staggered fields sharing the same padded plane.
"""
import ctypes

import numpy as np

from ._lib import GTFV3Error, check, dptr, lib

NG = 3

DEFAULT_CONFIG = dict(
    npx=49, npz=72, nq=4, layout_x=1, layout_y=1, dt=900.0, k_split=1, n_split=6,
    hord_mt=6, hord_vt=6, hord_tm=6, hord_dp=6, hord_tr=6,
    kord_mt=9, kord_wz=9, kord_tr=9, kord_tm=-9,
    dddmp=0.2, d2_bg=0.0, p_fac=0.05, fill=1, adiabatic=0, ptop=1.0,
)


def config_string(cfg: dict) -> bytes:
    return ";".join(f"{k}={v}" for k, v in cfg.items()).encode()


class Domain:
    def __init__(self, rank=0, nranks=1, nccl_id: bytes = None, **cfg):
        self.cfg = dict(DEFAULT_CONFIG)
        self.cfg.update(cfg)
        L = lib()
        idp = None
        if nccl_id is not None:
            self._id = ctypes.create_string_buffer(bytes(nccl_id), 128)
            idp = ctypes.cast(self._id, ctypes.c_void_p)
        self.h = L.gtfv3_create(config_string(self.cfg), rank, nranks, idp)
        if not self.h:
            from ._lib import last_error
            raise GTFV3Error(last_error())
        out = (ctypes.c_int * 10)()
        check(L.gtfv3_dims(self.h, out))
        (self.nx, self.ny, self.pitch, self.nj, self.nsub, self.npz, self.N,
         self.layout_x, self.layout_y, self.nq) = list(out)
        self.rank, self.nranks = rank, nranks
        self.subs = []
        for s in range(self.nsub):
            o = (ctypes.c_int * 8)()
            check(L.gtfv3_sub_info(self.h, s, o))
            self.subs.append(dict(tile=o[0], ioff=o[1], joff=o[2], N=o[3], flags=o[4], gid=o[5]))

    # ---- lifecycle ----
    def close(self):
        if getattr(self, "h", None):
            lib().gtfv3_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- shapes ----
    def shape(self, nk):
        return (self.nsub, nk, self.nj, self.pitch)

    def zeros(self, nk):
        return np.zeros(self.shape(nk))

    # ---- grid ----
    def metric(self, name):
        out = np.zeros((self.nsub, self.nj, self.pitch))
        check(lib().gtfv3_get_metric(self.h, name.encode(), dptr(out)))
        return out

    def corner_xyz(self):
        H = NG + 1
        out = np.zeros((self.nsub, self.ny + 2 * H + 1, self.nx + 2 * H + 1, 3))
        check(lib().gtfv3_get_xyz(self.h, dptr(out)))
        return out

    def scalars(self):
        out = np.zeros(2 + 12 * self.nsub)
        check(lib().gtfv3_get_scalars(self.h, dptr(out)))
        return dict(da_min=out[0], da_min_c=out[1], corner_w=out[2:].reshape(self.nsub, 4, 3))

    def level_damping(self):
        """the namelist's column of d_sw damping parameters (damp.hip column_damping): a list of
        per-level dicts and n_con, the number of top levels the d_con heat reaches"""
        out = np.zeros((self.npz, 10))
        n_con = lib().gtfv3_level_damping(self.h, dptr(out), self.npz)
        if n_con < 0:
            check(n_con)
        keys = ("d2_divg", "vt4", "dp4", "w4", "pt4", "d_con", "nord", "nord_v", "nord_w", "nord_t")
        return [dict(zip(keys, row)) for row in out], n_con

    # ---- fields ----
    def create(self, name, nk):
        check(lib().gtfv3_field_create(self.h, name.encode(), nk))

    def nk_of(self, name):
        return lib().gtfv3_field_nk(self.h, name.encode())

    def upload(self, name, arr):
        arr = np.ascontiguousarray(arr, dtype=np.float64)
        if arr.ndim != 4 or arr.shape[0] != self.nsub or arr.shape[2:] != (self.nj, self.pitch):
            raise ValueError(f"{name}: array shape {arr.shape} is not (nsub, nk, nj, pitch)")
        check(lib().gtfv3_field_upload(self.h, name.encode(), arr.shape[1], dptr(arr)))

    def upload_levels(self, name, k0, arr):
        """levels k0 .. k0 + arr.shape[1] - 1 of an existing field (every sub-domain)"""
        arr = np.ascontiguousarray(arr, dtype=np.float64)
        if arr.ndim != 4 or arr.shape[0] != self.nsub or arr.shape[2:] != (self.nj, self.pitch):
            raise ValueError(f"{name}: array shape {arr.shape} is not (nsub, nk, nj, pitch)")
        check(lib().gtfv3_field_upload_levels(self.h, name.encode(), k0, arr.shape[1], dptr(arr)))

    def download(self, name):
        nk = self.nk_of(name)
        if nk <= 0:
            raise GTFV3Error(f"no field {name}")
        out = np.zeros(self.shape(nk))
        check(lib().gtfv3_field_download(self.h, name.encode(), dptr(out)))
        return out

    def download_levels(self, name, k0, nk):
        """levels k0 .. k0 + nk - 1 of a field, every sub-domain: (nsub, nk, nj, pitch)"""
        out = np.zeros(self.shape(nk))
        check(lib().gtfv3_field_download_levels(self.h, name.encode(), int(k0), int(nk), dptr(out)))
        return out

    def device_ptr(self, name):
        """raw device pointer; valid until the next step() (q ping-pongs between planes)"""
        return lib().gtfv3_field_ptr(self.h, name.encode())

    # ---- operations ----
    def halo_update(self, spec: str):
        check(lib().gtfv3_halo_update(self.h, spec.encode()))

    def stencil(self, name, fields, params=()):
        p = np.ascontiguousarray(params, dtype=np.float64) if len(params) else np.zeros(1)
        check(lib().gtfv3_stencil(self.h, name.encode(), ",".join(fields).encode(), dptr(p), len(params)))

    def tracer_stats(self):
        """(nq, 4) array per tracer of the device state: sum(q * delp * area) over the compute
        domain, min q, max q, count of non-finite q (the "tracer_stats" stencil)"""
        self.stencil("tracer_stats", [])
        return self.download("tracer_stats")[0, 0].ravel()[:4 * self.nq].reshape(self.nq, 4)

    def set_vertical(self, ak, bk, ks):
        ak = np.ascontiguousarray(ak, dtype=np.float64)
        bk = np.ascontiguousarray(bk, dtype=np.float64)
        check(lib().gtfv3_set_vertical(self.h, dptr(ak), dptr(bk), int(ks)))

    def step(self, n=1):
        check(lib().gtfv3_step(self.h, n))

    def sync(self):
        check(lib().gtfv3_sync(self.h))

    def stream(self):
        return lib().gtfv3_stream(self.h)

    def kernel_timing(self, on=True):
        check(lib().gtfv3_kernel_timing(self.h, 1 if on else 0))

    def kernel_timing_filter(self, kernel=None):
        """time only `kernel` (its launch name) while timing is on; None: every kernel"""
        check(lib().gtfv3_kernel_timing_filter(self.h, kernel.encode() if kernel else None))

    def set_streams(self, n):
        """1: every kernel of the step on one stream; 3: the default fork onto side streams"""
        check(lib().gtfv3_set_streams(self.h, int(n)))

    def kernel_stats(self):
        """{kernel: (total_ms, launches, algorithmic_bytes)} since kernel_timing(True)"""
        buf = ctypes.create_string_buffer(1 << 16)
        check(lib().gtfv3_kernel_stats(self.h, buf, 1 << 16))
        out = {}
        for item in buf.value.decode().split(";"):
            if "=" in item:
                k, v = item.split("=")
                ms, n, b = v.split(",")
                out[k] = (float(ms), int(n), float(b))
        return out

    def step_times(self, reset=True):
        """device ms of each step completed since the last reset (HIP events on the library
        stream around fv_dynamics), oldest first"""
        n = lib().gtfv3_step_times(self.h, None, 0, 0)
        if n < 0:
            raise GTFV3Error("gtfv3_step_times failed")
        out = np.zeros(max(n, 1))
        n2 = lib().gtfv3_step_times(self.h, dptr(out), len(out), 1 if reset else 0)
        if n2 < 0:
            raise GTFV3Error("gtfv3_step_times failed")
        return out[:n2].tolist()

    def timers(self):
        buf = ctypes.create_string_buffer(8192)
        check(lib().gtfv3_timers(self.h, buf, 8192))
        out = {}
        for item in buf.value.decode().split(";"):
            if "=" in item:
                k, v = item.split("=")
                out[k] = float(v)
        return out


def unique_id() -> bytes:
    buf = ctypes.create_string_buffer(128)
    check(lib().gtfv3_get_unique_id(ctypes.cast(buf, ctypes.c_void_p)))
    return buf.raw
