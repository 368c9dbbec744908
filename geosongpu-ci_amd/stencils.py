"""NDSL-style stencil surface backed by the HIP library.

Two factories:
  * get_factories_single_tile(nx, ny, nz, nhalo): host numpy arrays in and out (the DSL
    pattern programs' single-tile numpy setup);
  * get_factories_cubed_sphere(npx, npz, nq, layout): device-resident quantities on the whole
    cubed sphere for the dycore stencils (c_sw, d_sw, fv_tp_2d, riem_solver_c, riem_solver3,
    update_dz_d, a2b_ord4, held_suarez, the moist columns ...), called the NDSL way --
    `self.c_sw = stencil_factory.from_dims_halo(func=c_sw, compute_dims=[X_DIM, Y_DIM, Z_DIM])`,
    `self.c_sw(delp, pt, w, u, v, uc, vc, ua, va, ut, vt, delpc, ptc, wc, dt2=dt2)` -- with the
    fields staying in HBM between calls (host views are synchronised lazily).

Mirrors the call shapes the reference's DSL pattern programs use
(dsl_patterns/Do__get_top_of_the_column.py:28-55, Do__while_in_gt_functions.py:15-52,
WIP__hybrid_index_2dout.py:25-65):

    stencil_factory, quantity_factory = get_factories_single_tile(nx, ny, nz, nhalo)
    tmp = quantity_factory.zeros([X_DIM, Y_DIM], "n/a")
    st = stencil_factory.from_dims_halo(func=column_top, compute_dims=[X_DIM, Y_DIM, Z_DIM])
    st(field_in, field_out)              # numpy (nx, ny, nz) arrays or Quantities, outputs in place

`func` names one of the library's HIP stencils (a `StencilDef` below) instead of a
gtscript function: there is no DSL compiler here, every stencil is a hand-written
kernel.  Arrays are indexed [i, j, k] like NDSL's numpy views.  Each call uploads
the arguments to the device, launches the kernel and downloads the outputs, so this
surface is for validation-sized work; the dycore itself keeps its state in HBM
(Domain / gtfv3_step).
"""
from dataclasses import dataclass
from typing import Sequence, Tuple

import numpy as np

from .domain import NG, Domain

X_DIM, Y_DIM, Z_DIM = "x", "y", "z"
X_INTERFACE_DIM, Y_INTERFACE_DIM, Z_INTERFACE_DIM = "x_interface", "y_interface", "z_interface"


@dataclass(frozen=True)
class StencilDef:
    """A library stencil: registry name, positional argument count, which arguments
    are written (downloaded after the call) and the names of its scalar parameters."""
    name: str
    nargs: int
    outputs: Tuple[int, ...]
    params: Tuple[str, ...] = ()


column_top = StencilDef("column_top", 2, (1,))
column_while_lt = StencilDef("column_while_lt", 2, (1,), ("thr",))
column_gather_k = StencilDef("column_gather_k", 4, (3,))

# dycore stencils (csrc/stencils_registry.cpp; argument order = the FV3 routine's)
c_sw = StencilDef("c_sw", 14, tuple(range(5, 14)), ("dt2",))
d_sw = StencilDef("d_sw", 18, (0, 1, 2, 3, 4) + tuple(range(9, 18)),
                  ("dt", "dddmp", "d2_bg", "hord_mt", "hord_vt", "hord_tm", "hord_dp"))
fv_tp_2d = StencilDef("fv_tp_2d", 11, (9, 10), ("ord", "nt"))
fv_tp_2d_pair = StencilDef("fv_tp_2d_pair", 12, (8, 9, 10, 11), ("ord",))
riem_solver_c = StencilDef("riem_solver_c", 6, (4, 5), ("dt2", "ptop", "p_fac", "dz_min"))
riem_solver3 = StencilDef("riem_solver3", 12, (2, 4) + tuple(range(5, 12)), ("dt", "ptop", "p_fac", "dz_min", "last_call"))
edge_profile = StencilDef("edge_profile", 8, (4, 5, 6, 7), ("variant",))
update_dz_d = StencilDef("update_dz_d", 5, (0,), ("hord",))
a2b_ord4 = StencilDef("a2b_ord4", 2, (1,))
p_grad_c = StencilDef("p_grad_c", 5, (3, 4), ("dt2",))
nh_p_grad = StencilDef("nh_p_grad", 6, (4, 5), ("dt", "ptop"))
held_suarez = StencilDef("held_suarez", 4, (1, 2, 3), ("dt",))
moist_qsat = StencilDef("moist_qsat", 5, (2, 3, 4))
fillq2zero = StencilDef("fillq2zero", 3, (0, 2))
gfdl_1m = StencilDef("gfdl_1m", 13, tuple(range(7)) + (9, 10, 11, 12), ("dt",))
evap_subl_pdf = StencilDef("evap_subl_pdf", 11, tuple(range(8)), ("dt",))
radcouple = StencilDef("radcouple", 22, tuple(range(13, 22)))
aer_activation = StencilDef("aer_activation", 8, (5, 6, 7))
moist_prep = StencilDef("moist_prep", 5, (2, 3, 4))
cup_gf_sh = StencilDef("cup_gf_sh", 14, (0, 1, 7, 8, 9, 10, 11, 12, 13), ("dt",))
buoyancy = StencilDef("buoyancy", 8, (4, 5, 6, 7))


class Quantity:
    """Field with dims/units and a numpy `view` indexed [i, j(, k)] (NDSL Quantity shape)."""

    def __init__(self, dims: Sequence[str], units: str, shape: Tuple[int, ...], dtype=np.float64):
        self.dims = tuple(dims)
        self.units = units
        self.data = np.zeros(shape, dtype=dtype)

    @property
    def view(self):
        return self.data


class QuantityFactory:
    def __init__(self, nx: int, ny: int, nz: int, nhalo: int):
        self.sizes = {X_DIM: nx, Y_DIM: ny, Z_DIM: nz, X_INTERFACE_DIM: nx + 1, Y_INTERFACE_DIM: ny + 1,
                      Z_INTERFACE_DIM: nz + 1}
        self.nhalo = nhalo

    def zeros(self, dims, units, dtype=np.float64):
        return Quantity(dims, units, tuple(self.sizes[d] for d in dims), dtype)

    def ones(self, dims, units, dtype=np.float64):
        q = self.zeros(dims, units, dtype)
        q.data[...] = 1
        return q


class FrozenStencil:
    def __init__(self, factory: "StencilFactory", sdef: StencilDef, compute_dims):
        if not isinstance(sdef, StencilDef):
            raise TypeError("from_dims_halo: func must be a StencilDef of the HIP library "
                            "(column_top, column_while_lt, column_gather_k, ...)")
        self.f, self.sdef, self.compute_dims = factory, sdef, tuple(compute_dims)

    def __call__(self, *args, **params):
        sd = self.sdef
        if len(args) != sd.nargs:
            raise TypeError(f"{sd.name}: expected {sd.nargs} fields, got {len(args)}")
        arrs = [a.data if isinstance(a, Quantity) else a for a in args]
        names = [f"_ndsl_{sd.name}_{n}" for n in range(len(arrs))]
        for n, (nm, a) in enumerate(zip(names, arrs)):
            self.f._upload(nm, np.asarray(a))
        p = [float(params[k]) for k in sd.params]
        self.f.domain.stencil(sd.name, names, p)
        for n in sd.outputs:
            out = self.f._download(names[n], arrs[n].shape)
            arrs[n][...] = out.astype(arrs[n].dtype)


class StencilFactory:
    """Single-tile stencil factory on a device Domain (tile 0 of a small cube)."""

    def __init__(self, nx: int, ny: int, nz: int, nhalo: int = 0):
        if nhalo > NG:
            raise ValueError(f"nhalo {nhalo} > {NG}")
        self.nx, self.ny, self.nz = nx, ny, nz
        n = max(nx, ny, 4)
        self.domain = Domain(npx=n + 1, npz=nz, nq=1)

    def from_dims_halo(self, func, compute_dims, compute_halos=()):
        return FrozenStencil(self, func, compute_dims)

    def _upload(self, name, a):
        d = self.domain
        a3 = a.reshape(a.shape + (1,)) if a.ndim == 2 else a
        nk = a3.shape[2]
        buf = d.zeros(nk)
        buf[0, :, NG:NG + a3.shape[1], NG:NG + a3.shape[0]] = np.transpose(a3, (2, 1, 0))
        d.upload(name, buf)

    def _download(self, name, shape):
        full = self.domain.download(name)
        nk = full.shape[1]
        out = np.transpose(full[0, :, NG:NG + shape[1], NG:NG + shape[0]], (2, 1, 0))
        return out[..., 0] if len(shape) == 2 else out.reshape(shape[0], shape[1], nk)

    def close(self):
        self.domain.close()


def get_factories_single_tile(nx: int, ny: int, nz: int, nhalo: int):
    """(StencilFactory, QuantityFactory) like ndsl.boilerplate.get_factories_single_tile_numpy."""
    return StencilFactory(nx, ny, nz, nhalo), QuantityFactory(nx, ny, nz, nhalo)


class DeviceQuantity:
    """A Domain field with NDSL Quantity semantics: dims, units, and a host `view`
    (nsub, nk, nj, pitch) that is downloaded on first access after a stencil wrote the
    field and uploaded before the next stencil that reads it (every view access marks the
    host copy as the newer one)."""

    def __init__(self, factory, name, dims, units, nk):
        self.f, self.name, self.dims, self.units, self.nk = factory, name, tuple(dims), units, nk
        factory.domain.create(name, nk)
        self._host = None
        self._host_newer = False

    @property
    def view(self):
        if self._host is None:
            self._host = self.f.domain.download(self.name)
        self._host_newer = True
        return self._host

    @property
    def data(self):
        return self.view

    def compute(self):
        """compute-domain copy indexed [s, k, j, i] (staggered dims +1)"""
        d = self.f.domain
        sx = 1 if X_INTERFACE_DIM in self.dims else 0
        sy = 1 if Y_INTERFACE_DIM in self.dims else 0
        return self.view[..., NG:NG + d.ny + sy, NG:NG + d.nx + sx].copy()

    def _sync_to_device(self):
        if self._host_newer:
            self.f.domain.upload(self.name, self._host)
            self._host_newer = False

    def _device_written(self):
        self._host = None
        self._host_newer = False


class DeviceQuantityFactory:
    def __init__(self, sf: "CubedSphereStencilFactory"):
        self.sf = sf
        self._n = 0

    def zeros(self, dims, units, dtype=np.float64, nk=None):
        if dtype != np.float64:
            raise TypeError("device quantities are fp64")
        d = self.sf.domain
        if nk is None:
            nk = 1 if Z_DIM not in dims and Z_INTERFACE_DIM not in dims else \
                (d.npz + 1 if Z_INTERFACE_DIM in dims else d.npz)
        self._n += 1
        return DeviceQuantity(self.sf, f"_q{self._n}_{units.replace('/', '_')}", dims, units, nk)


class DeviceStencil:
    def __init__(self, sf, sdef, compute_dims):
        if not isinstance(sdef, StencilDef):
            raise TypeError("from_dims_halo: func must be a StencilDef of the HIP library")
        self.sf, self.sdef, self.compute_dims = sf, sdef, tuple(compute_dims)

    def __call__(self, *args, **params):
        sd = self.sdef
        if len(args) != sd.nargs:
            raise TypeError(f"{sd.name}: expected {sd.nargs} fields, got {len(args)}")
        names = []
        for a in args:
            if a is None:
                names.append("-")  # optional field (e.g. fv_tp_2d without mass fluxes)
                continue
            if not isinstance(a, DeviceQuantity):
                raise TypeError(f"{sd.name}: arguments are DeviceQuantity objects of this factory")
            a._sync_to_device()
            names.append(a.name)
        missing = [k for k in sd.params if k not in params]
        if missing:
            raise TypeError(f"{sd.name}: missing parameters {missing}")
        self.sf.domain.stencil(sd.name, names, [float(params[k]) for k in sd.params])
        for n in sd.outputs:
            if args[n] is not None:
                args[n]._device_written()


class CubedSphereStencilFactory:
    """All tiles of a cubed sphere on the current GPU; stencils run on every sub-domain."""

    def __init__(self, npx, npz, nq=1, layout=(1, 1)):
        self.domain = Domain(npx=npx, npz=npz, nq=nq, layout_x=layout[0], layout_y=layout[1])

    def from_dims_halo(self, func, compute_dims, compute_halos=()):
        return DeviceStencil(self, func, compute_dims)

    def close(self):
        self.domain.close()


def get_factories_cubed_sphere(npx: int, npz: int, nq: int = 1, layout=(1, 1)):
    """(stencil factory, quantity factory) for device-resident dycore stencils on all six
    tiles (sub-domain layout per tile), the NDSL surface of pyFV3's DynamicalCore pieces."""
    sf = CubedSphereStencilFactory(npx, npz, nq, layout)
    return sf, DeviceQuantityFactory(sf)


def orchestrate(obj=None, config=None):
    """ndsl.orchestrate: nothing to orchestrate, the kernels are compiled ahead of time."""
    return obj
