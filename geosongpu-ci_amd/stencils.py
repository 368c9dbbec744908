"""NDSL-style stencil surface backed by the HIP library.

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


def orchestrate(obj=None, config=None):
    """ndsl.orchestrate: nothing to orchestrate, the kernels are compiled ahead of time."""
    return obj
