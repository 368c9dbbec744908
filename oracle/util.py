"""Oracle helpers: NaN-padded shifts and region masks in the HBM plane layout
(TEST INFRASTRUCTURE ONLY).  A NaN leaking into a compared region flags a stencil
that reads outside the allocated halo."""
import numpy as np

from . import NG


def sh(a, di=0, dj=0):
    """b[..., j, i] = a[..., j+dj, i+di]; NaN where the source is outside the plane."""
    out = np.full_like(a, np.nan)
    nj, ni = a.shape[-2:]
    j0, j1 = max(0, -dj), min(nj, nj - dj)
    i0, i1 = max(0, -di), min(ni, ni - di)
    if j1 > j0 and i1 > i0:
        out[..., j0:j1, i0:i1] = a[..., j0 + dj:j1 + dj, i0 + di:i1 + di]
    return out


class Plane:
    """Index helper for one sub-domain plane (nj, pitch)."""

    def __init__(self, sub, nx, ny, nj, pitch):
        self.io, self.jo, self.N = sub["ioff"], sub["joff"], sub["N"]
        self.nx, self.ny, self.nj, self.pitch = nx, ny, nj, pitch
        self.li = (np.arange(pitch) - NG)[None, :]
        self.lj = (np.arange(nj) - NG)[:, None]
        self.I = self.li + self.io
        self.J = self.lj + self.jo

    def reg(self, i0, i1, j0, j1):
        """local inclusive ranges"""
        return (self.li >= i0) & (self.li <= i1) & (self.lj >= j0) & (self.lj <= j1)

    def greg(self, I0, I1, J0, J1):
        """global inclusive ranges"""
        return (self.I >= I0) & (self.I <= I1) & (self.J >= J0) & (self.J <= J1)

    def at(self, I, J):
        """mask of the single global point (I, J) (empty if not in the plane)"""
        return (self.I == I) & (self.J == J)

    def owns(self, I, J):
        """True if global corner point (I, J) is inside this sub's compute corner range"""
        return self.io <= I <= self.io + self.nx and self.jo <= J <= self.jo + self.ny

    def slot(self, I, J):
        """(j, i) array slot of global point (I, J)"""
        return J - self.jo + NG, I - self.io + NG


def where(mask, new, old):
    return np.where(mask, new, old)
