"""Oracle for the K-column primitives (csrc/column.hip) — TEST INFRASTRUCTURE ONLY.

Pure-Python restatements of the reference's DSL pattern known-answer programs,
arrays indexed [i, j, k] like the NDSL numpy views they use:
  column_top       dsl_patterns/Do__get_top_of_the_column.py:33-38
                   (FORWARD interval(-1, None) into a 2-D temporary, PARALLEL broadcast)
  column_while_lt  dsl_patterns/Do__while_in_gt_functions.py:23-32
                   (`while field[0, 0, lev] < 4: lev += 1`, K-relative offset per level;
                   bounded at the last level, where the GT4Py program would read past it)
  column_gather_k  dsl_patterns/WIP__hybrid_index_2dout.py:34-42
                   (FORWARD: if k_mask == k_index_desired: out2d = data)
Pinned by the reference programs' own asserts (tests/test_column_kat.py).
"""
import numpy as np


def column_top(a):
    nx, ny, nz = a.shape
    tmp = np.zeros((nx, ny))
    for k in range(nz - 1, nz):          # interval(-1, None)
        tmp[:, :] = a[:, :, k]
    out = np.empty_like(a)
    for k in range(nz):                  # PARALLEL interval(...)
        out[:, :, k] = tmp
    return out


def column_while_lt(a, thr):
    nx, ny, nz = a.shape
    out = np.zeros_like(a)
    for i in range(nx):
        for j in range(ny):
            for k in range(nz):
                lev = 0
                while k + lev < nz - 1 and a[i, j, k + lev] < thr:
                    lev += 1
                out[i, j, k] = lev
    return out


def column_gather_k(data, kmask, kidx, out2d):
    out = np.array(out2d, dtype=np.float64, copy=True)
    nx, ny, nz = data.shape
    for k in range(nz):                  # FORWARD interval(...)
        hit = kmask[:, :, k] == kidx
        out[hit] = data[:, :, k][hit]
    return out
