"""CPU model of csrc/blockscan.hpp's partitioned Thomas solve (tri_solve), lane for lane:
NB blocks of M rows, DPP hand-overs as shifts over the block axis, Kogge-Stone scans of the
affine maps and of the Möbius pivot maps.  Against a sequential sweep in extended precision:

  * pp-type systems (strongly diagonally dominant, d ~ 2(1 + g), a = 1, c = g): the Möbius
    pivots are as accurate as the sequential sweep;
  * w-type systems (a scaled discrete Laplacian plus small layer masses): the Möbius pivots
    lose digits to cancellation between normalised block products (their matrices are a Jordan
    block), the serial pivots do not -- which is why riem_scan_k solves the w system with serial
    pivots and affine scans.
"""
import numpy as np
import pytest


def prev(v):
    o = np.zeros_like(v)
    o[1:] = v[:-1]
    return o


def nxt(v):
    o = np.zeros_like(v)
    o[:-1] = v[1:]
    return o


def _ks(v, nb, dn, comb):
    s, b = 1, np.arange(nb)
    while s < nb:
        if dn:
            o = tuple(np.concatenate([np.full(s, np.nan), x[:-s]]) for x in v)
            on = b >= s
        else:
            o = tuple(np.concatenate([x[s:], np.full(s, np.nan)]) for x in v)
            on = b + s < nb
        f = comb(v, o)
        v = tuple(np.where(on, fi, vi) for fi, vi in zip(f, v))
        s *= 2
    return v


def scan_aff(A, B, nb, dn):
    return _ks((A, B), nb, dn, lambda f, g: (f[0] * g[0], f[0] * g[1] + f[1]))


def _norm(t):
    sc = 1.0 / sum(np.abs(x) for x in t)
    return tuple(x * sc for x in t)


def scan_mob(t, nb):
    return _ks(t, nb, True, lambda f, g: _norm((f[0] * g[0] + f[1] * g[2], f[0] * g[1] + f[1] * g[3],
                                                f[2] * g[0] + f[3] * g[2], f[2] * g[1] + f[3] * g[3])))


def tri_solve(a, d, c, r, M, NB, mobius):
    """a, d, c, r: (NB, M) rows of one column"""
    b = np.arange(NB)
    last = b == NB - 1
    cprev = np.where(b == 0, 0.0, prev(c[:, M - 1]))
    c_up = lambda m: c[:, m - 1] if m > 0 else cprev
    gam, rbs = np.zeros((NB, M)), np.zeros((NB, M))

    def eliminate(rb, mask):
        for m in range(M):
            gm = c_up(m) * rb
            rb = 1.0 / (d[:, m] - a[:, m] * gm)
            gam[mask, m], rbs[mask, m] = gm[mask], rb[mask]
        return rb

    if mobius:
        T = (np.ones(NB), np.zeros(NB), np.zeros(NB), np.ones(NB))
        for m in range(M):
            e = a[:, m] * c_up(m)
            T = (d[:, m] * T[0] - e * T[2], d[:, m] * T[1] - e * T[3], T[0], T[1])
        T = scan_mob(_norm(T), NB)
        pu, pv = prev(T[0]), prev(T[2])
        eliminate(np.where(b == 0, 0.0, pv / np.where(b == 0, 1.0, pu)), np.ones(NB, bool))
    else:
        rb_in = np.zeros(NB)
        for rr in range(NB):
            eliminate(rb_in, b == rr)
            rb_in = np.where(b == rr + 1, prev(rbs[:, M - 1]), rb_in)
    yh, A = np.zeros(NB), np.ones(NB)
    for m in range(M):
        yh = (r[:, m] - a[:, m] * yh) * rbs[:, m]
        A = -a[:, m] * A * rbs[:, m]
    gnb = nxt(gam[:, 0])
    gnext = lambda m: gam[:, m + 1] if m + 1 < M else np.where(last, 0.0, gnb)
    Bc = np.ones(NB)
    for m in range(M - 1, -1, -1):
        Bc = -gnext(m) * Bc
    F = scan_aff(A, yh, NB, True)
    y = np.where(b == 0, 0.0, prev(F[1]))
    x = np.zeros((NB, M))
    for m in range(M):
        y = (r[:, m] - a[:, m] * y) * rbs[:, m]
        x[:, m] = y
    xh = np.zeros(NB)
    for m in range(M - 1, -1, -1):
        xh = x[:, m] - gnext(m) * xh
    H = scan_aff(Bc, xh, NB, False)
    xi = np.where(last, 0.0, nxt(H[1]))
    for m in range(M - 1, -1, -1):
        xi = x[:, m] - gnext(m) * xi
        x[:, m] = xi
    return x.ravel()


def thomas(a, d, c, r, dt=np.float64):
    a, d, c, r = (np.asarray(v, dtype=dt) for v in (a, d, c, r))
    n = len(d)
    gam, y = np.zeros(n, dt), np.zeros(n, dt)
    bet = d[0]
    y[0] = r[0] / bet
    for k in range(1, n):
        gam[k] = c[k - 1] / bet
        bet = d[k] - a[k] * gam[k]
        y[k] = (r[k] - a[k] * y[k - 1]) / bet
    x = y.copy()
    for k in range(n - 2, -1, -1):
        x[k] = y[k] - gam[k + 1] * x[k + 1]
    return x


def system(kind, r, n=72):
    dm = 100.0 + 900.0 * r.random(n)
    if kind == "pp":
        g = np.append(dm[:-1] / dm[1:], 0.0)
        a, d, c = np.ones(n), 2.0 * (1.0 + g), g
        d[-1] = 2.0
        rhs = 3e3 * r.standard_normal(n)
    else:
        dz = -(50.0 + 500.0 * r.random(n))
        pem = 1e5 * np.linspace(1e-5, 1.0, n + 1)
        aa = np.zeros(n + 1)
        aa[1:n] = 5.7e5 / (dz[:-1] + dz[1:]) * pem[1:n]
        p1 = 5.7e5 / dz[-1] * pem[n]
        a, c = aa[:n].copy(), np.append(aa[1:n], 0.0)
        d = dm - aa[:n] - np.append(aa[1:n], p1)
        rhs = dm * r.standard_normal(n) + 1e3 * r.standard_normal(n)
    a[0] = 0.0
    return a, d, c, rhs


@pytest.mark.parametrize("kind,mobius,bar", [("pp", True, 1e-14), ("w", False, 2e-13)])
def test_tri_solve_model_matches_sequential(kind, mobius, bar):
    r = np.random.default_rng(3)
    for _ in range(20):
        a, d, c, rhs = system(kind, r)
        want = thomas(a, d, c, rhs, np.longdouble).astype(np.float64)
        x = tri_solve(*(v.reshape(8, 9) for v in (a, d, c, rhs)), 9, 8, mobius)
        seq = thomas(a, d, c, rhs)
        sc = np.abs(want).mean()
        assert np.abs(x - want).max() / sc <= max(bar, 10 * np.abs(seq - want).max() / sc)


def test_mobius_pivots_lose_digits_on_the_w_system():
    """the reason for the serial pivots: on w-type systems the Möbius block products cancel"""
    r = np.random.default_rng(4)
    worst_mob = worst_ser = 0.0
    for _ in range(20):
        a, d, c, rhs = system("w", r)
        want = thomas(a, d, c, rhs, np.longdouble).astype(np.float64)
        sc = np.abs(want).mean()
        rows = [v.reshape(8, 9) for v in (a, d, c, rhs)]
        worst_mob = max(worst_mob, np.abs(tri_solve(*rows, 9, 8, True) - want).max() / sc)
        worst_ser = max(worst_ser, np.abs(tri_solve(*rows, 9, 8, False) - want).max() / sc)
    assert worst_ser < 2e-13 and worst_mob > 5 * worst_ser
