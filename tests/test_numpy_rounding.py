"""The rounding of numpy's small BLAS / LAPACK calls that the reference's values carry,
restated as the scalar formulas csrc/gtf_math.h and oracle/cpu_ref.cpp use.

numpy 2.2 calls OpenBLAS 0.3.29 for `dot` / `@` / `np.linalg.inv`; its x86-64 kernels
fuse multiply-adds in fixed orders. Each rule below is checked bit for bit against numpy
on random operands (fma from the C library through ctypes):

  x @ y (1-D, ddot)        s = x0*y0; s = fma(x1, y1, s); ...
  A @ x (gemv_n, 3x3)      s = A_i1*x1; s = fma(A_i0, x0, s); s = fma(A_i2, x2, s)
  x @ A (gemv_t)           s = x0*A_0j; s = fma(x1, A_1j, s); s = fma(x2, A_2j, s)
  A @ B, A @ B.T (3x3)     s = A_i0*B_0j; s = fma(A_i1, B_1j, s); s = fma(A_i2, B_2j, s)
  np.linalg.inv (2x2)      getf2 + trsm: l = q0 * (1/p0); u22 = q1 - l*p1;
                           x1 = y1 * (1/u22); x0 = fma(-x1, p1, y0) * (1/p0)

and the clustering functions built from them (clustering.py:11-105) equal the oracle's
(= the reference's numpy expressions) bit for bit. If numpy / OpenBLAS change on the
host, this test says so before the parity tests do.
"""
import ctypes
import itertools

import numpy as np
import pytest

import gtf_oracle as O

_libm = ctypes.CDLL("libm.so.6")
fma = _libm.fma
fma.restype = ctypes.c_double
fma.argtypes = [ctypes.c_double] * 3

N = 3000


def inv2(a, b, c, d):
    sw = abs(c) > abs(a)
    p0, p1 = (c, d) if sw else (a, b)
    q0, q1 = (a, b) if sw else (c, d)
    rp = 1.0 / p0
    l_ = q0 * rp
    u22 = q1 - l_ * p1
    ru = 1.0 / u22
    cols = []
    for e0, e1 in (((0.0, 1.0) if sw else (1.0, 0.0)), ((1.0, 0.0) if sw else (0.0, 1.0))):
        y1 = e1 - l_ * e0
        x1 = y1 * ru
        cols.append((fma(-x1, p1, e0) * rp, x1))
    return np.array([[cols[0][0], cols[1][0]], [cols[0][1], cols[1][1]]])


def inv3(m):
    r = np.zeros((3, 3))
    r[:2, :2] = inv2(m[0, 0], m[0, 1], m[1, 0], m[1, 1])
    r[2, 2] = 1.0 / m[2, 2]
    return r


def gemv_n(A, x):
    return np.array([fma(A[i, 2], x[2], fma(A[i, 0], x[0], A[i, 1] * x[1])) for i in range(3)])


def gemv_t(x, A):
    return np.array([fma(x[2], A[2, j], fma(x[1], A[1, j], x[0] * A[0, j])) for j in range(3)])


def ddot(x, y):
    s = x[0] * y[0]
    for i in range(1, len(x)):
        s = fma(x[i], y[i], s)
    return s


def gemm(A, B):
    C = np.zeros((3, 3))
    for i, j in itertools.product(range(3), range(3)):
        s = A[i, 0] * B[0, j]
        s = fma(A[i, 1], B[1, j], s)
        C[i, j] = fma(A[i, 2], B[2, j], s)
    return C


@pytest.fixture
def rng():
    return np.random.default_rng(20260)


def _cov(rng):
    A = rng.normal(size=(2, 2)) * 10 ** rng.uniform(-3, 1)
    C = np.zeros((3, 3))
    C[:2, :2] = A @ A.T + 1e-6 * np.eye(2)
    C[2, 2] = 10 ** rng.uniform(-4, 1)
    return C


def test_blas_kernels(rng):
    for _ in range(N):
        A = rng.normal(size=(3, 3)) * 10 ** rng.uniform(-3, 3, (3, 3))
        B = rng.normal(size=(3, 3)) * 10 ** rng.uniform(-3, 3, (3, 3))
        x = rng.normal(size=3) * 10 ** rng.uniform(-3, 3, 3)
        y = rng.normal(size=6) * 10 ** rng.uniform(-3, 3, 6)
        z = rng.normal(size=6)
        assert np.array_equal(A.dot(x), gemv_n(A, x))
        assert np.array_equal(x.dot(A), gemv_t(x, A))
        assert np.array_equal(A.dot(B), gemm(A, B))
        assert np.array_equal(A.dot(B.T), gemm(A, B.T))
        assert y.dot(z) == ddot(y, z)
        M = rng.normal(size=(2, 2)) * 10 ** rng.uniform(-4, 4)
        assert np.array_equal(np.linalg.inv(M), inv2(M[0, 0], M[0, 1], M[1, 0], M[1, 1]))


def test_clustering_functions(rng):
    for _ in range(N):
        c1, c2 = _cov(rng), _cov(rng)
        m1, m2 = rng.normal(size=3), rng.normal(size=3)
        assert np.array_equal(np.linalg.inv(c1), inv3(c1))
        # KLDistance (clustering.py:90-94)
        i1, i2 = inv3(c1), inv3(c2)
        d = (c1 - c2) * (i2 - i1)
        dm = m1 - m2
        assert (d[0, 0] + d[1, 1]) + d[2, 2] + ddot(gemv_t(dm, i1 + i2), dm) == O.KLDistance(m1, c1, m2, c2)
        # merge_states (clustering.py:97-105)
        mc = inv3(i1 + i2)
        mm = gemv_n(mc, gemv_n(i1, m1) + gemv_n(i2, m2))
        rm, rc = O.merge_states(m1, c1, m2, c2)
        assert np.array_equal(mm, rm) and np.array_equal(mc, rc)
        # mahalanobis_distance (clustering.py:11-78)
        na, nb, nc = (np.array([rng.normal() * 600, 0.0, rng.normal() * 500, rng.uniform(30, 1000)]) for _ in range(3))
        r = m1[:2] - m2[:2]
        I = inv2(c1[0, 0] + c2[0, 0], c1[0, 1] + c2[0, 1], c1[1, 0] + c2[1, 0], c1[1, 1] + c2[1, 1])
        t = (fma(r[1], I[1, 0], r[0] * I[0, 0]), fma(r[1], I[1, 1], r[0] * I[0, 1]))
        d1 = fma(t[1], r[1], t[0] * r[0])
        (za, ra), (zb, rb), (zc, rc_) = (na[2], na[3]), (nb[2], nb[3]), (nc[2], nc[3])
        j2, j3 = 1 / (rb - ra), -1 / (rc_ - ra)
        j5, j6 = -(zb - za) / (rb - ra) ** 2, (zc - za) / (rc_ - ra) ** 2
        J = [-j3 - j2, j2, j3, -j5 - j6, j5, j6]
        sz = [0.4 if abs(n[0]) >= 550.0 else 0.6 for n in (na, nb, nc)]
        sr = [0.6 if abs(n[0]) >= 550.0 else 0.4 for n in (na, nb, nc)]
        s = [q * q for q in sz + sr]
        cdt = ddot([J[i] * s[i] for i in range(6)], J)
        res = (zb - za) / (rb - ra) - (zc - za) / (rc_ - ra)
        got = d1 + res ** 2 * (1 / cdt)
        assert got == O.mahalanobis_distance(m1, c1, m2, c2, na, nb, nc, 0.4, 0.6, 550.0)


def qdiv(x, d, r):
    """csrc/gtf_math.h qdiv: x / d from r = 1.0 / d"""
    q = x * r
    m = abs(q)
    if 2.0 ** -960 <= m <= 2.0 ** 1000:
        return fma(fma(-q, d, x), r, q)
    return x / d if d != 0 else (np.float64(x) / np.float64(d))


def test_shared_reciprocal_division_is_exact(rng):
    """Markstein: with r = RN(1/d), RN(q + (x - d q) r) for q = RN(x r) is RN(x / d)"""
    xs = list(rng.normal(size=40000) * 10.0 ** rng.uniform(-40, 40, 40000))
    ds = list(rng.normal(size=40000) * 10.0 ** rng.uniform(-40, 40, 40000))
    # significands near 1 and near 2 (the hard cases of reciprocal-based division)
    m1 = 1 + rng.integers(0, 2 ** 52, 20000) / 2.0 ** 52
    m2 = 2 - rng.integers(1, 2 ** 20, 20000) / 2.0 ** 52
    e = rng.integers(-60, 60, (2, 20000))
    xs += list(np.ldexp(m1, e[0])) + list(np.ldexp(m2, e[0]))
    ds += list(np.ldexp(m2, e[1])) + list(np.ldexp(m1, e[1]))
    with np.errstate(all="ignore"):
        for x, d in zip(xs, ds):
            x, d = float(x), float(d)
            assert qdiv(x, d, 1.0 / d) == x / d
        for x, d in ((0.0, 3.0), (-0.0, 3.0), (1.0, 1e308), (1e-300, 1e10), (5e-324, 3.0), (1e308, 1e-10),
                     (2.0, float("inf")), (float("inf"), 2.0), (float("nan"), 2.0)):
            ref = np.float64(x) / np.float64(d)
            got = qdiv(x, d, float(np.float64(1.0) / np.float64(d)))
            assert got == ref or (np.isnan(got) and np.isnan(ref)), (x, d)
