"""Per-call netlib BLAS layer (libcyclone_blas.so).

CPU: the library exports every symbol include/cyclone_blas.h declares, the
Python signatures cover the header, and argument errors follow XERBLA's
numbering (checked before any device work).  GPU: the known answers of
mllib-local/src/test/scala/org/apache/spark/ml/linalg/BLASSuite.scala
(scal :61, axpy :73, dot :105, spr :135, syr :160, gemm :209, gemv :305,
spmv :432) and random operands against numpy (fp64, 1e-12 relative -- MFMA
summation order differs from netlib's loop order)."""
import subprocess

import numpy as np
import pytest

from cycloneml_amd import _native as N
from cycloneml_amd import blas


def test_blas_exports_every_declared_symbol():
    lib = blas.load()
    syms = blas.header_symbols()
    assert len(syms) == 21
    assert set(syms) == set(blas.SIGNATURES)
    nm = subprocess.run(["nm", "-D", "--defined-only", blas.LIB_PATH], capture_output=True,
                        text=True, check=True).stdout
    exported = {line.split()[-1] for line in nm.splitlines() if line.strip()}
    assert set(syms) <= exported
    assert all(hasattr(lib, s) for s in syms)


@pytest.mark.parametrize("call,info", [
    (lambda: blas.nativeBLAS.dgemm("X", "N", 1, 1, 1, 1.0, np.ones(1), 1, np.ones(1), 1, 0.0,
                                   np.ones(1), 1), 1),
    (lambda: blas.nativeBLAS.dgemm("N", "Q", 1, 1, 1, 1.0, np.ones(1), 1, np.ones(1), 1, 0.0,
                                   np.ones(1), 1), 2),
    (lambda: blas.nativeBLAS.dgemm("N", "N", -1, 1, 1, 1.0, np.ones(1), 1, np.ones(1), 1, 0.0,
                                   np.ones(1), 1), 3),
    (lambda: blas.nativeBLAS.dgemm("N", "N", 2, 1, 1, 1.0, np.ones(2), 1, np.ones(1), 1, 0.0,
                                   np.ones(2), 2), 8),
    (lambda: blas.nativeBLAS.dgemm("T", "N", 2, 1, 3, 1.0, np.ones(6), 2, np.ones(3), 3, 0.0,
                                   np.ones(2), 2), 8),
    (lambda: blas.nativeBLAS.dgemm("N", "N", 2, 2, 3, 1.0, np.ones(6), 2, np.ones(6), 2, 0.0,
                                   np.ones(4), 2), 10),
    (lambda: blas.nativeBLAS.dgemm("N", "N", 2, 1, 1, 1.0, np.ones(2), 2, np.ones(1), 1, 0.0,
                                   np.ones(2), 1), 13),
    (lambda: blas.nativeBLAS.dgemv("Z", 1, 1, 1.0, np.ones(1), 1, np.ones(1), 1, 0.0,
                                   np.ones(1), 1), 1),
    (lambda: blas.nativeBLAS.dgemv("N", 3, 1, 1.0, np.ones(3), 2, np.ones(1), 1, 0.0,
                                   np.ones(3), 1), 6),
    (lambda: blas.nativeBLAS.dgemv("N", 1, 1, 1.0, np.ones(1), 1, np.ones(1), 0, 0.0,
                                   np.ones(1), 1), 8),
    (lambda: blas.nativeBLAS.dgemv("N", 1, 1, 1.0, np.ones(1), 1, np.ones(1), 1, 0.0,
                                   np.ones(1), 0), 11),
    (lambda: blas.nativeBLAS.dspr("A", 1, 1.0, np.ones(1), 1, np.ones(1)), 1),
    (lambda: blas.nativeBLAS.dspr("U", -2, 1.0, np.ones(1), 1, np.ones(1)), 2),
    (lambda: blas.nativeBLAS.dspr("U", 1, 1.0, np.ones(1), 0, np.ones(1)), 5),
    (lambda: blas.nativeBLAS.dsyr("U", 3, 1.0, np.ones(3), 1, np.ones(9), 2), 7),
    (lambda: blas.nativeBLAS.dger(-1, 1, 1.0, np.ones(1), 1, np.ones(1), 1, np.ones(1), 1), 1),
    (lambda: blas.nativeBLAS.dger(1, 1, 1.0, np.ones(1), 1, np.ones(1), 0, np.ones(1), 1), 7),
    (lambda: blas.nativeBLAS.dger(3, 1, 1.0, np.ones(3), 1, np.ones(1), 1, np.ones(3), 2), 9),
    (lambda: blas.nativeBLAS.dspmv("U", 1, 1.0, np.ones(1), np.ones(1), 1, 0.0, np.ones(1), 0),
     9),
])
def test_xerbla_numbering(call, info):
    with pytest.raises(N.IllegalArgumentException, match=f"parameter number {info} had"):
        call()


def test_require_messages():
    with pytest.raises(N.IllegalArgumentException, match="columns of A don't match the rows"):
        blas.gemm(1.0, np.ones((2, 3), order="F"), np.ones((2, 2), order="F"), 0.0,
                  np.ones((2, 2), order="F"))
    with pytest.raises(N.IllegalArgumentException, match="C.isTransposed must be false"):
        blas.gemm(1.0, np.ones((2, 2), order="F"), np.ones((2, 3), order="F"), 0.0,
                  np.ones((2, 3)))
    with pytest.raises(N.IllegalArgumentException, match="not a square matrix"):
        blas.syr(0.1, np.ones(3), np.ones((3, 4), order="F"))
    with pytest.raises(N.IllegalArgumentException, match="doesn't match the rank of A"):
        blas.syr(0.1, np.ones(4), np.ones((3, 3), order="F"))


# ---------------------------------------------------------------- GPU


def _F(rows, cols, vals):
    """DenseMatrix(rows, cols, values) -- column-major."""
    return np.array(vals, dtype=np.float64).reshape(cols, rows).T.copy(order="F")


@pytest.mark.gpu
def test_gemm_known_answers(cuda):
    dA = _F(4, 3, [0.0, 1.0, 0.0, 0.0, 2.0, 0.0, 1.0, 0.0, 0.0, 0.0, 0.0, 3.0])
    dA2 = np.array([0.0, 2.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 3.0]).reshape(4, 3)
    B = _F(3, 2, [1.0, 0.0, 0.0, 0.0, 2.0, 1.0])
    expected = _F(4, 2, [0.0, 1.0, 0.0, 0.0, 4.0, 0.0, 2.0, 3.0])
    C1 = _F(4, 2, [1.0, 0.0, 2.0, 1.0, 0.0, 0.0, 1.0, 0.0])
    expected2 = _F(4, 2, [2.0, 1.0, 4.0, 2.0, 4.0, 0.0, 4.0, 3.0])
    expected3 = _F(4, 2, [2.0, 2.0, 4.0, 2.0, 8.0, 0.0, 6.0, 6.0])
    expected4 = _F(4, 2, [5.0, 0.0, 10.0, 5.0, 0.0, 0.0, 5.0, 0.0])
    for A in (dA, dA2):  # dA2: the transposed (row-major) DenseMatrix of BLASSuite:232
        C = np.zeros((4, 2), order="F")
        np.testing.assert_array_equal(blas.gemm(1.0, A, B, 0.0, C), expected)
        np.testing.assert_array_equal(blas.gemm(1.0, A, B, 2.0, C1.copy(order="F")), expected2)
        np.testing.assert_array_equal(blas.gemm(2.0, A, B, 2.0, C1.copy(order="F")), expected3)
        np.testing.assert_array_equal(blas.gemm(0.0, A, B, 5.0, C1.copy(order="F")), expected4)
        np.testing.assert_array_equal(blas.gemm(0.0, A, B, 1.0, C1.copy(order="F")), C1)
    # B transposed as well
    Bt = np.ascontiguousarray(B)
    np.testing.assert_array_equal(blas.gemm(1.0, dA2, Bt, 2.0, C1.copy(order="F")), expected2)


@pytest.mark.gpu
def test_gemv_known_answers(cuda):
    dA = _F(4, 3, [0.0, 1.0, 0.0, 0.0, 2.0, 0.0, 1.0, 0.0, 0.0, 0.0, 0.0, 3.0])
    dA2 = np.array([0.0, 2.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 3.0]).reshape(4, 3)
    dx = np.array([1.0, 2.0, 3.0])
    y1 = np.array([1.0, 3.0, 1.0, 0.0])
    for A in (dA, dA2):
        np.testing.assert_array_equal(blas.gemv(1.0, A, dx, 0.0, np.zeros(4)), [4.0, 1.0, 2.0, 9.0])
        np.testing.assert_array_equal(blas.gemv(1.0, A, dx, 2.0, y1.copy()), [6.0, 7.0, 4.0, 9.0])
        np.testing.assert_array_equal(blas.gemv(2.0, A, dx, 2.0, y1.copy()),
                                      [10.0, 8.0, 6.0, 18.0])


@pytest.mark.gpu
def test_spr_syr_spmv_known_answers(cuda):
    U = np.array([1.0, 2, 2, 3, 3, 3, 4, 4, 4, 4])
    blas.spr(0.1, np.array([1.0, 2, 2.1, 4]), U)
    np.testing.assert_allclose(U, [1.1, 2.2, 2.4, 3.21, 3.42, 3.441, 4.4, 4.8, 4.84, 5.6],
                               rtol=0, atol=1e-9)
    dA = _F(4, 4, [0.0, 1.2, 2.2, 3.1, 1.2, 3.2, 5.3, 4.6, 2.2, 5.3, 1.8, 3.0, 3.1, 4.6, 3.0, 0.8])
    blas.syr(0.15, np.array([0.0, 2.7, 3.5, 2.1]), dA)
    np.testing.assert_allclose(dA, _F(4, 4, [0.0, 1.2, 2.2, 3.1, 1.2, 4.2935, 6.7175, 5.4505, 2.2,
                                             6.7175, 3.6375, 4.1025, 3.1, 5.4505, 4.1025, 1.4615]),
                               rtol=0, atol=1e-15)
    A = np.array([3.0, -2.0, -8.0, 2.0, 4.0, -3.0, -4.0, 7.0, -3.0, 0.0])
    x = np.array([5.0, 2.0, -1.0, -9.0])
    y0 = np.array([-3.0, 6.0, -8.0, -3.0])
    cases = [(1.0, 1.0, [42.0, -87.0, 40.0, -6.0]), (0.5, 1.0, [19.5, -40.5, 16.0, -4.5]),
             (-0.5, 1.0, [-25.5, 52.5, -32.0, -1.5]), (0.0, 1.0, [-3.0, 6.0, -8.0, -3.0]),
             (1.0, 0.5, [43.5, -90.0, 44.0, -4.5]), (1.0, -0.5, [46.5, -96.0, 52.0, -1.5]),
             (1.0, 0.0, [45.0, -93.0, 48.0, -3.0])]
    for alpha, beta, exp in cases:
        np.testing.assert_allclose(blas.dspmv(4, alpha, A, x, beta, y0.copy()), exp, rtol=0,
                                   atol=1e-8)


@pytest.mark.gpu
def test_level1_known_answers(cuda):
    dx = np.array([1.0, 0.0, -2.0])
    assert blas.dot(dx, np.array([2.0, 1.0, 0.0])) == 2.0
    assert blas.dot(dx, dx) == 5.0
    np.testing.assert_array_equal(blas.scal(0.1, dx.copy()), np.array([0.1, 0.0, -0.2]))
    np.testing.assert_array_equal(blas.axpy(2.0, dx, np.array([2.0, 1.0, 0.0])), [4.0, 1.0, -4.0])
    y = np.zeros(3)
    blas.nativeBLAS.dcopy(3, dx, 1, y, 1)
    np.testing.assert_array_equal(y, dx)
    assert blas.nativeBLAS.dnrm2(3, dx, 1) == np.sqrt(5.0)


@pytest.mark.gpu
@pytest.mark.parametrize("ta,tb", [("N", "N"), ("T", "N"), ("N", "T"), ("T", "T")])
@pytest.mark.parametrize("m,n,k", [(1, 1, 1), (65, 33, 17), (130, 200, 257), (64, 64, 64)])
def test_dgemm_random(cuda, ta, tb, m, n, k):
    rng = np.random.default_rng(m * 7 + n * 3 + k)
    lda, ldb, ldc = (m if ta == "N" else k) + 3, (k if tb == "N" else n) + 1, m + 2
    A = rng.normal(size=(lda, k if ta == "N" else m))
    B = rng.normal(size=(ldb, n if tb == "N" else k))
    C = rng.normal(size=(ldc, n))
    opA = A[:m, :k] if ta == "N" else A[:k, :m].T
    opB = B[:k, :n] if tb == "N" else B[:n, :k].T
    alpha, beta = 1.5, -0.5
    exp = C.copy()
    exp[:m] = alpha * (opA @ opB) + beta * C[:m]
    flatC = C.ravel(order="F").copy()
    blas.nativeBLAS.dgemm(ta, tb, m, n, k, alpha, A.ravel(order="F").copy(), lda,
                          B.ravel(order="F").copy(), ldb, beta, flatC, ldc)
    got = flatC.reshape(n, ldc).T
    np.testing.assert_allclose(got, exp, rtol=1e-12, atol=1e-12 * np.abs(exp).max())
    np.testing.assert_array_equal(got[m:], C[m:])  # rows beyond m untouched


@pytest.mark.gpu
@pytest.mark.parametrize("layout", [101, 102])
def test_cblas_dgemm_layouts(cuda, layout):
    rng = np.random.default_rng(layout)
    m, n, k = 37, 21, 50
    A, B, C = rng.normal(size=(m, k)), rng.normal(size=(k, n)), rng.normal(size=(m, n))
    order = "C" if layout == 101 else "F"
    a, b, c = (M.copy(order=order) for M in (A, B, C))
    lda, ldb, ldc = (k, n, n) if order == "C" else (m, k, m)
    blas.load().cblas_dgemm(layout, 111, 111, m, n, k, 2.0, a.ctypes.data, lda, b.ctypes.data,
                            ldb, 0.5, c.ctypes.data, ldc)
    np.testing.assert_allclose(c, 2.0 * A @ B + 0.5 * C, rtol=1e-12, atol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("trans", ["N", "T"])
@pytest.mark.parametrize("incx,incy", [(1, 1), (2, -1), (-3, 2)])
def test_dgemv_strides(cuda, trans, incx, incy):
    rng = np.random.default_rng(abs(incx) * 10 + abs(incy))
    m, n, lda = 300, 129, 305
    A = rng.normal(size=(lda, n))
    lx, ly = (n, m) if trans == "N" else (m, n)
    x = rng.normal(size=1 + (lx - 1) * abs(incx))
    y = rng.normal(size=1 + (ly - 1) * abs(incy))
    # BLAS stride rule: logical element i sits at start + i*inc, start = 0 or
    # (1-len)*inc for inc < 0 -- exactly numpy's x[::inc] on these sizes
    opA = A[:m] if trans == "N" else A[:m].T
    exp = 0.7 * (opA @ x[::incx]) - 1.25 * y[::incy]
    blas.nativeBLAS.dgemv(trans, m, n, 0.7, A.ravel(order="F").copy(), lda, x, incx, -1.25, y,
                          incy)
    got = y[::incy]
    np.testing.assert_allclose(got, exp, rtol=1e-12, atol=1e-12 * np.abs(exp).max())


@pytest.mark.gpu
@pytest.mark.parametrize("uplo", ["U", "L"])
def test_dspr_dsyr_dger_random(cuda, uplo):
    rng = np.random.default_rng(3)
    n = 333
    x = rng.normal(size=n)
    full = rng.normal(size=(n, n))
    full = full + full.T
    tri = np.triu_indices(n) if uplo == "U" else np.tril_indices(n)
    # column-major packed order: sort by (col, row)
    order = np.lexsort((tri[0], tri[1]))
    rows, cols = tri[0][order], tri[1][order]
    ap = full[rows, cols].copy()
    blas.nativeBLAS.dspr(uplo, n, 0.3, x, 1, ap)
    exp = full + 0.3 * np.outer(x, x)
    np.testing.assert_allclose(ap, exp[rows, cols], rtol=1e-13, atol=1e-13)
    a = np.asfortranarray(full).ravel(order="F").copy()
    blas.nativeBLAS.dsyr(uplo, n, 0.3, x, 1, a, n)
    a = a.reshape(n, n).T
    mask = np.zeros((n, n), bool)
    mask[tri] = True
    np.testing.assert_allclose(a[mask], exp[mask], rtol=1e-13, atol=1e-13)
    np.testing.assert_array_equal(a[~mask], full[~mask])
    m = 101
    y = rng.normal(size=n)
    g = rng.normal(size=(m, n))
    flat = np.asfortranarray(g).ravel(order="F").copy()
    blas.nativeBLAS.dger(m, n, -2.0, x[:m], 1, y, 1, flat, m)
    np.testing.assert_allclose(flat.reshape(n, m).T, g - 2.0 * np.outer(x[:m], y), rtol=1e-13,
                               atol=1e-13)


@pytest.mark.gpu
def test_level1_random(cuda):
    rng = np.random.default_rng(4)
    n = 100_003
    x, y = rng.normal(size=n), rng.normal(size=n)
    assert abs(blas.nativeBLAS.ddot(n, x, 1, y, 1) - x @ y) <= 1e-10 * np.abs(x * y).sum()
    assert abs(blas.nativeBLAS.dnrm2(n, x, 1) - np.linalg.norm(x)) <= 1e-12 * np.linalg.norm(x)
    yy = y.copy()
    blas.nativeBLAS.daxpy(n, 0.25, x, 1, yy, 1)
    np.testing.assert_array_equal(yy, y + 0.25 * x)
    xx = x.copy()
    blas.nativeBLAS.dscal(n // 2, 3.0, xx, 2)
    exp = x.copy()
    exp[0:2 * (n // 2):2] *= 3.0
    np.testing.assert_array_equal(xx, exp)
    assert blas.nativeBLAS.ddot(0, x, 1, y, 1) == 0.0
