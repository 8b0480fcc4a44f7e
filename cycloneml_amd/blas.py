"""Python mirror of the per-call BLAS layer (libcyclone_blas.so).

Two surfaces, both over the netlib Fortran ABI the library exports:

* ``NativeBLAS`` -- the ``dev.ludovic.netlib.blas.BLAS`` methods the
  reference calls through ``BLAS.nativeBLAS`` / ``BLAS.getBLAS(n)``
  (mllib-local/src/main/scala/org/apache/spark/ml/linalg/BLAS.scala:42-55):
  dgemm, dgemv, dspr, dsyr, dger, dspmv, ddot, daxpy, dscal, dcopy, dnrm2,
  with netlib's argument order (column-major numpy buffers, leading
  dimensions, increments).
* module functions with the ``ml.linalg.BLAS`` object's semantics for dense
  operands: ``gemm`` (BLAS.scala:374-425), ``gemv`` (BLAS.scala:540-632),
  ``spr`` (BLAS.scala:277-285), ``syr`` (BLAS.scala:323-346), ``dspmv``
  (BLAS.scala:264-273), ``dot``,
  ``axpy``, ``scal``.

Every call copies its host operands to the device, runs a gfx950 kernel and
copies the result back (netlib's synchronous host-pointer contract); it is
the drop-in layer, not the hot path.  Invalid arguments raise
IllegalArgumentException with XERBLA's message; there is no CPU fallback.
"""
import ctypes
import os
import re
import threading

import numpy as np

from . import _native

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.environ.get("CYC_LIB_DIR") or _HERE, "libcyclone_blas.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "cyclone_blas.h")

_P = ctypes.c_void_p
_C = ctypes.c_char_p
_I = ctypes.c_int
_D = ctypes.c_double
_PI = ctypes.POINTER(ctypes.c_int)
_PD = ctypes.POINTER(ctypes.c_double)

SIGNATURES = {
    "dgemm_": (None, [_C, _C, _PI, _PI, _PI, _PD, _P, _PI, _P, _PI, _PD, _P, _PI]),
    "dgemv_": (None, [_C, _PI, _PI, _PD, _P, _PI, _P, _PI, _PD, _P, _PI]),
    "dspr_": (None, [_C, _PI, _PD, _P, _PI, _P]),
    "dsyr_": (None, [_C, _PI, _PD, _P, _PI, _P, _PI]),
    "dger_": (None, [_PI, _PI, _PD, _P, _PI, _P, _PI, _P, _PI]),
    "dspmv_": (None, [_C, _PI, _PD, _P, _P, _PI, _PD, _P, _PI]),
    "ddot_": (_D, [_PI, _P, _PI, _P, _PI]),
    "daxpy_": (None, [_PI, _PD, _P, _PI, _P, _PI]),
    "dscal_": (None, [_PI, _PD, _P, _PI]),
    "dcopy_": (None, [_PI, _P, _PI, _P, _PI]),
    "dnrm2_": (_D, [_PI, _P, _PI]),
    "cblas_dgemm": (None, [_I, _I, _I, _I, _I, _I, _D, _P, _I, _P, _I, _D, _P, _I]),
    "cblas_dgemv": (None, [_I, _I, _I, _I, _D, _P, _I, _P, _I, _D, _P, _I]),
    "cblas_dspr": (None, [_I, _I, _I, _D, _P, _I, _P]),
    "cblas_dsyr": (None, [_I, _I, _I, _D, _P, _I, _P, _I]),
    "cblas_dger": (None, [_I, _I, _I, _D, _P, _I, _P, _I, _P, _I]),
    "cblas_ddot": (_D, [_I, _P, _I, _P, _I]),
    "cblas_daxpy": (None, [_I, _D, _P, _I, _P, _I]),
    "cblas_dscal": (None, [_I, _D, _P, _I]),
    "cblas_dcopy": (None, [_I, _P, _I, _P, _I]),
    "cblas_dnrm2": (_D, [_I, _P, _I]),
}

_lib = None
_lock = threading.Lock()


def load():
    """Load libcyclone_blas.so (and libcyclone.so); raises if missing."""
    global _lib
    with _lock:
        if _lib is None:
            base = _native.load()
            if not os.path.exists(LIB_PATH):
                raise ImportError(f"libcyclone_blas.so not found at {LIB_PATH}; build it with "
                                  "make -C cycloneml_amd/csrc")
            L = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            _lib = (L, base)
    return _lib[0]


def header_symbols(path: str = HEADER_PATH):
    txt = re.sub(r"/\*.*?\*/", "", open(path).read(), flags=re.S)
    return sorted(set(re.findall(r"\b((?:cblas_)?d[a-z0-9]+_?)\s*\(", txt)))


def _check():
    msg = _native.load().cyc_last_error().decode(errors="replace")
    if not msg:
        return
    if "illegal value" in msg:
        raise _native.IllegalArgumentException(msg)
    raise _native.CycloneError(_native.CYC_ERR_HIP, msg)


def _buf(a, writable=False):
    if not isinstance(a, np.ndarray) or a.dtype != np.float64:
        raise TypeError("BLAS operands are float64 numpy arrays")
    if writable and not a.flags.writeable:
        raise ValueError("output operand is read-only")
    if not (a.flags.f_contiguous or a.flags.c_contiguous):
        raise ValueError("BLAS operands must be contiguous buffers")
    return a.ctypes.data_as(_P)


def _i(v):
    return ctypes.byref(ctypes.c_int(int(v)))


def _d(v):
    return ctypes.byref(ctypes.c_double(float(v)))


class NativeBLAS:
    """dev.ludovic.netlib.blas.BLAS surface (Fortran argument order; arrays
    are flat column-major float64 buffers, no offsets)."""

    def dgemm(self, transa, transb, m, n, k, alpha, a, lda, b, ldb, beta, c, ldc):
        load().dgemm_(transa.encode(), transb.encode(), _i(m), _i(n), _i(k), _d(alpha), _buf(a),
                      _i(lda), _buf(b), _i(ldb), _d(beta), _buf(c, True), _i(ldc))
        _check()

    def dgemv(self, trans, m, n, alpha, a, lda, x, incx, beta, y, incy):
        load().dgemv_(trans.encode(), _i(m), _i(n), _d(alpha), _buf(a), _i(lda), _buf(x),
                      _i(incx), _d(beta), _buf(y, True), _i(incy))
        _check()

    def dspr(self, uplo, n, alpha, x, incx, ap):
        load().dspr_(uplo.encode(), _i(n), _d(alpha), _buf(x), _i(incx), _buf(ap, True))
        _check()

    def dsyr(self, uplo, n, alpha, x, incx, a, lda):
        load().dsyr_(uplo.encode(), _i(n), _d(alpha), _buf(x), _i(incx), _buf(a, True), _i(lda))
        _check()

    def dger(self, m, n, alpha, x, incx, y, incy, a, lda):
        load().dger_(_i(m), _i(n), _d(alpha), _buf(x), _i(incx), _buf(y), _i(incy),
                     _buf(a, True), _i(lda))
        _check()

    def dspmv(self, uplo, n, alpha, ap, x, incx, beta, y, incy):
        load().dspmv_(uplo.encode(), _i(n), _d(alpha), _buf(ap), _buf(x), _i(incx), _d(beta),
                      _buf(y, True), _i(incy))
        _check()

    def ddot(self, n, x, incx, y, incy):
        r = load().ddot_(_i(n), _buf(x), _i(incx), _buf(y), _i(incy))
        _check()
        return r

    def daxpy(self, n, alpha, x, incx, y, incy):
        load().daxpy_(_i(n), _d(alpha), _buf(x), _i(incx), _buf(y, True), _i(incy))
        _check()

    def dscal(self, n, alpha, x, incx):
        load().dscal_(_i(n), _d(alpha), _buf(x, True), _i(incx))
        _check()

    def dcopy(self, n, x, incx, y, incy):
        load().dcopy_(_i(n), _buf(x), _i(incx), _buf(y, True), _i(incy))
        _check()

    def dnrm2(self, n, x, incx):
        r = load().dnrm2_(_i(n), _buf(x), _i(incx))
        _check()
        return r


nativeBLAS = NativeBLAS()


def _require(cond, msg):
    if not cond:
        raise _native.IllegalArgumentException("requirement failed: " + msg)


def _colmajor(A):
    """(flat column-major buffer, rows, cols) of a 2-D array; a transposed
    view (C-contiguous) is passed as 'T' of its Fortran-order transpose."""
    if A.flags.f_contiguous:
        return A, False
    return A.T, True  # A.T is F-contiguous with shape (cols, rows)


def gemm(alpha, A, B, beta, C):
    """C := alpha * A * B + beta * C (ml/linalg/BLAS.scala:374-425)."""
    _require(C.flags.f_contiguous, "The matrix C cannot be the product of a transpose() call. "
                                    "C.isTransposed must be false.")
    mA, nA = A.shape
    mB, nB = B.shape
    _require(nA == mB, f"The columns of A don't match the rows of B. A: {nA}, B: {mB}")
    _require(mA == C.shape[0], f"The rows of C don't match the rows of A. C: {C.shape[0]}, A: {mA}")
    _require(nB == C.shape[1],
             f"The columns of C don't match the columns of B. C: {C.shape[1]}, A: {nB}")
    if alpha == 0.0 and beta == 1.0:
        return C
    if alpha == 0.0:
        C *= beta  # BLAS.scala:390 dscal path
        return C
    a, ta = _colmajor(A)
    b, tb = _colmajor(B)
    nativeBLAS.dgemm("T" if ta else "N", "T" if tb else "N", mA, nB, nA, alpha, a,
                     a.shape[0], b, b.shape[0], beta, C, mA)
    return C


def gemv(alpha, A, x, beta, y):
    """y := alpha * A * x + beta * y (ml/linalg/BLAS.scala:540-632)."""
    mA, nA = A.shape
    _require(nA == x.size, f"The columns of A don't match the number of elements of x. "
                           f"A: {nA}, x: {x.size}")
    _require(mA == y.size, f"The rows of A don't match the number of elements of y. "
                           f"A: {mA}, y:{y.size}")
    if alpha == 0.0 and beta == 1.0:
        return y
    a, ta = _colmajor(A)
    if ta:
        nativeBLAS.dgemv("T", nA, mA, alpha, a, nA, x, 1, beta, y, 1)
    else:
        nativeBLAS.dgemv("N", mA, nA, alpha, a, mA, x, 1, beta, y, 1)
    return y


def spr(alpha, v, U):
    """U += alpha * v * v^T, U packed upper column-major (BLAS.scala:277-285)."""
    n = v.size
    _require(U.size == n * (n + 1) // 2, "packed size mismatch")
    nativeBLAS.dspr("U", n, alpha, v, 1, U)
    return U


def syr(alpha, x, A):
    """A += alpha * x * x^T, upper triangle (BLAS.scala:323-337)."""
    mA, nA = A.shape
    _require(mA == nA, f"A is not a square matrix (and hence is not symmetric). A: {mA} x {nA}")
    _require(mA == x.size, f"The size of x doesn't match the rank of A. A: {mA} x {nA}, "
                           f"x: {x.size}")
    nativeBLAS.dsyr("U", x.size, alpha, x, 1, A, mA)
    iu = np.triu_indices(mA, 1)  # fill the lower triangle (BLAS.scala:338-346)
    A[iu[1], iu[0]] = A[iu]
    return A


def dspmv(n, alpha, A, x, beta, y):
    """y := alpha * A * x + beta * y, A packed upper (BLAS.scala:264-273)."""
    nativeBLAS.dspmv("U", n, alpha, A, x, 1, beta, y, 1)
    return y


def dot(x, y):
    _require(x.size == y.size, f"BLAS.dot(x: Vector, y:Vector) was given Vectors with "
                               f"non-matching sizes: x.size = {x.size}, y.size = {y.size}")
    return nativeBLAS.ddot(x.size, x, 1, y, 1)


def axpy(a, x, y):
    _require(x.size == y.size, "Vector sizes must match")
    nativeBLAS.daxpy(x.size, a, x, 1, y, 1)
    return y


def scal(a, x):
    nativeBLAS.dscal(x.size, a, x, 1)
    return x
