"""ctypes wrapper around the CPU restatement in cyclone_oracle.c.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py as the parity checker.  The product package
(cycloneml_amd) never imports this module.

Each wrapper cites the reference Scala it restates (paths relative to
/root/reference).  Arrays are numpy float64 / int32 / int64, C-contiguous.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# CYC_ORACLE_LIB: a prebuilt copy to load instead (tools/asan_cpu.sh: the
# AddressSanitizer build, `make -C oracle asan`)
_LIB_PATH = os.environ.get("CYC_ORACLE_LIB") or os.path.join(_HERE, "liboracle.so")
_lib = None
_lock = threading.Lock()

_D = ctypes.POINTER(ctypes.c_double)
_I32 = ctypes.POINTER(ctypes.c_int32)
_I64 = ctypes.POINTER(ctypes.c_int64)
_i64 = ctypes.c_int64


def build() -> str:
    """Compile liboracle.so with the committed Makefile (gcc, -ffp-contract=off)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    with _lock:
        if _lib is None:
            src = os.path.join(_HERE, "cyclone_oracle.c")
            if not os.environ.get("CYC_ORACLE_LIB") and (
                    not os.path.exists(_LIB_PATH)
                    or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src)):
                build()
            L = ctypes.CDLL(_LIB_PATH)
            sig = {
                "orc_norm2": (ctypes.c_double, [_D, _i64]),
                "orc_sqdist": (ctypes.c_double, [_D, _D, _i64]),
                "orc_kmeans_stats": (None, [_D, _i64, _i64, _D]),
                "orc_take_require_failure": (ctypes.c_int, [_D, _D]),
                "orc_find_closest_stats": (None, [_D, _D, _i64, _i64, _D, _D, ctypes.c_double,
                                                  _I32, _D]),
                "orc_find_closest": (None, [_D, _D, _i64, _i64, _D, ctypes.c_double, _I32, _D]),
                "orc_point_costs": (ctypes.c_double, [_D, _D, _i64, _i64, _D, _D, _i64, _I32,
                                                      _D]),
                "orc_point_costs_sparse": (ctypes.c_double, [_I64, _I32, _D, _D, _i64, _i64, _D,
                                                             _D, _i64, _I32, _D]),
                "orc_find_closest_stats_sparse": (None, [_D, _D, _i64, _i64, _D, _I32, _D, _i64,
                                                         ctypes.c_double, _I32, _D]),
                "orc_kmeans_partition": (None, [_D, _D, _D, _i64, _i64, _D, _D, _D, _i64, _I32,
                                                _D, _D, _D, _D]),
                "orc_axpy": (None, [_i64, ctypes.c_double, _D, _D]),
                "orc_kmeans_update_centers": (ctypes.c_int, [_D, _D, _D, _D, _i64, _i64,
                                                             ctypes.c_double]),
                "orc_ddot": (ctypes.c_double, [_D, _D, _i64]),
                "orc_take_assert_failure": (ctypes.c_int, []),
                "orc_cos_stats": (None, [_D, _D, _i64, _i64, _D]),
                "orc_cos_find_closest_stats": (None, [_D, _D, _i64, _i64, _D, _D,
                                                      ctypes.c_double, _I32, _D]),
                "orc_cos_find_closest": (None, [_D, _D, _i64, _i64, _D, ctypes.c_double, _I32,
                                                _D]),
                "orc_cos_point_costs": (ctypes.c_double, [_D, _D, _i64, _i64, _D, _D, _i64,
                                                          _I32, _D]),
                "orc_cos_kmeans_partition": (None, [_D, _D, _D, _i64, _i64, _D, _D, _D, _i64,
                                                    _I32, _D, _D, _D, _D]),
                "orc_cos_update_centers": (ctypes.c_int, [_D, _D, _D, _D, _i64, _i64,
                                                          ctypes.c_double]),
                "orc_cos_point_costs_sparse": (ctypes.c_double, [_I64, _I32, _D, _D, _i64, _i64,
                                                                 _D, _D, _i64, _I32, _D]),
                "orc_cos_kmeans_partition_sparse": (None, [_I64, _I32, _D, _D, _D, _i64, _i64,
                                                           _D, _D, _D, _i64, _I32, _D, _D, _D,
                                                           _D]),
                "orc_log1pexp": (ctypes.c_double, [ctypes.c_double]),
                "orc_softmax": (None, [_D, _i64, _i64, _i64]),
                "orc_hinge_add_dense": (None, [_i64, _i64, _D, _D, _D, _D, ctypes.c_int, _D, _D,
                                               _D, _D]),
                "orc_hinge_add_csr": (None, [_i64, _i64, _I64, _I32, _D, _D, _D, _D,
                                             ctypes.c_int, _D, _D, _D, _D]),
                "orc_huber_add_block": (None, [_i64, _i64, _D, _I64, _I32, _D, _D, _D,
                                               ctypes.c_int, ctypes.c_double, _D, _D, _D, _D]),
                "orc_aft_add_block": (None, [_i64, _i64, _D, _I64, _I32, _D, _D, _D, ctypes.c_int,
                                             _D, _D, _D, _D]),
                "orc_least_squares_add_block": (None, [_i64, _i64, _D, _I64, _I32, _D, _D, _D,
                                                       _D, ctypes.c_int, ctypes.c_double,
                                                       ctypes.c_double, _D, _D, _D, _D]),
                "orc_binary_logistic_add_dense": (None, [_i64, _i64, _D, _D, _D, _D, ctypes.c_int,
                                                         ctypes.c_int, _D, _D, _D, _D]),
                "orc_binary_logistic_add_csr": (None, [_i64, _i64, _I64, _I32, _D, _D, _D, _D,
                                                       ctypes.c_int, ctypes.c_int, _D, _D, _D,
                                                       _D]),
                "orc_multinomial_logistic_add_dense": (None, [_i64, _i64, _i64, _D, _D, _D, _D,
                                                              ctypes.c_int, ctypes.c_int, _D, _D,
                                                              _D, _D]),
                "orc_multinomial_logistic_add_csr": (None, [_i64, _i64, _i64, _I64, _I32, _D, _D,
                                                            _D, _D, ctypes.c_int, ctypes.c_int,
                                                            _D, _D, _D, _D]),
                "orc_kmeans_partition_sparse": (None, [_I64, _I32, _D, _D, _D, _i64, _i64, _D,
                                                       _D, _D, _i64, _I32, _D, _D, _D, _D]),
                "orc_row_norms_csr": (None, [_I64, _D, _i64, _D]),
                "orc_summ_init": (None, [_i64, _D]),
                "orc_summ_add_row": (None, [_i64, _D, _I32, _D, _i64, ctypes.c_double]),
                "orc_summ_merge": (None, [_i64, _D, _D]),
                "orc_summarize": (None, [_i64, _i64, _D, _I64, _I32, _D, _D, _i64, _D]),
                "orc_summ_metrics": (None, [_i64, _D, _D]),
                "orc_label_summarize": (None, [_i64, _D, _D, _i64, _i64, _D, _I64, _I64]),
                "orc_dspr_upper": (None, [_i64, ctypes.c_double, _D, _D]),
                "orc_spr_sparse": (None, [ctypes.c_double, _I32, _D, _i64, _D]),
                "orc_gramian_partition": (None, [_D, _i64, _i64, _D, _D]),
                "orc_triu_to_full": (None, [_i64, _D, _D]),
                "orc_silhouette": (ctypes.c_int, [_D, _i64, _i64, _I32, _D, _i64, ctypes.c_int,
                                                  _D, _D]),
                "orc_blokify": (_i64, [_i64, _i64, _I64, _D, _i64, _I64,
                                       ctypes.POINTER(ctypes.c_uint8)]),
            }
            for name, (res, args) in sig.items():
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            _lib = L
    return _lib


class IllegalArgumentException(ValueError):
    """A Scala `require` failed (the restatement's IllegalArgumentException)."""


def java_double(x: float) -> str:
    """java.lang.Double.toString: shortest round-trip digits, plain decimal
    for 1e-3 <= |x| < 1e7 ("1.0", "0.001"), else "d.dddE<n>" ("1.0E7")."""
    x = float(x)
    if x != x:
        return "NaN"
    if x in (float("inf"), float("-inf")):
        return "Infinity" if x > 0 else "-Infinity"
    if x == 0.0:
        return "-0.0" if np.signbit(x) else "0.0"
    r = repr(abs(x))                       # shortest round-trip digits
    mant, _, exp = r.partition("e")
    ip, _, fp = mant.partition(".")
    digits = (ip + fp).lstrip("0")
    e10 = (int(exp) if exp else 0) + len(ip.lstrip("0")) - 1 if ip.strip("0") else \
        (int(exp) if exp else 0) - (len(fp) - len(fp.lstrip("0"))) - 1
    digits = digits.rstrip("0") or "0"
    sign = "-" if x < 0 else ""
    if 1e-3 <= abs(x) < 1e7:
        if e10 >= 0:
            ipart = digits[:e10 + 1].ljust(e10 + 1, "0")
            fpart = digits[e10 + 1:] or "0"
        else:
            ipart, fpart = "0", "0" * (-e10 - 1) + digits
        return f"{sign}{ipart}.{fpart}"
    return f"{sign}{digits[0]}.{digits[1:] or '0'}E{e10}"


def _raise_require():
    """Rethrow a failed MLUtils.fastSquaredDistance require (MLUtils.scala:
    542-543) recorded by the restatement on this thread."""
    n1, n2 = ctypes.c_double(), ctypes.c_double()
    if lib().orc_take_require_failure(ctypes.byref(n1), ctypes.byref(n2)):
        raise IllegalArgumentException(
            "requirement failed: Both norms should be greater or equal to 0.0, found "
            f"norm1={java_double(n1.value)}, norm2={java_double(n2.value)}")


def _p(a, ty=_D):
    if a is None:
        return None
    return a.ctypes.data_as(ty)


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


# --------------------------------------------------------------------------
# Vectors / KMeans
# --------------------------------------------------------------------------

def norm2(x) -> float:
    """mllib/linalg/Vectors.scala:489-514"""
    x = _f64(x)
    return lib().orc_norm2(_p(x), x.size)


def row_norms(X) -> np.ndarray:
    X = _f64(X)
    return np.array([norm2(X[i]) for i in range(X.shape[0])], dtype=np.float64)


def sqdist(a, b) -> float:
    """mllib/linalg/Vectors.scala:580-587"""
    a, b = _f64(a), _f64(b)
    return lib().orc_sqdist(_p(a), _p(b), a.size)


def kmeans_stats(C) -> np.ndarray:
    """DistanceMeasure.scala:48-76 computeStatistics (Euclidean :275-277)."""
    C = _f64(C)
    k, d = C.shape
    out = np.empty(k * (k + 1) // 2, dtype=np.float64)
    lib().orc_kmeans_stats(_p(C), k, d, _p(out))
    _raise_require()
    return out


def find_closest_stats(C, cnorm, stats, x, xnorm):
    """DistanceMeasure.scala:282-313"""
    C, cnorm, stats, x = _f64(C), _f64(cnorm), _f64(stats), _f64(x)
    idx = ctypes.c_int32()
    dist = ctypes.c_double()
    lib().orc_find_closest_stats(_p(C), _p(cnorm), C.shape[0], C.shape[1], _p(stats), _p(x),
                                 float(xnorm), ctypes.byref(idx), ctypes.byref(dist))
    _raise_require()
    return idx.value, dist.value


def find_closest(C, cnorm, x, xnorm):
    """DistanceMeasure.scala:318-340"""
    C, cnorm, x = _f64(C), _f64(cnorm), _f64(x)
    idx = ctypes.c_int32()
    dist = ctypes.c_double()
    lib().orc_find_closest(_p(C), _p(cnorm), C.shape[0], C.shape[1], _p(x), float(xnorm),
                           ctypes.byref(idx), ctypes.byref(dist))
    return idx.value, dist.value


def point_costs(X, xnorm, C, cnorm):
    """DistanceMeasure.pointCost (:152-156) per row (findClosest without
    statistics, :318-340) and the sequential RDD.sum of one partition
    (KMeansModel.computeCost, KMeansModel.scala:110-117).
    Returns (assign, cost, sum)."""
    X, xnorm, C, cnorm = _f64(X), _f64(xnorm), _f64(C), _f64(cnorm)
    n, d = X.shape
    a = np.zeros(n, dtype=np.int32)
    c = np.zeros(n)
    s = lib().orc_point_costs(_p(X), _p(xnorm), n, d, _p(C), _p(cnorm), C.shape[0], _p(a, _I32),
                              _p(c))
    return a, c, s


def point_costs_sparse(csr, xnorm, C, cnorm):
    """point_costs for CSR rows (csr = (rowptr int64, colidx int32, values))."""
    rowptr, colidx, vals = csr
    rowptr = np.ascontiguousarray(rowptr, dtype=np.int64)
    colidx = np.ascontiguousarray(colidx, dtype=np.int32)
    vals, xnorm, C, cnorm = _f64(vals), _f64(xnorm), _f64(C), _f64(cnorm)
    n = rowptr.size - 1
    a = np.zeros(n, dtype=np.int32)
    c = np.zeros(n)
    s = lib().orc_point_costs_sparse(_p(rowptr, _I64), _p(colidx, _I32), _p(vals), _p(xnorm), n,
                                     C.shape[1], _p(C), _p(cnorm), C.shape[0], _p(a, _I32), _p(c))
    return a, c, s


def find_closest_stats_sparse(C, cnorm, stats, idx, val, xnorm):
    """DistanceMeasure.scala:282-313 with a SparseVector point (MLUtils.scala:560-573)."""
    C, cnorm, stats, val = _f64(C), _f64(cnorm), _f64(stats), _f64(val)
    idx = np.ascontiguousarray(idx, dtype=np.int32)
    oi = ctypes.c_int32()
    od = ctypes.c_double()
    lib().orc_find_closest_stats_sparse(_p(C), _p(cnorm), C.shape[0], C.shape[1], _p(stats),
                                        _p(idx, _I32), _p(val), idx.size, float(xnorm),
                                        ctypes.byref(oi), ctypes.byref(od))
    _raise_require()
    return oi.value, od.value


def kmeans_partition(X, xnorm, w, C, cnorm, stats, want_assign=True):
    """KMeans.scala:287-306 mapPartitions body over one partition.

    Returns (assign, dist, sums[k,d], wsum[k], cost)."""
    X, xnorm, C, cnorm, stats = _f64(X), _f64(xnorm), _f64(C), _f64(cnorm), _f64(stats)
    w = None if w is None else _f64(w)
    n, d = X.shape
    k = C.shape[0]
    assign = np.empty(n, dtype=np.int32) if want_assign else None
    dist = np.empty(n, dtype=np.float64) if want_assign else None
    sums = np.zeros((k, d), dtype=np.float64)
    wsum = np.zeros(k, dtype=np.float64)
    cost = ctypes.c_double(0.0)
    lib().orc_kmeans_partition(_p(X), _p(xnorm), _p(w), n, d, _p(C), _p(cnorm), _p(stats), k,
                               _p(assign, _I32), _p(dist), _p(sums), _p(wsum),
                               ctypes.byref(cost))
    _raise_require()
    return assign, dist, sums, wsum, cost.value


def row_norms_csr(rowptr, vals) -> np.ndarray:
    """Vectors.norm(sparse, 2) per CSR row (mllib/linalg/Vectors.scala:489-514)."""
    rp = np.ascontiguousarray(rowptr, dtype=np.int64)
    v = _f64(vals)
    out = np.empty(len(rp) - 1)
    lib().orc_row_norms_csr(_p(rp, _I64), _p(v), len(rp) - 1, _p(out))
    return out


def kmeans_partition_sparse(csr, xnorm, w, C, cnorm, stats):
    """KMeans.scala:299-304 over sparse points (norm-trick findClosest, sparse
    axpy sums).  Returns (assign, dist, sums (k x d), wsum, cost)."""
    rp = np.ascontiguousarray(csr[0], dtype=np.int64)
    ci = np.ascontiguousarray(csr[1], dtype=np.int32)
    v = _f64(csr[2])
    C = _f64(C)
    k, d = C.shape
    n = len(rp) - 1
    a = np.empty(n, np.int32)
    dist = np.empty(n)
    sums = np.zeros(k * d)
    wsum = np.zeros(k)
    cost = np.zeros(1)
    lib().orc_kmeans_partition_sparse(_p(rp, _I64), _p(ci, _I32), _p(v), _p(_f64(xnorm)),
                                      _p(None if w is None else _f64(w)), n, d, _p(C),
                                      _p(_f64(cnorm)), _p(_f64(stats)), k, _p(a, _I32), _p(dist),
                                      _p(sums), _p(wsum), _p(cost))
    _raise_require()
    return a, dist, sums.reshape(k, d), wsum, cost[0]


def kmeans_iteration(X, xnorm, w, C, cnorm, num_partitions=1, threads=None):
    """One Lloyd iteration, KMeans.scala:275-334, with the rows split into
    `num_partitions` contiguous Spark partitions run on `threads` host threads
    (Spark local[N]).  Partition results merge in partition order with
    axpy(1.0, ...) (the reduceByKey combiner :308-310).

    Returns dict(assign, dist, sums, wsum, cost, centers, cnorm, converged)
    where centers/cnorm are the updated model (:322-330)."""
    X, xnorm, C, cnorm = _f64(X), _f64(xnorm), _f64(C), _f64(cnorm)
    n = X.shape[0]
    stats = kmeans_stats(C)
    bounds = np.linspace(0, n, num_partitions + 1).astype(np.int64)

    def run(p):
        a, b = bounds[p], bounds[p + 1]
        return kmeans_partition(X[a:b], xnorm[a:b], None if w is None else w[a:b], C, cnorm,
                                stats)

    if threads and threads > 1 and num_partitions > 1:
        with ThreadPoolExecutor(threads) as ex:
            parts = list(ex.map(run, range(num_partitions)))
    else:
        parts = [run(p) for p in range(num_partitions)]
    assign = np.concatenate([p[0] for p in parts])
    dist = np.concatenate([p[1] for p in parts])
    sums = parts[0][2].copy()
    wsum = parts[0][3].copy()
    cost = 0.0
    for p in parts:
        cost += p[4]
    for p in parts[1:]:
        for j in range(sums.shape[0]):
            if p[3][j] > 0:
                if wsum[j] > 0:
                    lib().orc_axpy(sums.shape[1], 1.0, _p(np.ascontiguousarray(p[2][j])),
                                   sums[j].ctypes.data_as(_D))
                else:
                    sums[j] = p[2][j]
                wsum[j] = wsum[j] + p[3][j]
    C2, cn2 = C.copy(), cnorm.copy()
    conv = update_centers(C2, cn2, sums, wsum)
    return dict(assign=assign, dist=dist, sums=sums, wsum=wsum, cost=cost, centers=C2,
                cnorm=cn2, converged=conv, stats=stats)


def update_centers(C, cnorm, sums, wsum, epsilon=1e-4) -> bool:
    """KMeans.scala:322-330 centroid + isCenterConverged, in place."""
    assert C.flags.c_contiguous and cnorm.flags.c_contiguous
    sums, wsum = _f64(sums), _f64(wsum)
    k, d = C.shape
    return bool(lib().orc_kmeans_update_centers(_p(C), _p(cnorm), _p(sums), _p(wsum), k, d,
                                                float(epsilon)))


# --------------------------------------------------------------------------
# KMeans with CosineDistanceMeasure (DistanceMeasure.scala:395-514)
# --------------------------------------------------------------------------

class JavaAssertionError(AssertionError):
    """A Scala `assert` failed (java.lang.AssertionError)."""


COSINE_ASSERT = "assertion failed: Cosine distance is not defined for zero-length vectors."


def _raise_assert():
    if lib().orc_take_assert_failure():
        raise JavaAssertionError(COSINE_ASSERT)


def cos_stats(C, cnorm) -> np.ndarray:
    """computeStatistics with the cosine statistic (:48-76, :412-417)."""
    C, cnorm = _f64(C), _f64(cnorm)
    k, d = C.shape
    out = np.empty(k * (k + 1) // 2)
    lib().orc_cos_stats(_p(C), _p(cnorm), k, d, _p(out))
    _raise_assert()
    return out


def cos_find_closest_stats(C, cnorm, stats, x, xnorm):
    C, cnorm, stats, x = _f64(C), _f64(cnorm), _f64(stats), _f64(x)
    i, dd = ctypes.c_int32(), ctypes.c_double()
    lib().orc_cos_find_closest_stats(_p(C), _p(cnorm), C.shape[0], C.shape[1], _p(stats), _p(x),
                                     float(xnorm), ctypes.byref(i), ctypes.byref(dd))
    _raise_assert()
    return i.value, dd.value


def cos_find_closest(C, cnorm, x, xnorm):
    C, cnorm, x = _f64(C), _f64(cnorm), _f64(x)
    i, dd = ctypes.c_int32(), ctypes.c_double()
    lib().orc_cos_find_closest(_p(C), _p(cnorm), C.shape[0], C.shape[1], _p(x), float(xnorm),
                               ctypes.byref(i), ctypes.byref(dd))
    _raise_assert()
    return i.value, dd.value


def cos_point_costs(X, xnorm, C, cnorm):
    """pointCost with the cosine distance for every row; (assign, cost, sum)."""
    X, xnorm, C, cnorm = _f64(X), _f64(xnorm), _f64(C), _f64(cnorm)
    n, d = X.shape
    a = np.empty(n, dtype=np.int32)
    c = np.empty(n)
    s = lib().orc_cos_point_costs(_p(X), _p(xnorm), n, d, _p(C), _p(cnorm), C.shape[0],
                                  _p(a, _I32), _p(c))
    _raise_assert()
    return a, c, s


def cos_kmeans_partition(X, xnorm, w, C, cnorm, stats):
    X, xnorm, C, cnorm, stats = _f64(X), _f64(xnorm), _f64(C), _f64(cnorm), _f64(stats)
    n, d = X.shape
    k = C.shape[0]
    a = np.full(n, -1, dtype=np.int32)
    dist = np.full(n, np.nan)
    sums = np.zeros(k * d)
    wsum = np.zeros(k)
    cost = np.zeros(1)
    lib().orc_cos_kmeans_partition(_p(X), _p(xnorm), _p(None if w is None else _f64(w)), n, d,
                                   _p(C), _p(cnorm), _p(stats), k, _p(a, _I32), _p(dist),
                                   _p(sums), _p(wsum), _p(cost))
    _raise_assert()
    return a, dist, sums.reshape(k, d), wsum, cost[0]


def cos_point_costs_sparse(csr, xnorm, C, cnorm):
    rp, ci, v, d = csr
    rp = np.ascontiguousarray(rp, dtype=np.int64)
    ci = np.ascontiguousarray(ci, dtype=np.int32)
    v, C, cnorm = _f64(v), _f64(C), _f64(cnorm)
    n = rp.shape[0] - 1
    a = np.empty(n, dtype=np.int32)
    c = np.empty(n)
    s = lib().orc_cos_point_costs_sparse(_p(rp, _I64), _p(ci, _I32), _p(v), _p(_f64(xnorm)), n,
                                         d, _p(C), _p(cnorm), C.shape[0], _p(a, _I32), _p(c))
    _raise_assert()
    return a, c, s


def cos_kmeans_partition_sparse(csr, xnorm, w, C, cnorm, stats):
    """csr = (rowptr, colidx, values, numFeatures)."""
    rp, ci, v, d = csr
    rp = np.ascontiguousarray(rp, dtype=np.int64)
    ci = np.ascontiguousarray(ci, dtype=np.int32)
    v, C, cnorm, stats = _f64(v), _f64(C), _f64(cnorm), _f64(stats)
    n, k = rp.shape[0] - 1, C.shape[0]
    a = np.full(n, -1, dtype=np.int32)
    dist = np.full(n, np.nan)
    sums = np.zeros(k * d)
    wsum = np.zeros(k)
    cost = np.zeros(1)
    lib().orc_cos_kmeans_partition_sparse(_p(rp, _I64), _p(ci, _I32), _p(v), _p(_f64(xnorm)),
                                          _p(None if w is None else _f64(w)), n, d, _p(C),
                                          _p(cnorm), _p(stats), k, _p(a, _I32), _p(dist),
                                          _p(sums), _p(wsum), _p(cost))
    _raise_assert()
    return a, dist, sums.reshape(k, d), wsum, cost[0]


def cos_update_centers(C, cnorm, sums, wsum, epsilon=1e-4) -> bool:
    """centroid + isCenterConverged of the cosine measure, in place."""
    assert C.flags.c_contiguous and cnorm.flags.c_contiguous
    sums, wsum = _f64(sums), _f64(wsum)
    k, d = C.shape
    return bool(lib().orc_cos_update_centers(_p(C), _p(cnorm), _p(sums), _p(wsum), k, d,
                                             float(epsilon)))


def cos_kmeans_iteration(X, xnorm, w, C, cnorm, epsilon=1e-4):
    """One cosine Lloyd iteration over a single partition (KMeans.scala:
    275-334): dict(assign, dist, sums, wsum, cost, centers, cnorm,
    converged, stats)."""
    C, cnorm = _f64(C), _f64(cnorm)
    stats = cos_stats(C, cnorm)
    a, dist, sums, wsum, cost = cos_kmeans_partition(X, xnorm, w, C, cnorm, stats)
    C2, cn2 = C.copy(), cnorm.copy()
    conv = cos_update_centers(C2, cn2, sums, wsum, epsilon)
    return dict(assign=a, dist=dist, sums=sums, wsum=wsum, cost=cost, centers=C2, cnorm=cn2,
                converged=conv, stats=stats)


# --------------------------------------------------------------------------
# Logistic aggregators
# --------------------------------------------------------------------------

def log1pexp(x: float) -> float:
    return lib().orc_log1pexp(float(x))


def binary_logistic_add(block, coef, fit_intercept, fit_with_mean, scaled_mean, state):
    """BinaryLogisticBlockAggregator.add (.scala:81-145).

    block: dict(labels, weights|None, X (dense S x F) | rowptr/colidx/values, F)
    state: dict(grad, loss, weight) updated in place."""
    L = lib()
    coef = _f64(coef)
    sm = None if scaled_mean is None else _f64(scaled_mean)
    labels = _f64(block["labels"])
    weights = None if block.get("weights") is None else _f64(block["weights"])
    loss = ctypes.c_double(state["loss"])
    wsum = ctypes.c_double(state["weight"])
    g = state["grad"]
    if "X" in block:
        X = _f64(block["X"])
        L.orc_binary_logistic_add_dense(X.shape[0], X.shape[1], _p(X), _p(labels), _p(weights),
                                        _p(coef), int(fit_intercept), int(fit_with_mean), _p(sm),
                                        _p(g), ctypes.byref(loss), ctypes.byref(wsum))
    else:
        rp = np.ascontiguousarray(block["rowptr"], dtype=np.int64)
        ci = np.ascontiguousarray(block["colidx"], dtype=np.int32)
        v = _f64(block["values"])
        L.orc_binary_logistic_add_csr(rp.size - 1, block["F"], _p(rp, _I64), _p(ci, _I32), _p(v),
                                      _p(labels), _p(weights), _p(coef), int(fit_intercept),
                                      int(fit_with_mean), _p(sm), _p(g), ctypes.byref(loss),
                                      ctypes.byref(wsum))
    state["loss"], state["weight"] = loss.value, wsum.value


def hinge_add(block, coef, fit_intercept, scaled_mean, state):
    """HingeBlockAggregator.add (ml/optim/aggregator/HingeBlockAggregator.scala:81-141).

    block / state as binary_logistic_add."""
    L = lib()
    coef = _f64(coef)
    sm = None if scaled_mean is None else _f64(scaled_mean)
    labels = _f64(block["labels"])
    weights = None if block.get("weights") is None else _f64(block["weights"])
    loss = ctypes.c_double(state["loss"])
    wsum = ctypes.c_double(state["weight"])
    g = state["grad"]
    if "X" in block:
        X = _f64(block["X"])
        L.orc_hinge_add_dense(X.shape[0], X.shape[1], _p(X), _p(labels), _p(weights), _p(coef),
                              int(fit_intercept), _p(sm), _p(g), ctypes.byref(loss),
                              ctypes.byref(wsum))
    else:
        rp = np.ascontiguousarray(block["rowptr"], dtype=np.int64)
        ci = np.ascontiguousarray(block["colidx"], dtype=np.int32)
        v = _f64(block["values"])
        L.orc_hinge_add_csr(rp.size - 1, block["F"], _p(rp, _I64), _p(ci, _I32), _p(v),
                            _p(labels), _p(weights), _p(coef), int(fit_intercept), _p(sm), _p(g),
                            ctypes.byref(loss), ctypes.byref(wsum))
    state["loss"], state["weight"] = loss.value, wsum.value


def huber_add(block, params, fit_intercept, epsilon, scaled_mean, state):
    """HuberBlockAggregator.add (.scala:80-141); params = linear, intercept, sigma."""
    L = lib()
    params = _f64(params)
    sm = None if scaled_mean is None else _f64(scaled_mean)
    labels = _f64(block["labels"])
    weights = None if block.get("weights") is None else _f64(block["weights"])
    loss = ctypes.c_double(state["loss"])
    wsum = ctypes.c_double(state["weight"])
    if "X" in block:
        X = _f64(block["X"])
        S, F, rp, ci, v = X.shape[0], X.shape[1], None, None, X
    else:
        rp = np.ascontiguousarray(block["rowptr"], dtype=np.int64)
        ci = np.ascontiguousarray(block["colidx"], dtype=np.int32)
        v = _f64(block["values"])
        S, F = rp.size - 1, block["F"]
    L.orc_huber_add_block(S, F, _p(v), None if rp is None else _p(rp, _I64),
                          None if ci is None else _p(ci, _I32), _p(labels), _p(weights),
                          _p(params), int(fit_intercept), float(epsilon), _p(sm),
                          _p(state["grad"]), ctypes.byref(loss), ctypes.byref(wsum))
    state["loss"], state["weight"] = loss.value, wsum.value


def aft_add(block, coef, fit_intercept, scaled_mean, state):
    """AFTBlockAggregator.add (.scala:76-130); block["weights"] = censors."""
    L = lib()
    coef = _f64(coef)
    sm = None if scaled_mean is None else _f64(scaled_mean)
    labels = _f64(block["labels"])
    cens = None if block.get("weights") is None else _f64(block["weights"])
    loss = ctypes.c_double(state["loss"])
    wsum = ctypes.c_double(state["weight"])
    if "X" in block:
        X = _f64(block["X"])
        S, F, rp, ci, v = X.shape[0], X.shape[1], None, None, X
    else:
        rp = np.ascontiguousarray(block["rowptr"], dtype=np.int64)
        ci = np.ascontiguousarray(block["colidx"], dtype=np.int32)
        v = _f64(block["values"])
        S, F = rp.size - 1, block["F"]
    L.orc_aft_add_block(S, F, _p(v), None if rp is None else _p(rp, _I64),
                        None if ci is None else _p(ci, _I32), _p(labels), _p(cens), _p(coef),
                        int(fit_intercept), _p(sm), _p(state["grad"]), ctypes.byref(loss),
                        ctypes.byref(wsum))
    state["loss"], state["weight"] = loss.value, wsum.value


def least_squares_add(block, coef, inverse_std, fit_intercept, label_std, label_mean,
                      scaled_mean, state):
    """LeastSquaresBlockAggregator.add (.scala:70-101); dim = numFeatures.
    block / state as binary_logistic_add."""
    L = lib()
    coef, inv = _f64(coef), _f64(inverse_std)
    sm = None if scaled_mean is None else _f64(scaled_mean)
    labels = _f64(block["labels"])
    weights = None if block.get("weights") is None else _f64(block["weights"])
    loss = ctypes.c_double(state["loss"])
    wsum = ctypes.c_double(state["weight"])
    if "X" in block:
        X = _f64(block["X"])
        S, F, rp, ci, v = X.shape[0], X.shape[1], None, None, X
    else:
        rp = np.ascontiguousarray(block["rowptr"], dtype=np.int64)
        ci = np.ascontiguousarray(block["colidx"], dtype=np.int32)
        v = _f64(block["values"])
        S, F = rp.size - 1, block["F"]
    L.orc_least_squares_add_block(S, F, _p(v), None if rp is None else _p(rp, _I64),
                                  None if ci is None else _p(ci, _I32), _p(labels), _p(weights),
                                  _p(coef), _p(inv), int(fit_intercept), float(label_std),
                                  float(label_mean), _p(sm), _p(state["grad"]),
                                  ctypes.byref(loss), ctypes.byref(wsum))
    state["loss"], state["weight"] = loss.value, wsum.value


def multinomial_logistic_add(block, coef, num_classes, fit_intercept, fit_with_mean,
                             scaled_mean, state):
    """MultinomialLogisticBlockAggregator.add (.scala:101-189)."""
    L = lib()
    coef = _f64(coef)
    sm = None if scaled_mean is None else _f64(scaled_mean)
    labels = _f64(block["labels"])
    weights = None if block.get("weights") is None else _f64(block["weights"])
    loss = ctypes.c_double(state["loss"])
    wsum = ctypes.c_double(state["weight"])
    g = state["grad"]
    if "X" in block:
        X = _f64(block["X"])
        L.orc_multinomial_logistic_add_dense(X.shape[0], X.shape[1], num_classes, _p(X),
                                             _p(labels), _p(weights), _p(coef),
                                             int(fit_intercept), int(fit_with_mean), _p(sm),
                                             _p(g), ctypes.byref(loss), ctypes.byref(wsum))
    else:
        rp = np.ascontiguousarray(block["rowptr"], dtype=np.int64)
        ci = np.ascontiguousarray(block["colidx"], dtype=np.int32)
        v = _f64(block["values"])
        L.orc_multinomial_logistic_add_csr(rp.size - 1, block["F"], num_classes, _p(rp, _I64),
                                           _p(ci, _I32), _p(v), _p(labels), _p(weights),
                                           _p(coef), int(fit_intercept), int(fit_with_mean),
                                           _p(sm), _p(g), ctypes.byref(loss),
                                           ctypes.byref(wsum))
    state["loss"], state["weight"] = loss.value, wsum.value


# --------------------------------------------------------------------------
# Gramian
# --------------------------------------------------------------------------

def dspr_upper(x, U, alpha=1.0):
    x = _f64(x)
    lib().orc_dspr_upper(x.size, float(alpha), _p(x), _p(U))


def spr_sparse(idx, val, U, alpha=1.0):
    idx = np.ascontiguousarray(idx, dtype=np.int32)
    val = _f64(val)
    lib().orc_spr_sparse(float(alpha), _p(idx, _I32), _p(val), idx.size, _p(U))


def gramian_partition(X, mean=None, U=None):
    """RowMatrix.scala:139-158 seqOp (or :171-190 with mean)."""
    X = _f64(X)
    rows, n = X.shape
    if U is None:
        U = np.zeros(n * (n + 1) // 2, dtype=np.float64)
    lib().orc_gramian_partition(_p(X), rows, n, _p(None if mean is None else _f64(mean)), _p(U))
    return U


def triu_to_full(n, U) -> np.ndarray:
    """RowMatrix.scala:845-867; returns the column-major n*n array."""
    U = _f64(U)
    G = np.empty(n * n, dtype=np.float64)
    lib().orc_triu_to_full(n, _p(U), _p(G))
    return G


def gramian_csr(rowptr, colidx, vals, n, U=None):
    """computeGramianMatrix's seqOp over SparseVector rows: the sparse spr
    branch (mllib/linalg/BLAS.scala:269-298) per row, in row order."""
    if U is None:
        U = np.zeros(n * (n + 1) // 2, dtype=np.float64)
    for r in range(len(rowptr) - 1):
        a, b = int(rowptr[r]), int(rowptr[r + 1])
        if b > a:
            spr_sparse(colidx[a:b], vals[a:b], U)
    return U


def is_sparse_matrix(row_nnz, ncols) -> bool:
    """RowMatrix.isSparseMatrix (RowMatrix.scala:439-441): no row with
    sparsity() = 1.0 - numNonzeros / size below 0.5."""
    nz = np.asarray(row_nnz, dtype=np.float64)
    return not bool(np.any(1.0 - nz / float(ncols) < 0.5))


def sparse_vector_covariance(n, U, mean, m):
    """computeSparseVectorCovariance (RowMatrix.scala:222-246) on the packed
    Gramian: column-major n*n, the i <= j loop mirrored."""
    G = triu_to_full(n, U).reshape(n, n).T.copy()      # G[i, j]
    m1 = m - 1.0
    for i in range(n):
        alpha = m / m1 * mean[i]
        for j in range(i, n):
            gij = G[i, j] / m1 - alpha * mean[j]
            G[i, j] = gij
            G[j, i] = gij
    return G


def dense_vector_covariance(n, U, m):
    """computeDenseVectorCovariance's finish (:203-217): full(U) / (m - 1)."""
    return triu_to_full(n, U).reshape(n, n).T / (m - 1.0)


# --------------------------------------------------------------------------
# java.util.Random (for regenerating the reference suites' datasets)
# --------------------------------------------------------------------------

class JavaRandom:
    """java.util.Random: 48-bit LCG, nextDouble, nextGaussian (polar method).

    Used to regenerate DistanceMeasureSuite.scala:37-53 inputs.  StrictMath
    log/sqrt are replaced by Python's math (correctly rounded sqrt; log may
    differ by an ulp in rare cases, which only perturbs test data)."""

    def __init__(self, seed: int):
        self.seed = (seed ^ 0x5DEECE66D) & ((1 << 48) - 1)
        self._next_gaussian = None

    def _next(self, bits: int) -> int:
        self.seed = (self.seed * 0x5DEECE66D + 0xB) & ((1 << 48) - 1)
        r = self.seed >> (48 - bits)
        if r >= 1 << (bits - 1):
            r -= 1 << bits
        return r

    def next_double(self) -> float:
        hi = self._next(26) & ((1 << 26) - 1)
        lo = self._next(27) & ((1 << 27) - 1)
        return ((hi << 27) + lo) * (1.0 / (1 << 53))

    def next_gaussian(self) -> float:
        import math
        if self._next_gaussian is not None:
            g, self._next_gaussian = self._next_gaussian, None
            return g
        while True:
            v1 = 2 * self.next_double() - 1
            v2 = 2 * self.next_double() - 1
            s = v1 * v1 + v2 * v2
            if 0 < s < 1:
                break
        mul = math.sqrt(-2 * math.log(s) / s)
        self._next_gaussian = v2 * mul
        return v1 * mul


class XORShiftRandom(JavaRandom):
    """org.apache.spark.util.random.XORShiftRandom
    (core/src/main/scala/org/apache/spark/util/random/XORShiftRandom.scala:36-67):
    java.util.Random's nextDouble / nextGaussian over an xorshift next(bits),
    the seed hashed by scala.util.hashing.MurmurHash3.bytesHash (scala-library
    2.12, not in the reference tree: its published x86_32 MurmurHash3 with
    arraySeed 0x3c074a61).  Pinned by RandomSuite.scala:26,29: Rand(30) ->
    0.2762195585886885, Rand(null = 0) -> 0.7604953758285915."""

    _M32 = 0xFFFFFFFF
    _M64 = (1 << 64) - 1

    def __init__(self, seed: int):
        b = (seed & self._M64).to_bytes(8, "big")          # ByteBuffer.putLong
        lo = _murmur3_bytes(b, 0x3C074A61)
        hi = _murmur3_bytes(b, lo)
        self.seed = ((hi << 32) | lo) & self._M64
        self._next_gaussian = None

    def _next(self, bits: int) -> int:
        x = self.seed ^ ((self.seed << 21) & self._M64)
        x ^= x >> 35
        x ^= (x << 4) & self._M64
        self.seed = x
        r = x & ((1 << bits) - 1)
        if bits == 32 and r >= 1 << 31:
            r -= 1 << 32
        return r


def kmeans_parallel_sample(costs, part_starts, first_index, seed, step, k, sum_costs):
    """One k-means|| step's filter (KMeans.scala:398-404) per partition:
    XORShiftRandom(seed ^ (step << 16) ^ index) (Int arithmetic, widened to
    Long), keep the point iff rand.nextDouble() < 2.0 * c * k / sumCosts.
    Returns the uint8 mask."""
    def i32(v):
        v &= 0xFFFFFFFF
        return v - (1 << 32) if v >= 1 << 31 else v
    costs = np.asarray(costs, dtype=np.float64)
    out = np.zeros(costs.size, dtype=np.uint8)
    for p in range(len(part_starts) - 1):
        init = i32(i32(seed) ^ i32(step << 16) ^ i32(first_index + p))
        rand = XORShiftRandom(init)
        for i in range(int(part_starts[p]), int(part_starts[p + 1])):
            out[i] = 1 if rand.next_double() < 2.0 * float(costs[i]) * k / sum_costs else 0
    return out


def local_kmeans_pp(points, weights, k, max_iterations, seed, closest=None):
    """LocalKMeans.kMeansPlusPlus (mllib/clustering/LocalKMeans.scala:35-134)
    in plain loops: k-means++ seeding with java.util.Random(seed), then
    Lloyd rounds with EuclideanDistanceMeasure.findClosest (orc_find_closest).
    closest(C) -> (index, cost) of every point against centers C replaces both
    distance steps for points that are sparse in the reference (e.g.
    point_costs_sparse over the points' CSR: fastSquaredDistance(dense
    center, sparse point))."""
    points = _f64(points)
    w = [float(v) for v in weights]
    m, d = points.shape
    rand = JavaRandom(seed)

    def next_int(bound):
        r = rand._next(31) & 0x7FFFFFFF
        mm = bound - 1
        if bound & mm == 0:
            return (bound * r) >> 31
        u = r
        while True:
            r = u % bound
            v = (u - r + mm) & 0xFFFFFFFF
            if v < 1 << 31:
                return r
            u = rand._next(31) & 0x7FFFFFFF

    tot = 0.0
    for v in w:
        tot += v
    r = rand.next_double() * tot
    i, cur = 0, 0.0
    while i < m and cur < r:
        cur += w[i]
        i += 1
    centers = [points[i - 1].copy()]
    if closest is None:
        cost = [sqdist(points[p], centers[0]) for p in range(m)]
    else:
        cost = [float(v) for v in closest(np.array([centers[0]]))[1]]
    for c in range(1, k):
        s = 0.0
        for p in range(m):
            s += cost[p] * w[p]
        r = rand.next_double() * s
        cum, j = 0.0, 0
        while j < m and cum < r:
            cum += w[j] * cost[j]
            j += 1
        centers.append(points[0].copy() if j == 0 else points[j - 1].copy())
        if closest is None:
            nc = [sqdist(points[p], centers[c]) for p in range(m)]
        else:
            nc = [float(v) for v in closest(np.array([centers[c]]))[1]]
        for p in range(m):
            cost[p] = min(nc[p], cost[p])
    old = [-1] * m
    it, moved = 0, True
    while moved and it < max_iterations:
        moved = False
        C = np.array(centers)
        cn = row_norms(C)
        counts = [0.0] * k
        sums = np.zeros((k, d))
        ids = None if closest is None else closest(C)[0]
        for p in range(m):
            if ids is None:
                idx, _ = find_closest(C, cn, points[p], norm2(points[p]))
            else:
                idx = int(ids[p])
            if w[p] != 0.0:
                sums[idx] = sums[idx] + w[p] * points[p]
            counts[idx] += w[p]
            if idx != old[p]:
                moved = True
                old[p] = idx
        for j in range(k):
            if counts[j] == 0.0:
                centers[j] = points[next_int(m)].copy()
            else:
                centers[j] = (1.0 / counts[j]) * sums[j]
        it += 1
    return np.array(centers)


def _murmur3_bytes(data: bytes, seed: int) -> int:
    """scala.util.hashing.MurmurHash3.bytesHash (x86_32, little-endian blocks)."""
    M = 0xFFFFFFFF

    def rotl(x, r):
        return ((x << r) | (x >> (32 - r))) & M

    def mix_last(h, k):
        k = (k * 0xCC9E2D51) & M
        k = rotl(k, 15)
        k = (k * 0x1B873593) & M
        return h ^ k

    h = seed & M
    n = len(data)
    i = 0
    while n - i >= 4:
        k = data[i] | data[i + 1] << 8 | data[i + 2] << 16 | data[i + 3] << 24
        h = mix_last(h, k)
        h = (rotl(h, 13) * 5 + 0xE6546B64) & M
        i += 4
    rem, k = n - i, 0
    if rem == 3:
        k ^= data[i + 2] << 16
    if rem >= 2:
        k ^= data[i + 1] << 8
    if rem >= 1:
        k ^= data[i]
        h = mix_last(h, k)
    h ^= n
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & M
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & M
    h ^= h >> 16
    return h


def generate_multinomial_logistic_input(weights, xMean, xVariance, addIntercept, nPoints, seed):
    """LogisticRegressionSuite.generateMultinomialLogisticInput
    (mllib/src/test/scala/org/apache/spark/ml/classification/LogisticRegressionSuite.scala:3061-3128),
    scala.util.Random(seed) = java.util.Random.  Returns (labels, X)."""
    import math
    rnd = JavaRandom(seed)
    xDim = len(xMean)
    xwi = xDim + 1 if addIntercept else xDim
    nClasses = len(weights) // xwi + 1
    X = np.empty((nPoints, xDim))
    for i in range(nPoints):
        for j in range(xDim):
            X[i, j] = rnd.next_gaussian()
    for i in range(nPoints):
        for j in range(xDim):
            X[i, j] = X[i, j] * math.sqrt(xVariance[j]) + xMean[j]
    y = np.empty(nPoints)
    for idx in range(nPoints):
        margins = [0.0] * nClasses
        for i in range(nClasses - 1):
            for j in range(xDim):
                margins[i + 1] += weights[i * xwi + j] * X[idx, j]
            if addIntercept:
                margins[i + 1] += weights[(i + 1) * xwi - 1]
        mx = max(margins)
        if mx > 0:
            margins = [m - mx for m in margins]
        probs = [math.exp(m) for m in margins]
        norm = 0.0
        for pr in probs:
            norm += pr
        probs = [pr / norm for pr in probs]
        for i in range(1, nClasses):
            probs[i] += probs[i - 1]
        p = rnd.next_double()
        lab = 0
        for i in range(nClasses):
            if p < probs[i]:
                lab = i
                break
        y[idx] = lab
    return y, X


def generate_logistic_input(offset, scale, nPoints, seed):
    """LogisticRegressionSuite.generateLogisticInput (:3021-3036)."""
    import math
    rnd = JavaRandom(seed)
    x1 = np.array([rnd.next_gaussian() for _ in range(nPoints)])
    y = np.empty(nPoints)
    for i in range(nPoints):
        p = 1.0 / (1.0 + math.exp(-(offset + scale * x1[i])))
        y[i] = 1.0 if rnd.next_double() < p else 0.0
    return y, x1.reshape(-1, 1)


def spark_rand_column(seed, nRows, numSlices):
    """functions.rand(seed) over sc.parallelize(rows, numSlices): partition i
    holds rows [i n / s, (i + 1) n / s) (ParallelCollectionRDD.slice,
    core/src/main/scala/org/apache/spark/rdd/ParallelCollectionRDD.scala:116-128)
    and draws XORShiftRandom(seed + i).nextDouble() per row (Rand,
    sql/catalyst/.../expressions/randomExpressions.scala:43-44)."""
    out = np.empty(nRows)
    for i in range(numSlices):
        a, b = (i * nRows) // numSlices, ((i + 1) * nRows) // numSlices
        r = XORShiftRandom(seed + i)
        for j in range(a, b):
            out[j] = r.next_double()
    return out


# --------------------------------------------------------------------------
# Summarizer pre-pass (ml/stat/Summarizer.scala:428-770,
# ml/stat/MultiClassSummarizer.scala:30-98)
# --------------------------------------------------------------------------

SUMM_FIELDS = 8
SUMM_SCALARS = 5
SUMM_METRICS = ("mean", "variance", "std", "sum", "numNonzeros", "max", "min", "normL2",
                "normL1")


def summarizer_new(F):
    st = np.empty(SUMM_FIELDS * F + SUMM_SCALARS)
    lib().orc_summ_init(F, _p(st))
    return st


def summarizer_add(st, F, x=None, idx=None, val=None, weight=1.0):
    """SummarizerBuffer.add(vector, weight): dense x, or sparse (idx, val)."""
    if x is not None:
        x = _f64(x)
        lib().orc_summ_add_row(F, _p(st), None, _p(x), len(x), float(weight))
    else:
        idx = np.ascontiguousarray(idx, dtype=np.int32)
        val = _f64(val)
        lib().orc_summ_add_row(F, _p(st), _p(idx, _I32), _p(val), len(val), float(weight))
    return st


def summarizer_merge(F, a, b):
    """a.merge(b), in place on a."""
    lib().orc_summ_merge(F, _p(a), _p(_f64(b)))
    return a


def summarize(F, X=None, csr=None, w=None, rows_per_partition=1 << 62):
    """Partitions of rows_per_partition rows, each add()-ed in order, merged in
    partition order (the device's schedule)."""
    out = np.empty(SUMM_FIELDS * F + SUMM_SCALARS)
    wp = None if w is None else _f64(w)
    if X is not None:
        X = _f64(X)
        lib().orc_summarize(X.shape[0], F, _p(X), None, None, None, _p(wp),
                            int(rows_per_partition), _p(out))
    else:
        rp = np.ascontiguousarray(csr[0], dtype=np.int64)
        ci = np.ascontiguousarray(csr[1], dtype=np.int32)
        v = _f64(csr[2])
        lib().orc_summarize(len(rp) - 1, F, None, _p(rp, _I64), _p(ci, _I32), _p(v), _p(wp),
                            int(rows_per_partition), _p(out))
    return out


def summarizer_metrics(F, st):
    out = np.empty(9 * F)
    lib().orc_summ_metrics(F, _p(_f64(st)), _p(out))
    m = {name: out[i * F:(i + 1) * F].copy() for i, name in enumerate(SUMM_METRICS)}
    m["count"] = st[SUMM_FIELDS * F]
    m["weightSum"] = st[SUMM_FIELDS * F + 1]
    return m


def label_summarize(y, w=None, rows_per_partition=1 << 62, max_classes=1024):
    """(histogram[:numClasses], countInvalid, numClasses)."""
    y = _f64(y)
    hist = np.empty(max_classes)
    inv = np.zeros(1, np.int64)
    mx = np.zeros(1, np.int64)
    lib().orc_label_summarize(len(y), _p(y), _p(None if w is None else _f64(w)),
                              int(rows_per_partition), int(max_classes), _p(hist),
                              _p(inv, _I64), _p(mx, _I64))
    nc = int(mx[0]) + 1
    return hist[:nc].copy(), int(inv[0]), nc


def row_numnonzeros(X=None, csr=None):
    """Vector.numNonzeros per row (values != 0, explicit zeros excluded)."""
    if X is not None:
        return np.count_nonzero(np.asarray(X) != 0.0, axis=1).astype(np.int64)
    rp, _, v = csr
    nz = (np.asarray(v) != 0.0).astype(np.int64)
    c = np.concatenate([[0], np.cumsum(nz)])
    rp = np.asarray(rp, dtype=np.int64)
    return (c[rp[1:]] - c[rp[:-1]]).astype(np.int64)


def blokify(F, row_nnz, weights, max_mem_usage):
    """InstanceBlock.blokifyWithMaxMemUsage (Instance.scala:146-180):
    (starts[nblocks + 1], dense[nblocks] bool)."""
    if not max_mem_usage > 0:
        raise IllegalArgumentException("requirement failed")
    nnz = np.ascontiguousarray(row_nnz, dtype=np.int64)
    n = nnz.size
    starts = np.zeros(n + 1, np.int64)
    dense = np.zeros(max(n, 1), np.uint8)
    nb = lib().orc_blokify(n, int(F), _p(nnz, _I64), _p(None if weights is None else _f64(weights)),
                           int(max_mem_usage), _p(starts, _I64),
                           dense.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
    return starts[:nb + 1].copy(), dense[:nb].astype(bool)


def parse_libsvm(text, num_features=-1):
    """Pure-Python restatement of MLUtils.parseLibSVMFile / parseLibSVMRecord /
    computeNumFeatures (mllib/util/MLUtils.scala:91-151), small inputs only.
    Returns (labels, (rowptr, colidx, values), numFeatures); raises
    ValueError with the reference's require text on a bad record."""
    labels, rowptr, colidx, values = [], [0], [], []
    max_index = -1
    for raw in text.split("\n"):
        line = raw.strip("".join(chr(c) for c in range(33)))   # String.trim
        if not line or line.startswith("#"):
            continue
        items = line.split(" ")
        labels.append(float(items[0]))
        previous = -1
        for item in items[1:]:
            if not item:
                continue
            iv = item.split(":")
            current = int(iv[0]) - 1
            value = float(iv[1])
            if not current > previous:
                raise ValueError("requirement failed: indices should be one-based and in "
                                 f"ascending order; found current={current}, "
                                 f'previous={previous}; line="{line}"')
            previous = current
            colidx.append(current)
            values.append(value)
        max_index = max(max_index, previous if previous >= 0 else 0)
        rowptr.append(len(colidx))
    nf = num_features if num_features > 0 else (max_index + 1 if labels else 1)
    return (np.array(labels, dtype=np.float64),
            (np.array(rowptr, dtype=np.int64), np.array(colidx, dtype=np.int32),
             np.array(values, dtype=np.float64)), nf)


# --------------------------------------------------------------------------
# ClusteringEvaluator Silhouette
# --------------------------------------------------------------------------

def silhouette(X, pred, k, weights=None, cosine=False):
    """ml/evaluation/ClusteringMetrics.scala SquaredEuclideanSilhouette
    (:254-400) / CosineSilhouette (:403-600), one partition: returns (score,
    stats) with stats = [featureSum | squaredNormSum | weightSum | rows];
    raises JavaAssertionError when fewer than two clusters have rows."""
    X = _f64(X)
    n, d = X.shape
    pred = np.ascontiguousarray(pred, dtype=np.int32)
    w = None if weights is None else _f64(weights)
    stats = np.zeros(k * d + 3 * k, dtype=np.float64)
    score = ctypes.c_double()
    rc = lib().orc_silhouette(_p(X), n, d, _p(pred, _I32), _p(w), k, 1 if cosine else 0,
                              _p(stats), ctypes.byref(score))
    if rc != 0:
        raise JavaAssertionError("assertion failed: Number of clusters must be greater than one.")
    return score.value, stats
