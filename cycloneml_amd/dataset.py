"""Host-pointer layer over libcyclone's resident datasets (cyc_dataset_*).

This is what a JVM shim binds: numpy host arrays in, numpy
host arrays out, the partition's rows resident in HBM between calls.  Each
method cites the reference loop it replaces; see include/cyclone.h.
"""
import ctypes

import numpy as np

from . import _native as N


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _f64(a):
    return None if a is None else np.ascontiguousarray(a, dtype=np.float64)


class ResidentDataset:
    """One partition's rows, resident on the current device.

    dense:  ``ResidentDataset.dense(F, capacity)`` then ``append_dense(X, ...)``
    CSR:    ``ResidentDataset.csr(F, capacity, capacity_nnz)`` then
            ``append_csr(rowptr, colidx, values, ...)``
    """

    def __init__(self, handle, numFeatures):
        self._h = handle
        self.numFeatures = numFeatures

    @classmethod
    def dense(cls, numFeatures, capacity_rows, labels=False, weights=False):
        h = ctypes.c_void_p()
        N.check(N.load().cyc_dataset_dense_create(numFeatures, capacity_rows, int(labels),
                                                  int(weights), ctypes.byref(h)))
        return cls(h, numFeatures)

    @classmethod
    def csr(cls, numFeatures, capacity_rows, capacity_nnz, labels=False, weights=False):
        h = ctypes.c_void_p()
        N.check(N.load().cyc_dataset_csr_create(numFeatures, capacity_rows, capacity_nnz,
                                                int(labels), int(weights), ctypes.byref(h)))
        return cls(h, numFeatures)

    def close(self):
        if self._h is not None and self._h.value:
            N.load().cyc_dataset_destroy(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def numRows(self):
        return int(N.load().cyc_dataset_rows(self._h))

    def append_dense(self, X, labels=None, weights=None):
        X = np.ascontiguousarray(X, dtype=np.float64)
        if X.ndim != 2 or X.shape[1] != self.numFeatures:
            raise N.IllegalArgumentException(
                f"requirement failed: expected rows of {self.numFeatures} features")
        labels, weights = _f64(labels), _f64(weights)
        N.check(N.load().cyc_dataset_append_dense(self._h, _p(X), _p(labels), _p(weights),
                                                  X.shape[0]))
        return self

    def append_csr(self, rowptr, colidx, values, labels=None, weights=None):
        rowptr = np.ascontiguousarray(rowptr, dtype=np.int64)
        colidx = np.ascontiguousarray(colidx, dtype=np.int32)
        values = _f64(values)
        labels, weights = _f64(labels), _f64(weights)
        N.check(N.load().cyc_dataset_append_csr(self._h, _p(rowptr), _p(colidx), _p(values),
                                                _p(labels), _p(weights), rowptr.size - 1))
        return self

    # ---- per-iteration entry points (outputs are ADDED to)
    def kmeans_iter(self, centers, sums=None, wsum=None, cost=None, want_assign=False,
                    distanceMeasure="euclidean", center_norms=None):
        """One partition of a Lloyd iteration (KMeans.scala:287-311) with the
        given DistanceMeasure; center_norms: the centers' VectorWithNorm
        norms (None = computed)."""
        from .clustering import _decode_measure
        measure = _decode_measure(distanceMeasure)
        centers = np.ascontiguousarray(centers, dtype=np.float64)
        k, d = centers.shape
        sums = np.zeros((k, d)) if sums is None else sums
        wsum = np.zeros(k) if wsum is None else wsum
        cost = np.zeros(1) if cost is None else cost
        assign = np.empty(self.numRows, dtype=np.int32) if want_assign else None
        cn = None if center_norms is None else np.ascontiguousarray(center_norms,
                                                                   dtype=np.float64)
        N.check(N.load().cyc_kmeans_iter_measure(self._h, measure, _p(centers), _p(cn), k,
                                                 _p(sums), _p(wsum), _p(cost), _p(assign)))
        return sums, wsum, cost, assign

    def _logreg(self, C, coef, fi, fwm, scaledMean, grad, loss_weight):
        coef = _f64(coef)
        grad = np.zeros(coef.size) if grad is None else grad
        lw = np.zeros(2) if loss_weight is None else loss_weight
        sm = _f64(scaledMean)
        lib = N.load()
        l_p = ctypes.c_void_p(lw.ctypes.data)
        w_p = ctypes.c_void_p(lw.ctypes.data + 8)
        if C == 1:
            rc = lib.cyc_logreg_binary_eval(self._h, _p(coef), int(fi), int(fwm), _p(sm),
                                            _p(grad), l_p, w_p)
        else:
            rc = lib.cyc_logreg_multinomial_eval(self._h, C, _p(coef), int(fi), int(fwm), _p(sm),
                                                 _p(grad), l_p, w_p)
        N.check(rc)
        return grad, lw

    def binary_logistic_eval(self, coef, fitIntercept, fitWithMean=False, scaledMean=None,
                             grad=None, loss_weight=None):
        """RDDLossFunction seqOp with BinaryLogisticBlockAggregator.add.
        Returns (grad, [lossSum, weightSum])."""
        return self._logreg(1, coef, fitIntercept, fitWithMean, scaledMean, grad, loss_weight)

    def multinomial_logistic_eval(self, numClasses, coef, fitIntercept, fitWithMean=False,
                                  scaledMean=None, grad=None, loss_weight=None):
        return self._logreg(numClasses, coef, fitIntercept, fitWithMean, scaledMean, grad,
                            loss_weight)

    def _linear(self, fn, coef, args_before, args_after, grad, loss_weight):
        coef = _f64(coef)
        grad = np.zeros(coef.size) if grad is None else grad
        lw = np.zeros(2) if loss_weight is None else loss_weight
        l_p = ctypes.c_void_p(lw.ctypes.data)
        w_p = ctypes.c_void_p(lw.ctypes.data + 8)
        N.check(fn(self._h, _p(coef), *args_before, *args_after, _p(grad), l_p, w_p))
        return grad, lw

    def hinge_eval(self, coef, fitIntercept, scaledMean=None, grad=None, loss_weight=None):
        """RDDLossFunction seqOp with HingeBlockAggregator.add (LinearSVC)."""
        return self._linear(N.load().cyc_svc_hinge_eval, coef, (int(fitIntercept),),
                            (_p(_f64(scaledMean)),), grad, loss_weight)

    def least_squares_eval(self, coef, inverseStd, fitIntercept, labelStd, labelMean,
                           scaledMean=None, grad=None, loss_weight=None):
        """... with LeastSquaresBlockAggregator.add (LinearRegression, dim F)."""
        inv = _f64(inverseStd)
        return self._linear(N.load().cyc_linreg_least_squares_eval, coef,
                            (_p(inv), int(fitIntercept), float(labelStd), float(labelMean)),
                            (_p(_f64(scaledMean)),), grad, loss_weight)

    def huber_eval(self, params, fitIntercept, epsilon, scaledMean=None, grad=None,
                   loss_weight=None):
        """... with HuberBlockAggregator.add (params: linear, intercept, sigma)."""
        return self._linear(N.load().cyc_linreg_huber_eval, params,
                            (int(fitIntercept), float(epsilon)), (_p(_f64(scaledMean)),), grad,
                            loss_weight)

    def aft_eval(self, coef, fitIntercept, scaledMean=None, grad=None, loss_weight=None):
        """... with AFTBlockAggregator.add (the dataset's weights are censors)."""
        return self._linear(N.load().cyc_aft_eval, coef, (int(fitIntercept),),
                            (_p(_f64(scaledMean)),), grad, loss_weight)

    def gramian(self, mean=None, U=None):
        """Packed upper Gramian (RowMatrix.scala:130-161); centered if mean."""
        n = self.numFeatures
        U = np.zeros(n * (n + 1) // 2) if U is None else U
        N.check(N.load().cyc_gramian(self._h, _p(_f64(mean)), _p(U)))
        return U

    def col_sums(self, sums=None):
        sums = np.zeros(self.numFeatures) if sums is None else sums
        N.check(N.load().cyc_col_sums(self._h, _p(sums)))
        return sums
