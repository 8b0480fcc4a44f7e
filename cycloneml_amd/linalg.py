"""RowMatrix on MI355X: host-side mirror of
mllib/linalg/distributed/RowMatrix.scala (Gramian, covariance, PCA).

`rows` is this rank's device-resident shard: a torch fp64 CUDA tensor (n x p,
row-major: an RDD of DenseVector rows) or a CSRRows triple (an RDD of
SparseVector rows; rowptr int64, colidx int32, values fp64).  computeGramianMatrix /
computeCovariance run the fp64-MFMA syrk of libcyclone and, when
torch.distributed is initialised, merge the packed triangle with one
all-reduce (the treeAggregate combOp U1 += U2, :149-157).  The eigensolve of
PCA stays on the host (breeze svd on the driver in the reference, :501).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native as N
from . import parallel


def _torch():
    import torch
    return torch


def _dist():
    torch = _torch()
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        return torch.distributed
    return None


class GramianPlan:
    def __init__(self, ncols):
        self._lib = N.load()
        h = ctypes.c_void_p()
        N.check(self._lib.cyc_gramian_plan_create(int(ncols), ctypes.byref(h)))
        self.handle = h
        self.p = int(ncols)

    def close(self):
        if self.handle:
            self._lib.cyc_gramian_plan_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def accumulate(self, X, U, mean=None, stream=None):
        N.check(self._lib.cyc_gramian_accumulate_dev(self.handle, N.ptr(X), int(X.shape[0]),
                                                     N.ptr(mean), N.ptr(U),
                                                     N.stream_handle(stream)))

    def col_sums(self, X, out, stream=None):
        N.check(self._lib.cyc_col_sums_dev(self.handle, N.ptr(X), int(X.shape[0]), N.ptr(out),
                                           N.stream_handle(stream)))

    def accumulate_csr(self, rows: "CSRRows", U, mean=None, stream=None):
        N.check(self._lib.cyc_gramian_accumulate_csr_dev(
            self.handle, N.ptr(rows.rowptr), N.ptr(rows.colidx), N.ptr(rows.values), rows.n,
            N.ptr(mean), N.ptr(U), N.stream_handle(stream)))

    def col_sums_csr(self, rows: "CSRRows", out, stream=None):
        N.check(self._lib.cyc_col_sums_csr_dev(
            self.handle, N.ptr(rows.rowptr), N.ptr(rows.colidx), N.ptr(rows.values), rows.n,
            N.ptr(out), N.stream_handle(stream)))


class CSRRows:
    """SparseVector rows of a RowMatrix shard in HBM (CSR, rowptr may start at
    any base)."""

    def __init__(self, rowptr, colidx, values, numCols: int):
        self.rowptr, self.colidx, self.values = rowptr, colidx, values
        self.numCols = int(numCols)
        self.n = int(rowptr.shape[0]) - 1
        self.device = values.device


def triu_to_full(n, U, stream=None):
    """RowMatrix.triuToFull (:845-867) on device; returns the (n, n) matrix."""
    torch = _torch()
    G = torch.empty(n * n, dtype=torch.float64, device=U.device)
    N.check(N.load().cyc_triu_to_full_dev(int(n), N.ptr(U), N.ptr(G), N.stream_handle(stream)))
    return G.view(n, n).t()   # column-major storage -> G[i, j]


class RowMatrix:
    """RowMatrix(rows) over a device-resident shard (dense tensor or CSRRows)."""

    def __init__(self, rows, nRows: int = 0, nCols: int = 0):
        self.rows = rows
        self._nRows = nRows
        self._nCols = nCols
        self._plan_ = None

    def close(self):
        """Release the cached syrk plan and its split-K slab in HBM (about
        0.3-0.5 GB at n = 1024).  The host-returning compute* methods call
        it on return; the *Device / *Packed forms keep the plan for the
        next pass (a loop over passes, as bench.py's), until close()."""
        if self._plan_ is not None:
            self._plan_.close()
            self._plan_ = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _plan(self) -> GramianPlan:
        """One syrk plan per matrix: its split-K slab is reused by every pass
        until close()."""
        n = self.numCols()
        if self._plan_ is None or self._plan_.p != n:
            self._plan_ = GramianPlan(n)
        return self._plan_

    @property
    def _sparse(self):
        return isinstance(self.rows, CSRRows)

    @property
    def _device(self):
        return self.rows.device

    def _local_rows(self):
        return self.rows.n if self._sparse else int(self.rows.shape[0])

    def numCols(self) -> int:
        if self._nCols <= 0:
            if self._sparse:
                self._nCols = self.rows.numCols
            else:
                if self.rows.shape[0] == 0 and _dist() is None:
                    raise RuntimeError("Cannot determine the number of cols because it is not "
                                       "specified in the constructor and the rows RDD is empty.")
                self._nCols = int(self.rows.shape[1])
        return self._nCols

    def numRows(self) -> int:
        if self._nRows <= 0:
            n = self._local_rows()
            d = _dist()
            if d is not None:
                t = _torch().tensor([n], dtype=_torch().int64, device=self._device)
                d.all_reduce(t)
                n = int(t.item())
            if n == 0:
                raise RuntimeError("Cannot determine the number of rows because it is not "
                                   "specified in the constructor and the rows RDD is empty.")
            self._nRows = n
        return self._nRows

    @staticmethod
    def _checkNumColumns(cols):
        if cols > 65535:
            raise N.IllegalArgumentException(f"Argument with more than 65535 cols: {cols}")

    def _packed(self, mean=None):
        torch = _torch()
        n = self.numCols()
        self._checkNumColumns(n)
        U = torch.zeros(n * (n + 1) // 2, dtype=torch.float64, device=self._device)
        plan = self._plan()
        if self._sparse:
            plan.accumulate_csr(self.rows, U, mean)
        else:
            plan.accumulate(self.rows, U, mean)
        parallel.allreduce_(U)             # treeAggregate combOp U1 += U2
        return U

    def computeGramianMatrixPacked(self):
        return self._packed()

    def computeGramianMatrix(self) -> np.ndarray:
        """RowMatrix.scala:130-161; returns the full n x n matrix (host)."""
        n = self.numCols()
        try:
            return triu_to_full(n, self._packed()).cpu().numpy()
        finally:
            self.close()

    def _column_mean(self):
        torch = _torch()
        n = self.numCols()
        s = torch.zeros(n, dtype=torch.float64, device=self._device)
        if self._sparse:
            self._plan().col_sums_csr(self.rows, s)
        else:
            self._plan().col_sums(self.rows, s)
        parallel.allreduce_(s)
        m = self.numRows()
        return s / m, m

    # rows of the first isSparseMatrix round per rank, and the growth factor
    SPARSITY_SCAN_FIRST = 1 << 16
    SPARSITY_SCAN_GROWTH = 4

    def _dense_rows(self, a: int, b: int):
        """Rows of [a, b) of this shard with sparsity() < 0.5 (device count)."""
        torch = _torch()
        cnt = torch.zeros(1, dtype=torch.int64, device=self._device)
        if b > a:
            if self._sparse:
                N.check(N.load().cyc_rowmatrix_dense_rows_dev(
                    None, N.ptr(self.rows.rowptr[a:b + 1]), N.ptr(self.rows.values), b - a,
                    self.numCols(), N.ptr(cnt), N.stream_handle()))
            else:
                N.check(N.load().cyc_rowmatrix_dense_rows_dev(
                    N.ptr(self.rows[a:b]), None, None, b - a, self.numCols(), N.ptr(cnt),
                    N.stream_handle()))
        return cnt

    def isSparseMatrix(self) -> bool:
        """RowMatrix.isSparseMatrix (:439-442): rows.filter(_.sparsity() < 0.5)
        .isEmpty().  isEmpty is take(1) (RDD.scala:1577-1579, :1443-1478): Spark
        scans one partition, then 4x as many (the scale-up factor) and so on,
        only until one dense row turns up, so a dense matrix costs it one row.
        Here every rank scans its shard in growing row
        ranges (SPARSITY_SCAN_FIRST rows, then x SPARSITY_SCAN_GROWTH) and one
        all-reduce per round of [dense rows found, rows left] stops all ranks
        together at the first round that finds one (over all ranks)."""
        torch = _torch()
        n = self._local_rows()
        a, size = 0, self.SPARSITY_SCAN_FIRST
        while True:
            b = min(n, a + size)
            t = torch.zeros(2, dtype=torch.float64, device=self._device)
            t[0] = self._dense_rows(a, b)[0]
            t[1] = n - b
            parallel.allreduce_(t)
            found, left = t.tolist()
            if found > 0:
                return False
            if left == 0:
                return True
            a, size = b, size * self.SPARSITY_SCAN_GROWTH

    def computeCovariance(self) -> np.ndarray:
        """RowMatrix.scala:452-467: computeDenseVectorCovariance (:163-220) or,
        when every row has sparsity >= 0.5, computeSparseVectorCovariance
        (:222-246) from the Gramian."""
        try:
            return self.computeCovarianceDevice().cpu().numpy()
        finally:
            self.close()

    def computeCovarianceDevice(self):
        """computeCovariance with the n x n result left in HBM (a torch view
        G[i, j] of the column-major matrix)."""
        torch = _torch()
        n = self.numCols()
        self._checkNumColumns(n)
        mean, m = self._column_mean()
        if not m > 1:
            raise N.IllegalArgumentException(
                f"RowMatrix.computeCovariance called on matrix with only {m} rows.  Cannot "
                "compute the covariance of a RowMatrix with <= 1 row.")
        G = torch.empty(n * n, dtype=torch.float64, device=self._device)
        if not self.isSparseMatrix():
            U = self._packed(mean)
            N.check(N.load().cyc_covariance_finalize_dev(int(n), N.ptr(U), int(m), N.ptr(G),
                                                         N.stream_handle()))
        else:
            U = self._packed()
            N.check(N.load().cyc_sparse_covariance_finalize_dev(
                int(n), N.ptr(U), int(m), N.ptr(mean), N.ptr(G), N.stream_handle()))
        return G.view(n, n).t()

    def computePrincipalComponentsAndExplainedVariance(self, k: int):
        """RowMatrix.scala:486-513 (n <= 65535 branch); eigensolve on host."""
        n = self.numCols()
        if not (0 < k <= n):
            raise N.IllegalArgumentException(f"k = {k} out of range (0, n = {n}]")
        cov = self.computeCovariance()
        u, s, _ = np.linalg.svd(cov)
        explained = s / s.sum()
        return u[:, :k].copy(), explained[:k].copy()

    def computePrincipalComponents(self, k: int):
        return self.computePrincipalComponentsAndExplainedVariance(k)[0]
