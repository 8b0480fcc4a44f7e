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
import os

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

    def col_moments(self, X, sums, sumsq, stream=None):
        N.check(self._lib.cyc_col_moments_dev(self.handle, N.ptr(X), int(X.shape[0]),
                                              N.ptr(sums), N.ptr(sumsq),
                                              N.stream_handle(stream)))

    def col_moments_csr(self, rows: "CSRRows", sums, sumsq, stream=None):
        N.check(self._lib.cyc_col_moments_csr_dev(
            self.handle, N.ptr(rows.rowptr), N.ptr(rows.colidx), N.ptr(rows.values), rows.n,
            N.ptr(sums), N.ptr(sumsq), N.stream_handle(stream)))

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
        mean, m, _ = self._column_moments(squares=False)
        return mean, m

    def _column_moments(self, squares=True, rows=None):
        """(mean, m, sum of squares or None): the colStats pass (:456) -- the
        column sums, and beside them in the same pass the sums of squares
        -- merged over ranks; over `rows` (a leading slice of this shard,
        with m their count over ranks) when given."""
        torch = _torch()
        n = self.numCols()
        s = torch.zeros(2 * n + 1 if squares else n, dtype=torch.float64, device=self._device)
        sq = s[n:2 * n] if squares else None
        rows = self.rows if rows is None else rows
        if self._sparse:
            self._plan().col_moments_csr(rows, s[:n], sq)
        else:
            self._plan().col_moments(rows, s[:n], sq)
        if rows is self.rows:
            parallel.allreduce_(s)         # one all-reduce for both
            m = self.numRows()
        else:
            s[2 * n] = rows.n if self._sparse else int(rows.shape[0])
            parallel.allreduce_(s)
            m = int(s[2 * n].item())
        return s[:n] / max(m, 1), m, sq

    def _packed_sums(self):
        """(U, sums): the plain syrk with the column sums riding it (one pass
        over dense rows, cyc_gramian_accumulate_sums_dev; CSR rows add the
        column-sum pass), merged over ranks in one all-reduce."""
        torch = _torch()
        n = self.numCols()
        nt = n * (n + 1) // 2
        B = torch.zeros(nt + n, dtype=torch.float64, device=self._device)
        U, S = B[:nt], B[nt:]
        plan = self._plan()
        if self._sparse:
            plan.accumulate_csr(self.rows, U)
            plan.col_sums_csr(self.rows, S)
        else:
            N.check(plan._lib.cyc_gramian_accumulate_sums_dev(
                plan.handle, N.ptr(self.rows), int(self.rows.shape[0]), N.ptr(U), N.ptr(S),
                N.stream_handle()))
        parallel.allreduce_(B)
        return U, S

    # computeCovariance's dense form: "auto" (below), "centred" (the
    # reference's centred spr, always) or "uncentred" (the Gramian finish,
    # always; for tests).  CYC_COV_FORM sets the default.
    covarianceForm = os.environ.get("CYC_COV_FORM", "auto")
    # the uncentred form needs mean^2 <= COV_MEAN_RATIO2 * variance in every
    # column; "auto" first checks the leading COV_SAMPLE_ROWS rows of each
    # shard to pick the pass order
    COV_MEAN_RATIO2 = 64.0
    COV_SAMPLE_ROWS = 1 << 16

    def _near_centred(self, mean, sumsq, m) -> bool:
        """The bound that lets the dense covariance skip the centring.  The
        reference centres every row (computeDenseVectorCovariance,
        :163-220) so that a large mean cannot cancel; the uncentred Gramian
        finish -- the reference's own computeSparseVectorCovariance formula
        (:222-246), G / (m-1) - m/(m-1) mean_i mean_j -- costs the plain syrk
        instead of the centred one, and its cancellation is bounded by the
        data: sum x_i^2 = (m-1) var_i + m mean_i^2, so with mean_i^2 <= R
        var_i for every column the rounding error of each entry is at most
        (1 + R m/(m-1)) times the centred form's, in units of sqrt(var_i
        var_j) (R = 64: ~65x an error of a few ulp, far inside the 1e-10 the
        parity tests hold).  A column failing it (a large mean, zero
        variance, NaN/Inf) keeps the whole matrix centred.  Every rank sees
        the same merged moments, so every rank decides the same."""
        var = (sumsq - m * mean * mean) / (m - 1)
        return bool((mean * mean <= self.COV_MEAN_RATIO2 * var).all().item())

    def _dense_covariance(self, m, G):
        """The dense covariance into G; returns (form, passes over the rows).
        "auto": the leading rows' moments choose the order --
          near-centred: the plain syrk with the column sums riding it, the
          exact bound from its diagonal (sum x_i^2) and sums, and the
          centred syrk after it only if the whole matrix fails the bound;
          otherwise: the moments pass, then the form the bound allows."""
        torch = _torch()
        n = self.numCols()
        form = self.covarianceForm
        from .config import strict_parity
        if strict_parity() and form == "auto":
            form = "centred"          # CYCLONE_STRICT_PARITY: the reference's dense form
        if form not in ("auto", "centred", "uncentred"):
            raise N.IllegalArgumentException(f"covarianceForm {form!r}: auto, centred or "
                                             "uncentred")
        lib = N.load()
        passes = []

        def centred(mean):
            passes.append("centred syrk")
            U = self._packed(mean)
            N.check(lib.cyc_covariance_finalize_dev(int(n), N.ptr(U), int(m), N.ptr(G),
                                                    N.stream_handle()))
            return "centred", passes

        def uncentred(U, mean):
            N.check(lib.cyc_sparse_covariance_finalize_dev(int(n), N.ptr(U), int(m),
                                                           N.ptr(mean), N.ptr(G),
                                                           N.stream_handle()))
            return "uncentred", passes

        if form == "centred":
            passes.append("column sums")
            return centred(self._column_moments(squares=False)[0])
        sample_ok = form == "uncentred"
        if form == "auto":
            k = min(self._local_rows(), self.COV_SAMPLE_ROWS)
            if self._sparse:
                r = self.rows
                head = CSRRows(r.rowptr[:k + 1], r.colidx, r.values, r.numCols)
            else:
                head = self.rows[:k]
            passes.append(f"moments of the leading {k} rows")
            ms, mk, sqs = self._column_moments(rows=head)
            sample_ok = mk > 1 and self._near_centred(ms, sqs, mk)
        if sample_ok:
            passes.append("syrk + column sums")
            U, S = self._packed_sums()
            mean = S / m
            if form == "uncentred":
                return uncentred(U, mean)
            i = torch.arange(n, device=self._device)
            if self._near_centred(mean, U[i * (i + 1) // 2 + i], m):
                return uncentred(U, mean)
            return centred(mean)
        passes.append("column moments")
        mean, _, sumsq = self._column_moments()
        if self._near_centred(mean, sumsq, m):
            passes.append("syrk")
            return uncentred(self._packed(), mean)
        return centred(mean)

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
        (:222-246) from the Gramian.  The dense form is the centred syrk, or
        the Gramian finish when the column moments bound its cancellation
        (_near_centred, _dense_covariance); lastCovarianceForm names the one
        that ran, lastCovariancePasses the passes over the rows."""
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
        m = self.numRows()
        if not m > 1:
            raise N.IllegalArgumentException(
                f"RowMatrix.computeCovariance called on matrix with only {m} rows.  Cannot "
                "compute the covariance of a RowMatrix with <= 1 row.")
        G = torch.empty(n * n, dtype=torch.float64, device=self._device)
        if not self.isSparseMatrix():
            form, passes = self._dense_covariance(m, G)
        else:                              # the Gramian finish (:222-246)
            mean = self._column_mean()[0]
            U = self._packed()
            N.check(N.load().cyc_sparse_covariance_finalize_dev(
                int(n), N.ptr(U), int(m), N.ptr(mean), N.ptr(G), N.stream_handle()))
            form, passes = "sparse", ["column sums", "syrk"]
        self.lastCovarianceForm, self.lastCovariancePasses = form, passes
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
