"""Logistic-regression loss aggregation on MI355X.

Host-side mirror of
  ml/optim/aggregator/DifferentiableLossAggregator.scala:30-80
  ml/optim/aggregator/BinaryLogisticBlockAggregator.scala:41-146
  ml/optim/aggregator/MultinomialLogisticBlockAggregator.scala:45-190
  ml/optim/loss/RDDLossFunction.scala:47-70 (+ L2Regularization)
with the same names, argument meaning and `require` messages.  A "block" is
a device-resident InstanceBlock (ml/feature/Instance.scala:39-106): all
blocks of a shard concatenated into one dense row-major (n x F) tensor or one
CSR triple, with labels and optional weights (None = the empty weights array
of an all-unit-weight block).  `add` runs the whole shard through
libcyclone's aggregator kernels; `merge` and `RDDLossFunction.calculate`
reproduce treeAggregate, with an RCCL all-reduce across ranks.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native as N
from . import parallel


def _torch():
    import torch
    return torch


class SparseTiles:
    """RAII wrapper of cyc_tiles: the row-block x column-tile layout of a CSR
    shard (cycloneml_amd/csrc/tiles.hip) that the binary aggregators' sparse
    path runs on -- 12 B per nonzero (format "wide") or 10 B per entry
    ("compact": 16-bit ids, ~1-3 % filler entries; "auto" picks it for dense
    enough segments), built by appending CSR rows (whole row blocks of
    ROW_BLOCK rows, except the last append); the CSR can be freed
    afterwards."""

    ROW_BLOCK = 2048          # cyc_tiles_row_block()
    FORMATS = {"auto": 0, "wide": 1, "compact": 2}   # CYC_TILES_AUTO / WIDE / COMPACT

    def __init__(self, numFeatures: int, capacity_rows: int, capacity_nnz: int,
                 format: str = "auto"):
        self._lib = N.load()
        h = ctypes.c_void_p()
        N.check(self._lib.cyc_tiles_create(int(numFeatures), int(capacity_rows),
                                           int(capacity_nnz), ctypes.byref(h)))
        self.handle = h
        self.numFeatures = int(numFeatures)
        if format not in self.FORMATS:
            raise ValueError(f"format must be one of {sorted(self.FORMATS)}")
        if format != "auto":
            N.check(self._lib.cyc_tiles_set_format(self.handle, self.FORMATS[format]))

    def append(self, rowptr, colidx, values, stream=None):
        n = int(rowptr.shape[0]) - 1
        N.check(self._lib.cyc_tiles_append_dev(self.handle, N.ptr(rowptr), N.ptr(colidx),
                                               N.ptr(values), n, N.stream_handle(stream)))
        return self

    @staticmethod
    def from_csr(rowptr, colidx, values, numFeatures, stream=None, format="auto"):
        n = int(rowptr.shape[0]) - 1
        t = SparseTiles(numFeatures, n, int(colidx.shape[0]), format=format)
        return t.append(rowptr, colidx, values, stream)

    @property
    def format(self):
        """"wide" / "compact" once decided ("auto" before the first append)."""
        f = int(self._lib.cyc_tiles_format(self.handle))
        return {v: k for k, v in self.FORMATS.items()}[f]

    @property
    def entries(self):
        return int(self._lib.cyc_tiles_entries(self.handle))

    @property
    def rows(self):
        return int(self._lib.cyc_tiles_rows(self.handle))

    @property
    def nnz(self):
        return int(self._lib.cyc_tiles_nnz(self.handle))

    @property
    def nbytes(self):
        return int(self._lib.cyc_tiles_bytes(self.handle))

    def close(self):
        if getattr(self, "handle", None):
            self._lib.cyc_tiles_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceInstanceBlock:
    """InstanceBlock rows resident in HBM (dense or CSR, isTransposed=true).
    A sparse block may hold its CSR arrays, a SparseTiles layout, or both
    (prepare(layout="tiles") derives the layout; release_csr() then drops the
    CSR so the layout is the only copy)."""

    def __init__(self, labels, weights=None, X=None, rowptr=None, colidx=None, values=None,
                 numFeatures=None, tiles=None):
        self.labels = labels
        self.weights = weights
        self.X = X
        self.rowptr, self.colidx, self.values = rowptr, colidx, values
        self.tiles = tiles
        if X is not None:
            self.numFeatures = int(X.shape[1])
            self.size = int(X.shape[0])
        else:
            if numFeatures is None:
                raise N.IllegalArgumentException("numFeatures is required for CSR blocks")
            self.numFeatures = int(numFeatures)
            self.size = int(rowptr.shape[0]) - 1 if rowptr is not None else tiles.rows
        if int(labels.shape[0]) != self.size:
            raise N.IllegalArgumentException("requirement failed")  # Instance.scala:43
        if weights is not None and int(weights.shape[0]) != self.size:
            raise N.IllegalArgumentException("requirement failed")  # Instance.scala:46

        self.csc = None

    @property
    def is_sparse(self):
        return self.X is None

    def prepare(self, stream=None, layout="csc", tiles_format="auto"):
        """Derive a layout of a CSR shard once, outside the training loop.
        layout="csc": the row-blocked column-major copy (cyc_csc_build_dev)
        the multinomial / summarizer CSR paths use (12 bytes per nonzero of
        HBM); layout="tiles": the row-block x column-tile layout
        (SparseTiles, entry format `tiles_format`: 12 bytes per nonzero
        wide, ~10 compact) the binary aggregators run on."""
        if self.is_sparse and layout == "tiles":
            if self.tiles is None:
                self.tiles = SparseTiles.from_csr(self.rowptr, self.colidx, self.values,
                                                  self.numFeatures, stream, format=tiles_format)
            return self
        if self.is_sparse and self.csc is None:
            h = ctypes.c_void_p()
            N.check(N.load().cyc_csc_build_dev(N.ptr(self.rowptr), N.ptr(self.colidx),
                                               N.ptr(self.values), self.size, self.numFeatures,
                                               N.stream_handle(stream), ctypes.byref(h)))
            self.csc = h
        return self

    def release_csr(self):
        """Drop the CSR arrays (and a CSC copy) once the tiles layout exists:
        the binary aggregators then read only the layout."""
        if self.tiles is None:
            raise N.IllegalArgumentException("prepare(layout='tiles') first")
        self.drop_derived()
        self.rowptr = self.colidx = self.values = None

    def drop_derived(self):
        """Forget the CSC copy (after the values change, e.g. standardization)."""
        if getattr(self, "csc", None):
            N.load().cyc_csc_destroy(self.csc)
            self.csc = None

    def __del__(self):
        try:
            if getattr(self, "csc", None):
                N.load().cyc_csc_destroy(self.csc)
                self.csc = None
        except Exception:
            pass

    @staticmethod
    def from_numpy(labels, weights=None, X=None, csr=None, numFeatures=None, device="cuda"):
        torch = _torch()
        t = lambda a, dt: None if a is None else torch.as_tensor(np.ascontiguousarray(a, dtype=dt), device=device)
        if csr is not None:
            rp, ci, v = csr
            return DeviceInstanceBlock(t(labels, np.float64), t(weights, np.float64),
                                       rowptr=t(rp, np.int64), colidx=t(ci, np.int32),
                                       values=t(v, np.float64), numFeatures=numFeatures)
        return DeviceInstanceBlock(t(labels, np.float64), t(weights, np.float64),
                                   X=t(X, np.float64))


def blokify(block: "DeviceInstanceBlock", maxBlockSizeInMB: float = 1.0, stream=None):
    """InstanceBlock.blokifyWithMaxMemUsage (ml/feature/Instance.scala:146-187)
    over a device shard with maxMemUsage = ceil(maxBlockSizeInMB * 2^20)
    (LogisticRegression.scala:967): (starts int64[nblocks + 1], dense
    bool[nblocks]) as device tensors -- the reference's block boundaries and
    each block's dense-or-CSR storage, computed where the rows live."""
    import math
    torch = _torch()
    if block.rowptr is None and block.X is None:
        raise N.IllegalArgumentException("blokify needs the block's rows (dense or CSR)")
    maxMem = int(math.ceil(maxBlockSizeInMB * 1024 * 1024))
    dev = block.labels.device
    n = block.size
    starts = torch.empty(n + 1, dtype=torch.int64, device=dev)
    dense = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
    nb = torch.empty(1, dtype=torch.int64, device=dev)
    N.check(N.load().cyc_blokify_dev(N.ptr(block.X), N.ptr(block.rowptr), N.ptr(block.values),
                                     N.ptr(block.weights), n, block.numFeatures, maxMem,
                                     N.ptr(starts), N.ptr(dense), N.ptr(nb),
                                     N.stream_handle(stream)))
    k = int(nb.item())
    return starts[:k + 1], dense[:k].bool()


_PLANS = {}
_PINNED = {}


def _pinned(n):
    """Page-locked host staging of n doubles, reused per size: the per-
    evaluation model broadcast (host -> HBM) and gradient collect (HBM ->
    host) go by DMA instead of through pageable bounce copies."""
    torch = _torch()
    t = _PINNED.get(n)
    if t is None:
        t = _PINNED[n] = torch.empty(n, dtype=torch.float64, pin_memory=True)
    return t


def _upload(a, device):
    """Host coefficients -> a fresh device tensor (synchronous copy from the
    pinned staging buffer, so the buffer is free again on return)."""
    torch = _torch()
    a = np.ascontiguousarray(a, dtype=np.float64).ravel()
    dev = torch.device(device)
    if dev.type != "cuda" or a.size == 0:
        return torch.as_tensor(a, device=dev)
    st = _pinned(a.size)
    st.copy_(torch.from_numpy(a))   # torch's threaded copy (8 MB: 0.4 vs 1.1 ms)
    out = torch.empty(a.size, dtype=torch.float64, device=dev)
    out.copy_(st)
    return out


def _dev_vector(x, device):
    """bcScaledMean-style model constants on the device: a device tensor is
    used as is (the caller broadcast it once), host arrays are uploaded."""
    if x is None:
        return None
    torch = _torch()
    if torch.is_tensor(x):
        return x.to(device=device, dtype=torch.float64)
    return torch.as_tensor(np.asarray(x, dtype=np.float64), device=device)


def _download(t):
    """Device vector -> new host numpy array via the pinned staging buffer."""
    if t.device.type != "cuda" or t.numel() == 0:
        return t.cpu().numpy().copy()
    torch = _torch()
    st = _pinned(t.numel())
    st.copy_(t)
    # out of the staging buffer by torch's threaded copy (8 MB: 0.5 vs 0.9 ms)
    return torch.empty(t.numel(), dtype=torch.float64).copy_(st).numpy()


def _logistic_plan(F, C, fit_intercept, fit_with_mean, device, hinge=False):
    """Plans own device scratch; one per shape and device, reused across the
    aggregators RDDLossFunction creates every evaluation."""
    key = (int(F), int(C), bool(fit_intercept), bool(fit_with_mean), str(device), bool(hinge))
    p = _PLANS.get(key)
    if p is None:
        p = _PLANS[key] = _LogisticPlan(F, C, fit_intercept, fit_with_mean, hinge)
    return p


class _LogisticPlan:
    def __init__(self, F, C, fit_intercept, fit_with_mean, hinge=False):
        self._lib = N.load()
        h = ctypes.c_void_p()
        if hinge:
            N.check(self._lib.cyc_hinge_plan_create(int(F), int(bool(fit_intercept)),
                                                    ctypes.byref(h)))
        else:
            N.check(self._lib.cyc_logistic_plan_create(int(F), int(C), int(bool(fit_intercept)),
                                                       int(bool(fit_with_mean)),
                                                       ctypes.byref(h)))
        self.handle = h

    def __del__(self):
        try:
            if self.handle:
                self._lib.cyc_logistic_plan_destroy(self.handle)
                self.handle = None
        except Exception:
            pass


class DifferentiableLossAggregator:
    """State {weightSum, lossSum, gradientSumArray} kept on the device."""

    dim: int

    def _init_state(self, device):
        torch = _torch()
        self._state = torch.zeros(self.dim + 2, dtype=torch.float64, device=device)

    @property
    def gradientSumArray(self):
        return self._state[:self.dim]

    @property
    def _loss_sum(self):
        return self._state[self.dim:self.dim + 1]

    @property
    def _weight_sum(self):
        return self._state[self.dim + 1:self.dim + 2]

    @property
    def weight(self) -> float:
        return float(self._state[self.dim + 1].item())

    def merge(self, other):
        """DifferentiableLossAggregator.scala:49-59"""
        if self.dim != other.dim:
            raise N.IllegalArgumentException(
                f"Dimensions mismatch when merging with another {type(self).__name__}. "
                f"Expecting {self.dim} but got {other.dim}.")
        if other.weight != 0:
            self._state += other._state
        return self

    def allreduce(self, group=None):
        """treeAggregate across ranks: one RCCL (or gloo) all-reduce of the
        [gradientSum | lossSum | weightSum] buffer."""
        parallel.allreduce_(self._state, group=group)
        return self

    @property
    def gradient(self) -> np.ndarray:
        """DifferentiableLossAggregator.scala:62-68"""
        ws = self.weight
        if not ws > 0.0:
            raise N.IllegalArgumentException(
                f"The effective number of instances should be greater than 0.0, but was {ws}.")
        # BLAS.scal(1.0 / weightSum, ...) on the device, then one copy out
        return _download(self.gradientSumArray * (1.0 / ws))

    @property
    def loss(self) -> float:
        """DifferentiableLossAggregator.scala:74-78"""
        ws = self.weight
        if not ws > 0.0:
            raise N.IllegalArgumentException(
                f"The effective number of instances should be greater than 0.0, but was {ws}.")
        return float(self._state[self.dim].item()) / ws


def _check_block(agg, block):
    if agg.numFeatures != block.numFeatures:
        raise N.IllegalArgumentException(
            "Dimensions mismatch when adding new instance. Expecting "
            f"{agg.numFeatures} but got {block.numFeatures}.")
    if block.weights is not None and bool((block.weights < 0).any().item()):
        w = block.weights.cpu().numpy()
        raise N.IllegalArgumentException(
            f"instance weights {'[' + ','.join(map(str, w)) + ']'} has to be >= 0.0")


def _tiles_add(agg, block, stream, inverseStd=None):
    """The binary aggregators' add over a block's SparseTiles layout
    (cyc_binary_add_tiles_dev; the plan carries the loss kind)."""
    N.check(N.load().cyc_binary_add_tiles_dev(
        agg._plan.handle, block.tiles.handle, N.ptr(block.labels), N.ptr(block.weights),
        N.ptr(agg.coef), N.ptr(inverseStd), N.ptr(agg.scaledMean),
        N.ptr(agg.gradientSumArray), N.ptr(agg._loss_sum), N.ptr(agg._weight_sum),
        N.stream_handle(stream)))
    return agg


class BinaryLogisticBlockAggregator(DifferentiableLossAggregator):
    """BinaryLogisticBlockAggregator(bcInverseStd, bcScaledMean, fitIntercept,
    fitWithMean)(bcCoefficients)."""

    def __init__(self, inverseStd, scaledMean, fitIntercept, fitWithMean, coefficients,
                 device="cuda"):
        torch = _torch()
        inverseStd = np.asarray(inverseStd, dtype=np.float64)
        if fitWithMean:
            if not fitIntercept:
                raise N.IllegalArgumentException(
                    "requirement failed: for training without intercept, should not center "
                    "the vectors")
            if scaledMean is None or len(scaledMean) != len(inverseStd):
                raise N.IllegalArgumentException(
                    "requirement failed: scaled means is required when center the vectors")
        if not isinstance(coefficients, (np.ndarray, list, tuple)) and not torch.is_tensor(
                coefficients):
            raise N.IllegalArgumentException(
                f"coefficients only supports dense vector but got type {type(coefficients)}.)")
        self.numFeatures = len(inverseStd)
        self.fitIntercept, self.fitWithMean = bool(fitIntercept), bool(fitWithMean)
        self.coef = _upload(coefficients, device) \
            if not torch.is_tensor(coefficients) else coefficients.to(device, torch.float64)
        self.dim = int(self.coef.shape[0])
        self.scaledMean = _dev_vector(scaledMean, device)
        self._plan = _logistic_plan(self.numFeatures, 1, self.fitIntercept, self.fitWithMean,
                                    device)
        self._init_state(device)

    def add(self, block: DeviceInstanceBlock, stream=None):
        """BinaryLogisticBlockAggregator.scala:81-145 over every block of the shard."""
        _check_block(self, block)
        lib = N.load()
        s = N.stream_handle(stream)
        if block.is_sparse and block.tiles is not None:
            return _tiles_add(self, block, stream)
        if block.is_sparse:
            N.check(lib.cyc_binary_logistic_add_csr_dev(
                self._plan.handle, N.ptr(block.rowptr), N.ptr(block.colidx), N.ptr(block.values),
                N.ptr(block.labels), N.ptr(block.weights), block.size, N.ptr(self.coef),
                N.ptr(self.scaledMean), N.ptr(self.gradientSumArray), N.ptr(self._loss_sum),
                N.ptr(self._weight_sum), block.csc, s))
        else:
            N.check(lib.cyc_binary_logistic_add_dense_dev(
                self._plan.handle, N.ptr(block.X), N.ptr(block.labels), N.ptr(block.weights),
                block.size, N.ptr(self.coef), N.ptr(self.scaledMean),
                N.ptr(self.gradientSumArray), N.ptr(self._loss_sum), N.ptr(self._weight_sum), s))
        return self


class HingeBlockAggregator(DifferentiableLossAggregator):
    """HingeBlockAggregator(bcInverseStd, bcScaledMean, fitIntercept)(bcCoefficients)
    (ml/optim/aggregator/HingeBlockAggregator.scala:41-141, LinearSVC's loss):
    the binary block kernels with the hinge epilogue; centers whenever it fits
    an intercept."""

    def __init__(self, inverseStd, scaledMean, fitIntercept, coefficients, device="cuda"):
        torch = _torch()
        inverseStd = np.asarray(inverseStd, dtype=np.float64)
        if fitIntercept and (scaledMean is None or len(scaledMean) != len(inverseStd)):
            raise N.IllegalArgumentException(
                "requirement failed: scaled means is required when center the vectors")
        if not isinstance(coefficients, (np.ndarray, list, tuple)) and not torch.is_tensor(
                coefficients):
            raise N.IllegalArgumentException(
                f"coefficients only supports dense vector but got type {type(coefficients)}.)")
        self.numFeatures = len(inverseStd)
        self.fitIntercept = bool(fitIntercept)
        self.coef = _upload(coefficients, device) \
            if not torch.is_tensor(coefficients) else coefficients.to(device, torch.float64)
        self.dim = int(self.coef.shape[0])
        self.scaledMean = _dev_vector(scaledMean, device)
        self._plan = _logistic_plan(self.numFeatures, 1, self.fitIntercept, self.fitIntercept,
                                    device, hinge=True)
        self._init_state(device)

    def add(self, block: DeviceInstanceBlock, stream=None):
        """HingeBlockAggregator.scala:81-141 over every block of the shard."""
        _check_block(self, block)
        lib = N.load()
        s = N.stream_handle(stream)
        if block.is_sparse and block.tiles is not None:
            return _tiles_add(self, block, stream)
        if block.is_sparse:
            N.check(lib.cyc_hinge_add_csr_dev(
                self._plan.handle, N.ptr(block.rowptr), N.ptr(block.colidx), N.ptr(block.values),
                N.ptr(block.labels), N.ptr(block.weights), block.size, N.ptr(self.coef),
                N.ptr(self.scaledMean), N.ptr(self.gradientSumArray), N.ptr(self._loss_sum),
                N.ptr(self._weight_sum), block.csc, s))
        else:
            N.check(lib.cyc_hinge_add_dense_dev(
                self._plan.handle, N.ptr(block.X), N.ptr(block.labels), N.ptr(block.weights),
                block.size, N.ptr(self.coef), N.ptr(self.scaledMean),
                N.ptr(self.gradientSumArray), N.ptr(self._loss_sum), N.ptr(self._weight_sum), s))
        return self


class LeastSquaresBlockAggregator(DifferentiableLossAggregator):
    """LeastSquaresBlockAggregator(bcInverseStd, bcScaledMean, fitIntercept,
    labelStd, labelMean)(bcCoefficients)
    (ml/optim/aggregator/LeastSquaresBlockAggregator.scala:31-101): the binary
    block kernels with the squared-error epilogue; dim = numFeatures."""

    def __init__(self, inverseStd, scaledMean, fitIntercept, labelStd, labelMean, coefficients,
                 device="cuda"):
        torch = _torch()
        if not labelStd > 0.0:
            raise N.IllegalArgumentException(
                "requirement failed: LeastSquaresBlockAggregator requires the label standard "
                "deviation to be positive.")
        if not isinstance(coefficients, (np.ndarray, list, tuple)) and not torch.is_tensor(
                coefficients):
            raise N.IllegalArgumentException(
                f"coefficients only supports dense vector but got type {type(coefficients)}.)")
        inv = np.asarray(inverseStd, dtype=np.float64)
        self.numFeatures = len(inv)
        self.fitIntercept = bool(fitIntercept)
        self.inverseStd = torch.as_tensor(inv, device=device)
        self.coef = _upload(coefficients, device) \
            if not torch.is_tensor(coefficients) else coefficients.to(device, torch.float64)
        self.dim = self.numFeatures
        self.scaledMean = _dev_vector(scaledMean, device)
        key = ("ls", self.numFeatures, self.fitIntercept, float(labelStd), float(labelMean),
               str(device))
        self._plan = _PLANS.get(key)
        if self._plan is None:
            self._plan = _PLANS[key] = _LeastSquaresPlan(self.numFeatures, self.fitIntercept,
                                                         labelStd, labelMean)
        self._init_state(device)

    def add(self, block: DeviceInstanceBlock, stream=None):
        """LeastSquaresBlockAggregator.scala:70-101 over every block of the shard."""
        _check_block(self, block)
        lib = N.load()
        s = N.stream_handle(stream)
        if block.is_sparse and block.tiles is not None:
            return _tiles_add(self, block, stream, self.inverseStd)
        if block.is_sparse:
            N.check(lib.cyc_least_squares_add_csr_dev(
                self._plan.handle, N.ptr(block.rowptr), N.ptr(block.colidx), N.ptr(block.values),
                N.ptr(block.labels), N.ptr(block.weights), block.size, N.ptr(self.coef),
                N.ptr(self.inverseStd), N.ptr(self.scaledMean), N.ptr(self.gradientSumArray),
                N.ptr(self._loss_sum), N.ptr(self._weight_sum), block.csc, s))
        else:
            N.check(lib.cyc_least_squares_add_dense_dev(
                self._plan.handle, N.ptr(block.X), N.ptr(block.labels), N.ptr(block.weights),
                block.size, N.ptr(self.coef), N.ptr(self.inverseStd), N.ptr(self.scaledMean),
                N.ptr(self.gradientSumArray), N.ptr(self._loss_sum), N.ptr(self._weight_sum), s))
        return self


class HuberBlockAggregator(DifferentiableLossAggregator):
    """HuberBlockAggregator(bcInverseStd, bcScaledMean, fitIntercept, epsilon)
    (bcParameters) (ml/optim/aggregator/HuberBlockAggregator.scala:41-141):
    the binary block kernels with the Huber epilogue; parameters = linear
    terms, intercept (if fitIntercept), sigma."""

    def __init__(self, inverseStd, scaledMean, fitIntercept, epsilon, parameters,
                 device="cuda"):
        torch = _torch()
        inv = np.asarray(inverseStd, dtype=np.float64)
        if fitIntercept and (scaledMean is None or len(scaledMean) != len(inv)):
            raise N.IllegalArgumentException(
                "requirement failed: scaled means is required when center the vectors")
        self.numFeatures = len(inv)
        self.fitIntercept = bool(fitIntercept)
        self.coef = _upload(parameters, device) \
            if not torch.is_tensor(parameters) else parameters.to(device, torch.float64)
        self.dim = int(self.coef.shape[0])
        if self.dim != self.numFeatures + (2 if self.fitIntercept else 1):
            raise N.IllegalArgumentException(
                f"requirement failed: parameters size {self.dim} does not match numFeatures "
                f"{self.numFeatures} (+ intercept) + sigma")
        self.scaledMean = _dev_vector(scaledMean, device)
        key = ("huber", self.numFeatures, self.fitIntercept, float(epsilon), str(device))
        self._plan = _PLANS.get(key)
        if self._plan is None:
            self._plan = _PLANS[key] = _HuberPlan(self.numFeatures, self.fitIntercept, epsilon)
        self._init_state(device)

    def add(self, block: DeviceInstanceBlock, stream=None):
        """HuberBlockAggregator.scala:80-141 over every block of the shard."""
        _check_block(self, block)
        lib = N.load()
        s = N.stream_handle(stream)
        if block.is_sparse and block.tiles is not None:
            return _tiles_add(self, block, stream)
        if block.is_sparse:
            N.check(lib.cyc_huber_add_csr_dev(
                self._plan.handle, N.ptr(block.rowptr), N.ptr(block.colidx), N.ptr(block.values),
                N.ptr(block.labels), N.ptr(block.weights), block.size, N.ptr(self.coef),
                N.ptr(self.scaledMean), N.ptr(self.gradientSumArray), N.ptr(self._loss_sum),
                N.ptr(self._weight_sum), block.csc, s))
        else:
            N.check(lib.cyc_huber_add_dense_dev(
                self._plan.handle, N.ptr(block.X), N.ptr(block.labels), N.ptr(block.weights),
                block.size, N.ptr(self.coef), N.ptr(self.scaledMean),
                N.ptr(self.gradientSumArray), N.ptr(self._loss_sum), N.ptr(self._weight_sum), s))
        return self


class _HuberPlan(_LogisticPlan):
    def __init__(self, F, fit_intercept, epsilon):
        self._lib = N.load()
        h = ctypes.c_void_p()
        N.check(self._lib.cyc_huber_plan_create(int(F), int(bool(fit_intercept)), float(epsilon),
                                                ctypes.byref(h)))
        self.handle = h


class AFTBlockAggregator(DifferentiableLossAggregator):
    """AFTBlockAggregator(bcScaledMean, fitIntercept)(bcCoefficients)
    (ml/optim/aggregator/AFTBlockAggregator.scala:30-130): the binary block
    kernels with the AFT survival epilogue.  coefficients = F linear terms,
    intercept, log(sigma); a block's `weights` carry the censors, as the
    reference's InstanceBlock does (:97)."""

    def __init__(self, scaledMean, fitIntercept, coefficients, device="cuda"):
        torch = _torch()
        if not isinstance(coefficients, (np.ndarray, list, tuple)) and not torch.is_tensor(
                coefficients):
            raise N.IllegalArgumentException(
                f"coefficients only supports dense vector but got type {type(coefficients)}.")
        self.coef = _upload(coefficients, device) \
            if not torch.is_tensor(coefficients) else coefficients.to(device, torch.float64)
        self.dim = int(self.coef.shape[0])
        self.numFeatures = self.dim - 2
        self.fitIntercept = bool(fitIntercept)
        if self.fitIntercept and (scaledMean is None or len(scaledMean) != self.numFeatures):
            raise N.IllegalArgumentException(
                "requirement failed: scaled means is required when center the vectors")
        self.scaledMean = _dev_vector(scaledMean, device)
        key = ("aft", self.numFeatures, self.fitIntercept, str(device))
        self._plan = _PLANS.get(key)
        if self._plan is None:
            self._plan = _PLANS[key] = _AFTPlan(self.numFeatures, self.fitIntercept)
        self._init_state(device)

    def add(self, block: DeviceInstanceBlock, stream=None):
        """AFTBlockAggregator.scala:76-130 over every block of the shard."""
        if self.numFeatures != block.numFeatures:
            raise N.IllegalArgumentException(
                "requirement failed: Dimensions mismatch when adding new instance. Expecting "
                f"{self.numFeatures} but got {block.numFeatures}.")
        if block.size and bool((block.labels <= 0).any().item()):      # :81
            raise N.IllegalArgumentException(
                "requirement failed: The lifetime or label should be greater than 0.")
        lib = N.load()
        s = N.stream_handle(stream)
        if block.is_sparse and block.tiles is not None:
            return _tiles_add(self, block, stream)
        if block.is_sparse:
            N.check(lib.cyc_aft_add_csr_dev(
                self._plan.handle, N.ptr(block.rowptr), N.ptr(block.colidx), N.ptr(block.values),
                N.ptr(block.labels), N.ptr(block.weights), block.size, N.ptr(self.coef),
                N.ptr(self.scaledMean), N.ptr(self.gradientSumArray), N.ptr(self._loss_sum),
                N.ptr(self._weight_sum), block.csc, s))
        else:
            N.check(lib.cyc_aft_add_dense_dev(
                self._plan.handle, N.ptr(block.X), N.ptr(block.labels), N.ptr(block.weights),
                block.size, N.ptr(self.coef), N.ptr(self.scaledMean),
                N.ptr(self.gradientSumArray), N.ptr(self._loss_sum), N.ptr(self._weight_sum), s))
        return self


class _AFTPlan(_LogisticPlan):
    def __init__(self, F, fit_intercept):
        self._lib = N.load()
        h = ctypes.c_void_p()
        N.check(self._lib.cyc_aft_plan_create(int(F), int(bool(fit_intercept)), ctypes.byref(h)))
        self.handle = h


class _LeastSquaresPlan(_LogisticPlan):
    def __init__(self, F, fit_intercept, label_std, label_mean):
        self._lib = N.load()
        h = ctypes.c_void_p()
        N.check(self._lib.cyc_least_squares_plan_create(int(F), int(bool(fit_intercept)),
                                                        float(label_std), float(label_mean),
                                                        ctypes.byref(h)))
        self.handle = h


class MultinomialLogisticBlockAggregator(DifferentiableLossAggregator):
    """MultinomialLogisticBlockAggregator: coefficients column-major
    (numClasses x numFeatures) followed by numClasses intercepts."""

    def __init__(self, inverseStd, scaledMean, fitIntercept, fitWithMean, coefficients,
                 device="cuda"):
        torch = _torch()
        inverseStd = np.asarray(inverseStd, dtype=np.float64)
        if fitWithMean:
            if not fitIntercept:
                raise N.IllegalArgumentException(
                    "requirement failed: for training without intercept, should not center "
                    "the vectors")
            if scaledMean is None or len(scaledMean) != len(inverseStd):
                raise N.IllegalArgumentException(
                    "requirement failed: scaled means is required when center the vectors")
        self.numFeatures = len(inverseStd)
        self.fitIntercept, self.fitWithMean = bool(fitIntercept), bool(fitWithMean)
        self.coef = _upload(coefficients, device) \
            if not torch.is_tensor(coefficients) else coefficients.to(device, torch.float64)
        self.dim = int(self.coef.shape[0])
        fpi = self.numFeatures + 1 if self.fitIntercept else self.numFeatures
        self.numClasses = self.dim // fpi
        if self.dim != self.numClasses * fpi:
            raise N.IllegalArgumentException("requirement failed")
        self.scaledMean = _dev_vector(scaledMean, device)
        self._plan = _logistic_plan(self.numFeatures, self.numClasses, self.fitIntercept,
                                    self.fitWithMean, device)
        self._init_state(device)

    def add(self, block: DeviceInstanceBlock, stream=None):
        """MultinomialLogisticBlockAggregator.scala:101-189 over the shard."""
        _check_block(self, block)
        if block.is_sparse:
            if block.rowptr is None:
                raise N.IllegalArgumentException(
                    "the multinomial aggregator needs the block's CSR rows (release_csr dropped "
                    "them)")
            block.prepare(stream)          # CSC copy for the gradient (built once)
            N.check(N.load().cyc_multinomial_logistic_add_csr_dev(
                self._plan.handle, N.ptr(block.rowptr), N.ptr(block.colidx),
                N.ptr(block.values), N.ptr(block.labels), N.ptr(block.weights), block.size,
                N.ptr(self.coef), N.ptr(self.scaledMean), N.ptr(self.gradientSumArray),
                N.ptr(self._loss_sum), N.ptr(self._weight_sum), block.csc,
                N.stream_handle(stream)))
            return self
        N.check(N.load().cyc_multinomial_logistic_add_dense_dev(
            self._plan.handle, N.ptr(block.X), N.ptr(block.labels), N.ptr(block.weights),
            block.size, N.ptr(self.coef), N.ptr(self.scaledMean), N.ptr(self.gradientSumArray),
            N.ptr(self._loss_sum), N.ptr(self._weight_sum), N.stream_handle(stream)))
        return self


class L2Regularization:
    """ml/optim/loss/DifferentiableRegularization.scala L2Regularization:
    loss = 0.5 * regParam * sum(coef_j^2) over regularized indices, gradient
    regParam * coef_j (applyFeaturesStd = None branch)."""

    def __init__(self, regParam, shouldApply=lambda j: True):
        self.regParam = regParam
        self.shouldApply = shouldApply

    def calculate(self, coefficients):
        c = np.asarray(coefficients, dtype=np.float64)
        grad = np.zeros_like(c)
        s = 0.0
        for j, v in enumerate(c):
            if self.shouldApply(j):
                s += v * v
                grad[j] = v * self.regParam
        return 0.5 * s * self.regParam, grad


class RDDLossFunction:
    """ml/optim/loss/RDDLossFunction.scala:47-70: one full data pass per
    evaluation.  `blocks` are this rank's device-resident shard(s); the
    treeAggregate merge is an all-reduce when torch.distributed is initialised."""

    def __init__(self, blocks, getAggregator, regularization=None):
        self.blocks = blocks if isinstance(blocks, (list, tuple)) else [blocks]
        self.getAggregator = getAggregator
        self.regularization = regularization

    def calculate(self, coefficients):
        agg = self.getAggregator(coefficients)
        for b in self.blocks:
            agg.add(b)
        agg.allreduce()
        gradient = agg.gradient
        loss = agg.loss
        if self.regularization is not None:
            regLoss, regGrad = self.regularization.calculate(coefficients)
            gradient = gradient + regGrad          # BLAS.axpy(1.0, regGradient, gradient)
            loss = loss + regLoss
        return loss, gradient
