"""KMeans on MI355X: host-side mirror of org.apache.spark.mllib.clustering.

Mirrors mllib/clustering/KMeans.scala (the Lloyd loop :240-349 and its
parameters) and KMeansModel; the per-partition body runs in libcyclone
(cycloneml_amd/csrc/kmeans.hip).  Data stays resident in HBM: `run` takes a
torch CUDA fp64 tensor of shape (n, d) -- one process per GPU holding its
shard of the rows (the Spark partitions assigned to that GPU).  When
torch.distributed is initialised, the reduceByKey/collectAsMap merge
(KMeans.scala:308-311) and the DoubleAccumulator cost are one all-reduce of
[sums | weights | cost] over RCCL (backend "nccl"), and every rank applies the
same centroid update (:322-330).
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


EUCLIDEAN = "euclidean"
COSINE = "cosine"
_MEASURES = {EUCLIDEAN: N.CYC_DISTANCE_EUCLIDEAN, COSINE: N.CYC_DISTANCE_COSINE}


def _decode_measure(dm: str) -> int:
    """DistanceMeasure.decodeFromString (DistanceMeasure.scala:241-247)."""
    if dm not in _MEASURES:
        raise N.IllegalArgumentException(
            f"distanceMeasure must be one of: {EUCLIDEAN}, {COSINE}. {dm} provided.")
    return _MEASURES[dm]


def xorshift_next_int(seed: int) -> int:
    """new XORShiftRandom(seed).nextInt() (core/.../util/random/
    XORShiftRandom.scala:44-66): the hashed state (cyc_xorshift_hash_seed)
    advanced once, its low 32 bits as a signed Int.  KMeans.scala:377 seeds
    the k-means|| steps with it."""
    m64 = (1 << 64) - 1
    x = int(N.load().cyc_xorshift_hash_seed(int(seed))) & m64
    x ^= (x << 21) & m64
    x ^= x >> 35
    x ^= (x << 4) & m64
    v = x & 0xFFFFFFFF
    return v - (1 << 32) if v >= 1 << 31 else v


IMAGE_MAX_D = 512   # the i8 row image's widest rows (kmeans_i8.hpp kMaxD)


class KMeansPlan:
    """RAII wrapper of cyc_kmeans_plan (device scratch for one (d, k) shape
    and one DistanceMeasure)."""

    def __init__(self, d: int, k: int, max_rows: int = 1, distanceMeasure: str = EUCLIDEAN):
        self._lib = N.load()
        measure = _decode_measure(distanceMeasure)
        h = ctypes.c_void_p()
        N.check(self._lib.cyc_kmeans_plan_create(int(d), int(k), int(max_rows), ctypes.byref(h)))
        self.handle = h
        self.d, self.k = int(d), int(k)
        self.distanceMeasure = distanceMeasure
        if measure != N.CYC_DISTANCE_EUCLIDEAN:
            N.check(self._lib.cyc_kmeans_plan_set_distance_measure(h, measure))

    def close(self):
        if self.handle:
            self._lib.cyc_kmeans_plan_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def stats(self, C, out=None, stream=None):
        N.check(self._lib.cyc_kmeans_stats_dev(self.handle, N.ptr(C), N.ptr(out),
                                               N.stream_handle(stream)))
        return out

    def rows(self, X, stream=None):
        """Per-fit row image of X for the exact-integer i8 screen (built once,
        like the norms KMeans.scala:263-270 caches); X must stay unchanged."""
        return KMeansRows(self, X, stream)

    def assign(self, X, xnorm, C, cnorm, assign, cost, stream=None, count_exact=False,
               rows=None):
        n_exact = ctypes.c_int64(0)
        N.check(self._lib.cyc_kmeans_assign_dev(
            self.handle, N.ptr(X), N.ptr(xnorm), _rows_handle(rows), int(X.shape[0]), N.ptr(C),
            N.ptr(cnorm), N.ptr(assign), N.ptr(cost),
            ctypes.byref(n_exact) if count_exact else None, N.stream_handle(stream)))
        return n_exact.value

    def point_cost(self, X, xnorm, C, cnorm, assign, cost, stream=None, rows=None):
        """findClosest(centers, point) without statistics for every row
        (DistanceMeasure.pointCost, DistanceMeasure.scala:152-156, 318-340)."""
        N.check(self._lib.cyc_kmeans_point_cost_dev(
            self.handle, N.ptr(X), N.ptr(xnorm), _rows_handle(rows), int(X.shape[0]), N.ptr(C),
            N.ptr(cnorm), N.ptr(assign), N.ptr(cost), N.stream_handle(stream)))

    def point_cost_csr(self, rowptr, colidx, values, xnorm, C, cnorm, assign, cost, stream=None):
        N.check(self._lib.cyc_kmeans_point_cost_csr_dev(
            self.handle, N.ptr(rowptr), N.ptr(colidx), N.ptr(values), N.ptr(xnorm),
            int(rowptr.shape[0]) - 1, N.ptr(C), N.ptr(cnorm), N.ptr(assign), N.ptr(cost),
            N.stream_handle(stream)))

    def last_tiers(self):
        """(rows left to the fp64 screen, rows left to the exact loop) of the
        last assign(count_exact=True)."""
        a, b = ctypes.c_int64(0), ctypes.c_int64(0)
        N.check(self._lib.cyc_kmeans_last_tiers(self.handle, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def last_screen(self):
        """Rows the two-limb i8 pass left to the three-limb pass on the last
        assign(count_exact=True) (-1: that call ran no two-limb pass)."""
        a = ctypes.c_int64(0)
        N.check(self._lib.cyc_kmeans_last_screen(self.handle, ctypes.byref(a)))
        return a.value

    def last_candidates(self):
        """Rows the two-limb pass handed to its candidate pass on the last
        assign(count_exact=True) (-1: no two-limb pass)."""
        a = ctypes.c_int64(0)
        N.check(self._lib.cyc_kmeans_last_candidates(self.handle, ctypes.byref(a)))
        return a.value

    def last_candidates3(self):
        """Of last_candidates(), the rows the three-limb candidate tier left to
        the fp64 candidate pass on the last assign(count_exact=True) (-1: the
        tier did not run)."""
        a = ctypes.c_int64(0)
        N.check(self._lib.cyc_kmeans_last_candidates3(self.handle, ctypes.byref(a)))
        return a.value

    def last_refine(self):
        """(rows the one-limb pass listed, rows handed to the full two-limb
        pass, candidate centers the refinement screened in total) of the
        last i8 screen; (-1, -1, -1) when it ran the two-limb pass over every
        center (k <= 96)."""
        a, b, c = ctypes.c_int64(0), ctypes.c_int64(0), ctypes.c_int64(0)
        N.check(self._lib.cyc_kmeans_last_refine(self.handle, ctypes.byref(a), ctypes.byref(b),
                                                 ctypes.byref(c)))
        return a.value, b.value, c.value

    def accumulate(self, X, xnorm, weights, C, cnorm, sums, wsum, cost_sum, assign=None,
                   cost=None, stream=None, rows=None):
        N.check(self._lib.cyc_kmeans_accumulate_dev(
            self.handle, N.ptr(X), N.ptr(xnorm), _rows_handle(rows), N.ptr(weights),
            int(X.shape[0]), N.ptr(C), N.ptr(cnorm), N.ptr(sums), N.ptr(wsum), N.ptr(cost_sum),
            N.ptr(assign), N.ptr(cost), N.stream_handle(stream)))

    def assign_csr(self, rowptr, colidx, values, xnorm, C, cnorm, assign, cost, stream=None):
        """findClosest for CSR rows (sparse points, dense centers); statistics
        from the last stats() call."""
        N.check(self._lib.cyc_kmeans_assign_csr_dev(
            self.handle, N.ptr(rowptr), N.ptr(colidx), N.ptr(values), N.ptr(xnorm),
            int(rowptr.shape[0]) - 1, N.ptr(C), N.ptr(cnorm), N.ptr(assign), N.ptr(cost),
            N.stream_handle(stream)))

    def accumulate_csr(self, rowptr, colidx, values, xnorm, weights, C, cnorm, sums, wsum,
                       cost_sum, assign=None, cost=None, stream=None):
        N.check(self._lib.cyc_kmeans_accumulate_csr_dev(
            self.handle, N.ptr(rowptr), N.ptr(colidx), N.ptr(values), N.ptr(xnorm),
            N.ptr(weights), int(rowptr.shape[0]) - 1, N.ptr(C), N.ptr(cnorm), N.ptr(sums),
            N.ptr(wsum), N.ptr(cost_sum), N.ptr(assign), N.ptr(cost), N.stream_handle(stream)))

    def update(self, C, cnorm, sums, wsum, epsilon, converged, stream=None):
        N.check(self._lib.cyc_kmeans_update_dev(self.handle, N.ptr(C), N.ptr(cnorm), N.ptr(sums),
                                                N.ptr(wsum), float(epsilon), N.ptr(converged),
                                                N.stream_handle(stream)))


class KMeansRows:
    """RAII wrapper of cyc_kmeans_rows: the int8 three-limb image of a fixed
    row block (3 bytes per element), built once per fit."""

    def __init__(self, plan: KMeansPlan, X, stream=None):
        self._lib = N.load()
        h = ctypes.c_void_p()
        N.check(self._lib.cyc_kmeans_rows_create(plan.handle, N.ptr(X), int(X.shape[0]),
                                                 N.stream_handle(stream), ctypes.byref(h)))
        self.handle = h
        self.X = X            # keeps the rows alive while the image is in use

    @property
    def nbytes(self):
        return int(self._lib.cyc_kmeans_rows_bytes(self.handle)) if self.handle else 0

    def set_bounds(self, enable: bool):
        """Carried bounds across this fit's Lloyd iterations (on by default,
        cyclone.h cyc_kmeans_rows_set_bounds): rows whose Hamerly bounds still
        certify their center skip the screen; either setting drops the state."""
        N.check(self._lib.cyc_kmeans_rows_set_bounds(self.handle, 1 if enable else 0))

    def set_incremental(self, enable: bool):
        """Incremental cluster sums across this fit's Lloyd iterations (on by
        default, cyclone.h cyc_kmeans_rows_set_incremental): with the carried
        bounds, unit weights and no per-row costs, a call folds only the rows
        that changed center into the carried sums; either setting drops the
        state."""
        N.check(self._lib.cyc_kmeans_rows_set_incremental(self.handle, 1 if enable else 0))

    def incremental_info(self):
        """(calls that took the incremental path, moved rows they folded);
        synchronises the device."""
        a, b = ctypes.c_int64(0), ctypes.c_int64(0)
        N.check(self._lib.cyc_kmeans_rows_incremental_info(self.handle, ctypes.byref(a),
                                                           ctypes.byref(b)))
        return a.value, b.value

    def bounds_rechecked(self):
        """Rows re-checked against their carried candidate sets (all calls;
        synchronises the device)."""
        a = ctypes.c_int64(0)
        N.check(self._lib.cyc_kmeans_rows_bounds_rechecked(self.handle, ctypes.byref(a)))
        return a.value

    def bounds_info(self):
        """(accumulate calls that used the bounds, rows those calls screened);
        synchronises the device."""
        a, b = ctypes.c_int64(0), ctypes.c_int64(0)
        N.check(self._lib.cyc_kmeans_rows_bounds_info(self.handle, ctypes.byref(a),
                                                      ctypes.byref(b)))
        return a.value, b.value

    def close(self):
        if self.handle:
            self._lib.cyc_kmeans_rows_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _rows_handle(rows):
    return None if rows is None else rows.handle


def row_norms(X, out=None, stream=None):
    """Vectors.norm(v, 2.0) per row, bit-exact (mllib/linalg/Vectors.scala:489-514)."""
    torch = _torch()
    if out is None:
        out = torch.empty(X.shape[0], dtype=torch.float64, device=X.device)
    N.check(N.load().cyc_row_norms_dev(N.ptr(X), int(X.shape[0]), int(X.shape[1]), N.ptr(out),
                                       N.stream_handle(stream)))
    return out


def row_norms_csr(rowptr, values, out=None, stream=None):
    """Vectors.norm(sparse, 2.0) per CSR row (stored values, in order)."""
    torch = _torch()
    n = int(rowptr.shape[0]) - 1
    if out is None:
        out = torch.empty(n, dtype=torch.float64, device=values.device)
    N.check(N.load().cyc_row_norms_csr_dev(N.ptr(rowptr), N.ptr(values), n, N.ptr(out),
                                           N.stream_handle(stream)))
    return out


class KMeansModel:
    """mllib/clustering/KMeansModel.scala: centers (k x d), distanceMeasure,
    cost, numIter."""

    def __init__(self, clusterCenters, trainingCost=0.0, numIter=0,
                 distanceMeasure: str = EUCLIDEAN):
        _decode_measure(distanceMeasure)
        self.clusterCenters = np.ascontiguousarray(clusterCenters, dtype=np.float64)
        self.trainingCost = float(trainingCost)
        self.numIter = int(numIter)
        self.distanceMeasure = distanceMeasure

    @property
    def k(self):
        return self.clusterCenters.shape[0]

    # ---- persistence (KMeansModel.scala:148-224, format "2.0") -----------
    def save(self, path, overwrite=False):
        from . import persist
        persist.save_kmeans_model(self, path, getattr(self, "distanceMeasure", "euclidean"),
                                  overwrite=overwrite)

    @staticmethod
    def load(path):
        from . import persist
        return persist.load_kmeans_model(path)

    # ---- device-side scoring (KMeansModel.scala:82-117) -----------------
    def _device_state(self, device, n, csr_d=None):
        torch = _torch()
        key = (str(device), csr_d)
        st = getattr(self, "_dev", None)
        if st is None or st["key"] != key:
            C = torch.from_numpy(self.clusterCenters).to(device)
            d = self.clusterCenters.shape[1]
            plan = KMeansPlan(d if csr_d is None else csr_d, self.k, max(1, n),
                              self.distanceMeasure)
            cnorm = row_norms(C)
            # the model's lazy statistics (KMeansModel.scala:51-56)
            plan.stats(C)
            st = self._dev = {"key": key, "C": C, "cnorm": cnorm, "plan": plan}
        return st

    def predict(self, X, xnorm=None, stream=None):
        """predict(points): findClosest(centersWithNorm, statistics, point)._1
        for every row of the device matrix X (KMeansModel.scala:82-97).
        Returns an int32 device tensor."""
        torch = _torch()
        n = int(X.shape[0])
        st = self._device_state(X.device, n)
        xn = row_norms(X, stream=stream) if xnorm is None else xnorm
        a = torch.empty(n, dtype=torch.int32, device=X.device)
        c = torch.empty(n, dtype=torch.float64, device=X.device)
        if n:
            st["plan"].assign(X, xn, st["C"], st["cnorm"], a, c, stream=stream)
        return a

    def predict_csr(self, rowptr, colidx, values, xnorm=None, stream=None):
        """predict for CSR rows (SparseVector points; libsvm input)."""
        torch = _torch()
        n = int(rowptr.shape[0]) - 1
        st = self._device_state(values.device, n, csr_d=self.clusterCenters.shape[1])
        xn = row_norms_csr(rowptr, values, stream=stream) if xnorm is None else xnorm
        a = torch.empty(n, dtype=torch.int32, device=values.device)
        c = torch.empty(n, dtype=torch.float64, device=values.device)
        if n:
            st["plan"].assign_csr(rowptr, colidx, values, xn, st["C"], st["cnorm"], a, c,
                                  stream=stream)
        return a

    def pointCosts(self, X, xnorm=None, stream=None):
        """DistanceMeasure.pointCost (DistanceMeasure.scala:152-156) for every
        row: (assign int32, cost fp64) device tensors."""
        torch = _torch()
        n = int(X.shape[0])
        st = self._device_state(X.device, n)
        xn = row_norms(X, stream=stream) if xnorm is None else xnorm
        a = torch.empty(n, dtype=torch.int32, device=X.device)
        c = torch.empty(n, dtype=torch.float64, device=X.device)
        if n:
            st["plan"].point_cost(X, xn, st["C"], st["cnorm"], a, c, stream=stream)
        return a, c

    def pointCosts_csr(self, rowptr, colidx, values, xnorm=None, stream=None):
        torch = _torch()
        n = int(rowptr.shape[0]) - 1
        st = self._device_state(values.device, n, csr_d=self.clusterCenters.shape[1])
        xn = row_norms_csr(rowptr, values, stream=stream) if xnorm is None else xnorm
        a = torch.empty(n, dtype=torch.int32, device=values.device)
        c = torch.empty(n, dtype=torch.float64, device=values.device)
        if n:
            st["plan"].point_cost_csr(rowptr, colidx, values, xn, st["C"], st["cnorm"], a, c,
                                      stream=stream)
        return a, c

    def computeCost(self, X, xnorm=None, stream=None):
        """computeCost(data) = data.map(pointCost).sum() (KMeansModel.scala:
        110-117): per-row costs bit-identical to the reference; the sum runs
        in a fixed device order, then across ranks (one all-reduce, like the
        driver's fold over partitions)."""
        _, c = self.pointCosts(X, xnorm, stream)
        return self._sum_costs(c)

    def computeCost_csr(self, rowptr, colidx, values, xnorm=None, stream=None):
        _, c = self.pointCosts_csr(rowptr, colidx, values, xnorm, stream)
        return self._sum_costs(c)

    @staticmethod
    def _sum_costs(c):
        torch = _torch()
        tot = c.sum().reshape(1) if c.numel() else torch.zeros(1, dtype=torch.float64,
                                                               device=c.device)
        parallel.allreduce_(tot)
        return float(tot.item())


class KMeans:
    """mllib.clustering.KMeans with the reference's parameters and defaults
    (KMeans.scala:48-60: k=2, maxIterations=20, epsilon=1e-4)."""

    RANDOM = "random"
    K_MEANS_PARALLEL = "k-means||"

    def __init__(self, k: int = 2, maxIterations: int = 20, epsilon: float = 1e-4,
                 seed: int = 0):
        self.k = k
        self.maxIterations = maxIterations
        self.epsilon = epsilon
        self.seed = seed
        self.initialModel = None
        self.distanceMeasure = "euclidean"
        self.initializationMode = KMeans.K_MEANS_PARALLEL
        self.initializationSteps = 2

    def setInitializationMode(self, mode: str):
        """KMeans.scala:117-121 (validateInitMode's result is not checked
        there either; an unknown mode runs k-means||, :255-258)."""
        self.initializationMode = mode
        return self

    def setInitializationSteps(self, steps: int):
        if not steps > 0:
            raise N.IllegalArgumentException(
                f"requirement failed: Number of initialization steps must be positive but got "
                f"{steps}")
        self.initializationSteps = steps
        return self

    def setSeed(self, seed: int):
        self.seed = int(seed)
        return self

    def initial_centers(self, X, xnorm=None, partition_starts=None):
        """The initial centers of a run without an initial model
        (KMeans.scala:250-259): initRandom or initKMeansParallel over the
        shard split into Spark partitions at partition_starts (default: one
        partition).  Across ranks every process passes its own shard and
        partitions; the partitions are numbered in rank order and the
        driver-side sampling sees all of them (kmeans_init)."""
        from . import kmeans_init
        n = int(X.shape[0])
        starts = np.asarray([0, n] if partition_starts is None else partition_starts,
                            dtype=np.int64)
        if self.initializationMode == KMeans.RANDOM:
            return kmeans_init.init_random(X, self.k, self.seed, starts)
        return kmeans_init.init_kmeans_parallel(X, self.k, self.seed, self.initializationSteps,
                                                starts, self.distanceMeasure, xnorm)

    # Builder setters (KMeans.scala:87-200)
    def setK(self, k):
        if not k > 0:
            raise N.IllegalArgumentException(f"Number of clusters must be positive but got {k}")
        self.k = k
        return self

    def setMaxIterations(self, m):
        if not m >= 0:
            raise N.IllegalArgumentException(
                f"Maximum of iterations must be nonnegative but got {m}")
        self.maxIterations = m
        return self

    def setEpsilon(self, eps):
        if not eps >= 0:
            raise N.IllegalArgumentException(
                f"Distance threshold must be nonnegative but got {eps}")
        self.epsilon = eps
        return self

    def setInitialModel(self, model: KMeansModel):
        if model.k != self.k:
            raise N.IllegalArgumentException("mismatched cluster count")
        self.initialModel = model
        return self

    def setDistanceMeasure(self, dm: str):
        """KMeans.scala:184-188.  validateDistanceMeasure's result is not
        checked there, so an unknown name fails at the run's
        DistanceMeasure.decodeFromString (KMeans.scala:248), as here."""
        self.distanceMeasure = dm
        return self

    @staticmethod
    def updateParallelCosts(X, newCenters, costs=None, xnorm=None, stream=None,
                            distanceMeasure=EUCLIDEAN):
        """One k-means|| cost update on the device (KMeans.scala:392-396):
        costs = min(pointCost(newCenters, x), cost) per row, pointCost being
        findClosest without statistics (bit-exact per row).  costs=None starts
        from +Infinity (:375).  Returns (costs, sum of costs); the sum is the
        `costs.sum()` that scales the sampling probabilities (:398), one
        all-reduce across ranks.  The sampling (XORShiftRandom per partition)
        and LocalKMeans stay on the host, as in the reference driver."""
        torch = _torch()
        m = KMeansModel(np.asarray(newCenters, dtype=np.float64),
                        distanceMeasure=distanceMeasure)
        _, c = m.pointCosts(X, xnorm, stream)
        if costs is not None:
            c = torch.minimum(c, costs)   # math.min: NaN propagates either way
        tot = c.sum().reshape(1) if c.numel() else torch.zeros(1, dtype=torch.float64,
                                                               device=c.device)
        parallel.allreduce_(tot)
        return c, float(tot.item())

    @staticmethod
    def parallelSample(costs, sumCosts, seed, step, k, partition_starts, first_partition=0,
                       stream=None):
        """The executor side of one k-means|| step (KMeans.scala:398-404) on
        the device: a uint8 mask of the rows whose partition's
        XORShiftRandom(seed ^ (step << 16) ^ index) draws nextDouble() <
        2.0 * cost * k / sumCosts, one draw per row in partition order --
        the points the reference collects (X[mask.bool()] keeps their
        order).  costs: the updated point costs (updateParallelCosts);
        seed: xorshift_next_int(KMeans seed); partition_starts: the shard's
        rows split into Spark partitions (host ints, from 0), partition p
        having index first_partition + p."""
        torch = _torch()
        starts = np.ascontiguousarray(partition_starts, dtype=np.int64)
        if starts.size < 2 or starts[0] != 0 or starts[-1] != costs.numel():
            raise N.IllegalArgumentException(
                "partition_starts must run from 0 to the number of rows")
        mask = torch.empty(costs.numel(), dtype=torch.uint8, device=costs.device)
        N.check(N.load().cyc_kmeans_parallel_sample_dev(
            N.ptr(costs), starts.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
            int(starts.size - 1), int(first_partition), int(seed), int(step), int(k),
            float(sumCosts), N.ptr(mask), N.stream_handle(stream)))
        return mask

    def run(self, X, weights=None, xnorm=None, stream=None, iteration_callback=None,
            partition_starts=None):
        """Lloyd's algorithm, KMeans.scala:240-349, on a device-resident shard.

        X: torch.float64 CUDA tensor (n, d).  weights: optional (n,) tensor.
        Without an initial model the centers come from initial_centers
        (partition_starts: the Spark partitions of the shard's rows).
        Returns KMeansModel (centers on the host)."""
        torch = _torch()
        dev = X.device
        n, d = X.shape
        # the cached norms (KMeans.scala:263-270): with setInitialModel and a
        # Euclidean row image (d <= 512) the Lloyd loop needs none from the
        # caller -- the image carries norms for the screens' margins and the
        # exact tier computes the reference's own norm for the rows it takes
        # (cyclone.h cyc_kmeans_accumulate_dev, xnorm NULL)
        if xnorm is None and (self.initialModel is None or self.distanceMeasure != EUCLIDEAN
                              or d > IMAGE_MAX_D):
            xnorm = row_norms(X, stream=stream)
        if self.initialModel is None:
            C0 = self.initial_centers(X, xnorm, partition_starts)
            # the run's k is the number of initial centers (KMeans.scala:250-259
            # may return fewer than k distinct points)
            self.initialModel = KMeansModel(C0, distanceMeasure=self.distanceMeasure)
            try:
                return self._run(X, weights, xnorm, stream, iteration_callback, C0.shape[0])
            finally:
                self.initialModel = None
        return self._run(X, weights, xnorm, stream, iteration_callback, self.k)

    def _run(self, X, weights, xnorm, stream, iteration_callback, k):
        torch = _torch()
        dev = X.device
        n, d = X.shape
        plan = KMeansPlan(d, k, n, self.distanceMeasure)   # decodeFromString (:248)
        rows = plan.rows(X, stream=stream)     # once per fit, like the cached norms
        C = torch.from_numpy(self.initialModel.clusterCenters.copy()).to(dev)
        parallel.broadcast_(C)             # bcCenters (KMeans.scala:276)
        cnorm = row_norms(C, stream=stream)
        buf = torch.empty(k * d + k + 1, dtype=torch.float64, device=dev)
        sums, wsum, cost_sum = buf[:k * d], buf[k * d:k * d + k], buf[k * d + k:]
        converged_t = torch.zeros(1, dtype=torch.int32, device=dev)
        iteration, converged, cost = 0, False, 0.0
        trace = [] if os.environ.get("CYC_KMEANS_FIT_TRACE") == "1" else None
        while iteration < self.maxIterations and not converged:
            buf.zero_()
            plan.accumulate(X, xnorm, weights, C, cnorm, sums, wsum, cost_sum, stream=stream,
                            rows=rows)
            parallel.allreduce_(buf)       # reduceByKey + collectAsMap + costAccum
            plan.update(C, cnorm, sums, wsum, self.epsilon, converged_t, stream=stream)
            converged = bool(converged_t.item())
            cost = float(cost_sum.item())
            if trace is not None:        # CYC_KMEANS_FIT_TRACE=1: the carried state per iteration
                trace.append({"bounds": rows.bounds_info(), "rechecked": rows.bounds_rechecked(),
                              "incremental": rows.incremental_info()})
            if iteration_callback:
                iteration_callback(iteration, cost)
            iteration += 1
        # diagnostics of the carried state (cumulative over the fit)
        self.lastFitInfo = {"bounded_calls_and_screened_rows": rows.bounds_info(),
                            "rechecked_rows": rows.bounds_rechecked(),
                            "incremental_calls_and_moved_rows": rows.incremental_info(),
                            "per_iteration": trace}
        rows.close()
        plan.close()
        return KMeansModel(C.cpu().numpy(), cost, iteration, self.distanceMeasure)

    def initial_centers_csr(self, rowptr, colidx, values, numFeatures, xnorm=None,
                            partition_starts=None):
        """initial_centers for a CSR shard (dense centers)."""
        from . import kmeans_init
        _decode_measure(self.distanceMeasure)
        n = int(rowptr.shape[0]) - 1
        starts = np.asarray([0, n] if partition_starts is None else partition_starts,
                            dtype=np.int64)
        if self.initializationMode == KMeans.RANDOM:
            return kmeans_init.init_random_csr(rowptr, colidx, values, int(numFeatures), self.k,
                                               self.seed, starts)
        return kmeans_init.init_kmeans_parallel_csr(rowptr, colidx, values, int(numFeatures),
                                                    self.k, self.seed,
                                                    self.initializationSteps, starts, xnorm,
                                                    self.distanceMeasure)

    def run_csr(self, rowptr, colidx, values, numFeatures, weights=None, stream=None,
                iteration_callback=None, partition_starts=None):
        """Lloyd's algorithm over sparse points (libsvm input, KMeansExample):
        CSR rowptr (int64), colidx (int32), values (fp64) CUDA tensors; the
        centers are dense, as in the reference after the first iteration.
        Without an initial model the centers come from initial_centers_csr."""
        if self.initialModel is None:
            xn = row_norms_csr(rowptr, values, stream=stream)
            C0 = self.initial_centers_csr(rowptr, colidx, values, numFeatures, xn,
                                          partition_starts)
            self.initialModel = KMeansModel(C0, distanceMeasure=self.distanceMeasure)
            k0 = self.k
            self.k = C0.shape[0]
            try:
                return self.run_csr(rowptr, colidx, values, numFeatures, weights, stream,
                                    iteration_callback)
            finally:
                self.initialModel = None
                self.k = k0
        torch = _torch()
        dev = values.device
        d, k = int(numFeatures), self.k
        n = int(rowptr.shape[0]) - 1
        xnorm = row_norms_csr(rowptr, values, stream=stream)
        plan = KMeansPlan(d, k, n, self.distanceMeasure)
        C = torch.from_numpy(self.initialModel.clusterCenters.copy()).to(dev)
        parallel.broadcast_(C)
        cnorm = row_norms(C, stream=stream)
        buf = torch.empty(k * d + k + 1, dtype=torch.float64, device=dev)
        sums, wsum, cost_sum = buf[:k * d], buf[k * d:k * d + k], buf[k * d + k:]
        converged_t = torch.zeros(1, dtype=torch.int32, device=dev)
        iteration, converged, cost = 0, False, 0.0
        trace = [] if os.environ.get("CYC_KMEANS_FIT_TRACE") == "1" else None
        while iteration < self.maxIterations and not converged:
            buf.zero_()
            plan.accumulate_csr(rowptr, colidx, values, xnorm, weights, C, cnorm, sums, wsum,
                                cost_sum, stream=stream)
            parallel.allreduce_(buf)
            plan.update(C, cnorm, sums, wsum, self.epsilon, converged_t, stream=stream)
            converged = bool(converged_t.item())
            cost = float(cost_sum.item())
            if iteration_callback:
                iteration_callback(iteration, cost)
            iteration += 1
        plan.close()
        return KMeansModel(C.cpu().numpy(), cost, iteration, self.distanceMeasure)
