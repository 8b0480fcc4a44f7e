"""ClusteringEvaluator / ClusteringMetrics: host-side mirror of
org.apache.spark.ml.evaluation (ClusteringEvaluator.scala, ClusteringMetrics.scala).

The Silhouette of a clustering (KMeansExample's printed score): the
per-cluster statistics and every row's coefficient run in libcyclone
(cyc_kmeans_silhouette_{stats,score}_dev, csrc/silhouette.hip) over rows
resident in HBM.  With torch.distributed initialised each rank passes its
own shard; the aggregateByKey merge of computeClusterStats
(ClusteringMetrics.scala:299-337) and the two sums of overallScore (:101-103)
are one all-reduce each, as the broadcast of the merged statistics (:393) is
implicit in every rank holding them.
"""
from __future__ import annotations

from . import _native as N
from . import parallel
from .clustering import COSINE, EUCLIDEAN, KMeansPlan


def _torch():
    import torch
    return torch


SQUARED_EUCLIDEAN = "squaredEuclidean"
_EVAL_MEASURES = {SQUARED_EUCLIDEAN.lower(): EUCLIDEAN, COSINE: COSINE}


class ClusteringMetrics:
    """ClusteringMetrics (ClusteringMetrics.scala:34-60) over device rows X
    (n x d fp64), predictions (n, integer cluster ids; in [0, k) when k is
    given) and weights (n fp64 or None: lit(1.0))."""

    def __init__(self, X, predictions, weights=None, k=None):
        self.X = X
        self.predictions = predictions
        self.weights = weights
        self.k = k
        self.distanceMeasure = SQUARED_EUCLIDEAN

    def getDistanceMeasure(self) -> str:
        return self.distanceMeasure

    def setDistanceMeasure(self, value: str):
        # :41-45: require(equalsIgnoreCase("squaredEuclidean") || ... "cosine")
        if value.lower() not in _EVAL_MEASURES:
            raise N.IllegalArgumentException("requirement failed")
        self.distanceMeasure = value
        return self

    def silhouette(self, stream=None) -> float:
        """ClusteringMetrics.silhouette (:48-60): SquaredEuclideanSilhouette
        or CosineSilhouette .computeSilhouetteScore.

        Prediction ids may be any integers (the reference keys its cluster
        statistics by the prediction value, ClusteringMetrics.scala:299-337):
        with k=None they are mapped to 0..K-1 in sorted order over every
        rank's ids (the clustersStatsMap keys), which leaves the score as
        is; a given k asserts ids in [0, k) instead.  The device statistics
        sort handles K <= MAX_CLUSTERS distinct ids."""
        torch = _torch()
        X = self.X
        if X.dtype != torch.float64 or not X.is_cuda or X.dim() != 2:
            raise N.IllegalArgumentException("requirement failed: features must be a device "
                                             "fp64 matrix (n x d)")
        n, d = int(X.shape[0]), int(X.shape[1])
        pred = self.predictions.to(device=X.device)
        w = None
        if self.weights is not None:
            w = self.weights.to(device=X.device, dtype=torch.float64).contiguous()
        X = X.contiguous()
        k = self.k
        if k is None:
            pred, k = dense_cluster_ids(pred)
        else:
            pred = pred.to(torch.int32).contiguous()
        k = max(int(k), 1)
        if k > MAX_CLUSTERS:
            raise N.IllegalArgumentException(
                f"requirement failed: the device Silhouette supports at most {MAX_CLUSTERS} "
                f"distinct cluster ids, got {k}")
        measure = _EVAL_MEASURES[self.distanceMeasure.lower()]
        plan = KMeansPlan(d, k, max(n, 1), distanceMeasure=measure)
        try:
            lib = N.load()
            s = N.stream_handle(stream)
            stats = torch.zeros(k * d + 3 * k, dtype=torch.float64, device=X.device)
            # the per-rank input checks (ids in range, checkNonNegativeWeight)
            # run first inside the stats call: agreed across ranks before the
            # all-reduce, so every rank raises the same error
            parallel.agree(lambda: N.check(lib.cyc_kmeans_silhouette_stats_dev(
                plan.handle, N.ptr(X), None, n, N.ptr(pred), N.ptr(w), N.ptr(stats), s)))
            parallel.allreduce_(stats)   # combOp across executors
            partial = torch.zeros(2, dtype=torch.float64, device=X.device)
            # the one-cluster assert reads the merged statistics: every rank agrees
            N.check(lib.cyc_kmeans_silhouette_score_dev(plan.handle, N.ptr(X), None, n,
                                                        N.ptr(pred), N.ptr(w), N.ptr(stats),
                                                        N.ptr(partial), s))
            parallel.allreduce_(partial)
            total = partial.cpu()
        finally:
            plan.close()
        return float(total[0]) / float(total[1])


# the device counting sort's bound on distinct cluster ids (KMeansPlan's k)
MAX_CLUSTERS = 8192


def dense_cluster_ids(pred):
    """(ids in 0..K-1, K): every rank's distinct predictions, sorted and
    numbered, and this shard's predictions mapped onto them.  The reference
    casts the prediction column to double and keys the cluster statistics
    by that value (ClusteringMetrics.scala), so distinct doubles -- 0.5 and
    0.7 too -- stay distinct clusters.  Each rank checks its own distinct
    count against MAX_CLUSTERS before anything is gathered (every rank
    raises together through parallel.agree)."""
    torch = _torch()
    p = pred.to(torch.float64).reshape(-1)
    nan = torch.isnan(p)
    has_nan = bool(nan.any())
    # Spark groups every NaN prediction under ONE key (NaN equals NaN in
    # grouping and sorts after every other double); torch.unique would not
    local = torch.unique(p[~nan]) if has_nan else torch.unique(p)

    def bound():
        if local.numel() + has_nan > MAX_CLUSTERS:
            raise N.IllegalArgumentException(
                f"requirement failed: the device Silhouette supports at most {MAX_CLUSTERS} "
                f"distinct cluster ids, got at least {local.numel() + has_nan}")
    parallel.agree(bound)
    mine = (local.cpu().tolist(), has_nan)
    gathered = parallel.allgather_object(mine)
    keys = sorted(set().union(*[set(g) for g, _ in gathered]))
    any_nan = any(h for _, h in gathered)
    K = len(keys) + (1 if any_nan else 0)
    if K == 0:
        return torch.zeros(p.numel(), dtype=torch.int32, device=p.device), 1
    kt = torch.tensor(keys, dtype=torch.float64, device=p.device)
    ids = torch.searchsorted(kt, p) if keys else torch.zeros_like(p, dtype=torch.int64)
    if has_nan:
        ids = torch.where(nan, torch.full_like(ids, K - 1), ids)
    ids = ids.to(torch.int32).contiguous()
    if ids.numel() and int(ids.max()) >= K:   # the kernels index cluster statistics by id
        raise N.IllegalArgumentException(
            "requirement failed: a prediction maps outside the cluster ids")
    return ids, K


class ClusteringEvaluator:
    """ClusteringEvaluator (ClusteringEvaluator.scala): metricName
    "silhouette", distanceMeasure "squaredEuclidean" (default) or "cosine";
    evaluate(X, predictions, weights) plays evaluate(dataset) with the
    features / prediction / weight columns given as device tensors."""

    def __init__(self, distanceMeasure: str = SQUARED_EUCLIDEAN, metricName: str = "silhouette"):
        self.metricName = metricName
        self.distanceMeasure = distanceMeasure

    def setDistanceMeasure(self, value: str):
        # ParamValidators.inArray(Array("squaredEuclidean", "cosine")) (:89-92)
        if value not in (SQUARED_EUCLIDEAN, COSINE):
            raise N.IllegalArgumentException(
                f"ClusteringEvaluator_distanceMeasure parameter distanceMeasure given invalid "
                f"value {value}.")
        self.distanceMeasure = value
        return self

    def getDistanceMeasure(self) -> str:
        return self.distanceMeasure

    def setMetricName(self, value: str):
        if value != "silhouette":
            raise N.IllegalArgumentException(
                f"ClusteringEvaluator_metricName parameter metricName given invalid value "
                f"{value}.")
        self.metricName = value
        return self

    def isLargerBetter(self) -> bool:
        return True

    def getMetrics(self, X, predictions, weights=None, k=None) -> ClusteringMetrics:
        """getMetrics (:125-150)."""
        m = ClusteringMetrics(X, predictions, weights, k)
        m.setDistanceMeasure(self.distanceMeasure)
        return m

    def evaluate(self, X, predictions, weights=None, k=None, stream=None) -> float:
        """evaluate (:106-115)."""
        metrics = self.getMetrics(X, predictions, weights, k)
        if self.metricName == "silhouette":
            return metrics.silhouette(stream)
        raise N.IllegalArgumentException(f"No support for metric {self.metricName}")
