"""ClusteringEvaluator's Silhouette (ml/evaluation/ClusteringMetrics.scala
SquaredEuclideanSilhouette :254-400, CosineSilhouette :403-600).

The restatement (oracle/cyclone_oracle.c orc_silhouette) is pinned by the
reference's known answers (CPU tests): ClusteringEvaluatorSuite's iris
scores, "squared euclidean Silhouette" 0.6564679231 and "cosine Silhouette"
0.7222369298 (ClusteringEvaluatorSuite.scala:62-100; iris_libsvm.txt is the
reference's data/mllib file, committed under tests/golden), its weight
support, single-element-cluster and number-of-clusters assertions
(:126-204), and the pyspark doctest (python/pyspark/ml/evaluation.py:
701-721, 0.9079...).  The device path (cyc_kmeans_silhouette_*_dev) is
checked against the restatement at 1e-12 relative on the same inputs.
"""
import os

import numpy as np
import pytest

import oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def iris():
    rows = [ln.split() for ln in open(os.path.join(GOLD, "iris_libsvm.txt")) if ln.strip()]
    y = np.array([float(r[0]) for r in rows])
    X = np.zeros((len(rows), 4))
    for i, r in enumerate(rows):
        for t in r[1:]:
            a, b = t.split(":")
            X[i, int(a) - 1] = float(b)
    return X, y.astype(np.int32)


def rel(a, b):
    return abs(a - b) / max(abs(b), 1e-300)


# pyspark doctest (evaluation.py:701-721)
DOCTEST_X = np.array([[0.0, 0.5], [0.5, 0.0], [10.0, 11.0], [10.5, 11.5], [1.0, 1.0],
                      [8.0, 6.0]])
DOCTEST_P = np.array([0, 0, 1, 1, 0, 1], dtype=np.int32)
# "single-element clusters with weight" (ClusteringEvaluatorSuite.scala:190-203)
SINGLE_X = np.array([[5.1, 3.5, 1.4, 0.2], [7.0, 3.2, 4.7, 1.4], [6.3, 3.3, 6.0, 2.5]])
SINGLE_P = np.array([0, 1, 2], dtype=np.int32)
SINGLE_W = np.array([6.0, 0.25, 9.99])


# ---------------------------------------------------------------- oracle pins

@pytest.mark.parametrize("cosine,expected", [(False, 0.6564679231), (True, 0.7222369298)])
def test_oracle_iris_known_answers(cosine, expected):
    X, p = iris()
    assert rel(O.silhouette(X, p, 3, cosine=cosine)[0], expected) < 1e-5
    # newIrisDataset: features through Float (MLTestingUtils.scala:257-270)
    Xf = X.astype(np.float32).astype(np.float64)
    assert rel(O.silhouette(Xf, p, 3, cosine=cosine)[0], expected) < 1e-5


@pytest.mark.parametrize("cosine", [False, True])
def test_oracle_weight_support(cosine):
    X, p = iris()
    s1 = O.silhouette(X, p, 3, cosine=cosine)[0]
    for w in (0.25, 1.0, 10.0, 99.99):
        s2 = O.silhouette(X, p, 3, np.full(len(p), w), cosine=cosine)[0]
        assert rel(s2, s1) < 1e-6


def test_oracle_pyspark_doctest():
    s = O.silhouette(DOCTEST_X, DOCTEST_P, 2)[0]
    assert f"{s:.4f}".startswith("0.9079") or str(s).startswith("0.9079")
    sw = O.silhouette(DOCTEST_X, DOCTEST_P, 2, np.full(6, 2.5))[0]
    assert str(sw).startswith("0.9079")


@pytest.mark.parametrize("cosine", [False, True])
def test_oracle_single_element_clusters(cosine):
    X, p = iris()
    i0, i1 = int(np.where(p == 0)[0][0]), int(np.where(p == 1)[0][0])
    assert O.silhouette(X[[i0, i1]], p[[i0, i1]], 3, cosine=cosine)[0] == 0.0
    assert O.silhouette(SINGLE_X, SINGLE_P, 3, SINGLE_W, cosine=cosine)[0] == 0.0


@pytest.mark.parametrize("cosine", [False, True])
def test_oracle_number_of_clusters(cosine):
    X, p = iris()
    m = p == 0
    with pytest.raises(AssertionError, match="Number of clusters must be greater than one"):
        O.silhouette(X[m], p[m], 3, cosine=cosine)


# ---------------------------------------------------------------- device path

def _dev(cuda, *arrs):
    import torch
    return [None if a is None else torch.as_tensor(a, device=cuda) for a in arrs]


def _evaluate(cuda, X, p, k=None, w=None, cosine=False):
    from cycloneml_amd.evaluation import ClusteringEvaluator
    Xd, pd, wd = _dev(cuda, np.ascontiguousarray(X, dtype=np.float64), p, w)
    ev = ClusteringEvaluator(distanceMeasure="cosine" if cosine else "squaredEuclidean")
    return ev.evaluate(Xd, pd, wd, k=k)


@pytest.mark.gpu
@pytest.mark.parametrize("cosine,expected", [(False, 0.6564679231), (True, 0.7222369298)])
def test_device_iris(cuda, cosine, expected):
    X, p = iris()
    s = _evaluate(cuda, X, p, cosine=cosine)
    assert rel(s, O.silhouette(X, p, 3, cosine=cosine)[0]) < 1e-12
    assert rel(s, expected) < 1e-5
    for w in (0.25, 10.0, 99.99):
        sw = _evaluate(cuda, X, p, w=np.full(len(p), w), cosine=cosine)
        assert rel(sw, s) < 1e-6


@pytest.mark.gpu
def test_device_pyspark_doctest(cuda):
    assert str(_evaluate(cuda, DOCTEST_X, DOCTEST_P)).startswith("0.9079")
    assert str(_evaluate(cuda, DOCTEST_X, DOCTEST_P, w=np.full(6, 2.5))).startswith("0.9079")


@pytest.mark.gpu
@pytest.mark.parametrize("cosine", [False, True])
def test_device_single_element_clusters(cuda, cosine):
    X, p = iris()
    i0, i1 = int(np.where(p == 0)[0][0]), int(np.where(p == 1)[0][0])
    assert _evaluate(cuda, X[[i0, i1]], p[[i0, i1]], k=3, cosine=cosine) == 0.0
    assert _evaluate(cuda, SINGLE_X, SINGLE_P, w=SINGLE_W, cosine=cosine) == 0.0


@pytest.mark.gpu
@pytest.mark.parametrize("cosine", [False, True])
def test_device_errors(cuda, cosine):
    from cycloneml_amd import _native as N
    X, p = iris()
    m = p == 0
    with pytest.raises(N.JavaAssertionError,
                       match="assertion failed: Number of clusters must be greater than one."):
        _evaluate(cuda, X[m], p[m], k=3, cosine=cosine)
    w = np.ones(len(p))
    w[7] = -1.0
    with pytest.raises(N.IllegalArgumentException,
                       match=r"illegal weight value: -1\.0\. weight must be >= 0\.0\."):
        _evaluate(cuda, X, p, w=w, cosine=cosine)
    bad = p.copy()
    bad[3] = 5
    with pytest.raises(N.IllegalArgumentException, match="predictions must lie in"):
        _evaluate(cuda, X, bad, k=3, cosine=cosine)


@pytest.mark.gpu
@pytest.mark.parametrize("cosine", [False, True])
def test_device_arbitrary_cluster_ids(cuda, cosine):
    """Any integer ids (negative, past the device sort's 8192, sparse) give
    the score of the same clustering numbered 0..K-1 (the reference keys its
    statistics by the prediction value); more than 8192 distinct ids raise."""
    from cycloneml_amd import _native as N
    X, p = iris()
    ref = _evaluate(cuda, X, p, cosine=cosine)
    ids = np.array([-7, 40_000, 9_999_999_999], dtype=np.int64)
    assert _evaluate(cuda, X, ids[p], cosine=cosine) == ref
    rng = np.random.default_rng(3)
    n = 20_000
    many = rng.permutation(n).astype(np.int64) * 3
    with pytest.raises(N.IllegalArgumentException, match="at most 8192 distinct"):
        _evaluate(cuda, rng.normal(size=(n, 4)), many, cosine=cosine)


@pytest.mark.gpu
@pytest.mark.parametrize("n,d,k,weighted,cosine", [
    (200_003, 64, 50, True, False), (200_003, 64, 50, True, True),
    (65_536, 256, 1024, False, False), (70_001, 17, 3, True, False),
    (50_000, 300, 130, False, True)])
def test_device_matches_restatement(cuda, n, d, k, weighted, cosine):
    """Random clusterings (some clusters empty, zero weights present) at
    1e-12 relative; the statistics buffer against the restatement's."""
    import torch
    from cycloneml_amd import _native as N
    from cycloneml_amd.clustering import KMeansPlan
    rng = np.random.default_rng(n + d + k)
    C = rng.normal(size=(k, d)) * 4.0
    p = rng.integers(0, max(k - 3, 2), size=n).astype(np.int32)   # the last clusters empty
    X = C[p] + rng.normal(size=(n, d))
    w = None
    if weighted:
        w = rng.random(n) * 3.0
        w[rng.integers(0, n, size=n // 100)] = 0.0
    s_ref, st_ref = O.silhouette(X, p, k, w, cosine=cosine)
    s = _evaluate(cuda, X, p, k=k, w=w, cosine=cosine)
    assert rel(s, s_ref) < 1e-12
    # the statistics themselves (sorted fixed-order folds vs row order)
    Xd, pd, wd = _dev(cuda, X, p, w)
    plan = KMeansPlan(d, k, n, distanceMeasure="cosine" if cosine else "euclidean")
    stats = torch.zeros(k * d + 3 * k, dtype=torch.float64, device=cuda)
    N.check(N.load().cyc_kmeans_silhouette_stats_dev(plan.handle, N.ptr(Xd), None, n,
                                                     N.ptr(pd), N.ptr(wd), N.ptr(stats), None))
    got = stats.cpu().numpy()
    np.testing.assert_allclose(got, st_ref, rtol=1e-11, atol=1e-9)
    assert np.array_equal(got[-k:], st_ref[-k:])   # row counts exact
    plan.close()
