"""The reference's own assertions on KMeans runs WITHOUT an initial model
(initialisation "random" = initRandom, "k-means||" = initKMeansParallel,
mllib/clustering/KMeans.scala:354-432), through KMeans.run / run_csr on the
device:

- mllib KMeansSuite.scala:36-278 ("single cluster", "fewer distinct points
  than clusters", "unique cluster centers", "deterministic initialization",
  "single cluster with big dataset", "single cluster with sparse data",
  "k-means|| initialization", "two clusters"), the data partitioned as
  `sc.parallelize(seq[, numSlices])` under the suite's `local[2]`
  (MLlibTestSparkContext.scala:39: default parallelism 2);
- the pyspark doctest of ml.clustering.KMeans (python/pyspark/ml/
  clustering.py:588-626, `local[2]` at :1834): k=2, setSeed(1), weights 2.0,
  predict(head) == 0, clusterSizes [2, 2], trainingCost 4.0;
- examples ml.KMeansExample (KMeansExample.scala:45-49): libsvm input,
  k=2, setSeed(1L), the default k-means||.

The suite's unseeded `KMeans.train` calls draw their seed from
Utils.random (a random seed per run); their assertions hold for any seed,
so they run here over several seeds.
"""
import os

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SEEDS = (0, 1, 42, 12345, -7)


def slices(n, num_slices):
    """ParallelCollectionRDD.slice's partition starts: partition i holds
    positions [i * n / numSlices, (i + 1) * n / numSlices)."""
    return np.array([(i * n) // num_slices for i in range(num_slices + 1)], dtype=np.int64)


def _dev(a, cuda):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).to(cuda)


def _run(X, k, max_iter, mode, seed, num_slices, cuda, weights=None, steps=2):
    from cycloneml_amd.clustering import KMeans
    km = KMeans(k=k, maxIterations=max_iter).setInitializationMode(mode).setSeed(seed)
    km.setInitializationSteps(steps)
    w = None if weights is None else _dev(weights, cuda)
    return km.run(_dev(X, cuda), weights=w, partition_starts=slices(len(X), num_slices))


MODES = ("k-means||", "random")


@pytest.mark.parametrize("seed", SEEDS)
def test_single_cluster(cuda, seed):
    """KMeansSuite.scala:36-63: one cluster at the mean (1, 3, 4) whatever
    the iterations and initialisation mode."""
    X = np.array([[1.0, 2.0, 6.0], [1.0, 3.0, 0.0], [1.0, 4.0, 6.0]])
    for it, mode in ((1, "k-means||"), (2, "k-means||"), (5, "k-means||"), (1, "random")):
        m = _run(X, 1, it, mode, seed, 2, cuda)
        np.testing.assert_allclose(m.clusterCenters[0], [1.0, 3.0, 4.0], atol=1e-5)


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("seed", SEEDS)
def test_fewer_distinct_points_than_clusters(cuda, mode, seed):
    """KMeansSuite.scala:65-78: three equal points, k=2 -> one center."""
    X = np.array([[1.0, 2.0, 3.0]] * 3)
    m = _run(X, 2, 1, mode, seed, 2, cuda)
    assert m.clusterCenters.shape[0] == 1


def _unique_points():
    """KMeansSuite.scala:80-85: java.util.Random(42), 10 distinct points of 3
    nextDouble()s, each repeated 1 + nextInt(3) times, 2 slices."""
    from cycloneml_amd.kmeans_init import JavaRandom
    rng = JavaRandom(42)
    points = [[rng.next_double() for _ in range(3)] for _ in range(10)]
    data = []
    for p in points:
        data.extend([p] * (1 + rng.next_int(3)))
    return np.array(points), np.array(data)


def _distinct_count(C):
    return len({tuple(r) for r in np.asarray(C).tolist()})


def test_unique_cluster_centers(cuda):
    """KMeansSuite.scala:80-125 (seed 42): k-means|| with 10 steps gives
    distinct initial centers, at most the 10 distinct points for k=50 and
    exactly 10 for k=10; every final model has distinct centers, also with
    random initialisation."""
    from cycloneml_amd.clustering import KMeans
    points, data = _unique_points()
    Xd = _dev(data, cuda)
    starts = slices(len(data), 2)
    km = KMeans(k=50, maxIterations=5).setInitializationMode("k-means||") \
        .setInitializationSteps(10).setSeed(42)
    C0 = km.initial_centers(Xd, partition_starts=starts)
    assert C0.shape[0] == _distinct_count(C0) and C0.shape[0] <= 10
    fin = km.run(Xd, partition_starts=starts).clusterCenters
    assert fin.shape[0] == _distinct_count(fin)
    km2 = KMeans(k=10, maxIterations=5).setInitializationMode("k-means||") \
        .setInitializationSteps(10).setSeed(42)
    C2 = km2.initial_centers(Xd, partition_starts=starts)
    assert C2.shape[0] == _distinct_count(C2) == 10
    fin2 = km2.run(Xd, partition_starts=starts).clusterCenters
    assert fin2.shape[0] == _distinct_count(fin2)
    km3 = KMeans(k=10, maxIterations=5).setInitializationMode("random").setSeed(42)
    fin3 = km3.run(Xd, partition_starts=starts).clusterCenters
    assert fin3.shape[0] == _distinct_count(fin3)


@pytest.mark.parametrize("mode", MODES)
def test_deterministic_initialization(cuda, mode):
    """KMeansSuite.scala:127-146: points (n, n) for n < 1000 in 3 slices,
    k=10, two iterations, seed 42: two runs give the same centers (absTol
    1e-14; here bit for bit)."""
    X = np.array([[float(n), float(n)] for n in range(1000)])
    m1 = _run(X, 10, 2, mode, 42, 3, cuda)
    m2 = _run(X, 10, 2, mode, 42, 3, cuda)
    assert m1.clusterCenters.shape == (10, 2)
    np.testing.assert_array_equal(m1.clusterCenters, m2.clusterCenters)


@pytest.mark.parametrize("seed", SEEDS)
def test_single_cluster_big_dataset(cuda, seed):
    """KMeansSuite.scala:148-177: 100 copies of the three points, 4 slices."""
    small = np.array([[1.0, 2.0, 6.0], [1.0, 3.0, 0.0], [1.0, 4.0, 6.0]])
    X = np.tile(small, (100, 1))
    for it, mode in ((1, "k-means||"), (2, "k-means||"), (5, "k-means||"), (1, "random")):
        m = _run(X, 1, it, mode, seed, 4, cuda)
        assert m.clusterCenters.shape[0] == 1
        np.testing.assert_allclose(m.clusterCenters[0], [1.0, 3.0, 4.0], atol=1e-5)


@pytest.mark.parametrize("seed", SEEDS[:3])
def test_single_cluster_sparse_data(cuda, seed):
    """KMeansSuite.scala:179-216: 600 sparse rows of dimension 10,000 in 4
    slices (run_csr); the one center is (1, 3, 4, 0, ...)."""
    import torch
    from cycloneml_amd.clustering import KMeans
    n = 10000
    rows = []
    for i in range(1, 101):
        x = i / 1000.0
        rows += [[(0, 1.0 + x), (1, 2.0), (2, 6.0)], [(0, 1.0 - x), (1, 2.0), (2, 6.0)],
                 [(0, 1.0), (1, 3.0 + x)], [(0, 1.0), (1, 3.0 - x)],
                 [(0, 1.0), (1, 4.0), (2, 6.0 + x)], [(0, 1.0), (1, 4.0), (2, 6.0 - x)]]
    rowptr = np.concatenate([[0], np.cumsum([len(r) for r in rows])]).astype(np.int64)
    colidx = np.array([c for r in rows for c, _ in r], dtype=np.int32)
    vals = np.array([v for r in rows for _, v in r])
    dev = (torch.from_numpy(rowptr).to(cuda), torch.from_numpy(colidx).to(cuda),
           torch.from_numpy(vals).to(cuda))
    want = np.zeros(n)
    want[:3] = [1.0, 3.0, 4.0]
    for it, mode in ((1, "k-means||"), (2, "k-means||"), (5, "k-means||"), (1, "random")):
        km = KMeans(k=1, maxIterations=it).setInitializationMode(mode).setSeed(seed)
        m = km.run_csr(*dev, n, partition_starts=slices(len(rows), 4))
        np.testing.assert_allclose(m.clusterCenters[0], want, atol=1e-5)


@pytest.mark.parametrize("seed", SEEDS)
def test_kmeans_parallel_initialization(cuda, seed):
    """KMeansSuite.scala:218-253: five points, k=5: k-means|| places a center
    on every point (after 1 and after 10 Lloyd iterations)."""
    P = np.array([[1.0, 2.0, 6.0], [1.0, 3.0, 0.0], [1.0, 4.0, 6.0], [1.0, 0.0, 1.0],
                  [1.0, 1.0, 1.0]])
    for it in (1, 10):
        m = _run(P, 5, it, "k-means||", seed, 2, cuda)
        got = sorted(m.clusterCenters.tolist(), key=lambda r: -sum(v * v for v in r))
        want = sorted(P.tolist(), key=lambda r: -sum(v * v for v in r))
        np.testing.assert_allclose(got, want, atol=1e-5)


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("seed", SEEDS)
def test_two_clusters(cuda, mode, seed):
    """KMeansSuite.scala:255-278: six points in 3 slices, k=2, two
    iterations suffice from any initial centers."""
    X = np.array([[0.0, 0.0], [0.0, 0.1], [0.1, 0.0], [9.0, 0.0], [9.0, 0.2], [9.2, 0.0]])
    m = _run(X, 2, 2, mode, seed, 3, cuda)
    p = m.predict(_dev(X, cuda)).cpu().numpy()
    assert p[0] == p[1] == p[2] and p[3] == p[4] == p[5] and p[0] != p[3]


def test_pyspark_doctest_weighted(cuda):
    """python/pyspark/ml/clustering.py:588-626 under local[2] (:1834): four
    weighted points in 2 partitions, KMeans(k=2).setSeed(1), weightCol 2.0,
    default maxIter 20 / k-means|| / initSteps 2 / tol 1e-4:
    predict(head) == 0, two centers, rows 0/1 and 2/3 together,
    clusterSizes [2, 2], trainingCost 4.0."""
    X = np.array([[0.0, 0.0], [1.0, 1.0], [9.0, 8.0], [8.0, 9.0]])
    m = _run(X, 2, 20, "k-means||", 1, 2, cuda, weights=np.full(4, 2.0))
    assert m.clusterCenters.shape == (2, 2)
    p = m.predict(_dev(X, cuda)).cpu().numpy()
    assert int(p[0]) == 0
    assert p[0] == p[1] and p[2] == p[3]
    assert np.bincount(p, minlength=2).tolist() == [2, 2]
    assert m.trainingCost == 4.0


def test_kmeans_example_default_init(cuda):
    """examples ml.KMeansExample (KMeansExample.scala:45-49) as the reference
    runs it: data/mllib/sample_kmeans_data.txt read as libsvm (one file
    smaller than a split: 1 partition), KMeans().setK(2).setSeed(1L) with
    the default k-means|| initialisation, maxIter 20, tol 1e-4.  Clusters
    {0,1,2} / {3,4,5}, centers (0.1, 0.1, 0.1) / (9.1, 9.1, 9.1); the
    per-row costs of the fitted model bit-exact vs the restatement."""
    from cycloneml_amd import mlutils
    from cycloneml_amd.clustering import KMeans
    path = os.path.join(GOLD, "sample_kmeans_data.txt")
    blk = mlutils.loadLibSVMFile(path, device=cuda)
    km = KMeans().setK(2).setSeed(1)
    assert km.maxIterations == 20 and km.epsilon == 1e-4
    assert km.initializationMode == "k-means||" and km.initializationSteps == 2
    model = km.run_csr(blk.rowptr, blk.colidx, blk.values, blk.numFeatures,
                       partition_starts=slices(6, 1))
    np.testing.assert_allclose(sorted(model.clusterCenters.tolist()),
                               [[0.1, 0.1, 0.1], [9.1, 9.1, 9.1]], atol=1e-12)
    p = model.predict_csr(blk.rowptr, blk.colidx, blk.values).cpu().numpy()
    assert p[0] == p[1] == p[2] and p[3] == p[4] == p[5] and p[0] != p[3]
    _, csr, _ = oracle.parse_libsvm(open(path).read())
    C = model.clusterCenters
    _, want, _ = oracle.point_costs_sparse(csr, oracle.row_norms_csr(csr[0], csr[2]), C,
                                           oracle.row_norms(C))
    _, got = model.pointCosts_csr(blk.rowptr, blk.colidx, blk.values)
    assert np.array_equal(got.cpu().numpy(), want)
    # KMeansExample.scala:51-56: ClusteringEvaluator().evaluate(predictions),
    # the squared-Euclidean Silhouette of the fitted clustering (the sparse
    # rows' dot / axpy / norm visit the same nonzeros as their dense form)
    from cycloneml_amd.evaluation import ClusteringEvaluator
    rowptr, colidx, vals = csr
    Xd = np.zeros((6, blk.numFeatures))
    for i in range(6):
        Xd[i, colidx[rowptr[i]:rowptr[i + 1]]] = vals[rowptr[i]:rowptr[i + 1]]
    import torch
    sil = ClusteringEvaluator().evaluate(torch.as_tensor(Xd, device=cuda),
                                         torch.as_tensor(p, device=cuda))
    want_sil, _ = oracle.silhouette(Xd, p.astype(np.int32), 2)
    assert abs(sil - want_sil) <= 1e-12 * abs(want_sil)
    assert 0.99 < sil < 1.0
