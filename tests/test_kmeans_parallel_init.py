"""k-means|| initialisation, the executor side (mllib/clustering/KMeans.scala:
370-404): the per-partition XORShiftRandom draws of one step on the device
against the restatement (oracle.kmeans_parallel_sample over oracle's
XORShiftRandom, itself pinned by RandomSuite's known values in
test_oracle_golden.py).  Bar: the chosen mask bit-exact.

The driver side (takeSample of the first center, LocalKMeans.kMeansPlusPlus
over the candidates) stays on the host as in the reference and is not
restated here.
"""
import numpy as np
import pytest

import oracle


def test_hash_seed_and_next_int_match_restatement():
    """XORShiftRandom.hashSeed (C ABI, host) and nextInt() against the
    restated generator, negative and wide seeds included."""
    from cycloneml_amd import _native as N
    from cycloneml_amd.clustering import xorshift_next_int
    L = N.load()
    for s in [0, 1, 42, -7, 30, 2 ** 40, -2 ** 62, 2 ** 63 - 1]:
        assert int(L.cyc_xorshift_hash_seed(s)) == oracle.XORShiftRandom(s).seed
        assert xorshift_next_int(s) == oracle.XORShiftRandom(s)._next(32)


def test_partition_starts_validated():
    import torch
    from cycloneml_amd import _native as N
    from cycloneml_amd.clustering import KMeans
    c = torch.zeros(10, dtype=torch.float64)
    with pytest.raises(N.IllegalArgumentException, match="partition_starts"):
        KMeans.parallelSample(c, 1.0, 3, 0, 5, [0, 4])


@pytest.mark.gpu
@pytest.mark.parametrize("lens,first,seed,step", [
    ([1000], 0, 12345, 0),
    ([70, 0, 129, 64, 1], 3, -99, 1),
    ([200_000, 150_001], 7, 2 ** 31 - 1, 2),
    ([33] * 40, 0, -(2 ** 31), 5),
])
def test_parallel_sample_vs_restatement(cuda, lens, first, seed, step):
    import torch
    from cycloneml_amd.clustering import KMeans
    rng = np.random.default_rng(sum(lens) + step)
    n = sum(lens)
    costs = rng.exponential(size=n)
    costs[rng.random(n) < 0.05] = 0.0
    starts = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    k = 10
    sum_costs = float(costs.sum())
    mask = KMeans.parallelSample(torch.from_numpy(costs).to(cuda), sum_costs, seed, step, k,
                                 starts, first).cpu().numpy()
    ref = oracle.kmeans_parallel_sample(costs, starts, first, seed, step, k, sum_costs)
    np.testing.assert_array_equal(mask, ref)
    assert 0 < mask.sum() < n


@pytest.mark.gpu
def test_kmeans_parallel_steps_end_to_end(cuda):
    """Two k-means|| steps from a first center (KMeans.scala:372-407): cost
    update (pointCost min, bit-exact), sumCosts, the draw -- the candidate
    rows collected in the reference's order."""
    import torch
    from cycloneml_amd.clustering import KMeans, xorshift_next_int
    rng = np.random.default_rng(8)
    n, d, k = 20_000, 16, 12
    X = rng.normal(size=(n, d)) + rng.integers(0, 6, size=(n, 1)) * 3.0
    starts = np.array([0, 5000, 9000, 15000, n], dtype=np.int64)
    seed = xorshift_next_int(2024)
    Xd = torch.from_numpy(X).to(cuda)
    centers = [X[17].copy()]
    new = np.array(centers)
    costs_d = None
    costs_h = np.full(n, np.inf)
    for step in range(2):
        costs_d, total = KMeans.updateParallelCosts(Xd, new, costs_d)
        _, pc, _ = oracle.point_costs(X, oracle.row_norms(X), new, oracle.row_norms(new))
        costs_h = np.minimum(pc, costs_h)
        np.testing.assert_array_equal(costs_d.cpu().numpy(), costs_h)
        mask = KMeans.parallelSample(costs_d, total, seed, step, k, starts).cpu().numpy()
        ref = oracle.kmeans_parallel_sample(costs_h, starts, 0, seed, step, k, total)
        np.testing.assert_array_equal(mask, ref)
        new = X[mask.astype(bool)]
        assert new.shape[0] > 0
        centers.extend(new)


# ------------------------------------------------------- driver-side init

def test_java_random_known_values():
    """java.util.Random known answers: new Random(42).nextInt() =
    -1170105035, nextLong() = -5025562857975149833 for seed 42; the
    product generator equals the test-side restatement on nextDouble."""
    from cycloneml_amd.kmeans_init import JavaRandom, XORShiftRandom
    assert JavaRandom(42).next_int() == -1170105035
    assert JavaRandom(42).next_long() == -5025562857975149833
    a, b = JavaRandom(7), oracle.JavaRandom(7)
    assert [a.next_double() for _ in range(50)] == [b.next_double() for _ in range(50)]
    x, y = XORShiftRandom(30), oracle.XORShiftRandom(30)
    assert x.next_double() == 0.2762195585886885          # RandomSuite Rand(30)
    y.next_double()
    assert [x.next_double() for _ in range(50)] == [y.next_double() for _ in range(50)]
    r = JavaRandom(3)
    vals = [r.next_int(10) for _ in range(2000)] + [r.next_int(64) for _ in range(200)]
    assert min(vals) >= 0 and max(vals[:2000]) <= 9 and max(vals[2000:]) <= 63


def test_take_sample_shapes():
    """RDD.takeSample(false, num, seed): num distinct positions in range;
    num >= count returns every item permuted; deterministic in the seed."""
    from cycloneml_amd.kmeans_init import take_sample_indices
    lens = [1000, 0, 2500, 7]
    for num in (1, 5, 40):
        s = take_sample_indices(lens, num, 123)
        assert len(s) == num and len(set(s)) == num and all(0 <= i < 3507 for i in s)
        assert s == take_sample_indices(lens, num, 123)
    allp = take_sample_indices([3, 4], 10, 9)
    assert sorted(allp) == list(range(7))
    assert take_sample_indices([5], 0, 1) == [] and take_sample_indices([0, 0], 3, 1) == []


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["k-means||", "random"])
def test_kmeans_run_without_initial_model(cuda, mode):
    """KMeans.run with the default k-means|| (or random) initialisation
    (KMeans.scala:250-259): the initial centers equal the host composition
    of the restated pieces -- takeSample, the cost passes and draws of
    oracle.kmeans_parallel_sample, oracle.local_kmeans_pp -- and the Lloyd
    run from them equals a run from those centers given as the model."""
    import torch
    from cycloneml_amd.clustering import KMeans, KMeansModel, xorshift_next_int
    from cycloneml_amd.kmeans_init import take_sample_indices
    rng = np.random.default_rng(4)
    n, d, k = 3000, 8, 4
    X = rng.normal(size=(n, d)) + rng.integers(0, 4, size=(n, 1)) * 5.0
    starts = np.array([0, 1000, 2200, n], dtype=np.int64)
    Xd = torch.from_numpy(X).to(cuda)
    km = KMeans(k=k, maxIterations=10).setSeed(77).setInitializationMode(mode)
    C0 = km.initial_centers(Xd, partition_starts=starts)
    s = xorshift_next_int(77)
    lens = np.diff(starts)
    if mode == "random":
        ref = X[take_sample_indices(lens, k, s)]
    else:
        cands = [X[take_sample_indices(lens, 1, s)[0]]]
        new = np.array(cands)
        costs = np.full(n, np.inf)
        for step in range(2):
            _, pc, _ = oracle.point_costs(X, oracle.row_norms(X), new, oracle.row_norms(new))
            costs = np.minimum(pc, costs)
            total = float(torch.from_numpy(costs).to(cuda).sum().item())   # the device fold
            mask = oracle.kmeans_parallel_sample(costs, starts, 0, s, step, k, total)
            new = X[mask.astype(bool)]
            cands.extend(new)
        uniq = []
        for c in cands:
            if not any(np.array_equal(c, u) for u in uniq):
                uniq.append(c)
        uniq = np.array(uniq)
        if uniq.shape[0] > k:
            a, _, _ = oracle.point_costs(X, oracle.row_norms(X), uniq, oracle.row_norms(uniq))
            wts = np.bincount(a, minlength=uniq.shape[0]).astype(np.float64)
            ref = oracle.local_kmeans_pp(uniq, wts, k, 30, 0)
        else:
            ref = uniq
    np.testing.assert_array_equal(C0, ref)
    m1 = km.run(Xd, partition_starts=starts)
    km2 = KMeans(k=C0.shape[0], maxIterations=10).setInitialModel(KMeansModel(C0))
    m2 = km2.run(Xd)
    np.testing.assert_array_equal(m1.clusterCenters, m2.clusterCenters)
    assert m1.numIter == m2.numIter


def _sparse_data(rng, n, d):
    """CSR rows with ~8 nonzeros each around a few cluster patterns."""
    rows = []
    for _ in range(n):
        c = rng.integers(0, 4)
        cols = np.unique(np.concatenate([rng.choice(d, size=6, replace=False),
                                         [c * 5, c * 5 + 1]]))
        vals = rng.normal(size=cols.size) + (cols // 5 == c) * 4.0
        rows.append((cols, vals))
    rowptr = np.concatenate([[0], np.cumsum([r[0].size for r in rows])]).astype(np.int64)
    colidx = np.concatenate([r[0] for r in rows]).astype(np.int32)
    vals = np.concatenate([r[1] for r in rows])
    dense = np.zeros((n, d))
    for i, (c, v) in enumerate(rows):
        dense[i, c] = v
    return (rowptr, colidx, vals), dense


def _csr_of(rows):
    nz = rows != 0.0
    rp = np.concatenate([[0], np.cumsum(nz.sum(1))]).astype(np.int64)
    r, c = np.nonzero(nz)
    return rp, c.astype(np.int32), rows[r, c]


@pytest.mark.gpu
@pytest.mark.parametrize("mode,measure", [("k-means||", "euclidean"), ("random", "euclidean"),
                                          ("k-means||", "cosine")])
def test_kmeans_run_csr_without_initial_model(cuda, mode, measure):
    """KMeans.run over sparse points without an initial model: the initial
    centers equal the host composition over the CSR restatement
    (oracle.point_costs_sparse: fastSquaredDistance(dense center, sparse
    point)), LocalKMeans over the sparse candidates through the same
    restatement; the Lloyd run from them equals a run given those centers."""
    import torch
    from cycloneml_amd.clustering import KMeans, KMeansModel, xorshift_next_int
    from cycloneml_amd.kmeans_init import take_sample_indices
    rng = np.random.default_rng(12)
    n, d, k = 3000, 40, 4
    csr, X = _sparse_data(rng, n, d)
    xn = oracle.row_norms_csr(csr[0], csr[2])
    starts = np.array([0, 1100, 2000, n], dtype=np.int64)
    dev = [torch.from_numpy(a).to(cuda) for a in csr]
    km = KMeans(k=k, maxIterations=10).setSeed(5).setInitializationMode(mode)
    km.setDistanceMeasure(measure)
    C0 = km.initial_centers_csr(*dev, d, partition_starts=starts)
    if measure == "cosine":     # the run's measure for the costs and counts
        def run_costs(C):
            return oracle.cos_point_costs_sparse(csr + (d,), xn, C, oracle.row_norms(C))
    else:
        def run_costs(C):
            return oracle.point_costs_sparse(csr, xn, C, oracle.row_norms(C))
    s = xorshift_next_int(5)
    lens = np.diff(starts)
    if mode == "random":
        ref = X[take_sample_indices(lens, k, s)]
    else:
        cands = [X[take_sample_indices(lens, 1, s)[0]]]
        new = np.array(cands)
        costs = np.full(n, np.inf)
        for step in range(2):
            _, pc, _ = run_costs(new)
            costs = np.minimum(pc, costs)
            total = float(torch.from_numpy(costs).to(cuda).sum().item())   # the device fold
            mask = oracle.kmeans_parallel_sample(costs, starts, 0, s, step, k, total)
            new = X[mask.astype(bool)]
            cands.extend(new)
        uniq = []
        for c in cands:
            if not any(np.array_equal(c, u) for u in uniq):
                uniq.append(c)
        uniq = np.array(uniq)
        assert uniq.shape[0] > k
        a, _, _ = run_costs(uniq)
        wts = np.bincount(a, minlength=uniq.shape[0]).astype(np.float64)
        cc = _csr_of(uniq)
        cn = oracle.row_norms_csr(cc[0], cc[2])

        def closest(C):
            ia, ic, _ = oracle.point_costs_sparse(cc, cn, C, oracle.row_norms(C))
            return ia, ic

        ref = oracle.local_kmeans_pp(uniq, wts, k, 30, 0, closest=closest)
    np.testing.assert_array_equal(C0, ref)
    m1 = km.run_csr(*dev, d, partition_starts=starts)
    m2 = KMeans(k=C0.shape[0], maxIterations=10).setDistanceMeasure(measure).setInitialModel(
        KMeansModel(C0, distanceMeasure=measure)).run_csr(*dev, d)
    # the CSR cluster sums are device atomics: equal to rounding
    np.testing.assert_allclose(m1.clusterCenters, m2.clusterCenters, rtol=1e-12, atol=1e-12)


def test_distinct_rows_vector_equality():
    """`.distinct` with Vector.equals semantics (mllib Vectors.equals: `!=`
    on doubles): -0.0 equals 0.0 (the first occurrence is kept), NaN rows are
    never merged, order of first occurrence."""
    from cycloneml_amd.kmeans_init import _distinct_rows
    nan = float("nan")
    R = np.array([[0.0, 1.0], [-0.0, 1.0], [nan, 2.0], [nan, 2.0], [3.0, -0.0], [3.0, 0.0],
                  [0.0, 1.0]])
    got = _distinct_rows(R)
    assert got.shape == (4, 2)
    assert np.signbit(got[0, 0]) == False and got[0, 1] == 1.0       # noqa: E712
    assert np.isnan(got[1, 0]) and np.isnan(got[2, 0])
    assert got[3, 0] == 3.0 and np.signbit(got[3, 1])                 # first: -0.0
