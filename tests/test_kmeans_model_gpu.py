"""GPU parity tests: KMeansModel scoring on the device --
predict (findClosest with statistics, KMeansModel.scala:82-97), pointCost /
computeCost (findClosest WITHOUT statistics, DistanceMeasure.scala:152-156,
318-340; KMeansModel.scala:110-117), dense and CSR rows, against the CPU
restatement (oracle/: orc_find_closest_stats, orc_point_costs,
orc_point_costs_sparse).

Bar: indices and per-row costs bit-exact; the computeCost sum within 1e-12
relative (device summation order differs from a Spark partitioning).
"""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


def _dev(a, cuda):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(cuda)


def _model(C):
    from cycloneml_amd.clustering import KMeansModel
    return KMeansModel(C)


def test_two_clusters_predict_and_cost(cuda):
    # KMeansSuite "two clusters" (mllib KMeansSuite.scala:255-278) points
    X = np.array([[0.0, 0.0], [0.0, 0.1], [0.1, 0.0], [9.0, 0.0], [9.0, 0.2], [9.2, 0.0]])
    C = np.array([[0.1 / 3, 0.1 / 3], [9.2 / 3 + 6.0, 0.2 / 3]])
    m = _model(C)
    p = m.predict(_dev(X, cuda)).cpu().numpy()
    assert p[0] == p[1] == p[2] and p[3] == p[4] == p[5] and p[0] != p[3]
    a, c, s = oracle.point_costs(X, oracle.row_norms(X), C, oracle.row_norms(C))
    ga, gc = m.pointCosts(_dev(X, cuda))
    assert np.array_equal(ga.cpu().numpy(), a)
    assert np.array_equal(gc.cpu().numpy(), c)
    assert m.computeCost(_dev(X, cuda)) == pytest.approx(s, rel=1e-12)


@pytest.mark.parametrize("n,d,k", [(20000, 37, 50), (5000, 256, 300), (3000, 8, 1)])
def test_dense_point_cost_and_predict_bit_exact(cuda, n, d, k):
    rng = np.random.default_rng(n + d + k)
    X = rng.normal(size=(n, d)) + rng.integers(0, 6, size=(n, 1)) * 1.5
    C = X[rng.choice(n, size=k, replace=False)].copy()
    if k > 4:
        C[3] = C[1]                          # duplicate centers: ties -> exact tier
        X[:20] = C[2]                        # rows sitting on a center
        X[20:40] = 0.5 * (C[0] + C[4])       # near-equidistant rows
    # NaN norm: findClosest WITHOUT statistics never calls fastSquaredDistance
    # (every `lowerBoundOfSqDist < bestDistance` is false, :327-329), so
    # pointCost is +inf at index 0 and no require fails; predict (WITH
    # statistics) measures center 0 first and fails MLUtils.scala:542-543
    X[40, 0] = np.nan
    X[41, 1] = np.inf
    xn, cn = oracle.row_norms(X), oracle.row_norms(C)
    a, c, s = oracle.point_costs(X, xn, C, cn)
    m = _model(C)
    ga, gc = m.pointCosts(_dev(X, cuda))
    assert np.array_equal(ga.cpu().numpy(), a)
    assert np.array_equal(gc.cpu().numpy(), c, equal_nan=True)
    assert np.isinf(gc[40].item()) and np.isinf(gc[41].item())
    # predict: findClosest with the model's statistics (a1)
    from cycloneml_amd import _native as N
    stats = oracle.kmeans_stats(C)
    with pytest.raises(oracle.IllegalArgumentException) as want_err:
        oracle.find_closest_stats(C, cn, stats, X[40], xn[40])
    with pytest.raises(N.IllegalArgumentException) as got_err:
        m.predict(_dev(X, cuda))
    assert str(got_err.value) == str(want_err.value)
    keep = np.arange(n) != 40
    want = np.array([oracle.find_closest_stats(C, cn, stats, X[r], xn[r])[0]
                     for r in range(n) if keep[r]])
    assert np.array_equal(m.predict(_dev(X[keep], cuda)).cpu().numpy(), want)
    fin = np.isfinite(c)
    mf = _model(C)
    got = mf.computeCost(_dev(X[fin], cuda))
    assert got == pytest.approx(float(np.sum(c[fin])), rel=1e-12)


def _random_csr(rng, n, d, density):
    rows, cols, vals = [0], [], []
    for _ in range(n):
        mm = max(1, rng.binomial(d, density))
        cc = np.sort(rng.choice(d, size=mm, replace=False))
        cols.extend(cc.tolist())
        vals.extend((rng.normal(size=mm) * 3.0 + rng.integers(-2, 3)).tolist())
        rows.append(len(cols))
    return (np.array(rows, np.int64), np.array(cols, np.int32), np.array(vals))


def test_csr_point_cost_and_predict_bit_exact(cuda):
    rng = np.random.default_rng(7)
    n, d, k = 3000, 300, 40
    csr = _random_csr(rng, n, d, 0.05)
    rowptr, colidx, vals = csr
    Xd = np.zeros((n, d))
    for r in range(n):
        Xd[r, colidx[rowptr[r]:rowptr[r + 1]]] = vals[rowptr[r]:rowptr[r + 1]]
    C = Xd[rng.choice(n, size=k, replace=False)].copy()
    C[5] = C[6]
    xn = oracle.row_norms_csr(rowptr, vals)
    cn = oracle.row_norms(C)
    a, c, s = oracle.point_costs_sparse(csr, xn, C, cn)
    m = _model(C)
    R, I, V = (_dev(rowptr, cuda), _dev(colidx, cuda), _dev(vals, cuda))
    ga, gc = m.pointCosts_csr(R, I, V)
    assert np.array_equal(ga.cpu().numpy(), a)
    assert np.array_equal(gc.cpu().numpy(), c)
    assert m.computeCost_csr(R, I, V) == pytest.approx(s, rel=1e-12)
    stats = oracle.kmeans_stats(C)
    want = np.array([oracle.find_closest_stats_sparse(
        C, cn, stats, colidx[rowptr[r]:rowptr[r + 1]], vals[rowptr[r]:rowptr[r + 1]], xn[r])[0]
        for r in range(n)])
    assert np.array_equal(m.predict_csr(R, I, V).cpu().numpy(), want)


def test_empty_input(cuda):
    import torch
    m = _model(np.eye(3))
    X = torch.empty(0, 3, dtype=torch.float64, device=cuda)
    assert m.predict(X).numel() == 0
    assert m.computeCost(X) == 0.0


def test_kmeans_parallel_cost_updates(cuda):
    """k-means|| cost updates (KMeans.scala:375-398) on the device: costs start
    at +inf and take min(pointCost(newCenters), cost) per step; every step
    bit-exact vs the restatement's per-row findClosest without statistics."""
    from cycloneml_amd.clustering import KMeans
    rng = np.random.default_rng(11)
    X = rng.normal(size=(4000, 24)) + rng.integers(0, 5, size=(4000, 1)) * 3.0
    xn = oracle.row_norms(X)
    want = np.full(X.shape[0], np.inf)
    got, tot = None, 0.0
    Xd = _dev(X, cuda)
    for step in range(3):
        C = X[rng.choice(X.shape[0], size=5 + 3 * step, replace=False)]
        _, c, _ = oracle.point_costs(X, xn, C, oracle.row_norms(C))
        want = np.minimum(want, c)
        got, tot = KMeans.updateParallelCosts(Xd, C, got)
        assert np.array_equal(got.cpu().numpy(), want)
        assert tot == pytest.approx(float(want.sum()), rel=1e-12)


def test_point_cost_on_a_fresh_plan(cuda):
    """cyc_kmeans_point_cost_dev needs no prior cyc_kmeans_stats_dev: a fresh
    plan (no statistics, no center transpose yet) and a plan last used for
    OTHER centers both give the restatement's bits."""
    import torch
    from cycloneml_amd.clustering import KMeansPlan, row_norms
    rng = np.random.default_rng(21)
    n, d, k = 6000, 40, 64
    X = rng.normal(size=(n, d)) + rng.integers(0, 8, size=(n, 1)) * 2.0
    C = X[rng.choice(n, size=k, replace=False)].copy()
    C2 = C + 0.5
    a, c, _ = oracle.point_costs(X, oracle.row_norms(X), C, oracle.row_norms(C))
    Xd, Cd, C2d = _dev(X, cuda), _dev(C, cuda), _dev(C2, cuda)
    xn, cn = row_norms(Xd), row_norms(Cd)
    for warm in (False, True):
        plan = KMeansPlan(d, k, n)
        if warm:
            plan.stats(C2d)      # statistics / transpose of other centers
        ga = torch.empty(n, dtype=torch.int32, device=cuda)
        gc = torch.empty(n, dtype=torch.float64, device=cuda)
        plan.point_cost(Xd, xn, Cd, cn, ga, gc)
        assert np.array_equal(ga.cpu().numpy(), a)
        assert np.array_equal(gc.cpu().numpy(), c)
