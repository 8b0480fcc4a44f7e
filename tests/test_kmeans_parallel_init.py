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
