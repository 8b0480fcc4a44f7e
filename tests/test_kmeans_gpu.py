"""GPU parity tests: libcyclone KMeans kernels vs the CPU restatement (oracle/).

Bar (BASELINE.json north_star): assignments and per-point costs bit-exact;
sums / centers within 1e-10 relative (we assert tighter where the order is
known).  Every call goes through the C ABI (cycloneml_amd/_native.py).
"""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


def _dev(a, cuda):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(cuda)


def _plan(d, k, n=1):
    from cycloneml_amd.clustering import KMeansPlan
    return KMeansPlan(d, k, n)


def _gpu_assign(X, C, cuda, count_exact=True):
    import torch
    from cycloneml_amd.clustering import row_norms
    Xd, Cd = _dev(X, cuda), _dev(C, cuda)
    xn, cn = row_norms(Xd), row_norms(Cd)
    p = _plan(X.shape[1], C.shape[0], X.shape[0])
    p.stats(Cd)
    a = torch.empty(X.shape[0], dtype=torch.int32, device=cuda)
    c = torch.empty(X.shape[0], dtype=torch.float64, device=cuda)
    n_exact = p.assign(Xd, xn, Cd, cn, a, c, count_exact=count_exact)
    torch.cuda.synchronize()
    return a.cpu().numpy(), c.cpu().numpy(), n_exact, xn.cpu().numpy(), cn.cpu().numpy()


def _oracle_assign(X, C):
    xn, cn = oracle.row_norms(X), oracle.row_norms(C)
    stats = oracle.kmeans_stats(C)
    a, dist, *_ = oracle.kmeans_partition(X, xn, None, C, cn, stats)
    return a, dist


@pytest.mark.parametrize("n,d", [(1, 1), (63, 3), (1000, 8), (777, 13), (4096, 256), (300, 257)])
def test_row_norms_bitexact(cuda, n, d):
    from cycloneml_amd.clustering import row_norms
    rng = np.random.default_rng(n * 31 + d)
    X = rng.normal(size=(n, d)) * rng.uniform(0.1, 100, size=(n, 1))
    got = row_norms(_dev(X, cuda)).cpu().numpy()
    np.testing.assert_array_equal(got, oracle.row_norms(X))


@pytest.mark.parametrize("k,d", [(1, 4), (2, 3), (17, 5), (130, 64), (1024, 256)])
def test_stats_bitexact(cuda, k, d):
    import torch
    rng = np.random.default_rng(k + d)
    C = rng.normal(size=(k, d)) * 3.0
    p = _plan(d, k)
    out = torch.empty(k * (k + 1) // 2, dtype=torch.float64, device=cuda)
    p.stats(_dev(C, cuda), out)
    got = out.cpu().numpy()
    ref = oracle.kmeans_stats(C)          # every packed entry, k = 1024 included
    assert got.shape == ref.shape == (k * (k + 1) // 2,)
    np.testing.assert_array_equal(np.isnan(got), np.isnan(ref))
    np.testing.assert_array_equal(got[~np.isnan(got)], ref[~np.isnan(ref)])


@pytest.mark.parametrize("n,d,k", [(2000, 2, 2), (3000, 3, 5), (1000, 8, 10), (2500, 16, 37),
                                   (2000, 64, 130), (1500, 256, 300), (700, 300, 33),
                                   (500, 513, 20), (64, 1, 1)])
def test_assign_bitexact(cuda, n, d, k):
    rng = np.random.default_rng(n + d + k)
    true_c = rng.normal(scale=4.0, size=(max(k // 2, 1), d))
    X = true_c[rng.integers(0, true_c.shape[0], n)] + rng.normal(size=(n, d))
    C = X[rng.choice(n, size=k, replace=False)] if k <= n else rng.normal(size=(k, d))
    a, c, n_exact, xn, cn = _gpu_assign(X, C, cuda)
    np.testing.assert_array_equal(xn, oracle.row_norms(X))
    ra, rc = _oracle_assign(X, C)
    np.testing.assert_array_equal(a, ra)
    np.testing.assert_array_equal(c, rc)


def test_distance_measure_suite(cuda):
    """DistanceMeasureSuite.scala:28-63 data (java.util.Random(42), k=10, dim=8,
    1000 points): findClosest with and without statistics agree (reference
    assertion), and the GPU equals both bit for bit."""
    rng = oracle.JavaRandom(42)
    C = np.array([[rng.next_gaussian() for _ in range(8)] for _ in range(10)])
    X = np.array([[rng.next_gaussian() for _ in range(8)] for _ in range(1000)])
    cn = oracle.row_norms(C)
    stats = oracle.kmeans_stats(C)
    for x in X[:200]:
        xn = oracle.norm2(x)
        assert oracle.find_closest(C, cn, x, xn) == oracle.find_closest_stats(C, cn, stats, x, xn)
    a, c, *_ = _gpu_assign(X, C, cuda)
    ra, rc = _oracle_assign(X, C)
    np.testing.assert_array_equal(a, ra)
    np.testing.assert_array_equal(c, rc)


def test_assign_ties_and_duplicates(cuda):
    """Duplicate centers and points equidistant to two centers force the
    exact-emulation path; results must still be the reference's."""
    rng = np.random.default_rng(7)
    d = 24
    base = rng.normal(size=(6, d))
    C = np.vstack([base, base[:3], base[2:4] * 1.0])          # duplicated centers
    mid = 0.5 * (C[0] + C[1])
    X = np.vstack([rng.normal(size=(500, d)), np.repeat(mid[None], 50, 0), C,
                   C[:4] + 1e-13])
    a, c, n_exact, *_ = _gpu_assign(X, C, cuda)
    ra, rc = _oracle_assign(X, C)
    assert n_exact > 0
    np.testing.assert_array_equal(a, ra)
    np.testing.assert_array_equal(c, rc)


def test_assign_nonfinite(cuda):
    """+Inf norms pass the require (Inf >= 0.0) and rows with them keep the
    reference's index / cost; 1e200 rows overflow sqdist to +Inf."""
    rng = np.random.default_rng(3)
    X = rng.normal(size=(200, 16))
    X[7, 0] = np.inf
    X[8, 3] = -np.inf
    X[9, :] = 1e200
    C = rng.normal(size=(9, 16))
    a, c, n_exact, *_ = _gpu_assign(X, C, cuda)
    ra, rc = _oracle_assign(X, C)
    np.testing.assert_array_equal(a, ra)
    np.testing.assert_array_equal(c, rc)


def _require_message(fn):
    with pytest.raises(oracle.IllegalArgumentException) as e:
        fn()
    return str(e.value)


@pytest.mark.parametrize("case", ["row", "rows", "center0", "center_m", "k1_center", "csr"])
@pytest.mark.parametrize("path", ["assign", "accumulate"])
def test_nan_norm_require(cuda, case, path):
    """MLUtils.fastSquaredDistance's require(norm1 >= 0.0 && norm2 >= 0.0)
    (MLUtils.scala:542-543) on the with-statistics paths: a NaN-norm point
    fails at (center 0, point) (DistanceMeasure.scala:286), a NaN center
    fails computeStatistics' pair loop (:55-66).  The device returns
    CYC_ERR_INVALID_ARG with the restatement's exact message (Java
    Double.toString of the norms)."""
    import torch
    from cycloneml_amd import _native as N
    from cycloneml_amd.clustering import KMeansPlan, row_norms, row_norms_csr
    rng = np.random.default_rng(5)
    n, d, k = 300, 24, 1 if case == "k1_center" else 7
    X = rng.normal(size=(n, d)) * 3.0
    C = rng.normal(size=(k, d))
    if case == "row":
        X[117, 4] = np.nan
    elif case == "rows":
        X[[250, 33, 180], [0, 5, 23]] = np.nan
        X[10, 2] = np.inf                   # +Inf norm passes the require
    elif case == "center0":
        C[0, 3] = np.nan
    elif case in ("center_m", "k1_center"):
        C[k - 1 if case == "center_m" else 0, 1] = np.nan
        if case == "center_m":
            C[k - 3, 0] = np.nan            # the lowest NaN center is reported
    if case == "csr":
        X[X < 1.0] = 0.0                    # sparse rows
        X[41, 7] = np.nan
    xn, cn = oracle.row_norms(X), oracle.row_norms(C)
    if case == "csr":
        rowptr = np.concatenate([[0], np.cumsum((X != 0).sum(1))]).astype(np.int64)
        nz = np.nonzero(X != 0)
        colidx, vals = nz[1].astype(np.int32), X[nz]
        xn = oracle.row_norms_csr(rowptr, vals)
        want = _require_message(lambda: oracle.kmeans_partition_sparse(
            (rowptr, colidx, vals), xn, None, C, cn, oracle.kmeans_stats(C)))
    else:
        want = _require_message(lambda: oracle.kmeans_iteration(X, xn, None, C, cn))
    assert want.startswith("requirement failed: Both norms should be greater or equal to 0.0")
    Cd = _dev(C, cuda)
    cnd = row_norms(Cd)
    plan = KMeansPlan(d, k, n)
    a = torch.empty(n, dtype=torch.int32, device=cuda)
    c = torch.empty(n, dtype=torch.float64, device=cuda)
    sums = torch.zeros(k * d, dtype=torch.float64, device=cuda)
    wsum = torch.zeros(k, dtype=torch.float64, device=cuda)
    cost = torch.zeros(1, dtype=torch.float64, device=cuda)
    with pytest.raises(N.IllegalArgumentException) as got:
        if case == "csr":
            R, I, V = _dev(rowptr, cuda), _dev(colidx, cuda), _dev(vals, cuda)
            xnd = row_norms_csr(R, V)
            if path == "assign":
                try:
                    plan.stats(Cd)
                except N.IllegalArgumentException:
                    raise AssertionError("centers are finite")
                plan.assign_csr(R, I, V, xnd, Cd, cnd, a, c)
            else:
                plan.accumulate_csr(R, I, V, xnd, None, Cd, cnd, sums, wsum, cost)
        else:
            Xd = _dev(X, cuda)
            xnd = row_norms(Xd)
            if path == "assign":
                plan.stats(Cd)            # NaN centers fail here (computeStatistics)
                plan.assign(Xd, xnd, Cd, cnd, a, c, rows=plan.rows(Xd))
            else:
                plan.accumulate(Xd, xnd, None, Cd, cnd, sums, wsum, cost, rows=plan.rows(Xd))
    assert str(got.value) == want
    # the plan stays usable after the failure
    Xf = np.nan_to_num(X, nan=0.5)
    Cf = np.nan_to_num(C, nan=0.25)
    af, cf, *_ = _gpu_assign(Xf, Cf, cuda)
    ra, rc = _oracle_assign(Xf, Cf)
    np.testing.assert_array_equal(af, ra)
    np.testing.assert_array_equal(cf, rc)


@pytest.mark.parametrize("use_rows", [False, True])
@pytest.mark.parametrize("n,d,k,weighted", [(5000, 16, 12, False), (20000, 256, 64, True),
                                            (3000, 7, 1, False), (4000, 600, 9, True),
                                            (1500, 1100, 5, False),
                                            # >= 2^20 rows with the row image: the
                                            # parts pipeline (sums stream)
                                            (1_200_001, 32, 40, True)])
def test_lloyd_iteration(cuda, n, d, k, weighted, use_rows):
    import torch
    from cycloneml_amd.clustering import row_norms
    rng = np.random.default_rng(n + k)
    X = rng.normal(size=(n, d)) + rng.integers(0, 5, size=(n, 1)) * 3.0
    C = X[rng.choice(n, size=k, replace=False)].copy()
    w = rng.uniform(0.5, 2.0, size=n) if weighted else None
    ref = oracle.kmeans_iteration(X, oracle.row_norms(X), w, C, oracle.row_norms(C))
    Xd, Cd = _dev(X, cuda), _dev(C, cuda)
    wd = None if w is None else _dev(w, cuda)
    xn, cn = row_norms(Xd), row_norms(Cd)
    p = _plan(d, k, n)
    sums = torch.zeros(k * d, dtype=torch.float64, device=cuda)
    wsum = torch.zeros(k, dtype=torch.float64, device=cuda)
    cost = torch.zeros(1, dtype=torch.float64, device=cuda)
    a = torch.empty(n, dtype=torch.int32, device=cuda)
    pc = torch.empty(n, dtype=torch.float64, device=cuda)
    rows = p.rows(Xd) if use_rows else None
    p.accumulate(Xd, xn, wd, Cd, cn, sums, wsum, cost, a, pc, rows=rows)
    conv = torch.zeros(1, dtype=torch.int32, device=cuda)
    p.update(Cd, cn, sums, wsum, 1e-4, conv)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(a.cpu().numpy(), ref["assign"])
    np.testing.assert_array_equal(pc.cpu().numpy(), ref["dist"])
    np.testing.assert_allclose(wsum.cpu().numpy(), ref["wsum"], rtol=1e-12)
    np.testing.assert_allclose(sums.cpu().numpy().reshape(k, d), ref["sums"], rtol=1e-10,
                               atol=1e-10 * np.abs(ref["sums"]).max())
    assert abs(cost.item() - ref["cost"]) <= 1e-12 * abs(ref["cost"])
    np.testing.assert_allclose(Cd.cpu().numpy(), ref["centers"], rtol=1e-10,
                               atol=1e-12 * np.abs(ref["centers"]).max())
    np.testing.assert_allclose(cn.cpu().numpy(), ref["cnorm"], rtol=1e-12)
    assert bool(conv.item()) == ref["converged"]


@pytest.mark.parametrize("d", [64, 256, 255])
def test_rows_image_unaligned(cuda, d):
    """The row image from rows that start 8 bytes past a 16-byte boundary
    (k_rows_quantize's 8-byte load path; even d otherwise takes 16-byte
    loads) gives the oracle's assignment and distances."""
    import torch
    from cycloneml_amd.clustering import row_norms
    n, k = 3001, 24
    rng = np.random.default_rng(d)
    X = rng.normal(size=(n, d)) + rng.integers(0, 6, size=(n, 1)) * 2.5
    C = X[rng.choice(n, size=k, replace=False)].copy()
    buf = torch.empty(n * d + 1, dtype=torch.float64, device=cuda)
    Xd = buf[1:].view(n, d)
    Xd.copy_(torch.from_numpy(X))
    assert Xd.data_ptr() % 16 == 8
    Cd = _dev(C, cuda)
    xn, cn = row_norms(Xd), row_norms(Cd)
    p = _plan(d, k, n)
    a = torch.empty(n, dtype=torch.int32, device=cuda)
    c = torch.empty(n, dtype=torch.float64, device=cuda)
    p.assign(Xd, xn, Cd, cn, a, c, rows=p.rows(Xd))
    ra, rc = _oracle_assign(X, C)
    np.testing.assert_array_equal(a.cpu().numpy(), ra)
    np.testing.assert_array_equal(c.cpu().numpy(), rc)


def test_weighted_centers_exact(cuda):
    """ml/clustering/KMeansSuite.scala:323-411 'Two centers with weightCol':
    exact (===) centers after convergence, up to the order of the clusters."""
    from cycloneml_amd.clustering import KMeans, KMeansModel
    import torch
    pts = np.array([[0.0, 0.0], [0.0, 0.1], [0.1, 0.0], [9.0, 0.0], [9.0, 0.2], [9.2, 0.0]])
    for w, expect in [
        ([2.0] * 6, {(9.066666666666666, 0.06666666666666667),
                     (0.03333333333333333, 0.03333333333333333)}),
        ([1.0, 2.0, 3.0, 2.5, 1.0, 2.0], {(9.072727272727272, 0.03636363636363637),
                                          (0.05, 0.03333333333333333)}),
    ]:
        km = KMeans(k=2, maxIterations=10).setInitialModel(KMeansModel(pts[[0, 3]]))
        model = km.run(_dev(pts, cuda), weights=_dev(np.array(w), cuda))
        got = {tuple(map(float, c)) for c in model.clusterCenters}
        assert got == expect


@pytest.mark.timeout(900)
def test_full_config_all_rows(cuda):
    """BASELINE config 2 at full size on EXACTLY the rows bench.py times
    (bench.kmeans_data: the same seeds and 1M-row chunks) and its initial
    centers (rows 0..1023): EVERY row's assignment and cost equals the
    restatement bit for bit (oracle run as 16 row partitions on the host's
    threads, about a minute), the k = 1024 statistics equal the restatement's
    in all 524,800 packed entries, the cluster sums / weights / cost agree
    with the restatement's partition-ordered merge to 1e-10, and the
    size-independent identities hold (weights sum to n, cluster sums add up
    to the column sums of X).  The tier counts the bench line reports come
    from this data."""
    import os
    import sys
    import torch
    from cycloneml_amd.clustering import row_norms
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    n, d, k = 10_000_000, 256, 1024
    X = bench.kmeans_data(n, cuda, 0, d, k)
    C = X[:k].clone()
    st = torch.empty(k * (k + 1) // 2, dtype=torch.float64, device=cuda)
    _plan(d, k).stats(C, st)
    ref_st = oracle.kmeans_stats(C.cpu().numpy())
    np.testing.assert_array_equal(st.cpu().numpy(), ref_st)
    xn, cn = row_norms(X), row_norms(C)
    p = _plan(d, k, n)
    sums = torch.zeros(k * d, dtype=torch.float64, device=cuda)
    wsum = torch.zeros(k, dtype=torch.float64, device=cuda)
    cost = torch.zeros(1, dtype=torch.float64, device=cuda)
    a = torch.empty(n, dtype=torch.int32, device=cuda)
    pc = torch.empty(n, dtype=torch.float64, device=cuda)
    rows = p.rows(X)
    p.accumulate(X, xn, None, C, cn, sums, wsum, cost, a, pc, rows=rows)
    torch.cuda.synchronize()
    del rows
    assert wsum.sum().item() == n
    colsum = X.sum(0)
    np.testing.assert_allclose(sums.view(k, d).sum(0).cpu().numpy(), colsum.cpu().numpy(),
                               rtol=1e-9, atol=1e-6)
    assert abs(cost.item() - pc.sum().item()) <= 1e-10 * cost.item()
    # every row against the restatement (Spark local[16]: 16 partitions)
    threads = min(int(os.environ.get("OMP_NUM_THREADS", "0")) or 16, os.cpu_count() or 1, 16)
    Xh = X.cpu().numpy()
    del X
    xnh = xn.cpu().numpy()
    np.testing.assert_array_equal(xnh[:1000], oracle.row_norms(Xh[:1000]))
    Ch = C.cpu().numpy()
    ref = oracle.kmeans_iteration(Xh, xnh, None, Ch, oracle.row_norms(Ch),
                                  num_partitions=threads, threads=threads)
    ah, ch = a.cpu().numpy(), pc.cpu().numpy()
    bad = np.flatnonzero((ah != ref["assign"]) | (ch != ref["dist"]))
    assert bad.size == 0, f"{bad.size} rows differ, first {bad[:10]}"
    np.testing.assert_array_equal(wsum.cpu().numpy(), ref["wsum"])
    np.testing.assert_allclose(sums.cpu().numpy().reshape(k, d), ref["sums"], rtol=1e-10,
                               atol=1e-10 * np.abs(ref["sums"]).max())
    assert abs(cost.item() - ref["cost"]) <= 1e-10 * ref["cost"]


def _assign_variant(X, C, cuda, variant, monkeypatch, use_rows=False):
    """Assign through a plan built with CYC_KMEANS_ASSIGN=variant (and the
    i8 row image when use_rows); returns (assign, cost, fp64-screen rows,
    exact rows)."""
    import torch
    from cycloneml_amd.clustering import KMeansPlan, row_norms
    monkeypatch.setenv("CYC_KMEANS_ASSIGN", str(variant))
    Xd, Cd = _dev(X, cuda), _dev(C, cuda)
    xn, cn = row_norms(Xd), row_norms(Cd)
    p = KMeansPlan(X.shape[1], C.shape[0], X.shape[0])
    p.stats(Cd)
    a = torch.empty(X.shape[0], dtype=torch.int32, device=cuda)
    c = torch.empty(X.shape[0], dtype=torch.float64, device=cuda)
    rows = p.rows(Xd) if use_rows else None
    n_exact = p.assign(Xd, xn, Cd, cn, a, c, count_exact=True, rows=rows)
    torch.cuda.synchronize()
    t2, ex = p.last_tiers()
    assert ex == n_exact
    return a.cpu().numpy(), c.cpu().numpy(), t2, ex


@pytest.mark.parametrize("n,d,k", [(4000, 32, 7), (3000, 64, 130), (2000, 256, 300),
                                   (1000, 96, 1), (700, 512, 40), (5000, 128, 1024)])
def test_bf16_screen_matches_fp64_screen(cuda, monkeypatch, n, d, k):
    """Tier 1 (bf16x3 screen) + tier 2 (fp64 screen on its leftovers) equals
    the fp64 screen alone and the restatement, bit for bit; on separated
    clusters the bf16 screen decides most rows."""
    rng = np.random.default_rng(n + 3 * d + k)
    true_c = rng.normal(scale=4.0, size=(max(k, 1), d))
    X = true_c[rng.integers(0, true_c.shape[0], n)] + rng.normal(size=(n, d))
    C = true_c + rng.normal(scale=0.1, size=true_c.shape)
    a3, c3, t2, _ = _assign_variant(X, C, cuda, 3, monkeypatch)
    a2, c2, t2b, _ = _assign_variant(X, C, cuda, 2, monkeypatch)
    ra, rc = _oracle_assign(X, C)
    np.testing.assert_array_equal(a3, ra)
    np.testing.assert_array_equal(c3, rc)
    np.testing.assert_array_equal(a2, a3)
    np.testing.assert_array_equal(c2, c3)
    assert t2b == n                      # variant 2: every row through the fp64 screen
    assert t2 <= max(n // 20, 5), t2     # separated clusters: bf16 decides >= 95%


def test_bf16_screen_hard_cases(cuda, monkeypatch):
    """Near ties, duplicate centers, huge rows (> 2^56), tiny-scale rows and
    Inf rows fall through the bf16 screen to the fp64 screen / exact
    loop and still match the reference."""
    rng = np.random.default_rng(17)
    d, k = 64, 20
    C = rng.normal(scale=3.0, size=(k, d))
    C[7] = C[3]                                           # duplicate center
    X = np.vstack([
        C[rng.integers(0, k, 800)] + rng.normal(size=(800, d)),
        0.5 * (C[0] + C[1]) + rng.normal(scale=1e-9, size=(40, d)),   # near ties
        C[rng.integers(0, k, 30)] * 1e18,                 # |x| > 2^56
        C[rng.integers(0, k, 30)] * 1e-30,                # bf16 underflow scale
        C[:5] + 1e-14,
    ])
    X[805, 2] = np.inf                    # (NaN rows fail the require: test_nan_norm_require)
    X[806, 0] = -np.inf
    a3, c3, t2, ex = _assign_variant(X, C, cuda, 3, monkeypatch)
    ra, rc = _oracle_assign(X, C)
    np.testing.assert_array_equal(a3, ra)
    np.testing.assert_array_equal(c3, rc)
    assert t2 >= 100 and ex > 0


def test_bf16_screen_off_for_huge_center(cuda, monkeypatch):
    rng = np.random.default_rng(19)
    d, k, n = 32, 9, 1500
    C = rng.normal(size=(k, d))
    C[4] *= 1e20                                          # |c| > 2^56: screen off
    X = rng.normal(size=(n, d)) * 2
    a3, c3, t2, _ = _assign_variant(X, C, cuda, 3, monkeypatch)
    assert t2 == n
    ra, rc = _oracle_assign(X, C)
    np.testing.assert_array_equal(a3, ra)
    np.testing.assert_array_equal(c3, rc)


@pytest.mark.parametrize("n,d,k", [(4000, 32, 7), (3000, 64, 130), (2000, 256, 300),
                                   (1000, 96, 1), (700, 512, 40), (5000, 128, 1024),
                                   (900, 1, 3), (1200, 100, 33), (800, 300, 64)])
def test_i8_screen_matches_reference(cuda, monkeypatch, n, d, k):
    """Tier 1 = exact-integer i8 screen (row image), then the fp64 screen and
    the exact loop on its leftovers: bit-identical to the restatement and to
    the fp64 screen alone; on separated clusters the i8 screen decides
    (nearly) every row."""
    rng = np.random.default_rng(n + 5 * d + k)
    true_c = rng.normal(scale=4.0, size=(max(k, 1), d))
    X = true_c[rng.integers(0, true_c.shape[0], n)] + rng.normal(size=(n, d))
    C = true_c + rng.normal(scale=0.1, size=true_c.shape)
    a8, c8, t2, _ = _assign_variant(X, C, cuda, 2, monkeypatch, use_rows=True)
    a2, c2, _, _ = _assign_variant(X, C, cuda, 2, monkeypatch)
    ra, rc = _oracle_assign(X, C)
    np.testing.assert_array_equal(a8, ra)
    np.testing.assert_array_equal(c8, rc)
    np.testing.assert_array_equal(a2, a8)
    np.testing.assert_array_equal(c2, c8)
    assert t2 <= max(n // 100, 3), t2


def test_i8_screen_near_ties_and_dense_clusters(cuda, monkeypatch):
    """Centers drawn from the data itself (setInitialModel on rows, as in the
    bench config) and close center pairs: many near ties, all resolved to the
    reference's index."""
    rng = np.random.default_rng(23)
    n, d, k = 6000, 256, 256
    true_c = rng.normal(scale=4.0, size=(k // 2, d))
    X = true_c[rng.integers(0, k // 2, n)] + rng.normal(size=(n, d))
    C = X[:k].copy()
    a8, c8, t2, ex = _assign_variant(X, C, cuda, 2, monkeypatch, use_rows=True)
    ra, rc = _oracle_assign(X, C)
    np.testing.assert_array_equal(a8, ra)
    np.testing.assert_array_equal(c8, rc)


def test_i8_screen_hard_cases(cuda, monkeypatch):
    """Near ties, duplicate centers, huge rows (> 2^50), tiny-scale rows,
    all-zero rows and Inf rows fall through the i8 screen to the fp64
    screen / exact loop and still match the reference."""
    rng = np.random.default_rng(29)
    d, k = 64, 20
    C = rng.normal(scale=3.0, size=(k, d))
    C[7] = C[3]                                           # duplicate center
    X = np.vstack([
        C[rng.integers(0, k, 800)] + rng.normal(size=(800, d)),
        0.5 * (C[0] + C[1]) + rng.normal(scale=1e-9, size=(40, d)),   # near ties
        C[rng.integers(0, k, 30)] * 1e18,                 # beyond 2^50
        C[rng.integers(0, k, 30)] * 1e-30,                # tiny scale
        np.zeros((5, d)),
        C[:5] + 1e-14,
    ])
    X[805, 2] = np.inf                    # (NaN rows fail the require: test_nan_norm_require)
    X[806, 0] = -np.inf
    a8, c8, t2, ex = _assign_variant(X, C, cuda, 2, monkeypatch, use_rows=True)
    ra, rc = _oracle_assign(X, C)
    np.testing.assert_array_equal(a8, ra)
    np.testing.assert_array_equal(c8, rc)
    assert t2 >= 100 and ex > 0


@pytest.mark.parametrize("scale", [1e20, 1e-40])
def test_i8_screen_extreme_centers(cuda, monkeypatch, scale):
    """A center beyond 2^50 turns the i8 screen off for the launch; tiny
    centers still screen correctly (coarser grid)."""
    rng = np.random.default_rng(31)
    d, k, n = 32, 9, 1500
    C = rng.normal(size=(k, d))
    C[4] *= scale
    X = rng.normal(size=(n, d)) * 2
    a8, c8, t2, _ = _assign_variant(X, C, cuda, 2, monkeypatch, use_rows=True)
    if scale > 1:
        assert t2 == n
    ra, rc = _oracle_assign(X, C)
    np.testing.assert_array_equal(a8, ra)
    np.testing.assert_array_equal(c8, rc)


@pytest.mark.parametrize("n,d,k,sep", [(6000, 256, 1024, True), (5000, 128, 300, False),
                                       (3000, 200, 65, True), (2000, 512, 40, True)])
def test_i8_two_limb_pass(cuda, monkeypatch, n, d, k, sep):
    """d <= 256: the two-limb i8 pass screens every row and the three-limb
    pass only its leftovers (a subset of the rows), bit-identical to the
    restatement; separated clusters leave few rows to the three-limb pass.
    d > 256 runs no two-limb pass (-1)."""
    import torch
    from cycloneml_amd.clustering import KMeansPlan, row_norms
    monkeypatch.setenv("CYC_KMEANS_ASSIGN", "2")
    rng = np.random.default_rng(n + d + k)
    true_c = rng.normal(scale=4.0 if sep else 0.7, size=(k, d))
    X = true_c[rng.integers(0, k, n)] + rng.normal(size=(n, d))
    C = true_c + rng.normal(scale=0.1, size=true_c.shape) if sep else X[:k].copy()
    Xd, Cd = _dev(X, cuda), _dev(C, cuda)
    xn, cn = row_norms(Xd), row_norms(Cd)
    p = KMeansPlan(d, k, n)
    p.stats(Cd)
    a = torch.empty(n, dtype=torch.int32, device=cuda)
    c = torch.empty(n, dtype=torch.float64, device=cuda)
    ex = p.assign(Xd, xn, Cd, cn, a, c, count_exact=True, rows=p.rows(Xd))
    l3 = p.last_screen()
    t2, _ = p.last_tiers()
    ra, rc = _oracle_assign(X, C)
    np.testing.assert_array_equal(a.cpu().numpy(), ra)
    np.testing.assert_array_equal(c.cpu().numpy(), rc)
    if d > 256:
        assert l3 == -1
        return
    assert 0 <= t2 <= l3 <= n and ex <= t2
    if sep:
        assert l3 <= n // 10, l3


def test_rows_image_guard(cuda):
    """The row image is bound to its rows: other X or n is refused with the
    reference-style message."""
    import torch
    from cycloneml_amd import _native as N
    from cycloneml_amd.clustering import KMeansPlan, row_norms
    X = _dev(np.random.default_rng(1).normal(size=(100, 16)), cuda)
    C = X[:4].clone()
    p = KMeansPlan(16, 4, 100)
    p.stats(C)
    rows = p.rows(X)
    assert rows.nbytes == 100 * 3 * 128 + 100 * 8
    a = torch.empty(100, dtype=torch.int32, device=cuda)
    c = torch.empty(100, dtype=torch.float64, device=cuda)
    with pytest.raises(N.IllegalArgumentException, match="row image"):
        p.assign(X[:50], row_norms(X[:50]), C, row_norms(C), a, c, rows=rows)


@pytest.mark.parametrize("n,d,k,weighted", [(5000, 16, 12, False), (20000, 256, 64, True),
                                            (3000, 300, 7, True), (2000, 700, 5, False),
                                            (1_100_003, 256, 64, True), (1_048_579, 100, 3, False)])
def test_lloyd_iteration_no_row_costs(cuda, n, d, k, weighted):
    """accumulate without per-row outputs (the training loop's call): the
    streaming cluster-sum pass folds w (c - x)^2 per dimension; sums, weights
    and centers as with row costs, the cost total within 1e-12 relative."""
    import torch
    from cycloneml_amd.clustering import row_norms
    rng = np.random.default_rng(n + k + 1)
    X = rng.normal(size=(n, d)) + rng.integers(0, 5, size=(n, 1)) * 3.0
    C = X[rng.choice(n, size=k, replace=False)].copy()
    w = rng.uniform(0.5, 2.0, size=n) if weighted else None
    ref = oracle.kmeans_iteration(X, oracle.row_norms(X), w, C, oracle.row_norms(C))
    Xd, Cd = _dev(X, cuda), _dev(C, cuda)
    wd = None if w is None else _dev(w, cuda)
    xn, cn = row_norms(Xd), row_norms(Cd)
    p = _plan(d, k, n)
    sums = torch.zeros(k * d, dtype=torch.float64, device=cuda)
    wsum = torch.zeros(k, dtype=torch.float64, device=cuda)
    cost = torch.zeros(1, dtype=torch.float64, device=cuda)
    p.accumulate(Xd, xn, wd, Cd, cn, sums, wsum, cost, rows=p.rows(Xd))
    torch.cuda.synchronize()
    np.testing.assert_allclose(wsum.cpu().numpy(), ref["wsum"], rtol=1e-12)
    np.testing.assert_allclose(sums.cpu().numpy().reshape(k, d), ref["sums"], rtol=1e-10,
                               atol=1e-10 * np.abs(ref["sums"]).max())
    assert abs(cost.item() - ref["cost"]) <= 1e-12 * abs(ref["cost"])


@pytest.mark.parametrize("k,d,nostats", [(2500, 16, False), (2500, 16, True), (1030, 300, False)])
def test_exact_tier_many_centers(cuda, k, d, nostats):
    """Rows the screens cannot decide (exact ties between duplicated centers)
    go to the exact tier; with k > 1024 its distances are staged in several
    1024-center chunks.  Index and cost bit-exact vs the restatement, with
    statistics (findClosest :282-313) and without (pointCost :318-340)."""
    import torch
    from cycloneml_amd.clustering import KMeansModel
    rng = np.random.default_rng(k + d)
    base = rng.integers(-3, 4, size=(k // 2, d)).astype(np.float64)
    C = np.concatenate([base, base])[:k]            # every center twice
    if C.shape[0] < k:
        C = np.concatenate([C, base[: k - C.shape[0]]])
    rng.shuffle(C)
    X = C[rng.integers(0, k, 3000)] + rng.integers(0, 2, size=(3000, d)) * 0.5
    if nostats:
        a, c = KMeansModel(C).pointCosts(_dev(X, cuda))
        ra, rc, _ = oracle.point_costs(X, oracle.row_norms(X), C, oracle.row_norms(C))
        np.testing.assert_array_equal(a.cpu().numpy(), ra)
        np.testing.assert_array_equal(c.cpu().numpy(), rc)
        return
    a, c, n_exact, *_ = _gpu_assign(X, C, cuda)
    assert n_exact > 0
    ra, rc = _oracle_assign(X, C)
    np.testing.assert_array_equal(a, ra)
    np.testing.assert_array_equal(c, rc)


@pytest.mark.parametrize("n,d,k,sep,dup", [(200_000, 64, 128, 4.0, False),
                                           (120_000, 256, 1024, 4.0, False),
                                           (150_000, 200, 300, 1.5, True),
                                           (100_000, 32, 97, 4.0, False),
                                           (60_000, 256, 96, 4.0, False)])
def test_one_limb_refinement_lloyd(cuda, n, d, k, sep, dup):
    """d <= 256, k > 96: the i8 screen runs the one-limb pass over every
    center and the two-limb refinement over the union of each 32 rows'
    candidates (kmeans_i8.hip k_screen32r), the full two-limb pass only for
    the rows neither handles.  Over four Lloyd iterations (centers moving
    between them) every assignment and cost equals the restatement's bit
    for bit, sums within 1e-10.  Cases: separated clusters (d 64 / 256, k up
    to 1024), close clusters with near-duplicate centers (near ties), k = 97
    (the smallest refined k) and k = 96 (the two-limb pass over every
    center: no refinement)."""
    import torch
    from cycloneml_amd.clustering import KMeansPlan, row_norms
    rng = np.random.default_rng(n + d + k)
    true_c = rng.normal(scale=sep, size=(k, d))
    X = true_c[rng.integers(0, k, n)] + rng.normal(size=(n, d))
    C = X[:k].copy()
    if dup:
        C[k // 2:k // 2 + 10] = C[:10] + 1e-9          # near-duplicate centers
    Xd, Cd = _dev(X, cuda), _dev(C, cuda)
    xn, cn = row_norms(Xd), row_norms(Cd)
    p = KMeansPlan(d, k, n)
    rows = p.rows(Xd)
    a = torch.empty(n, dtype=torch.int32, device=cuda)
    pc = torch.empty(n, dtype=torch.float64, device=cuda)
    conv = torch.zeros(1, dtype=torch.int32, device=cuda)
    for it in range(4):
        Ch = Cd.cpu().numpy()
        ref = oracle.kmeans_iteration(X, oracle.row_norms(X), None, Ch, oracle.row_norms(Ch),
                                      num_partitions=8, threads=8)
        sums = torch.zeros(k * d, dtype=torch.float64, device=cuda)
        wsum = torch.zeros(k, dtype=torch.float64, device=cuda)
        cost = torch.zeros(1, dtype=torch.float64, device=cuda)
        p.accumulate(Xd, xn, None, Cd, cn, sums, wsum, cost, a, pc, rows=rows)
        listed, full, union = p.last_refine()
        torch.cuda.synchronize()
        bad = np.flatnonzero((a.cpu().numpy() != ref["assign"]) | (pc.cpu().numpy() != ref["dist"]))
        assert bad.size == 0, f"iteration {it}: {bad.size} rows differ, first {bad[:10]}"
        np.testing.assert_allclose(sums.cpu().numpy().reshape(k, d), ref["sums"], rtol=1e-10,
                                   atol=1e-10 * np.abs(ref["sums"]).max())
        if k <= 96:
            assert (listed, full, union) == (-1, -1, -1)
        else:
            assert 0 <= listed <= n and 0 <= full <= n and union >= 0
        p.update(Cd, cn, sums, wsum, 1e-4, conv)


@pytest.mark.parametrize("n,d,k", [(150_000, 200, 300), (100_000, 64, 128)])
@pytest.mark.parametrize("cands3", ["1", "0"])
def test_three_limb_candidate_tier(cuda, monkeypatch, n, d, k, cands3):
    """Rows the two-limb tiers hand to the candidate pass first meet the
    three-limb candidate tier (kmeans_i8.hip k_screen_cands3: exact integer
    limb products over the row's <= 6 candidates, the three-limb pass's
    bounds); the rows it cannot certify go on to the fp64 candidate pass.
    Close clusters with near-duplicate centers (near ties); d = 200 (16
    lanes per row) and d = 64 (8 lanes per row).  Index and cost bit-exact
    vs the restatement with the tier on and off (CYC_KMEANS_CANDS3=0); on,
    it leaves fewer rows to the fp64 pass than reach it."""
    import torch
    from cycloneml_amd.clustering import row_norms
    monkeypatch.setenv("CYC_KMEANS_CANDS3", cands3)
    rng = np.random.default_rng(n + d + k + 7)
    true_c = rng.normal(scale=1.5, size=(k, d))
    X = true_c[rng.integers(0, k, n)] + rng.normal(size=(n, d))
    C = X[:k].copy()
    C[k // 2:k // 2 + 10] = C[:10] + 1e-9
    Xd, Cd = _dev(X, cuda), _dev(C, cuda)
    xn, cn = row_norms(Xd), row_norms(Cd)
    p = _plan(d, k, n)
    p.stats(Cd)
    rows = p.rows(Xd)
    a = torch.empty(n, dtype=torch.int32, device=cuda)
    c = torch.empty(n, dtype=torch.float64, device=cuda)
    p.assign(Xd, xn, Cd, cn, a, c, count_exact=True, rows=rows)
    torch.cuda.synchronize()
    cand, fp64 = p.last_candidates(), p.last_candidates3()
    assert cand > 0
    if cands3 == "1":
        assert 0 <= fp64 < cand
    else:
        assert fp64 == -1
    ra, rc = _oracle_assign(X, C)
    np.testing.assert_array_equal(a.cpu().numpy(), ra)
    np.testing.assert_array_equal(c.cpu().numpy(), rc)


@pytest.mark.timeout(900)
def test_full_config_third_iteration(cuda):
    """BASELINE config 2 on bench.py's rows as the bench times it: two Lloyd
    iterations, then the third (centers that moved, as in the timed steps)
    compared with the restatement for EVERY row (assignment and cost bit for
    bit, sums within 1e-10); the one-limb pass + refinement handled it."""
    import os
    import sys
    import torch
    from cycloneml_amd.clustering import row_norms
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    n, d, k = 10_000_000, 256, 1024
    X = bench.kmeans_data(n, cuda, 0, d, k)
    C = X[:k].clone()
    xn, cn = row_norms(X), row_norms(C)
    p = _plan(d, k, n)
    rows = p.rows(X)
    conv = torch.zeros(1, dtype=torch.int32, device=cuda)
    a = torch.empty(n, dtype=torch.int32, device=cuda)
    pc = torch.empty(n, dtype=torch.float64, device=cuda)
    for it in range(3):
        if it == 2:
            Ch = C.cpu().numpy()
        sums = torch.zeros(k * d, dtype=torch.float64, device=cuda)
        wsum = torch.zeros(k, dtype=torch.float64, device=cuda)
        cost = torch.zeros(1, dtype=torch.float64, device=cuda)
        p.accumulate(X, xn, None, C, cn, sums, wsum, cost, a, pc, rows=rows)
        if it < 2:
            p.update(C, cn, sums, wsum, 1e-4, conv)
    listed, full, union = p.last_refine()
    torch.cuda.synchronize()
    assert 0 <= full < n // 4 and listed >= 0 and union >= 0
    del rows
    threads = min(int(os.environ.get("OMP_NUM_THREADS", "0")) or 16, os.cpu_count() or 1, 16)
    Xh = X.cpu().numpy()
    del X
    ref = oracle.kmeans_iteration(Xh, xn.cpu().numpy(), None, Ch, oracle.row_norms(Ch),
                                  num_partitions=threads, threads=threads)
    ah, ch = a.cpu().numpy(), pc.cpu().numpy()
    bad = np.flatnonzero((ah != ref["assign"]) | (ch != ref["dist"]))
    assert bad.size == 0, f"{bad.size} rows differ, first {bad[:10]}"
    np.testing.assert_array_equal(wsum.cpu().numpy(), ref["wsum"])
    np.testing.assert_allclose(sums.cpu().numpy().reshape(k, d), ref["sums"], rtol=1e-10,
                               atol=1e-10 * np.abs(ref["sums"]).max())


def _lloyd_run(Xd, Cd0, cuda, iters, bounds, hook=None):
    """`iters` Lloyd iterations through KMeansPlan.accumulate / update over a
    row image with carried bounds on or off; per iteration the host copies of
    (centers used, assign, cost, sums, wsum, cost_sum)."""
    import torch
    from cycloneml_amd.clustering import KMeansPlan, row_norms
    n, d = Xd.shape
    k = Cd0.shape[0]
    Cd = Cd0.clone()
    xn, cn = row_norms(Xd), row_norms(Cd)
    p = KMeansPlan(d, k, n)
    rows = p.rows(Xd)
    rows.set_bounds(bounds)
    a = torch.empty(n, dtype=torch.int32, device=cuda)
    pc = torch.empty(n, dtype=torch.float64, device=cuda)
    conv = torch.zeros(1, dtype=torch.int32, device=cuda)
    out = []
    for it in range(iters):
        if hook:
            hook(it, Cd, cn)
        Ch = Cd.cpu().numpy()
        sums = torch.zeros(k * d, dtype=torch.float64, device=cuda)
        wsum = torch.zeros(k, dtype=torch.float64, device=cuda)
        cost = torch.zeros(1, dtype=torch.float64, device=cuda)
        p.accumulate(Xd, xn, None, Cd, cn, sums, wsum, cost, a, pc, rows=rows)
        out.append((Ch, a.cpu().numpy(), pc.cpu().numpy(), sums.cpu().numpy(),
                    wsum.cpu().numpy(), cost.item()))
        p.update(Cd, cn, sums, wsum, 1e-4, conv)
    torch.cuda.synchronize()
    return out, rows.bounds_info()


@pytest.mark.parametrize("n,d,k,sep", [(200_000, 64, 128, 4.0), (120_000, 256, 1024, 3.0),
                                       (150_000, 200, 300, 1.5)])
def test_carried_bounds_bitwise(cuda, n, d, k, sep):
    """Carried (Hamerly) bounds across the Lloyd iterations of one fit
    (kmeans_i8.hpp Bounds): twelve iterations with the bounds on give the
    SAME bits as with them off -- every row's assignment and cost, the
    cluster sums, weights and cost -- and the last iteration equals the
    restatement (KMeans.scala:275-334 on the same centers) for every row; the
    bounds skipped the screen for rows (screened < n per call after the
    first) without changing a bit."""
    import torch
    rng = np.random.default_rng(n + d + k + 11)
    true_c = rng.normal(scale=sep, size=(k, d))
    X = true_c[rng.integers(0, k, n)] + rng.normal(size=(n, d))
    Xd = _dev(X, cuda)
    C0 = Xd[:k].clone()
    on, (calls, screened) = _lloyd_run(Xd, C0, cuda, 12, True)
    off, (calls_off, _) = _lloyd_run(Xd, C0, cuda, 12, False)
    assert calls == 12 and calls_off == 0
    assert n <= screened < 12 * n
    for it, (a, b) in enumerate(zip(on, off)):
        np.testing.assert_array_equal(a[0], b[0], err_msg=f"centers, iteration {it}")
        for j, name in ((1, "assign"), (2, "cost"), (3, "sums"), (4, "wsum")):
            np.testing.assert_array_equal(a[j], b[j], err_msg=f"{name}, iteration {it}")
        assert a[5] == b[5]
    Ch, ah, ch = on[-1][0], on[-1][1], on[-1][2]
    ref = oracle.kmeans_iteration(X, oracle.row_norms(X), None, Ch, oracle.row_norms(Ch),
                                  num_partitions=8, threads=8)
    bad = np.flatnonzero((ah != ref["assign"]) | (ch != ref["dist"]))
    assert bad.size == 0, f"{bad.size} rows differ, first {bad[:10]}"


def test_carried_bounds_moved_centers(cuda):
    """The bounds follow whatever centers the caller passes: between Lloyd
    iterations the centers are replaced (a jump of one center, a permutation
    of two, a NaN center for one iteration, then finite again, identical
    centers), and every iteration still equals the restatement bit for bit
    (the NaN iteration raises the reference's require, as without bounds)."""
    import torch
    n, d, k = 60_000, 64, 130
    rng = np.random.default_rng(5)
    true_c = rng.normal(scale=3.0, size=(k, d))
    X = true_c[rng.integers(0, k, n)] + rng.normal(size=(n, d))
    Xd = _dev(X, cuda)
    from cycloneml_amd.clustering import KMeansPlan, row_norms
    from cycloneml_amd import _native as N
    xn = row_norms(Xd)
    p = KMeansPlan(d, k, n)
    rows = p.rows(Xd)
    a = torch.empty(n, dtype=torch.int32, device=cuda)
    pc = torch.empty(n, dtype=torch.float64, device=cuda)
    Cd = Xd[:k].clone()
    conv = torch.zeros(1, dtype=torch.int32, device=cuda)
    for it in range(9):
        if it == 3:
            Cd[7] += 5.0                      # one center jumps
        if it == 4:
            Cd[[1, 2]] = Cd[[2, 1]].clone()   # two centers swap indices
        if it == 5:
            Cd[9] = float("nan")
        if it == 6:
            Cd[9] = Xd[999]
        if it == 7:
            Cd[11] = Cd[12]                   # identical centers: ties
        cn = row_norms(Cd)
        Ch = Cd.cpu().numpy()
        sums = torch.zeros(k * d, dtype=torch.float64, device=cuda)
        wsum = torch.zeros(k, dtype=torch.float64, device=cuda)
        cost = torch.zeros(1, dtype=torch.float64, device=cuda)
        if it == 5:
            with pytest.raises(N.IllegalArgumentException, match="norm2=NaN"):
                p.accumulate(Xd, xn, None, Cd, cn, sums, wsum, cost, a, pc, rows=rows)
            continue
        p.accumulate(Xd, xn, None, Cd, cn, sums, wsum, cost, a, pc, rows=rows)
        torch.cuda.synchronize()
        ref = oracle.kmeans_iteration(X, oracle.row_norms(X), None, Ch, oracle.row_norms(Ch),
                                      num_partitions=4, threads=4)
        bad = np.flatnonzero((a.cpu().numpy() != ref["assign"]) |
                             (pc.cpu().numpy() != ref["dist"]))
        assert bad.size == 0, f"iteration {it}: {bad.size} rows differ, first {bad[:10]}"
        p.update(Cd, cn, sums, wsum, 1e-4, conv)
    calls, screened = rows.bounds_info()
    assert calls == 9 and screened < 9 * n


def test_carried_bounds_scope(cuda):
    """Where the bounds do not apply they stay off: k <= 96 (no one-limb
    pass), the cosine measure, and the calls other than accumulate
    (assign / point_cost neither use nor move them)."""
    import torch
    from cycloneml_amd.clustering import KMeansPlan, row_norms
    n, d = 20_000, 32
    rng = np.random.default_rng(8)
    X = rng.normal(size=(n, d)) + rng.integers(0, 5, size=(n, 1)) * 3.0
    Xd = _dev(X, cuda)
    xn = row_norms(Xd)
    for k, measure in ((96, "euclidean"), (200, "cosine"), (200, "euclidean")):
        p = KMeansPlan(d, k, n, measure)
        rows = p.rows(Xd)
        Cd = Xd[:k].clone()
        cn = row_norms(Cd)
        a = torch.empty(n, dtype=torch.int32, device=cuda)
        pc = torch.empty(n, dtype=torch.float64, device=cuda)
        p.stats(Cd)
        p.assign(Xd, xn, Cd, cn, a, pc, rows=rows)
        p.point_cost(Xd, xn, Cd, cn, a, pc, rows=rows)
        assert rows.bounds_info() == (0, 0)
        sums = torch.zeros(k * d, dtype=torch.float64, device=cuda)
        wsum = torch.zeros(k, dtype=torch.float64, device=cuda)
        cost = torch.zeros(1, dtype=torch.float64, device=cuda)
        p.accumulate(Xd, xn, None, Cd, cn, sums, wsum, cost, a, pc, rows=rows)
        calls, screened = rows.bounds_info()
        assert (calls, screened) == ((1, n) if (k, measure) == (200, "euclidean") else (0, 0))


@pytest.mark.timeout(900)
def test_full_config_late_iteration(cuda):
    """BASELINE config 2 on bench.py's rows, one fit from setInitialModel
    (rows 0..1023) as the bench and KMeans.run drive it: the carried bounds
    and the incremental cluster sums on (the defaults), eleven Lloyd
    iterations without per-row costs, then the twelfth compared with the
    restatement on the same centers for EVERY row: the sums, weights and cost
    of the incremental call (sums within 1e-10, weights exact, cost within
    1e-12), then the assignment and cost of every row bit for bit (a second
    call with per-row costs on the same centers).  By then the bounds let most
    rows skip the screen and the sums are carried."""
    import os
    import sys
    import torch
    from cycloneml_amd.clustering import row_norms
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    n, d, k = 10_000_000, 256, 1024
    X = bench.kmeans_data(n, cuda, 0, d, k)
    C = X[:k].clone()
    xn, cn = row_norms(X), row_norms(C)
    p = _plan(d, k, n)
    rows = p.rows(X)
    conv = torch.zeros(1, dtype=torch.int32, device=cuda)
    a = torch.empty(n, dtype=torch.int32, device=cuda)
    pc = torch.empty(n, dtype=torch.float64, device=cuda)
    last = 11
    for it in range(last + 1):
        if it == last:
            Ch = C.cpu().numpy()
            _, before = rows.bounds_info()
        sums = torch.zeros(k * d, dtype=torch.float64, device=cuda)
        wsum = torch.zeros(k, dtype=torch.float64, device=cuda)
        cost = torch.zeros(1, dtype=torch.float64, device=cuda)
        p.accumulate(X, xn, None, C, cn, sums, wsum, cost, a, None, rows=rows)
        if it < last:
            p.update(C, cn, sums, wsum, 1e-4, conv)
    calls, after = rows.bounds_info()
    assert calls == last + 1
    screened = after - before
    assert 0 < screened < n // 2, screened
    assert rows.bounds_rechecked() > 0      # carried candidate sets re-checked
    inc_calls, moved = rows.incremental_info()
    assert inc_calls >= 4, (inc_calls, moved)   # the late iterations fold moved rows only
    a_inc = a.cpu().numpy()
    # the same centers again with per-row costs (the full pass): every row's cost
    s2 = torch.zeros(k * d, dtype=torch.float64, device=cuda)
    w2 = torch.zeros(k, dtype=torch.float64, device=cuda)
    c2 = torch.zeros(1, dtype=torch.float64, device=cuda)
    p.accumulate(X, xn, None, C, cn, s2, w2, c2, a, pc, rows=rows)
    np.testing.assert_array_equal(a.cpu().numpy(), a_inc)
    del rows
    threads = min(int(os.environ.get("OMP_NUM_THREADS", "0")) or 16, os.cpu_count() or 1, 16)
    Xh = X.cpu().numpy()
    del X
    ref = oracle.kmeans_iteration(Xh, xn.cpu().numpy(), None, Ch, oracle.row_norms(Ch),
                                  num_partitions=threads, threads=threads)
    ah, ch = a.cpu().numpy(), pc.cpu().numpy()
    bad = np.flatnonzero((ah != ref["assign"]) | (ch != ref["dist"]))
    assert bad.size == 0, f"{bad.size} rows differ, first {bad[:10]}"
    np.testing.assert_array_equal(wsum.cpu().numpy(), ref["wsum"])
    np.testing.assert_allclose(sums.cpu().numpy().reshape(k, d), ref["sums"], rtol=1e-10,
                               atol=1e-10 * np.abs(ref["sums"]).max())
    assert abs(cost.item() - ref["cost"]) <= 1e-12 * ref["cost"], (cost.item(), ref["cost"])
    np.testing.assert_array_equal(w2.cpu().numpy(), ref["wsum"])
    assert abs(c2.item() - ref["cost"]) <= 1e-12 * ref["cost"]


def _lloyd_inc(Xd, Cd0, cuda, iters, inc, hook=None, check=()):
    """`iters` Lloyd iterations through KMeansPlan.accumulate / update with
    the carried bounds on, no per-row costs (the incremental sums' case),
    incremental sums on or off; at the iterations in `check` the call is
    compared with the restatement on the same centers (assign exact, weights
    exact, sums within 1e-10, cost within 1e-12).  Returns the final
    centers and (incremental calls, moved rows)."""
    import torch
    from cycloneml_amd.clustering import KMeansPlan, row_norms
    n, d = Xd.shape
    k = Cd0.shape[0]
    Cd = Cd0.clone()
    xn, cn = row_norms(Xd), row_norms(Cd)
    p = KMeansPlan(d, k, n)
    rows = p.rows(Xd)
    rows.set_incremental(inc)
    a = torch.empty(n, dtype=torch.int32, device=cuda)
    conv = torch.zeros(1, dtype=torch.int32, device=cuda)
    Xh = Xd.cpu().numpy() if check else None
    for it in range(iters):
        if hook:
            hook(it, Cd, cn)
        sums = torch.zeros(k * d, dtype=torch.float64, device=cuda)
        wsum = torch.zeros(k, dtype=torch.float64, device=cuda)
        cost = torch.zeros(1, dtype=torch.float64, device=cuda)
        Ch = Cd.cpu().numpy()
        p.accumulate(Xd, xn, None, Cd, cn, sums, wsum, cost, a, None, rows=rows)
        if it in check:
            ref = oracle.kmeans_iteration(Xh, oracle.row_norms(Xh), None, Ch,
                                          oracle.row_norms(Ch), num_partitions=8, threads=8)
            np.testing.assert_array_equal(a.cpu().numpy(), ref["assign"],
                                          err_msg=f"assign, iteration {it}")
            np.testing.assert_array_equal(wsum.cpu().numpy(), ref["wsum"],
                                          err_msg=f"wsum, iteration {it}")
            np.testing.assert_allclose(sums.cpu().numpy().reshape(k, d), ref["sums"], rtol=1e-10,
                                       atol=1e-10 * np.abs(ref["sums"]).max(),
                                       err_msg=f"sums, iteration {it}")
            assert abs(cost.item() - ref["cost"]) <= 1e-12 * ref["cost"], (it, cost.item(),
                                                                          ref["cost"])
        p.update(Cd, cn, sums, wsum, 1e-4, conv)
    torch.cuda.synchronize()
    return Cd, rows.incremental_info()


@pytest.mark.parametrize("n,d,k,sep", [(200_000, 64, 128, 4.0), (120_000, 256, 1024, 3.0),
                                       (150_000, 200, 300, 1.5), (60_000, 700, 40, 2.0)])
def test_incremental_sums_fit(cuda, n, d, k, sep):
    """Incremental cluster sums (cyclone.h cyc_kmeans_rows_set_incremental)
    over a 14-iteration fit: every checked iteration equals the restatement
    on the same centers (assignments and weights exactly, sums within 1e-10,
    cost within 1e-12), most late iterations took the incremental path, and
    the fit's centers stay within 1e-9 of the fit with the full pass every
    iteration (d = 700 has no carried bounds: the full pass only)."""
    rng = np.random.default_rng(n + d + k + 29)
    true_c = rng.normal(scale=sep, size=(k, d))
    X = true_c[rng.integers(0, k, n)] + rng.normal(size=(n, d))
    Xd = _dev(X, cuda)
    C0 = Xd[:k].clone()
    C_on, (inc, moved) = _lloyd_inc(Xd, C0, cuda, 14, True, check=(0, 3, 7, 13))
    C_off, (inc_off, _) = _lloyd_inc(Xd, C0, cuda, 14, False)
    assert inc_off == 0
    if d <= 256 and k > 96:
        assert inc >= 6, (inc, moved)
        assert moved > 0
    else:
        assert inc == 0
    Con, Coff = C_on.cpu().numpy(), C_off.cpu().numpy()
    np.testing.assert_allclose(Con, Coff, rtol=1e-9, atol=1e-9 * np.abs(Coff).max())


def test_incremental_sums_edge_cases(cuda):
    """The incremental state under the caller's hand: a center thrown far
    away (the correction term's bound fails: the full pass), a center
    duplicated (its copy empties: weight exactly 0, the centroid not
    updated), a cluster emptied and refilled, the incremental switch toggled
    mid-fit, and a NaN center for one call (the reference's require; the
    next call starts over) -- every call equal to the restatement."""
    import torch
    from cycloneml_amd import _native as N
    n, d, k = 60_000, 64, 130
    rng = np.random.default_rng(17)
    true_c = rng.normal(scale=3.0, size=(k, d))
    X = true_c[rng.integers(0, k, n)] + rng.normal(size=(n, d))
    Xd = _dev(X, cuda)
    state = {}

    def hook(it, Cd, cn):
        from cycloneml_amd.clustering import row_norms
        if it == 5:
            Cd[7] += 50.0                       # far away: its rows leave
        elif it == 7:
            Cd[11] = Cd[12]                     # a duplicate: 12 empties
        elif it == 9:
            Cd[7] = Xd[3]                       # back among the rows
        cn.copy_(row_norms(Cd))
        state["it"] = it

    _, (inc, moved) = _lloyd_inc(Xd, Xd[:k].clone(), cuda, 13, True, hook=hook,
                                 check=tuple(range(13)))
    assert inc >= 4, (inc, moved)
    # toggling drops the state; a NaN center raises and the next call is full
    from cycloneml_amd.clustering import KMeansPlan, row_norms
    p = KMeansPlan(d, k, n)
    rows = p.rows(Xd)
    C = Xd[:k].clone()
    cn = row_norms(C)
    xn = row_norms(Xd)
    a = torch.empty(n, dtype=torch.int32, device=cuda)
    conv = torch.zeros(1, dtype=torch.int32, device=cuda)
    Xh = X
    for it in range(8):
        if it == 3:
            rows.set_incremental(False)
        if it == 4:
            rows.set_incremental(True)
        Cs = C.clone()
        if it == 5:
            Cs[2, 0] = float("nan")
            with pytest.raises(N.IllegalArgumentException):
                s0 = torch.zeros(k * d, dtype=torch.float64, device=cuda)
                p.accumulate(Xd, xn, None, Cs, row_norms(Cs), s0,
                             torch.zeros(k, dtype=torch.float64, device=cuda),
                             torch.zeros(1, dtype=torch.float64, device=cuda), a, None, rows=rows)
            torch.cuda.synchronize()
            continue
        sums = torch.zeros(k * d, dtype=torch.float64, device=cuda)
        wsum = torch.zeros(k, dtype=torch.float64, device=cuda)
        cost = torch.zeros(1, dtype=torch.float64, device=cuda)
        p.accumulate(Xd, xn, None, C, cn, sums, wsum, cost, a, None, rows=rows)
        Ch = C.cpu().numpy()
        ref = oracle.kmeans_iteration(Xh, oracle.row_norms(Xh), None, Ch, oracle.row_norms(Ch),
                                      num_partitions=8, threads=8)
        np.testing.assert_array_equal(a.cpu().numpy(), ref["assign"])
        np.testing.assert_array_equal(wsum.cpu().numpy(), ref["wsum"])
        np.testing.assert_allclose(sums.cpu().numpy().reshape(k, d), ref["sums"], rtol=1e-10,
                                   atol=1e-10 * np.abs(ref["sums"]).max())
        assert abs(cost.item() - ref["cost"]) <= 1e-12 * ref["cost"]
        p.update(C, cn, sums, wsum, 1e-4, conv)
    assert rows.incremental_info()[0] >= 1


@pytest.mark.parametrize("n,d,k,dup", [(60_000, 64, 130, True), (40_000, 256, 1024, False),
                                       (20_000, 300, 40, True)])
def test_accumulate_without_norms(cuda, n, d, k, dup):
    """cyc_kmeans_accumulate_dev with xnorm NULL and a Euclidean row image:
    the image's norms for the screens, the reference's own norm where its
    loop decides (k_assign_exact: duplicate centers force exact rows) --
    the same bits as with the caller's norms over three Lloyd iterations
    (assign, cost, sums, weights, cost sum), and the require message of a
    NaN row names the same norms."""
    import torch
    from cycloneml_amd import _native as N
    from cycloneml_amd.clustering import KMeansPlan, row_norms
    rng = np.random.default_rng(n + d + k)
    true_c = rng.normal(scale=2.5, size=(k, d))
    X = true_c[rng.integers(0, k, n)] + rng.normal(size=(n, d))
    Xd = _dev(X, cuda)
    C0 = Xd[:k].clone()
    if dup:
        C0[k // 2:k // 2 + 4] = C0[:4]                    # exact ties: the exact tier
    out = []
    for with_norms in (True, False):
        p = KMeansPlan(d, k, n)
        rows = p.rows(Xd)
        C = C0.clone()
        cn = row_norms(C)
        xn = row_norms(Xd) if with_norms else None
        a = torch.empty(n, dtype=torch.int32, device=cuda)
        pc = torch.empty(n, dtype=torch.float64, device=cuda)
        conv = torch.zeros(1, dtype=torch.int32, device=cuda)
        res = []
        for it in range(3):
            buf = torch.zeros(k * d + k + 1, dtype=torch.float64, device=cuda)
            sums, wsum, cost = buf[:k * d], buf[k * d:k * d + k], buf[k * d + k:]
            p.accumulate(Xd, xn, None, C, cn, sums, wsum, cost, a, pc, rows=rows)
            res.append((a.cpu().numpy(), pc.cpu().numpy(), buf.cpu().numpy()))
            p.update(C, cn, sums, wsum, 1e-4, conv)
        out.append(res)
    for (a1, c1, b1), (a2, c2, b2) in zip(*out):
        np.testing.assert_array_equal(a1, a2)
        np.testing.assert_array_equal(c1, c2)
        np.testing.assert_array_equal(b1, b2)
    Xn = X.copy()
    Xn[7, 3] = np.nan
    msgs = []
    for with_norms in (True, False):
        Xb = _dev(Xn, cuda)
        p = KMeansPlan(d, k, n)
        rows = p.rows(Xb)
        C = C0.clone()
        with pytest.raises(N.IllegalArgumentException) as e:
            p.accumulate(Xb, row_norms(Xb) if with_norms else None, None, C, row_norms(C),
                         torch.zeros(k * d, dtype=torch.float64, device=cuda),
                         torch.zeros(k, dtype=torch.float64, device=cuda),
                         torch.zeros(1, dtype=torch.float64, device=cuda), rows=rows)
        msgs.append(str(e.value))
    assert msgs[0] == msgs[1] and "norm2=NaN" in msgs[0]
    # k = 1 with a NaN center: the message names row 0's norm (recomputed)
    msgs = []
    for with_norms in (True, False):
        p = KMeansPlan(d, 1, n)
        rows = p.rows(Xd)
        C = torch.full((1, d), float("nan"), dtype=torch.float64, device=cuda)
        with pytest.raises(N.IllegalArgumentException) as e:
            p.accumulate(Xd, row_norms(Xd) if with_norms else None, None, C, row_norms(C),
                         torch.zeros(d, dtype=torch.float64, device=cuda),
                         torch.zeros(1, dtype=torch.float64, device=cuda),
                         torch.zeros(1, dtype=torch.float64, device=cuda), rows=rows)
        msgs.append(str(e.value))
    assert msgs[0] == msgs[1] and "norm1=NaN" in msgs[0], msgs


_RECHECK_CHILD = r'''
import os, sys, numpy as np, torch
sys.path.insert(0, os.getcwd())
from cycloneml_amd.clustering import KMeansPlan, row_norms
dev = torch.device("cuda", 0)
d, k, n = int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
rng = np.random.default_rng(11)
X = torch.as_tensor(rng.normal(scale=4.0, size=(k, d))[rng.integers(0, k, n)]
                    + rng.normal(size=(n, d)), device=dev)
C = X[:k].clone()
xn = row_norms(X)
p = KMeansPlan(d, k, n); rows = p.rows(X)
a = torch.empty(n, dtype=torch.int32, device=dev)
out, info = [], []
for it in range(8):
    cn = row_norms(C)
    s = torch.zeros(k * d, dtype=torch.float64, device=dev); w = torch.zeros(k, dtype=torch.float64, device=dev)
    c = torch.zeros(1, dtype=torch.float64, device=dev)
    p.accumulate(X, xn, None, C, cn, s, w, c, a, None, rows=rows)
    out.append(a.cpu().numpy().copy())
    info.append((rows.bounds_info()[1], rows.bounds_rechecked()))
    # the next centers: a fixed drift (not the sums), so both forms see the same centers
    C = C + torch.as_tensor(rng.normal(scale=0.02, size=(k, d)), device=dev)
np.save(sys.argv[1], np.stack(out))
print(" ".join(f"{x}:{y}" for x, y in info))
'''


@pytest.mark.parametrize("d,k,n", [(256, 300, 80000), (64, 200, 60000)])
def test_recheck_forms_identical(cuda, d, k, n):
    """The two-phase re-check (k_recheck, the default) against the one-phase
    k_screen_cands3<.., true> (CYC_KMEANS_RECHECK=1): the same centers each
    iteration give the same assignments, iteration by iteration, and the
    same carried-state traffic.  The counters are compared within 0.5 %:
    they vary by a few rows from run to run in EITHER form
    (tools/probe/recheck_forms_probe.py: two runs of one form differ by
    1-60 rows of ~10^5).  The screens' lists are appended in arbitrary
    order, and the two-limb refinement screens them 32 rows at a time over
    the union of their candidates: the grouping, and with it the carried
    lower bound a certified row keeps, follows that order.  d = 256 and 64: the S = 8 and S = 4
    instantiations."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    os.makedirs(os.path.join(root, "gpurun_out"), exist_ok=True)
    res = {}
    for form in ("0", "1"):
        f = os.path.join(root, "gpurun_out", f"recheck_{form}_{d}.npy")
        env = dict(os.environ, CYC_KMEANS_RECHECK=form)
        r = subprocess.run([sys.executable, "-c", _RECHECK_CHILD, f, str(d), str(k), str(n)],
                           env=env, cwd=root, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        res[form] = (np.load(f), r.stdout.split())
    np.testing.assert_array_equal(res["0"][0], res["1"][0])
    for e0, e1 in zip(res["0"][1], res["1"][1]):
        for v0, v1 in zip(e0.split(":"), e1.split(":")):
            assert abs(int(v0) - int(v1)) <= 0.005 * max(int(v0), int(v1)) + 2, (e0, e1)
    # the carried state was exercised: rows were re-checked after the first call
    assert int(res["0"][1][-1].split(":")[1]) > 0
