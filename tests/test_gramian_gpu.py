"""GPU parity: RowMatrix Gramian / covariance / PCA (fp64 MFMA syrk) vs the
CPU restatement (oracle: per-row netlib dspr "U") and the reference's known
answers.  Bar: 1e-10 relative (north_star); exact where the reference is."""
import json
import os

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu
GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden",
                                   "reference_known_answers.json")))


def _dev(a, cuda):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).to(cuda)


def test_gram_known_answer(cuda):
    from cycloneml_amd.linalg import RowMatrix
    g = GOLD["rowmatrix_gram"]
    G = RowMatrix(_dev(np.array(g["rows"]), cuda)).computeGramianMatrix()
    assert list(G.T.reshape(-1)) == g["expected_colmajor"]


def test_pca_known_answer(cuda):
    from cycloneml_amd.linalg import RowMatrix
    g = GOLD["rowmatrix_gram"]
    pca = GOLD["rowmatrix_pca"]
    pc_ref = np.array(pca["principal_components_rows"])
    for k in (1, 2, 3):
        pc, ev = RowMatrix(_dev(np.array(g["rows"]), cuda)) \
            .computePrincipalComponentsAndExplainedVariance(k)
        assert pc.shape == (3, k)
        for j in range(k):
            assert min(np.abs(pc[:, j] - pc_ref[:, j]).max(),
                       np.abs(pc[:, j] + pc_ref[:, j]).max()) < 1e-6
        np.testing.assert_allclose(ev, pca["explained_variance"][:k], atol=1e-6)


def test_covariance_accuracy(cuda):
    from cycloneml_amd.linalg import RowMatrix
    rows = np.array(GOLD["rowmatrix_cov_accuracy"]["rows"])
    cov = RowMatrix(_dev(rows, cuda)).computeCovariance()
    np.testing.assert_allclose(np.abs(cov), np.abs(np.cov(rows.T)), atol=1e-6)


@pytest.mark.parametrize("n,p", [(1, 1), (100, 3), (1000, 64), (777, 130), (5000, 257),
                                 (20000, 512), (3000, 1024),
                                 # even widths take k_gram_dma (8-row LDS-DMA chunks):
                                 # one row, rows not a multiple of 8, tiny and ragged panels
                                 (1, 2), (9, 128), (37, 256), (10001, 130), (15, 2)])
def test_gramian_vs_oracle(cuda, n, p):
    from cycloneml_amd.linalg import RowMatrix
    rng = np.random.default_rng(n + p)
    X = rng.uniform(0, 1, size=(n, p))
    U = RowMatrix(_dev(X, cuda)).computeGramianMatrixPacked().cpu().numpy()
    R = oracle.gramian_partition(X)
    np.testing.assert_allclose(U, R, rtol=1e-12)


@pytest.mark.parametrize("form", ["auto", "centred", "uncentred"])
@pytest.mark.parametrize("n,p", [(500, 7), (4000, 200), (13, 2), (1001, 130)])
def test_covariance_vs_oracle(cuda, n, p, form):
    """Both dense forms against the reference's centred restatement (mean
    3 sigma: "auto" takes the uncentred Gramian finish)."""
    from cycloneml_amd.linalg import RowMatrix
    rng = np.random.default_rng(p)
    X = rng.normal(size=(n, p)) + 3.0
    mat = RowMatrix(_dev(X, cuda))
    mat.covarianceForm = form
    cov = mat.computeCovariance()
    assert mat.lastCovarianceForm == ("uncentred" if form == "auto" else form)
    mean = X.sum(0) / n
    U = oracle.gramian_partition(X, mean)
    ref = oracle.triu_to_full(p, U).reshape(p, p).T / (n - 1.0)
    np.testing.assert_allclose(cov, ref, rtol=1e-10, atol=1e-12)
    assert (cov == cov.T).all()   # SPARK-10875 symmetry


def _cov_ref(X):
    n, p = X.shape
    U = oracle.gramian_partition(X, X.sum(0) / n)
    return np.asarray(oracle.triu_to_full(p, U)).reshape(p, p).T / (n - 1.0)


def _assert_entrywise(got, ref, tol, what=""):
    """|got - ref|_ij <= tol sqrt(ref_ii ref_jj) for EVERY entry: the
    per-entry bar in units of the two columns' standard deviations (a
    norm-wise bound says nothing about entries far below the largest)."""
    d = np.sqrt(np.clip(np.diag(ref), 0.0, None))
    lim = tol * np.outer(d, d)
    bad = np.abs(got - ref) > lim
    assert not bad.any(), (f"{what}: {int(bad.sum())} entries off, worst "
                           f"{float((np.abs(got - ref) / np.maximum(lim / tol, 1e-300)).max()):.3g}")


def test_covariance_entrywise_mixed_scales(cuda):
    """Both dense covariance forms per ENTRY (|dC_ij| <= 1e-10 sqrt(C_ii
    C_jj)) against the restatement of the reference's centred form
    (computeDenseVectorCovariance, RowMatrix.scala:163-220): columns of
    mixed scales (standard deviations 1e-3 .. 1e3 side by side) whose means
    sit just inside the uncentred form's bound (mean = 7.9 sd, mean^2 = 62.4
    variance) and exactly AT it (mean^2 = 64 variance, the bound's edge:
    the auto choice's own check decides), and the centred syrk on the same
    rows."""
    from cycloneml_amd.linalg import RowMatrix
    rng = np.random.default_rng(17)
    n, p = 6000, 48
    base = rng.normal(size=(n, p))
    base = (base - base.mean(0)) / base.std(0, ddof=1)
    scale = 10.0 ** rng.integers(-3, 4, size=p)
    for shift in (7.9, 8.0):
        X = (base + shift) * scale
        ref = _cov_ref(X)
        for form in ("auto", "uncentred", "centred"):
            mat = RowMatrix(_dev(X, cuda))
            mat.covarianceForm = form
            cov = mat.computeCovariance()
            if form == "auto" and shift == 7.9:
                assert mat.lastCovarianceForm == "uncentred"
            _assert_entrywise(cov, ref, 1e-10, f"shift {shift}, {form}")


def test_covariance_form_choice(cuda):
    """RowMatrix._near_centred / _dense_covariance: the uncentred finish
    only when every column has mean^2 <= 64 variance; a large mean, a
    constant nonzero column or a NaN keep the reference's centred syrk; at
    the bound the uncentred result still meets the 1e-10 parity bar
    (norm-wise).  Leading rows that pass while the whole matrix fails take
    the fused pass, then the centred syrk."""
    from cycloneml_amd import _native as N
    from cycloneml_amd.linalg import RowMatrix
    rng = np.random.default_rng(5)
    n, p = 3000, 40
    base = rng.normal(size=(n, p))
    base = (base - base.mean(0)) / base.std(0, ddof=1)    # mean 0, variance 1 exactly-ish
    cases = [(base + 7.9, "uncentred"), (base + 8.1, "centred"), (base * 1e-3 + 1e6, "centred")]
    const = base.copy()
    const[:, 3] = 2.5
    cases.append((const, "centred"))
    zero = base.copy()
    zero[:, 3] = 0.0
    cases.append((zero, "uncentred"))
    for X, want in cases:
        mat = RowMatrix(_dev(X, cuda))
        cov = mat.computeCovariance()
        assert mat.lastCovarianceForm == want
        ref = _cov_ref(X)
        np.testing.assert_allclose(cov, ref, rtol=1e-10, atol=1e-10 * np.abs(ref).max())
    fused = ["moments of the leading 3000 rows", "syrk + column sums"]
    mat = RowMatrix(_dev(base + 7.9, cuda))
    mat.computeCovariance()
    assert mat.lastCovariancePasses == fused
    mat = RowMatrix(_dev(base + 8.1, cuda))
    mat.computeCovariance()
    assert mat.lastCovariancePasses == ["moments of the leading 3000 rows", "column moments",
                                        "centred syrk"]
    # the leading 16 rows near-centred, the rest far off: fused pass, exact
    # bound fails, centred syrk
    misled = base * 1e-3 + 1e6
    misled[:16] = base[:16]
    mat = RowMatrix(_dev(misled, cuda))
    mat.COV_SAMPLE_ROWS = 16
    cov = mat.computeCovariance()
    assert mat.lastCovarianceForm == "centred"
    assert mat.lastCovariancePasses == ["moments of the leading 16 rows", "syrk + column sums",
                                        "centred syrk"]
    ref = _cov_ref(misled)
    np.testing.assert_allclose(cov, ref, rtol=1e-10, atol=1e-10 * np.abs(ref).max())
    nan = base.copy()
    nan[7, 2] = np.nan
    mat = RowMatrix(_dev(nan, cuda))
    cov = mat.computeCovariance()
    assert mat.lastCovarianceForm == "centred" and np.isnan(cov[2]).all()
    mat = RowMatrix(_dev(base, cuda))
    mat.covarianceForm = "both"
    with pytest.raises(N.IllegalArgumentException, match="covarianceForm"):
        mat.computeCovariance()


def test_gramian_accumulates_and_checks_columns(cuda):
    import torch
    from cycloneml_amd import _native as N
    from cycloneml_amd.linalg import GramianPlan
    rng = np.random.default_rng(1)
    X = rng.uniform(size=(300, 40))
    plan = GramianPlan(40)
    U = torch.zeros(40 * 41 // 2, dtype=torch.float64, device=cuda)
    plan.accumulate(_dev(X[:100], cuda), U)
    plan.accumulate(_dev(X[100:], cuda), U)
    np.testing.assert_allclose(U.cpu().numpy(), oracle.gramian_partition(X), rtol=1e-12)
    with pytest.raises(N.IllegalArgumentException, match="65535"):
        GramianPlan(65536)


def test_gramian_large_shard_properties(cuda):
    """Config 3 row width (1024 cols) on a 2M-row shard: compare against the
    oracle on a row subset folded into the same totals (linearity)."""
    import torch
    from cycloneml_amd.linalg import GramianPlan
    n, p = 2_000_000, 1024
    g = torch.Generator(device=cuda).manual_seed(3)
    X = torch.rand(n, p, generator=g, device=cuda, dtype=torch.float64)
    plan = GramianPlan(p)
    Ufull = torch.zeros(p * (p + 1) // 2, dtype=torch.float64, device=cuda)
    plan.accumulate(X, Ufull)
    Ua = torch.zeros_like(Ufull)
    plan.accumulate(X[: n // 2], Ua)
    plan.accumulate(X[n // 2:], Ua)
    torch.cuda.synchronize()
    np.testing.assert_allclose(Ua.cpu().numpy(), Ufull.cpu().numpy(), rtol=1e-11)
    # trace = sum of squared entries
    tr = sum(Ufull[j * (j + 1) // 2 + j].item() for j in range(p))
    assert abs(tr - (X * X).sum().item()) <= 1e-10 * tr
    sub = X[:2000].cpu().numpy()
    Us = torch.zeros_like(Ufull)
    plan.accumulate(X[:2000], Us)
    np.testing.assert_allclose(Us.cpu().numpy(), oracle.gramian_partition(sub), rtol=1e-11)


@pytest.fixture(scope="module")
def bench_gram_rows(cuda):
    """bench.py's gramian / pca shard at its benched size (bench.gramian_data:
    30M x 1024 = 246 GB, the largest resident shard of BASELINE configs[2];
    the first rows of the same stream if the device has less free memory),
    shared by the Gramian and covariance tests below."""
    import gc
    import sys
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    gc.collect()
    torch.cuda.empty_cache()
    free, _ = torch.cuda.mem_get_info(cuda)
    n = int(min(30_000_000, (free - (24 << 30)) // (8 * 1024)))
    n -= n % 1024
    X = bench.gramian_data(n, cuda, 0, 1024)
    yield X
    del X
    gc.collect()
    torch.cuda.empty_cache()


@pytest.mark.timeout(600)
def test_gramian_bench_shard(cuda, bench_gram_rows):
    """On the bench's rows: the whole-shard Gramian equals the sum of its two
    halves' (split-K sizing differs between them) within 1e-12, equals the
    restatement on a 2000-row subset, and satisfies G 1 = X^T (X 1)."""
    import torch
    from cycloneml_amd.linalg import GramianPlan
    p = 1024
    X = bench_gram_rows
    n = int(X.shape[0])
    plan = GramianPlan(p)
    U = torch.zeros(p * (p + 1) // 2, dtype=torch.float64, device=cuda)
    plan.accumulate(X, U)
    Uh = torch.zeros_like(U)
    h = n // 2 + 777
    plan.accumulate(X[:h], Uh)
    plan.accumulate(X[h:], Uh)
    torch.cuda.synchronize()
    np.testing.assert_allclose(Uh.cpu().numpy(), U.cpu().numpy(), rtol=1e-12)
    # G 1 = X^T (X 1), accumulated in 1M-row chunks
    w = torch.zeros(p, dtype=torch.float64, device=cuda)
    for s in range(0, n, 1 << 20):
        xs = X[s:s + (1 << 20)]
        w += xs.T @ xs.sum(1)
    Gf = np.asarray(oracle.triu_to_full(p, U.cpu().numpy())).reshape(p, p)
    np.testing.assert_allclose(Gf.sum(1), w.cpu().numpy(), rtol=1e-11)
    Us = torch.zeros_like(U)
    plan.accumulate(X[n - 2000:], Us)
    np.testing.assert_allclose(Us.cpu().numpy(),
                               oracle.gramian_partition(X[n - 2000:].cpu().numpy()), rtol=1e-11)


@pytest.mark.timeout(600)
def test_covariance_pca_bench_shard(cuda, bench_gram_rows):
    """The PCA variant of configs[2] at its shape, on the bench's rows
    (RowMatrix.computeCovariance, RowMatrix.scala:452-467 ->
    computeDenseVectorCovariance :163-220 -- the centred syrk with 16-row
    chunks and split-K over millions of rows, and the uncentred Gramian
    finish that "auto" picks for these rows; then
    computePrincipalComponentsAndExplainedVariance :486-513):
    - isSparseMatrix is false after its first round (take(1) semantics);
    - the centred packed sum equals its two unequal halves' (the whole
      shard's mean) within 1e-12 of its largest entry;
    - the first and the last 2000 rows' centred sums equal the restatement
      (x - mean, then netlib dspr per row) within 1e-10;
    - both forms are exactly symmetric, the uncentred one within 1e-10 of
      the centred one (norm-wise), and Cov 1 equals
      sum_r (x_r - mu) ((x_r - mu) . 1) / (m - 1) accumulated in 1M-row
      chunks (the identity (X^T (X 1) - m mu (mu . 1)) / (m - 1) without its
      cancellation) within 1e-11;
    - PCA (k = 3) returns unit principal components and explained variances
      that sum to at most 1."""
    import torch
    from cycloneml_amd.linalg import GramianPlan, RowMatrix
    p = 1024
    X = bench_gram_rows
    n = int(X.shape[0])
    mat = RowMatrix(X)
    assert not mat.isSparseMatrix()
    cov = mat.computeCovarianceDevice()          # U[0, 1): mean^2 = 3 variance
    assert mat.lastCovarianceForm == "uncentred"
    mat.covarianceForm = "centred"
    cov_c = mat.computeCovarianceDevice()        # the reference's centred syrk
    assert mat.lastCovarianceForm == "centred"
    torch.cuda.synchronize()
    mu = torch.zeros(p, dtype=torch.float64, device=cuda)
    for s in range(0, n, 1 << 20):
        mu += X[s:s + (1 << 20)].sum(0)
    mean, m = mat._column_mean()
    assert m == n
    plan = GramianPlan(p)
    U = torch.zeros(p * (p + 1) // 2, dtype=torch.float64, device=cuda)
    plan.accumulate(X, U, mean)
    Uh = torch.zeros_like(U)
    h = n // 3 + 4099
    plan.accumulate(X[:h], Uh, mean)
    plan.accumulate(X[h:], Uh, mean)
    torch.cuda.synchronize()
    Uw = U.cpu().numpy()             # norm-wise: off-diagonal sums are small (cancellation)
    np.testing.assert_allclose(Uh.cpu().numpy(), Uw, rtol=1e-12, atol=1e-12 * np.abs(Uw).max())
    mean_h = mean.cpu().numpy()
    np.testing.assert_allclose(mean_h, (mu / n).cpu().numpy(), rtol=1e-12)
    for a in (0, n - 2000):
        Us = torch.zeros_like(U)
        plan.accumulate(X[a:a + 2000], Us, mean)
        ref = oracle.gramian_partition(X[a:a + 2000].cpu().numpy(), mean_h)
        got = Us.cpu().numpy()
        scale = np.abs(ref).max()
        np.testing.assert_allclose(got, ref, rtol=1e-10, atol=1e-10 * scale)
        cref = oracle.dense_vector_covariance(p, ref, 2000)
        cgot = oracle.dense_vector_covariance(p, got, 2000)
        np.testing.assert_allclose(cgot, cref, rtol=1e-10, atol=1e-10 * np.abs(cref).max())
    C = cov_c.cpu().numpy()
    assert np.array_equal(C, C.T)                               # SPARK-10875
    np.testing.assert_allclose(C, oracle.dense_vector_covariance(p, U.cpu().numpy(), n),
                               rtol=1e-13, atol=0)
    # the uncentred finish against the centred syrk: 1e-10 of the largest
    # entry (the parity bar; the cancellation is bounded by mean^2 = 3 var)
    Cu = cov.cpu().numpy()
    assert np.array_equal(Cu, Cu.T)
    np.testing.assert_allclose(Cu, C, rtol=1e-10, atol=1e-10 * np.abs(C).max())
    # per entry, in units of the columns' standard deviations
    _assert_entrywise(Cu, C, 1e-10, "uncentred vs centred, whole shard")
    # each form on the head and tail 2000 rows against the restatement
    for a in (0, n - 2000):
        Xs = X[a:a + 2000]
        ref = _cov_ref(Xs.cpu().numpy())
        for form in ("auto", "centred"):
            sub = RowMatrix(Xs)
            sub.covarianceForm = form
            _assert_entrywise(sub.computeCovariance(), ref, 1e-10, f"rows {a}.., {form}")
    w = torch.zeros(p, dtype=torch.float64, device=cuda)
    for s in range(0, n, 1 << 20):
        xc = X[s:s + (1 << 20)] - mean
        w += xc.T @ xc.sum(1)
    w /= (n - 1.0)
    for CC in (C, Cu):
        np.testing.assert_allclose(CC.sum(1), w.cpu().numpy(), rtol=1e-11,
                                   atol=1e-11 * float(w.abs().max()))
    mat.covarianceForm = "auto"
    pc, ev = mat.computePrincipalComponentsAndExplainedVariance(3)
    assert pc.shape == (p, 3) and ev.shape == (3,)
    np.testing.assert_allclose(np.linalg.norm(pc, axis=0), 1.0, rtol=1e-12)
    assert np.all(ev > 0) and ev.sum() <= 1.0 and np.all(np.diff(ev) <= 0)


# -- SparseVector rows (CSR): sparse spr, isSparseMatrix, both covariances --

def _csr(rp, ci, v, n, cuda):
    import torch
    from cycloneml_amd.linalg import CSRRows
    return CSRRows(torch.as_tensor(np.asarray(rp, np.int64), device=cuda),
                   torch.as_tensor(np.asarray(ci, np.int32), device=cuda),
                   torch.as_tensor(np.asarray(v, np.float64), device=cuda), n)


SPARSE_DATA = ([0, 2, 5, 8, 10], [1, 2, 0, 1, 2, 0, 1, 2, 0, 2],
               [1.0, 2.0, 3.0, 4.0, 5.0, 6.0, 7.0, 8.0, 9.0, 1.0])


def test_sparse_rowmatrix_suite_known_answers(cuda):
    """RowMatrixSuite sparseMat (:45-50): gram exact (:95-102), PCA (:241-253),
    covariance = breeze cov (:318-324, closeToZero 1e-6)."""
    from cycloneml_amd.linalg import RowMatrix
    g = GOLD["rowmatrix_gram"]
    mat = RowMatrix(_csr(*SPARSE_DATA, 3, cuda))
    assert mat.numRows() == 4 and mat.numCols() == 3
    G = mat.computeGramianMatrix()
    assert list(G.T.reshape(-1)) == g["expected_colmajor"]
    assert not mat.isSparseMatrix()
    dense = np.array(g["rows"])
    np.testing.assert_allclose(mat.computeCovariance(), np.cov(dense.T), atol=1e-6)
    pc_ref = np.array(GOLD["rowmatrix_pca"]["principal_components_rows"])
    for k in (1, 2, 3):
        pc, _ = RowMatrix(_csr(*SPARSE_DATA, 3, cuda)) \
            .computePrincipalComponentsAndExplainedVariance(k)
        for j in range(k):
            assert min(np.abs(pc[:, j] - pc_ref[:, j]).max(),
                       np.abs(pc[:, j] + pc_ref[:, j]).max()) < 1e-6


def _sparse_rows(rng, n, p, nnz_max):
    lens = rng.integers(0, nnz_max + 1, size=n)
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    ci = np.concatenate([np.sort(rng.choice(p, size=l, replace=False)) for l in lens] or
                        [np.zeros(0)]).astype(np.int32)
    v = rng.random(rp[-1]) + 0.5
    return rp, ci, v


def test_csr_gramian_multi_chunk_vs_restatement(cuda):
    """70,000 CSR rows x 4,096 columns: three ~1 GiB densified chunks; the
    packed Gramian equals the per-row sparse spr restatement (1e-12)."""
    from cycloneml_amd.linalg import RowMatrix
    rng = np.random.default_rng(8)
    n, p = 70_000, 4096
    rp, ci, v = _sparse_rows(rng, n, p, 40)
    U = RowMatrix(_csr(rp, ci, v, p, cuda)).computeGramianMatrixPacked().cpu().numpy()
    ref = oracle.gramian_csr(rp, ci, v, p)
    nz = ref != 0
    np.testing.assert_allclose(U[nz], ref[nz], rtol=1e-12)
    assert np.all(U[~nz] == 0.0)


def test_sparse_covariance_path(cuda):
    """Every row at least half zeros -> computeSparseVectorCovariance (from
    the Gramian), for CSR rows and for the same rows as a dense tensor (the
    reference picks the path by the values, not the vector type)."""
    from cycloneml_amd.linalg import RowMatrix
    rng = np.random.default_rng(9)
    n, p = 3000, 64
    rp, ci, v = _sparse_rows(rng, n, p, 32)
    X = np.zeros((n, p))
    for r in range(n):
        X[r, ci[rp[r]:rp[r + 1]]] = v[rp[r]:rp[r + 1]]
    mean = X.mean(0)
    ref = oracle.sparse_vector_covariance(p, oracle.gramian_csr(rp, ci, v, p), mean, n)
    for mat in (RowMatrix(_csr(rp, ci, v, p, cuda)), RowMatrix(_dev(X, cuda))):
        assert mat.isSparseMatrix()
        C = mat.computeCovariance()
        np.testing.assert_allclose(C, ref, rtol=1e-9, atol=1e-13)
        np.testing.assert_allclose(C, np.cov(X.T), rtol=1e-8, atol=1e-12)
        assert np.array_equal(C, C.T)


def test_dense_covariance_on_csr_rows(cuda):
    """Rows denser than half -> the dense (centred) path on densified CSR rows
    equals the dense tensor's result and the restatement (1e-10)."""
    from cycloneml_amd.linalg import RowMatrix
    rng = np.random.default_rng(10)
    n, p = 5000, 48
    rp, ci, v = _sparse_rows(rng, n, p, 48)
    X = np.zeros((n, p))
    for r in range(n):
        X[r, ci[rp[r]:rp[r + 1]]] = v[rp[r]:rp[r + 1]]
    mat = RowMatrix(_csr(rp, ci, v, p, cuda))
    assert not mat.isSparseMatrix()
    C = mat.computeCovariance()
    Cd = RowMatrix(_dev(X, cuda)).computeCovariance()
    ref = oracle.dense_vector_covariance(p, oracle.gramian_partition(X, X.mean(0)), n)
    np.testing.assert_allclose(C, ref, rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(C, Cd, rtol=1e-12, atol=1e-14)


def test_csr_gramian_index_require(cuda):
    import cycloneml_amd._native as N
    from cycloneml_amd.linalg import RowMatrix
    with pytest.raises(N.IllegalArgumentException):
        RowMatrix(_csr([0, 2], [3, 1], [1.0, 2.0], 4, cuda)).computeGramianMatrix()


def test_is_sparse_matrix_scan_rounds(cuda, monkeypatch):
    """isSparseMatrix as take(1) (RDD.scala:1443-1478, 1577-1579): growing row
    ranges until one row with sparsity() < 0.5 turns up -- here the last row
    of the shard, so every round runs -- for dense tensors and CSR rows; a
    matrix without such a row is sparse."""
    import torch
    from cycloneml_amd.linalg import RowMatrix
    monkeypatch.setattr(RowMatrix, "SPARSITY_SCAN_FIRST", 7)
    rng = np.random.default_rng(4)
    n, p = 2000, 10
    X = np.zeros((n, p))
    for r in range(n):
        X[r, rng.choice(p, size=5, replace=False)] = rng.uniform(0.5, 1.5, size=5)  # sparsity 0.5
    assert RowMatrix(_dev(X, cuda)).isSparseMatrix()
    for last in (n - 1, 0, 900):
        Y = X.copy()
        Y[last] = 1.0
        assert not RowMatrix(_dev(Y, cuda)).isSparseMatrix()
        nz = Y != 0
        rp = np.concatenate([[0], np.cumsum(nz.sum(1))]).astype(np.int64)
        r_, c_ = np.nonzero(nz)
        assert not RowMatrix(_csr(rp, c_, Y[r_, c_], p, cuda)).isSparseMatrix()
    assert RowMatrix(torch.zeros(0, p, dtype=torch.float64, device=cuda), nCols=p) \
        .isSparseMatrix()
