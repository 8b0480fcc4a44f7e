"""Resident-dataset host layer (cyc_dataset_*, cyc_kmeans_iter,
cyc_logreg_*_eval, cyc_gramian, cyc_col_sums) against the CPU restatement.
Same bars as the _dev paths: KMeans assignments bit-exact, everything fp64
within 1e-10 relative."""
import numpy as np
import pytest

import oracle
from cycloneml_amd import _native as N
from cycloneml_amd.dataset import ResidentDataset


def test_dataset_requires_device_or_valid_args():
    import torch
    with pytest.raises(N.IllegalArgumentException, match="Number of features"):
        ResidentDataset.dense(0, 10)
    if torch.cuda.is_available():
        pytest.skip("device present")
    with pytest.raises(N.CycloneError) as e:
        ResidentDataset.dense(4, 10)
    assert e.value.code == N.CYC_ERR_NO_DEVICE


def _rel_close(got, ref, rtol=1e-10):
    got, ref = np.asarray(got), np.asarray(ref)
    scale = max(np.abs(ref).max(), 1e-300)
    np.testing.assert_allclose(got, ref, rtol=rtol, atol=rtol * scale)


def _csr(n, F, rng, nnz=8):
    rp, ci, vv = [0], [], []
    for _ in range(n):
        k = int(rng.integers(0, 2 * nnz + 1))
        cols = np.sort(rng.choice(F, size=min(k, F), replace=False))
        ci += list(cols)
        vv += list(rng.uniform(-1, 1, size=cols.size))
        rp.append(len(ci))
    return np.array(rp, np.int64), np.array(ci, np.int32), np.array(vv)


@pytest.mark.gpu
@pytest.mark.parametrize("weighted", [False, True])
def test_kmeans_iter_in_chunks(cuda, weighted):
    rng = np.random.default_rng(11)
    n, d, k = 5000, 40, 24
    X = rng.normal(size=(n, d)) + rng.integers(0, 6, size=(n, 1)) * 3.0
    w = rng.uniform(0.5, 2.0, size=n) if weighted else None
    C = X[:k].copy()
    ds = ResidentDataset.dense(d, n, weights=weighted)
    for s, e in ((0, 1000), (1000, 1001), (1001, n)):   # three appended blocks
        ds.append_dense(X[s:e], weights=None if w is None else w[s:e])
    assert ds.numRows == n
    sums, wsum, cost, assign = ds.kmeans_iter(C, want_assign=True)
    ref = oracle.kmeans_iteration(X, oracle.row_norms(X), w, C, oracle.row_norms(C))
    assert np.array_equal(assign, ref["assign"])
    _rel_close(sums, ref["sums"])
    _rel_close(wsum, ref["wsum"])
    assert abs(cost[0] - ref["cost"]) <= 1e-10 * ref["cost"]
    # outputs accumulate (aggregator add semantics)
    ds.kmeans_iter(C, sums, wsum, cost)
    _rel_close(sums, 2 * ref["sums"])
    # appending rows invalidates the cached norms
    X2 = rng.normal(size=(10, d))
    with pytest.raises(N.IllegalArgumentException, match="capacity exceeded"):
        ds.append_dense(X2, weights=np.ones(10) if weighted else None)


@pytest.mark.gpu
def test_kmeans_iter_norms_refresh_after_append(cuda):
    rng = np.random.default_rng(12)
    n, d, k = 600, 16, 5
    X = rng.normal(size=(n, d)) * 2
    C = X[:k].copy()
    ds = ResidentDataset.dense(d, n)
    ds.append_dense(X[:300])
    ds.kmeans_iter(C)
    ds.append_dense(X[300:])
    _, _, _, a = ds.kmeans_iter(C, want_assign=True)
    ref = oracle.kmeans_iteration(X, oracle.row_norms(X), None, C, oracle.row_norms(C))
    assert np.array_equal(a, ref["assign"])


@pytest.mark.gpu
@pytest.mark.parametrize("sparse", [False, True])
@pytest.mark.parametrize("fi,fwm", [(False, False), (True, False), (True, True)])
def test_binary_eval(cuda, sparse, fi, fwm):
    rng = np.random.default_rng(21 + fi + 2 * fwm)
    n, F = 3000, 50
    y = rng.integers(0, 2, size=n).astype(np.float64)
    w = rng.uniform(0.1, 2.0, size=n)
    coef = rng.normal(size=F + (1 if fi else 0)) * 0.3
    sm = rng.normal(size=F) * 0.1 if fwm else None
    st = dict(grad=np.zeros(coef.size), loss=0.0, weight=0.0)
    if sparse:
        rp, ci, vv = _csr(n, F, rng)
        ds = ResidentDataset.csr(F, n, ci.size, labels=True, weights=True)
        h = n // 2
        ds.append_csr(rp[:h + 1], ci[:rp[h]], vv[:rp[h]], y[:h], w[:h])
        ds.append_csr(rp[h:], ci[rp[h]:], vv[rp[h]:], y[h:], w[h:])  # rowptr base rp[h]
        blk = dict(labels=y, weights=w, rowptr=rp, colidx=ci, values=vv, F=F)
    else:
        X = rng.normal(size=(n, F))
        ds = ResidentDataset.dense(F, n, labels=True, weights=True).append_dense(X, y, w)
        blk = dict(labels=y, weights=w, X=X)
    oracle.binary_logistic_add(blk, coef, fi, fwm, sm, st)
    grad, lw = ds.binary_logistic_eval(coef, fi, fwm, sm)
    _rel_close(grad, st["grad"])
    assert abs(lw[0] - st["loss"]) <= 1e-10 * abs(st["loss"])
    assert abs(lw[1] - st["weight"]) <= 1e-12 * st["weight"]
    g2, _ = ds.binary_logistic_eval(coef, fi, fwm, sm)
    assert np.array_equal(g2, grad)  # deterministic run to run


@pytest.mark.gpu
def test_multinomial_eval(cuda):
    rng = np.random.default_rng(31)
    n, F, C = 2000, 48, 7
    X = rng.normal(size=(n, F))
    y = rng.integers(0, C, size=n).astype(np.float64)
    coef = rng.normal(size=C * F + C) / np.sqrt(F)
    sm = rng.normal(size=F) * 0.1
    ds = ResidentDataset.dense(F, n, labels=True).append_dense(X, y)
    st = dict(grad=np.zeros(coef.size), loss=0.0, weight=0.0)
    oracle.multinomial_logistic_add(dict(labels=y, weights=None, X=X), coef, C, True, True, sm,
                                    st)
    grad, lw = ds.multinomial_logistic_eval(C, coef, True, True, sm)
    _rel_close(grad, st["grad"])
    assert abs(lw[0] - st["loss"]) <= 1e-10 * abs(st["loss"])
    assert lw[1] == st["weight"]


@pytest.mark.gpu
def test_gramian_and_col_sums(cuda):
    rng = np.random.default_rng(41)
    n, F = 1500, 70
    X = rng.uniform(size=(n, F))
    ds = ResidentDataset.dense(F, n).append_dense(X)
    _rel_close(ds.gramian(), oracle.gramian_partition(X))
    mean = X.mean(axis=0)
    _rel_close(ds.gramian(mean=mean), oracle.gramian_partition(X, mean))
    _rel_close(ds.col_sums(), X.sum(axis=0), rtol=1e-12)


@pytest.mark.gpu
def test_csr_dataset_gramian_and_col_sums(cuda):
    """cyc_gramian / cyc_col_sums over a CSR dataset: the sparse spr seqOp
    (mllib/linalg/BLAS.scala:269-298) per row, and the centred variant."""
    rng = np.random.default_rng(42)
    n, F = 900, 50
    rows, cols, vals = [0], [], []
    for _ in range(n):
        c = np.sort(rng.choice(F, size=int(rng.integers(0, 12)), replace=False))
        cols.extend(c.tolist())
        vals.extend(rng.uniform(size=len(c)).tolist())
        rows.append(len(cols))
    rp, ci, v = np.array(rows, np.int64), np.array(cols, np.int32), np.array(vals)
    X = np.zeros((n, F))
    for r in range(n):
        X[r, ci[rp[r]:rp[r + 1]]] = v[rp[r]:rp[r + 1]]
    ds = ResidentDataset.csr(F, n, len(v)).append_csr(rp, ci, v)
    ref = oracle.gramian_csr(rp, ci, v, F)
    _rel_close(ds.gramian(), ref)
    mean = X.mean(axis=0)
    _rel_close(ds.gramian(mean=mean), oracle.gramian_partition(X, mean))
    _rel_close(ds.col_sums(), X.sum(axis=0), rtol=1e-12)


@pytest.mark.gpu
def test_dataset_errors(cuda):
    ds = ResidentDataset.csr(5, 4, 8, labels=True)
    with pytest.raises(N.IllegalArgumentException, match="out of range"):
        ds.append_csr(np.array([0, 1]), np.array([5]), np.array([1.0]), np.zeros(1))
    with pytest.raises(N.IllegalArgumentException, match="labels must not be null"):
        ds.append_csr(np.array([0, 1]), np.array([1]), np.array([1.0]))
    ds.append_csr(np.array([0, 1]), np.array([1]), np.array([1.0]), np.zeros(1))
    dd = ResidentDataset.dense(3, 2)
    with pytest.raises(N.IllegalArgumentException, match="holds no labels"):
        dd.binary_logistic_eval(np.zeros(3), False)


@pytest.mark.gpu
def test_dataset_csr_kmeans_iter(cuda):
    """cyc_kmeans_iter over a CSR dataset (sparse points, KMeansExample's input
    type): assignments bit-exact, sums / weights / cost to 1e-12 relative."""
    rng = np.random.default_rng(21)
    n, F, k = 700, 30, 6
    rows, cols, vals = [0], [], []
    for _ in range(n):
        c = np.sort(rng.choice(F, size=int(rng.integers(1, 8)), replace=False))
        cols.extend(c.tolist())
        vals.extend(rng.normal(size=len(c)).tolist())
        rows.append(len(cols))
    rp, ci, v = np.array(rows, np.int64), np.array(cols, np.int32), np.array(vals)
    w = rng.uniform(0.5, 1.5, n)
    C = rng.normal(size=(k, F)) * 0.3
    ds = ResidentDataset.csr(F, n, len(v), weights=True)
    ds.append_csr(rp[:301], ci[:rp[300]], v[:rp[300]], weights=w[:300])
    ds.append_csr(rp[300:] - rp[300], ci[rp[300]:], v[rp[300]:], weights=w[300:])
    sums, wsum, cost, assign = ds.kmeans_iter(C, want_assign=True)
    ra, _, rs, rw, rc = oracle.kmeans_partition_sparse((rp, ci, v), oracle.row_norms_csr(rp, v),
                                                       w, C, oracle.row_norms(C),
                                                       oracle.kmeans_stats(C))
    np.testing.assert_array_equal(assign, ra)
    _rel_close(sums, rs, rtol=1e-12)
    _rel_close(wsum, rw, rtol=1e-12)
    _rel_close(cost[0], rc, rtol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("sparse", [False, True])
@pytest.mark.parametrize("fi", [False, True])
def test_other_aggregator_evals(cuda, sparse, fi):
    """Resident-dataset evaluators of the hinge / least squares / Huber / AFT
    block aggregators vs the restatement (1e-10), dense and CSR rows appended
    in two pieces."""
    rng = np.random.default_rng(31 + fi + 2 * sparse)
    n, F = 2500, 40
    y01 = rng.integers(0, 2, size=n).astype(np.float64)
    yr = rng.normal(size=n) * 2.0
    yt = rng.exponential(2.0, size=n) + 1e-3
    w = rng.uniform(0.1, 2.0, size=n)
    cens = (rng.uniform(size=n) < 0.6).astype(np.float64)
    sm = rng.normal(size=F) * 0.1 if fi else None
    inv = rng.uniform(0.5, 2.0, size=F)
    inv[3] = 0.0
    if sparse:
        rp, ci, vv = _csr(n, F, rng)
        blk = lambda lab, wt: dict(labels=lab, weights=wt, rowptr=rp, colidx=ci, values=vv, F=F)
    else:
        X = rng.normal(size=(n, F))
        blk = lambda lab, wt: dict(labels=lab, weights=wt, X=X)

    def make(lab, wt):
        if sparse:
            ds = ResidentDataset.csr(F, n, ci.size, labels=True, weights=True)
            h = n // 2
            ds.append_csr(rp[:h + 1], ci[:rp[h]], vv[:rp[h]], lab[:h], wt[:h])
            ds.append_csr(rp[h:], ci[rp[h]:], vv[rp[h]:], lab[h:], wt[h:])
            return ds
        return ResidentDataset.dense(F, n, labels=True, weights=True).append_dense(X, lab, wt)

    def check(got, st):
        grad, lw = got
        _rel_close(grad, st["grad"])
        assert abs(lw[0] - st["loss"]) <= 1e-10 * abs(st["loss"])
        assert abs(lw[1] - st["weight"]) <= 1e-12 * st["weight"]

    coef = rng.normal(size=F + (1 if fi else 0)) * 0.3
    st = dict(grad=np.zeros(coef.size), loss=0.0, weight=0.0)
    oracle.hinge_add(blk(y01, w), coef, fi, sm, st)
    check(make(y01, w).hinge_eval(coef, fi, sm), st)

    coef = rng.normal(size=F) * 0.3
    st = dict(grad=np.zeros(F), loss=0.0, weight=0.0)
    oracle.least_squares_add(blk(yr, w), coef, inv, fi, 1.7, 0.2, sm, st)
    check(make(yr, w).least_squares_eval(coef, inv, fi, 1.7, 0.2, sm), st)

    params = np.concatenate([rng.normal(size=F) * 0.3, [0.4] if fi else [], [0.9]])
    st = dict(grad=np.zeros(params.size), loss=0.0, weight=0.0)
    oracle.huber_add(blk(yr, w), params, fi, 1.35, sm, st)
    check(make(yr, w).huber_eval(params, fi, 1.35, sm), st)

    coef = np.concatenate([rng.normal(size=F) * 0.1, [0.3 if fi else 0.0], [0.2]])
    st = dict(grad=np.zeros(coef.size), loss=0.0, weight=0.0)
    oracle.aft_add(blk(yt, cens), coef, fi, sm, st)
    check(make(yt, cens).aft_eval(coef, fi, sm), st)


@pytest.mark.gpu
def test_kmeans_iter_cosine_two_iterations(cuda):
    """The resident-dataset Lloyd body with the cosine measure
    (cyc_kmeans_iter_measure): the second iteration passes the updated
    centers' VectorWithNorm norms (1.0, DistanceMeasure.scala:477-483);
    dense and CSR datasets vs the restatement."""
    rng = np.random.default_rng(31)
    n, d, k = 4000, 24, 10
    X = rng.normal(size=(n, d)) + rng.integers(0, 5, size=(n, 1)) * 2.0
    C = X[:k].copy()
    ds = ResidentDataset.dense(d, n)
    ds.append_dense(X)
    xn = oracle.row_norms(X)
    cn = oracle.row_norms(C)
    for it in range(2):
        sums, wsum, cost, assign = ds.kmeans_iter(C, want_assign=True, distanceMeasure="cosine",
                                                  center_norms=None if it == 0 else cn)
        ref = oracle.cos_kmeans_iteration(X, xn, None, C, cn)
        assert np.array_equal(assign, ref["assign"])
        _rel_close(sums, ref["sums"])
        _rel_close(wsum, ref["wsum"])
        assert abs(cost[0] - ref["cost"]) <= 1e-10 * abs(ref["cost"])
        C, cn = ref["centers"], ref["cnorm"]
    # CSR rows, every one with stored nonzeros (the cosine assert needs |x| > 0)
    rp, ci, vv = [0], [], []
    for _ in range(n):
        cols = np.sort(rng.choice(d, size=int(rng.integers(1, 9)), replace=False))
        ci += list(cols)
        vv += list(rng.uniform(0.1, 1.0, size=cols.size))
        rp.append(len(ci))
    rp, ci, vv = np.array(rp, np.int64), np.array(ci, np.int32), np.array(vv)
    dcs = ResidentDataset.csr(d, n, int(rp[-1]))
    dcs.append_csr(rp, ci, vv)
    C2 = rng.normal(size=(k, d))
    sums, wsum, cost, assign = dcs.kmeans_iter(C2, want_assign=True, distanceMeasure="cosine")
    c2n = oracle.row_norms(C2)
    xn2 = oracle.row_norms_csr(rp, vv)
    ra, rd, rs, rw, rc = oracle.cos_kmeans_partition_sparse((rp, ci, vv, d), xn2, None, C2, c2n,
                                                            oracle.cos_stats(C2, c2n))
    assert np.array_equal(assign, ra)
    _rel_close(sums, rs)
    # a zero-length row: the reference's AssertionError
    rp0 = np.array([0, 0, 1], np.int64)
    dz = ResidentDataset.csr(d, 2, 1)
    dz.append_csr(rp0, np.array([3], np.int32), np.array([1.0]))
    with pytest.raises(N.JavaAssertionError, match="Cosine distance is not defined"):
        dz.kmeans_iter(rng.normal(size=(2, d)), distanceMeasure="cosine")
