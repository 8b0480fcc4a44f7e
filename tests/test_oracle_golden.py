"""Pin the CPU restatement (oracle/) against the reference's own known-answer
tests and fixtures (tests/golden/reference_known_answers.json, each entry
citing its Scala source).  CPU only."""
import json
import os

import numpy as np
import pytest

import oracle

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden",
                                   "reference_known_answers.json")))


def test_gram_known_answer_dense_and_sparse():
    g = GOLD["rowmatrix_gram"]
    X = np.array(g["rows"])
    U = oracle.gramian_partition(X)
    assert list(oracle.triu_to_full(3, U)) == g["expected_colmajor"]
    U2 = np.zeros(6)
    for idx, val in g["sparse_rows"]:
        oracle.spr_sparse(idx, val, U2)
    assert list(oracle.triu_to_full(3, U2)) == g["expected_colmajor"]


def test_spr_known_answer():
    s = GOLD["blas_spr"]
    U = np.array(s["U"])
    oracle.dspr_upper(s["x"], U, s["alpha"])
    np.testing.assert_allclose(U, s["expected"], rtol=0, atol=s["abs_tol"])
    U2 = np.array(s["U"])
    oracle.spr_sparse(s["sparse_idx"], s["sparse_val"], U2, 0.1)
    np.testing.assert_allclose(U2, s["expected_sparse"], rtol=0, atol=s["abs_tol_sparse"])


def _cov_oracle(X):
    m = X.shape[0]
    mean = X.sum(0) / m
    n = X.shape[1]
    U = oracle.gramian_partition(X, mean)
    G = oracle.triu_to_full(n, U).reshape(n, n).T
    return G / (m - 1.0)


def test_covariance_and_pca_known_answers():
    g = GOLD["rowmatrix_gram"]
    X = np.array(g["rows"])
    cov = _cov_oracle(X)
    np.testing.assert_allclose(cov, np.cov(X.T), atol=1e-12)
    u, s, _ = np.linalg.svd(cov)
    pca = GOLD["rowmatrix_pca"]
    pc = np.array(pca["principal_components_rows"])
    for j in range(3):
        assert min(np.abs(u[:, j] - pc[:, j]).max(), np.abs(u[:, j] + pc[:, j]).max()) < 1e-6
    np.testing.assert_allclose(s / s.sum(), pca["explained_variance"], atol=1e-6)
    acc = np.array(GOLD["rowmatrix_cov_accuracy"]["rows"])
    np.testing.assert_allclose(np.abs(_cov_oracle(acc)), np.abs(np.cov(acc.T)), atol=1e-6)


def _lloyd(points, w, C, max_iter=20, eps=1e-4):
    C = np.array(C, dtype=np.float64)
    cn = oracle.row_norms(C)
    xn = oracle.row_norms(points)
    for _ in range(max_iter):
        r = oracle.kmeans_iteration(points, xn, w, C, cn)
        C, cn = r["centers"], r["cnorm"]
        if r["converged"]:
            break
    return C, r


def test_weighted_kmeans_exact_centers():
    g = GOLD["kmeans_weighted_two_centers"]
    pts = np.array(g["points"])
    for case in g["cases"]:
        C, _ = _lloyd(pts, np.array(case["weights"]), pts[[0, 3]])
        assert {tuple(c) for c in C} == {tuple(c) for c in case["centers"]}


def test_kmeans_example_sparse_path():
    """KMeansExample input through the sparse (norm-trick) findClosest."""
    g = GOLD["kmeans_example_data"]
    idx, val = [], []
    for line in g["libsvm"]:
        toks = line.split()[1:]
        idx.append([int(t.split(":")[0]) - 1 for t in toks])
        val.append([float(t.split(":")[1]) for t in toks])
    dense = np.zeros((6, 3))
    for r in range(6):
        dense[r, idx[r]] = val[r]
    C = dense[[0, 3]].copy()
    for _ in range(20):
        cn = oracle.row_norms(C)
        stats = oracle.kmeans_stats(C)
        assign = [oracle.find_closest_stats_sparse(C, cn, stats, idx[r], val[r],
                                                   oracle.norm2(val[r]))[0] for r in range(6)]
        newC = np.array([dense[[r for r in range(6) if assign[r] == j]].mean(0) for j in range(2)])
        if np.allclose(newC, C):
            break
        C = newC
    clusters = sorted(sorted(r for r in range(6) if assign[r] == j) for j in range(2))
    assert clusters == g["expected_clusters"]
    np.testing.assert_allclose(sorted(C.tolist()), g["expected_centers_approx"], atol=1e-12)


def test_distance_measure_suite_with_vs_without_stats():
    """DistanceMeasureSuite.scala:55-67 (java.util.Random(42), k=10, dim=8)."""
    rng = oracle.JavaRandom(42)
    C = np.array([[rng.next_gaussian() for _ in range(8)] for _ in range(10)])
    X = np.array([[rng.next_gaussian() for _ in range(8)] for _ in range(1000)])
    cn = oracle.row_norms(C)
    stats = oracle.kmeans_stats(C)
    for x in X:
        xn = oracle.norm2(x)
        i1, c1 = oracle.find_closest(C, cn, x, xn)
        i2, c2 = oracle.find_closest_stats(C, cn, stats, x, xn)
        assert i1 == i2
        assert abs(c1 - c2) <= 1e-10 * min(abs(c1), abs(c2)) or c1 == c2


def test_java_random_matches_known_sequence():
    # java.util.Random(42).nextDouble() / nextGaussian() published values
    r = oracle.JavaRandom(42)
    assert r.next_double() == 0.7275636800328681
    r = oracle.JavaRandom(42)
    assert abs(r.next_gaussian() - 1.1419053154730547) < 1e-15


def test_utils_softmax_and_log1pexp():
    a = np.array([1.0, 2.0, 3.0])
    oracle.lib().orc_softmax(a.ctypes.data_as(oracle._D), 3, 0, 1)
    e = np.exp(np.array([1.0, 2.0, 3.0]) - 3.0)
    np.testing.assert_allclose(a, e / e.sum(), rtol=1e-15)
    b = np.array([1.0, np.inf, 3.0, np.inf])
    oracle.lib().orc_softmax(b.ctypes.data_as(oracle._D), 4, 0, 1)
    assert list(b) == [0.0, 1.0, 0.0, np.inf * 0.0] or (b[1] == 1.0 and b[0] == 0.0)
    assert oracle.log1pexp(800.0) == 800.0
    assert oracle.log1pexp(-800.0) == 0.0
    assert abs(oracle.log1pexp(0.5) - np.log1p(np.exp(0.5))) < 1e-15


# ------------------------------------------------------------- aggregators

def _summ(instances):
    """Summarizer mean/std (weighted, unbiased; Summarizer.scala:673-690)."""
    X = np.array([f for _, _, f in instances])
    w = np.array([w for _, w, _ in instances])
    W = w.sum()
    mean = (w[:, None] * X).sum(0) / W
    denom = W - (w * w).sum() / W
    var = (w[:, None] * (X - mean) ** 2).sum(0) / denom
    return mean, np.sqrt(var)


def _blocks(scaled, bs, sparse):
    out = []
    for s in range(0, len(scaled), bs):
        grp = scaled[s:s + bs]
        labels = np.array([l for l, _, _ in grp])
        weights = np.array([w for _, w, _ in grp])
        X = np.array([f for _, _, f in grp])
        if sparse:
            rp, ci, vv = [0], [], []
            for row in X:
                nz = np.nonzero(row)[0]
                ci += list(nz)
                vv += list(row[nz])
                rp.append(len(ci))
            out.append(dict(labels=labels, weights=weights, rowptr=np.array(rp),
                            colidx=np.array(ci, dtype=np.int32), values=np.array(vv),
                            F=X.shape[1]))
        else:
            out.append(dict(labels=labels, weights=weights, X=X))
    return out


@pytest.mark.parametrize("fit_intercept,fit_with_mean", [(False, False), (True, False),
                                                         (True, True)])
def test_binary_aggregator_vs_naive_loop(fit_intercept, fit_with_mean):
    """BinaryLogisticBlockAggregatorSuite.scala:131-264 naive expectations."""
    g = GOLD["logistic_aggregator_instances"]
    inst = [(l, w, np.array(f)) for l, w, f in g["binary"]]
    mean, std = _summ(inst)
    inv = np.where(std != 0, 1.0 / std, 0.0)
    coef = np.array(g["binary_coef"])
    icpt = g["binary_intercept"] if fit_intercept else 0.0
    W = sum(w for _, w, _ in inst)
    loss, grad, gi = 0.0, np.zeros(2), 0.0
    for l, w, f in inst:
        x = f - mean if fit_with_mean else f
        margin = (coef / std) @ x + icpt
        prob = 1.0 / (1.0 + np.exp(-margin))
        loss += -w * l * np.log(prob) - w * (1.0 - l) * np.log1p(-prob)
        grad += w * (prob - l) * x / std
        gi += w * (prob - l)
    exp_loss = loss / W
    exp_grad = np.append(grad, gi) / W if fit_intercept else grad / W
    scaled = [(l, w, f * inv) for l, w, f in inst]
    full_coef = np.append(coef, icpt) if fit_intercept else coef
    for bs in g["block_sizes"]:
        for sparse in (False, True):
            st = dict(grad=np.zeros(full_coef.size), loss=0.0, weight=0.0)
            for b in _blocks(scaled, bs, sparse):
                oracle.binary_logistic_add(b, full_coef, fit_intercept, fit_with_mean,
                                           inv * mean if fit_with_mean else None, st)
            assert abs(st["loss"] / st["weight"] - exp_loss) <= 1e-9 * abs(exp_loss)
            np.testing.assert_allclose(st["grad"] / st["weight"], exp_grad, rtol=1e-9)


@pytest.mark.parametrize("fit_intercept,fit_with_mean", [(False, False), (True, False),
                                                         (True, True)])
def test_multinomial_aggregator_vs_naive_loop(fit_intercept, fit_with_mean):
    """MultinomialLogisticBlockAggregatorSuite.scala:134-346 naive expectations."""
    g = GOLD["logistic_aggregator_instances"]
    inst = [(l, w, np.array(f)) for l, w, f in g["multinomial"]]
    C, F = 3, 2
    mean, std = _summ(inst)
    inv = np.where(std != 0, 1.0 / std, 0.0)
    coef = np.array(g["multinomial_coef"])          # column-major C x F
    icpt = np.array(g["multinomial_intercept"]) if fit_intercept else np.zeros(C)
    Wm = np.array([[coef[f * C + c] / std[f] for f in range(F)] for c in range(C)])
    W = sum(w for _, w, _ in inst)
    loss = 0.0
    grad = np.zeros(C * F)
    gi = np.zeros(C)
    for l, w, f in inst:
        x = f - mean if fit_with_mean else f
        m = Wm @ x + icpt
        p = np.exp(m) / np.exp(m).sum()
        loss += w * (np.log(np.exp(m).sum()) - m[int(l)])
        for c in range(C):
            d = w * (p[c] - (1.0 if c == int(l) else 0.0))
            for ff in range(F):
                grad[ff * C + c] += d * x[ff] / std[ff]
            gi[c] += d
    exp_loss = loss / W
    exp_grad = (np.concatenate([grad, gi]) if fit_intercept else grad) / W
    scaled = [(l, w, f * inv) for l, w, f in inst]
    full = np.concatenate([coef, icpt]) if fit_intercept else coef
    for bs in g["block_sizes"]:
        for sparse in (False, True):
            st = dict(grad=np.zeros(full.size), loss=0.0, weight=0.0)
            for b in _blocks(scaled, bs, sparse):
                oracle.multinomial_logistic_add(b, full, C, fit_intercept, fit_with_mean,
                                                inv * mean if fit_with_mean else None, st)
            assert abs(st["loss"] / st["weight"] - exp_loss) <= 1e-9 * abs(exp_loss)
            np.testing.assert_allclose(st["grad"] / st["weight"], exp_grad, rtol=1e-9)


def test_point_costs_restate_find_closest_without_statistics():
    """orc_point_costs / orc_point_costs_sparse (pointCost, DistanceMeasure.scala:
    152-156, 318-340) against a pure-Python restatement of the loop, and the
    KMeansSuite "two clusters" points (mllib KMeansSuite.scala:255-278)."""
    import math
    rng = np.random.default_rng(3)
    X = rng.normal(size=(60, 5))
    C = X[:7].copy()
    C[4] = C[2]
    xn, cn = oracle.row_norms(X), oracle.row_norms(C)
    a, c, s = oracle.point_costs(X, xn, C, cn)
    for r in range(X.shape[0]):
        best, bi = math.inf, 0
        for i in range(C.shape[0]):
            lb = (cn[i] - xn[r]) ** 2
            if lb < best:
                dd = 0.0
                for j in range(X.shape[1]):
                    t = C[i, j] - X[r, j]
                    dd += t * t
                if dd < best:
                    best, bi = dd, i
        assert a[r] == bi and c[r] == best
    tot = 0.0
    for v in c:
        tot += v
    assert s == tot
    # sparse rows: the same points as CSR agree with the dense loop on indices
    rowptr = np.arange(0, X.size + 1, X.shape[1], dtype=np.int64)
    colidx = np.tile(np.arange(X.shape[1], dtype=np.int32), X.shape[0])
    a2, c2, _ = oracle.point_costs_sparse((rowptr, colidx, X.ravel()), xn, C, cn)
    assert np.array_equal(a2, a)
    np.testing.assert_allclose(c2, c, rtol=1e-12, atol=1e-12)
    P = np.array([[0.0, 0.0], [0.0, 0.1], [0.1, 0.0], [9.0, 0.0], [9.0, 0.2], [9.2, 0.0]])
    Cp = np.array([[0.1 / 3, 0.1 / 3], [9.2 / 3 + 6.0, 0.2 / 3]])
    ap, _, _ = oracle.point_costs(P, oracle.row_norms(P), Cp, oracle.row_norms(Cp))
    assert list(ap) == [0, 0, 0, 1, 1, 1]


@pytest.mark.parametrize("fit_intercept", [False, True])
def test_hinge_aggregator_vs_naive_loop(fit_intercept):
    """HingeBlockAggregatorSuite.scala:128-219 naive expectations (its three
    weighted instances, coefficients (1, 2), intercept 1.0; block sizes 1, 2,
    4; dense and sparse blocks; relTol 1e-9)."""
    inst = [(0.0, 0.1, np.array([1.0, 2.0])), (1.0, 0.5, np.array([1.5, 1.0])),
            (0.0, 0.3, np.array([4.0, 0.5]))]
    mean, std = _summ(inst)
    inv = np.where(std != 0, 1.0 / std, 0.0)
    coef = np.array([1.0, 2.0])
    icpt = 1.0 if fit_intercept else 0.0
    W = sum(w for _, w, _ in inst)
    loss, grad, gi = 0.0, np.zeros(2), 0.0
    for l, w, f in inst:
        x = f - mean if fit_intercept else f
        margin = (coef / std) @ x + icpt
        ls = 2 * l - 1.0
        if 1.0 > ls * margin:
            loss += (1.0 - ls * margin) * w
            grad += x * -ls * w / std
            gi += -ls * w
    exp_loss = loss / W
    exp_grad = np.append(grad, gi) / W if fit_intercept else grad / W
    scaled = [(l, w, f * inv) for l, w, f in inst]
    full_coef = np.append(coef, icpt) if fit_intercept else coef
    for bs in (1, 2, 4):
        for sparse in (False, True):
            st = dict(grad=np.zeros(full_coef.size), loss=0.0, weight=0.0)
            for b in _blocks(scaled, bs, sparse):
                oracle.hinge_add(b, full_coef, fit_intercept, inv * mean if fit_intercept else None,
                                 st)
            assert abs(st["loss"] / st["weight"] - exp_loss) <= 1e-9 * abs(exp_loss)
            np.testing.assert_allclose(st["grad"] / st["weight"], exp_grad, rtol=1e-9)


def test_least_squares_aggregator_vs_naive_loop():
    """LeastSquaresBlockAggregatorSuite.scala:122-178 "check correctness" (its
    three weighted instances, coefficients (1, 2), fitIntercept = true; block
    sizes 1, 2, 4; dense and sparse blocks; relTol 1e-9), plus the constant
    feature case (:45-49): effectiveCoef zeroes it."""
    inst = [(0.0, 0.1, np.array([1.0, 2.0])), (1.0, 0.5, np.array([1.5, 1.0])),
            (0.0, 0.3, np.array([4.0, 0.5]))]
    mean, std = _summ(inst)
    ymean, ystd = _summ([(0.0, w, np.array([l])) for l, w, _ in inst])
    ymean, ystd = float(ymean[0]), float(ystd[0])
    inv = np.where(std != 0, 1.0 / std, 0.0)
    coef = np.array([1.0, 2.0])
    W = sum(w for _, w, _ in inst)
    errs = [coef @ ((f - mean) / std) - (l - ymean) / ystd for l, _, f in inst]
    exp_loss = sum(w * e * e / 2.0 for e, (_, w, _) in zip(errs, inst)) / W
    exp_grad = sum(e * w * f / std for e, (_, w, f) in zip(errs, inst)) / W
    scaled = [(l, w, f * inv) for l, w, f in inst]
    for bs in (1, 2, 4):
        for sparse in (False, True):
            st = dict(grad=np.zeros(2), loss=0.0, weight=0.0)
            for b in _blocks(scaled, bs, sparse):
                oracle.least_squares_add(b, coef, inv, True, ystd, ymean, inv * mean, st)
            assert abs(st["loss"] / st["weight"] - exp_loss) <= 1e-9 * abs(exp_loss)
            np.testing.assert_allclose(st["grad"] / st["weight"], exp_grad, rtol=1e-9)
    # constant feature: the aggregator equals the one over the filtered feature
    const = [(0.0, 0.1, np.array([1.0, 2.0])), (1.0, 0.5, np.array([1.0, 1.0])),
             (1.0, 0.3, np.array([1.0, 0.5]))]
    m2, s2 = _summ(const)
    inv2 = np.where(s2 != 0, 1.0 / s2, 0.0)
    ym, ys = _summ([(0.0, w, np.array([l])) for l, w, _ in const])
    st = dict(grad=np.zeros(2), loss=0.0, weight=0.0)
    oracle.least_squares_add(_blocks([(l, w, f * inv2) for l, w, f in const], 3, False)[0],
                             coef, inv2, True, float(ys[0]), float(ym[0]), inv2 * m2, st)
    stf = dict(grad=np.zeros(1), loss=0.0, weight=0.0)
    oracle.least_squares_add(_blocks([(l, w, f[1:] * inv2[1:]) for l, w, f in const], 3,
                                     False)[0], coef[1:], inv2[1:], True, float(ys[0]),
                             float(ym[0]), (inv2 * m2)[1:], stf)
    assert st["grad"][0] == 0.0
    np.testing.assert_allclose(st["grad"][1:], stf["grad"], rtol=1e-12)
    assert st["loss"] == pytest.approx(stf["loss"], rel=1e-12)


@pytest.mark.parametrize("fit_intercept,sigma", [(False, 4.0), (True, 4.0), (True, 0.3),
                                                 (False, 0.3)])
def test_huber_aggregator_vs_naive_loop(fit_intercept, sigma):
    """HuberBlockAggregatorSuite.scala:132-250 naive expectations (its three
    instances, coefficients (1, 2), intercept 3.0, sigma 4.0, epsilon 1.35;
    block sizes 1, 2, 4; dense and sparse blocks; relTol 1e-9); sigma 0.3
    takes the suite's formulas into the linear branch too."""
    inst = [(0.0, 0.1, np.array([1.0, 2.0])), (1.0, 0.5, np.array([1.5, 1.0])),
            (0.0, 0.3, np.array([4.0, 0.5]))]
    eps = 1.35
    mean, std = _summ(inst)
    inv = np.where(std != 0, 1.0 / std, 0.0)
    coef = np.array([1.0, 2.0])
    icpt = 3.0 if fit_intercept else 0.0
    W = sum(w for _, w, _ in inst)
    loss, gc, gi, gs = 0.0, np.zeros(2), 0.0, 0.0
    for l, w, f in inst:
        x = f - mean if fit_intercept else f
        margin = (coef / std) @ x + icpt
        ll = l - margin
        if abs(ll) <= sigma * eps:
            loss += 0.5 * w * (sigma + ll ** 2 / sigma)
            gc += -1.0 * w * (ll / sigma) * (x / std)
            gi += -1.0 * w * (ll / sigma)
            gs += 0.5 * w * (1.0 - (ll / sigma) ** 2)
        else:
            loss += 0.5 * w * (sigma + 2.0 * eps * abs(ll) - sigma * eps * eps)
            sign = -1.0 if ll >= 0 else 1.0
            gc += w * sign * eps * (x / std)
            gi += w * sign * eps
            gs += 0.5 * w * (1.0 - eps * eps)
    exp_grad = (np.concatenate([gc, [gi, gs]]) if fit_intercept else np.append(gc, gs)) / W
    params = np.concatenate([coef, [icpt, sigma]]) if fit_intercept else np.append(coef, sigma)
    scaled = [(l, w, f * inv) for l, w, f in inst]
    for bs in (1, 2, 4):
        for sparse in (False, True):
            st = dict(grad=np.zeros(params.size), loss=0.0, weight=0.0)
            for b in _blocks(scaled, bs, sparse):
                oracle.huber_add(b, params, fit_intercept, eps,
                                 inv * mean if fit_intercept else None, st)
            assert abs(st["loss"] / st["weight"] - loss / W) <= 1e-9 * abs(loss / W)
            # entries that cancel to ~0 in the all-linear case: absolute 1e-12
            np.testing.assert_allclose(st["grad"] / st["weight"], exp_grad, rtol=1e-9,
                                       atol=1e-12)


@pytest.mark.parametrize("fit_intercept", [False, True])
def test_aft_aggregator_vs_naive_loop(fit_intercept):
    """AFTBlockAggregator (.scala:76-130) restatement against a per-instance
    loop on explicitly centred, scaled features (the reference has no
    AFTBlockAggregator suite; the expectations restate the aggregator's
    formulas: epsilon = (log t - margin) / sigma, loss = delta log sigma -
    delta epsilon + e^epsilon, multiplier (delta - e^epsilon) / sigma); block
    sizes 1, 2, 4; dense and sparse blocks; relTol 1e-9."""
    inst = [(1.218, 1.0, np.array([1.560, -0.605])), (2.949, 0.0, np.array([0.346, 2.158])),
            (3.627, 0.0, np.array([1.380, 0.231])), (0.273, 1.0, np.array([0.520, 1.151])),
            (4.199, 0.0, np.array([0.795, -0.226]))]
    X = np.array([f for _, _, f in inst])
    mean, std = X.mean(0), X.std(0, ddof=1)
    inv = 1.0 / std
    coef = np.array([0.3, -0.2, 0.5 if fit_intercept else 0.0, 0.1])   # linear, icpt, log sigma
    sigma = np.exp(coef[-1])
    loss, g = 0.0, np.zeros(4)
    for t, delta, f in inst:
        xs = (f - mean) * inv if fit_intercept else f * inv
        margin = coef[:2] @ xs + (coef[2] if fit_intercept else 0.0)
        eps = (np.log(t) - margin) / sigma
        loss += delta * np.log(sigma) - delta * eps + np.exp(eps)
        m = (delta - np.exp(eps)) / sigma
        g[:2] += m * xs
        if fit_intercept:
            g[2] += m
        g[3] += delta + m * sigma * eps
    scaled = [(t, d, f * inv) for t, d, f in inst]
    for bs in (1, 2, 4):
        for sparse in (False, True):
            st = dict(grad=np.zeros(4), loss=0.0, weight=0.0)
            for b in _blocks(scaled, bs, sparse):
                oracle.aft_add(b, coef, fit_intercept, inv * mean if fit_intercept else None, st)
            assert st["weight"] == len(inst)
            assert abs(st["loss"] - loss) <= 1e-9 * abs(loss)
            np.testing.assert_allclose(st["grad"], g, rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("x,s", [
    (1.0, "1.0"), (0.001, "0.001"), (1e-4, "1.0E-4"), (1e7, "1.0E7"), (9999999.0, "9999999.0"),
    (123.456, "123.456"), (-2.5e-4, "-2.5E-4"), (1.7976931348623157e308, "1.7976931348623157E308"),
    (float("nan"), "NaN"), (float("inf"), "Infinity"), (-0.0, "-0.0"), (0.1, "0.1"),
    (100.0, "100.0"), (1234567.0, "1234567.0"), (12345678.9, "1.23456789E7"),
    (0.3333333333333333, "0.3333333333333333"), (2.0 ** 0.5, "1.4142135623730951")])
def test_java_double_to_string(x, s):
    """java.lang.Double.toString, which Scala's s"$norm" interpolation uses in
    MLUtils.scala:542-543's require message."""
    assert oracle.java_double(x) == s


def test_fast_squared_distance_require():
    """MLUtils.scala:542-543: require(norm1 >= 0.0 && norm2 >= 0.0).  With
    statistics (Lloyd, predict) a NaN-norm point fails at center 0 and a NaN
    center fails computeStatistics; without statistics (pointCost) no
    distance with a NaN norm is ever measured, so nothing fails."""
    rng = np.random.default_rng(2)
    X = rng.normal(size=(50, 6))
    C = rng.normal(size=(4, 6))
    X[20, 1] = np.nan
    xn, cn = oracle.row_norms(X), oracle.row_norms(C)
    with pytest.raises(oracle.IllegalArgumentException) as e:
        oracle.kmeans_iteration(X, xn, None, C, cn)
    assert str(e.value) == ("requirement failed: Both norms should be greater or equal to 0.0, "
                            f"found norm1={oracle.java_double(cn[0])}, norm2=NaN")
    a, c, _ = oracle.point_costs(X, xn, C, cn)
    assert a[20] == 0 and c[20] == np.inf
    C[2, 0] = np.nan
    with pytest.raises(oracle.IllegalArgumentException, match="norm1=.*, norm2=NaN"):
        oracle.kmeans_stats(C)


def test_rowmatrix_sparse_paths_restated():
    """RowMatrixSuite sparseData (RowMatrixSuite.scala:45-50): the sparse spr
    Gramian is the exact gram [126, 54, 72, ...] (:95-102); the rows have
    sparsity 1/3 or 0, so isSparseMatrix is false and computeCovariance takes
    the dense path; a matrix whose rows are all at least half zeros takes
    computeSparseVectorCovariance, which equals breeze-style cov (np.cov)
    to rounding."""
    rp = np.array([0, 2, 5, 8, 10])
    ci = np.array([1, 2, 0, 1, 2, 0, 1, 2, 0, 2])
    v = np.array([1.0, 2.0, 3.0, 4.0, 5.0, 6.0, 7.0, 8.0, 9.0, 1.0])
    U = oracle.gramian_csr(rp, ci, v, 3)
    G = oracle.triu_to_full(3, U)
    assert list(G) == [126.0, 54.0, 72.0, 54.0, 66.0, 78.0, 72.0, 78.0, 94.0]
    assert not oracle.is_sparse_matrix(np.diff(rp), 3)
    assert oracle.is_sparse_matrix([2, 1, 0], 4)      # sparsity 0.5 is not < 0.5
    rng = np.random.default_rng(1)
    X = rng.normal(size=(50, 6))
    X[rng.random(X.shape) < 0.6] = 0.0
    X[:, 0] = np.where(np.arange(50) % 2 == 0, 0.0, 1.5)
    nz = np.count_nonzero(X, axis=1)
    X[nz > 3, 1:] = 0.0
    assert oracle.is_sparse_matrix(np.count_nonzero(X, axis=1), 6)
    U = oracle.gramian_partition(X)
    cov = oracle.sparse_vector_covariance(6, U, X.mean(0), 50)
    np.testing.assert_allclose(cov, np.cov(X.T), rtol=1e-10, atol=1e-12)
