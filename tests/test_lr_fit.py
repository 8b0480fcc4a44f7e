"""End-to-end LogisticRegression fits checked against the glmnet coefficients
LogisticRegressionSuite asserts (tests/golden/lr_glmnet_known_answers.json,
with the suite's own tolerances and Spark's TestingUtils semantics).

The suite's datasets are regenerated bit for bit where the JVM is
deterministic: generateMultinomialLogisticInput over java.util.Random(42)
(StrictMath.log / sqrt by Python's math, which can move a rare value by an
ulp) and the rand(42) weight column, XORShiftRandom(42 + partition) over 4
parallelize slices (pinned by RandomSuite's known values in
test_oracle_golden).

CPU tests: the estimator's driver logic (summaries -> optimizer -> solution
in the original space) with the ORACLE aggregator as the data pass over
explicitly standardized rows, i.e. the reference's own arrangement.  GPU
tests: LogisticRegression.fit over device blocks through libcyclone.
"""
import functools
import json
import os

import numpy as np
import pytest

import oracle
from cycloneml_amd import optimize
from cycloneml_amd.classification import LogisticRegression

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden",
                                     "lr_glmnet_known_answers.json")))
CASES = {c["id"]: c for c in GOLDEN["cases"]}


@functools.lru_cache(maxsize=None)
def dataset(name):
    d = GOLDEN["datasets"][name]
    y, X = oracle.generate_multinomial_logistic_input(d["weights"], d["xMean"], d["xVariance"],
                                                      True, d["nPoints"], d["seed"])
    w = oracle.spark_rand_column(d["seed"], d["nPoints"], d["slices"])
    return y, X, w


def spark_close(actual, expected, tol):
    """TestingUtils: relTol -> |x - y| < eps min(|x|, |y|) (x == y passes);
    absTol -> |x - y| < eps."""
    actual = np.ravel(np.asarray(actual, dtype=np.float64))
    expected = np.ravel(np.asarray(expected, dtype=np.float64))
    assert actual.shape == expected.shape
    for a, e in zip(actual, expected):
        if "rel" in tol:
            ok = a == e or abs(a - e) < tol["rel"] * min(abs(a), abs(e))
        else:
            ok = a == e or abs(a - e) < tol["abs"]
        assert ok, f"{a} vs {e} ({tol}); all: {actual} vs {expected}"


def estimator(case):
    p = dict(case["params"])
    lr = LogisticRegression(regParam=p.get("regParam", 0.0),
                            elasticNetParam=p.get("elasticNetParam", 0.0),
                            maxIter=p.get("maxIter", 100), tol=p.get("tol", 1e-6),
                            fitIntercept=p["fitIntercept"],
                            standardization=p["standardization"])
    for k in ("lowerBoundsOnCoefficients", "upperBoundsOnCoefficients",
              "lowerBoundsOnIntercepts", "upperBoundsOnIntercepts"):
        if k in p:
            getattr(lr, "set" + k[0].upper() + k[1:])(p[k])
    return lr


def check_model(case, model):
    nC = len(case["intercept"])
    if case.get("coef_check") == "bounded_mlor_equivalent":
        # checkBoundedMLORCoefficientsEquivalent (LogisticRegressionSuite.scala:3138-3144):
        # per feature, the class-wise differences to the expected column are equal
        # (absTol 1e-2) -- unregularized MLOR is identifiable only up to a shift
        diff = model.coefficientMatrix - np.asarray(case["coef"]).reshape(nC, -1)
        for j in range(diff.shape[1]):
            for a, b in zip(diff[:-1, j], diff[1:, j]):
                assert abs(a - b) < 1e-2, (j, diff[:, j])
    else:
        coef = model.coefficientMatrix.reshape(-1) if nC > 1 else model.coefficients
        spark_close(coef, case["coef"], case["coef_tol"])
    icpt = model.interceptVector if nC > 1 else [model.intercept]
    spark_close(icpt, case["intercept"], case["intercept_tol"])
    if case.get("centered"):
        np.testing.assert_allclose(model.coefficientMatrix.sum(axis=0), 0.0, atol=1e-5)
        np.testing.assert_allclose(model.interceptVector.sum(), 0.0, atol=1e-5)


def oracle_fit(case):
    y, X, w = dataset(case["data"])
    F = X.shape[1]
    m = oracle.summarizer_metrics(F, oracle.summarize(F, X=X, w=w))
    hist, invalid, _ = oracle.label_summarize(y, w)
    assert invalid == 0
    lr = estimator(case)

    def make_cost(numClasses, multinomial, fitWithMean, inverseStd):
        Xs = X * inverseStd                              # the StandardScaler pass
        scaledMean = inverseStd * m["mean"]
        blk = dict(labels=y, weights=w, X=Xs)

        def cost(coef):
            st = dict(grad=np.zeros(coef.size), loss=0.0, weight=0.0)
            if multinomial:
                oracle.multinomial_logistic_add(blk, coef, numClasses, lr.fitIntercept,
                                                fitWithMean, scaledMean, st)
            else:
                oracle.binary_logistic_add(blk, coef, lr.fitIntercept, fitWithMean,
                                           scaledMean, st)
            return st["loss"] / st["weight"], st["grad"] / st["weight"]
        return cost
    return lr.train_from_summary(F, hist, m["mean"], m["std"], make_cost)


@pytest.mark.parametrize("cid", sorted(CASES))
def test_fit_oracle_data_pass(cid):
    case = CASES[cid]
    check_model(case, oracle_fit(case))


def test_datasets_shape():
    y, X, w = dataset("binaryDataset")
    assert X.shape == (10000, 4) and set(np.unique(y)) == {0.0, 1.0}
    assert 0.0 <= w.min() and w.max() < 1.0
    y3, _, _ = dataset("multinomialDataset")
    assert set(np.unique(y3)) == {0.0, 1.0, 2.0}


def test_lbfgs_rosenbrock():
    def f(x):
        a, b = x
        v = (1 - a) ** 2 + 100 * (b - a * a) ** 2
        g = np.array([-2 * (1 - a) - 400 * a * (b - a * a), 200 * (b - a * a)])
        return v, g
    x = optimize.LBFGS(200, 10, 1e-12).minimize(f, np.array([-1.2, 1.0]))
    np.testing.assert_allclose(x, [1.0, 1.0], atol=1e-5)


def test_owlqn_lasso_zeroes():
    # min 0.5 |x - t|^2 + l |x|_1  ->  soft threshold of t
    t = np.array([3.0, -0.5, 0.2, -2.0])
    lam = 1.0

    def f(x):
        return 0.5 * float((x - t) @ (x - t)), x - t
    x = optimize.OWLQN(100, 10, np.full(4, lam), 1e-10).minimize(f, np.zeros(4))
    np.testing.assert_allclose(x, np.sign(t) * np.maximum(np.abs(t) - lam, 0), atol=1e-6)


def test_constant_label_shortcut():
    lr = LogisticRegression()
    m = lr.train_from_summary(3, [0.0, 5.0], np.zeros(3), np.ones(3),
                              lambda *a: pytest.fail("no data pass expected"))
    assert m.intercept == np.inf and np.all(m.coefficients == 0)


def test_param_checks():
    from cycloneml_amd import _native as N
    with pytest.raises(N.IllegalArgumentException):
        LogisticRegression(elasticNetParam=1.5)
    with pytest.raises(N.IllegalArgumentException, match="Binomial family only supports"):
        LogisticRegression(family="binomial").train_from_summary(
            2, [1.0, 2.0, 3.0], np.zeros(2), np.ones(2), None)


# -- GPU: the same fits with the data pass on the device ---------------------

def device_block(name, cuda):
    import torch
    from cycloneml_amd.optim import DeviceInstanceBlock
    y, X, w = dataset(name)
    return DeviceInstanceBlock(torch.as_tensor(y, device=cuda), torch.as_tensor(w, device=cuda),
                               X=torch.as_tensor(X, device=cuda))


@pytest.mark.gpu
@pytest.mark.parametrize("cid", sorted(CASES))
def test_fit_device(cid, cuda):
    case = CASES[cid]
    model = estimator(case).fit(device_block(case["data"], cuda))
    check_model(case, model)


@pytest.mark.gpu
def test_fit_device_csr_matches_dense(cuda):
    """The same binary fit from a CSR copy of the rows (the tiles layout)."""
    import torch
    from cycloneml_amd.optim import DeviceInstanceBlock
    y, X, w = dataset("binaryDataset")
    n, F = X.shape
    rp = torch.arange(0, n * F + 1, F, dtype=torch.int64, device=cuda)
    ci = torch.arange(F, dtype=torch.int32, device=cuda).repeat(n)
    blk = DeviceInstanceBlock(torch.as_tensor(y, device=cuda), torch.as_tensor(w, device=cuda),
                              rowptr=rp, colidx=ci,
                              values=torch.as_tensor(X.reshape(-1), device=cuda), numFeatures=F)
    blk.prepare(layout="tiles")
    case = CASES["binary_intercept_l2_std"]
    check_model(case, estimator(case).fit(blk))


def test_lbfgsb_box_quadratic_kkt():
    rng = np.random.default_rng(0)
    n = 8
    Q = rng.normal(size=(n, n))
    A = Q @ Q.T + n * np.eye(n)
    b = rng.normal(size=n) * 5
    lo, hi = np.full(n, -0.3), np.full(n, 0.4)
    x = optimize.LBFGSB(lo, hi, 500, 10, 1e-12).minimize(
        lambda z: (0.5 * z @ A @ z - b @ z, A @ z - b), np.zeros(n))
    g = A @ x - b
    assert np.abs(np.clip(x - g, lo, hi) - x).max() < 1e-8       # projected gradient = 0
    assert np.all(x >= lo) and np.all(x <= hi) and np.any(x == hi) and np.any(x == lo)


def test_bound_params_checks():
    from cycloneml_amd import _native as N
    hist, mean, std = [3.0, 4.0], np.zeros(4), np.ones(4)
    lr = LogisticRegression(elasticNetParam=0.5, regParam=0.1) \
        .setUpperBoundsOnCoefficients([[1.0, 0.0, 1.0, 0.0]])
    with pytest.raises(N.IllegalArgumentException, match="only supports L2 regularization"):
        lr.train_from_summary(4, hist, mean, std, None)
    lr = LogisticRegression(fitIntercept=False).setUpperBoundsOnIntercepts([1.0])
    with pytest.raises(N.IllegalArgumentException, match="bounds on intercepts"):
        lr.train_from_summary(4, hist, mean, std, None)
    lr = LogisticRegression().setUpperBoundsOnCoefficients([[1.0, 0.0, 1.0]])
    with pytest.raises(N.IllegalArgumentException, match="shape of upperBoundsOnCoefficients"):
        lr.train_from_summary(4, hist, mean, std, None)
    lr = LogisticRegression().setUpperBoundsOnCoefficients([[0.0] * 4]) \
        .setLowerBoundsOnCoefficients([[1.0] * 4])
    with pytest.raises(N.IllegalArgumentException, match="less than or equal"):
        lr.train_from_summary(4, hist, mean, std, None)


def test_initial_model_needs_same_fit_intercept():
    """createInitialSolution (LogisticRegression.scala:836-848): an initial
    model is used only when its shape AND its fitIntercept match; otherwise
    the fit starts from the histogram's intercept as without a model."""
    from cycloneml_amd.classification import LogisticRegressionModel
    F = 3
    hist = np.array([30.0, 70.0])
    std = np.array([1.0, 2.0, 0.5])
    lr = LogisticRegression(fitIntercept=True)
    base = lr._initial_solution(2, F, hist, std, False)
    m_no = LogisticRegressionModel([[0.5, -1.0, 2.0]], [0.25], 2, False, fitIntercept=False)
    lr.setInitialModel(m_no)
    assert np.array_equal(lr._initial_solution(2, F, hist, std, False), base)
    m_yes = LogisticRegressionModel([[0.5, -1.0, 2.0]], [0.25], 2, False, fitIntercept=True)
    lr.setInitialModel(m_yes)
    np.testing.assert_array_equal(lr._initial_solution(2, F, hist, std, False),
                                  [0.5, -2.0, 1.0, 0.25])
