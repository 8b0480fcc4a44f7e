"""GPU parity tests: the Summarizer pre-pass (csrc/summarizer.hip) vs the CPU
restatement (oracle/: SummarizerBuffer.add/merge/metrics, Summarizer.scala:
428-770; MultiClassSummarizer, MultiClassSummarizer.scala:30-98) and the
reference's SummarizerSuite known answers.

Bar: bit-exact buffers and metrics for the same partitioning (the device runs
the reference's per-element operation order, partitions merged in order);
the known answers at the suite's own absolute tolerances.
"""
import json
import os

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden",
                                   "summarizer_known_answers.json")))


def _dev(a, cuda):
    import torch
    return None if a is None else torch.from_numpy(np.ascontiguousarray(a)).to(cuda)


def _dense_data(rng, n, F, weighted):
    X = rng.normal(size=(n, F)) * rng.uniform(0.1, 5.0, size=F)
    X[rng.random((n, F)) < 0.3] = 0.0            # zeros are skipped (nonZeroIterator)
    X[:, 0] = 0.0                                # an all-zero column
    if F > 2:
        X[:, 2] = np.abs(X[:, 2]) + 1.0          # a strictly positive column (min > 0)
    w = None
    if weighted:
        w = rng.uniform(0.0, 2.0, n)
        w[rng.random(n) < 0.1] = 0.0             # rows of weight 0 are skipped
    return X, w


@pytest.mark.parametrize("n,F,R,weighted", [(1, 3, 7, False), (500, 7, 64, True),
                                            (4000, 33, 300, True), (20000, 300, 4096, False),
                                            (3000, 5, 1 << 15, True)])
def test_dense_buffer_and_metrics_bitexact(cuda, n, F, R, weighted):
    from cycloneml_amd.stat import SummarizerBuffer
    rng = np.random.default_rng(n + F)
    X, w = _dense_data(rng, n, F, weighted)
    ref = oracle.summarize(F, X=X, w=w, rows_per_partition=R)
    sb = SummarizerBuffer.of_dense(_dev(X, cuda), _dev(w, cuda), rows_per_partition=R)
    np.testing.assert_array_equal(sb.buf.cpu().numpy(), ref)
    m = oracle.summarizer_metrics(F, ref)
    for key in ("mean", "variance", "std", "sum", "numNonzeros", "max", "min", "normL2",
                "normL1"):
        np.testing.assert_array_equal(getattr(sb, key), m[key], err_msg=key)
    assert sb.count == int(m["count"]) and sb.weightSum == m["weightSum"]


def test_csr_buffer_bitexact_two_row_blocks(cuda):
    """CSR rows through the CSC copy: its row blocks (2^18 rows) are the
    partitions, so 300k rows give two partitions merged in order."""
    from cycloneml_amd.optim import DeviceInstanceBlock
    from cycloneml_amd.stat import SummarizerBuffer
    rng = np.random.default_rng(3)
    n, F, k = 300_000, 1000, 8
    # k distinct increasing columns per row (one per stratum of F / k), as a
    # SparseVector requires (Vectors.scala:617-625)
    cols = (np.arange(k) * (F // k) + rng.integers(0, F // k, size=(n, k))).astype(np.int32)
    vals = rng.normal(size=(n, k))
    vals[rng.random((n, k)) < 0.05] = 0.0        # explicit zeros are skipped
    rp = np.arange(0, n * k + 1, k, dtype=np.int64)
    w = rng.uniform(0.0, 1.0, n)
    blk = DeviceInstanceBlock.from_numpy(np.zeros(n), w, csr=(rp, cols.ravel(), vals.ravel()),
                                         numFeatures=F, device=cuda)
    sb = SummarizerBuffer.of_block(blk)
    ref = oracle.summarize(F, csr=(rp, cols.ravel(), vals.ravel()), w=w,
                           rows_per_partition=1 << 18)
    np.testing.assert_array_equal(sb.buf.cpu().numpy(), ref)


def test_merge_bitexact(cuda):
    from cycloneml_amd.stat import SummarizerBuffer
    rng = np.random.default_rng(8)
    X, w = _dense_data(rng, 900, 12, True)
    a = SummarizerBuffer.of_dense(_dev(X[:300], cuda), _dev(w[:300], cuda), rows_per_partition=50)
    b = SummarizerBuffer.of_dense(_dev(X[300:], cuda), _dev(w[300:], cuda), rows_per_partition=80)
    ra = oracle.summarize(12, X=X[:300], w=w[:300], rows_per_partition=50)
    rb = oracle.summarize(12, X=X[300:], w=w[300:], rows_per_partition=80)
    np.testing.assert_array_equal(a.merge(b).buf.cpu().numpy(),
                                  oracle.summarizer_merge(12, ra.copy(), rb))


def _rows_matrix(case):
    rows = case["rows"]
    F = len(rows[0]) if not isinstance(rows[0], dict) else rows[0]["sparse"][0]
    X = np.zeros((len(rows), F))
    for i, r in enumerate(rows):
        if isinstance(r, dict):
            for j, v in r["sparse"][1]:
                X[i, j] = v
        else:
            X[i] = r
    return X, F


@pytest.mark.parametrize("case", GOLD["cases"], ids=lambda c: c["name"])
def test_summarizer_suite_known_answers_on_device(cuda, case):
    from cycloneml_amd.stat import SummarizerBuffer
    X, F = _rows_matrix(case)
    for mode in ("weighted", "unweighted"):
        if mode not in case:
            continue
        w = np.array(case["weights"]) if mode == "weighted" else None
        split = case.get("split")
        if split is None:
            sb = SummarizerBuffer.of_dense(_dev(X, cuda), _dev(w, cuda))
        else:
            sb = SummarizerBuffer.of_dense(_dev(X[:split], cuda),
                                           None if w is None else _dev(w[:split], cuda)).merge(
                SummarizerBuffer.of_dense(_dev(X[split:], cuda),
                                          None if w is None else _dev(w[split:], cuda)))
        for key, want in case[mode].items():
            got = sb.count if key == "count" else getattr(
                sb, "numNonzeros" if key == "numNonZeros" else key)
            np.testing.assert_allclose(got, want, rtol=0, atol=case["abs_tol"], err_msg=key)


def test_errors(cuda):
    import cycloneml_amd._native as N
    from cycloneml_amd.stat import SummarizerBuffer
    X = np.ones((5, 3))
    w = np.array([1.0, 2.0, -0.5, 1.0, 1.0])
    sb = SummarizerBuffer.of_dense(_dev(X, cuda), _dev(w, cuda))
    with pytest.raises(N.IllegalArgumentException, match="sample weight, -0.5 has to be >= 0.0"):
        sb.mean
    empty = SummarizerBuffer.of_dense(_dev(np.zeros((0, 3)), cuda))
    assert empty.count == 0
    with pytest.raises(N.IllegalArgumentException, match="Nothing has been added"):
        empty.mean
    with pytest.raises(N.IllegalArgumentException, match="Nothing has been added"):
        empty.numNonzeros


def test_label_summarizer_vs_oracle(cuda):
    from cycloneml_amd.stat import MultiClassSummarizer
    rng = np.random.default_rng(4)
    n = 50_000
    y = rng.integers(0, 37, n).astype(np.float64)
    y[rng.random(n) < 0.01] = 2.5
    y[rng.random(n) < 0.01] = -1.0
    y[rng.random(n) < 0.005] = np.nan
    w = rng.uniform(0.0, 3.0, n)
    w[rng.random(n) < 0.05] = 0.0
    # max_classes 8 < numClasses exercises the second pass
    m = MultiClassSummarizer.of_labels(_dev(y, cuda), _dev(w, cuda), rows_per_partition=4096,
                                       max_classes=8)
    hist, inv, nc = oracle.label_summarize(y, w, rows_per_partition=4096, max_classes=64)
    assert m.numClasses == nc and m.countInvalid == inv
    np.testing.assert_array_equal(m.histogram, hist)
    g = GOLD["labels"]
    m2 = MultiClassSummarizer.of_labels(_dev(np.array(g["y"]), cuda), _dev(np.array(g["w"]), cuda),
                                        rows_per_partition=3)
    np.testing.assert_array_equal(m2.histogram, g["histogram"])
    assert m2.countInvalid == g["countInvalid"] and m2.numClasses == g["numClasses"]


def test_standardize_and_classification_summarizers(cuda):
    """LogisticRegression.train's pre-pass (:511-516, :957-965) on the device:
    summarizers, inverseStd, scaledMean, then the in-place scaling."""
    from cycloneml_amd.optim import DeviceInstanceBlock
    from cycloneml_amd.stat import getClassificationSummarizers, standardize_
    rng = np.random.default_rng(9)
    n, F = 5000, 16
    X, _ = _dense_data(rng, n, F, False)
    y = rng.integers(0, 3, n).astype(np.float64)
    blk = DeviceInstanceBlock.from_numpy(y, None, X=X, device=cuda)
    summ, lab = getClassificationSummarizers([blk], rows_per_partition=1000)
    ref = oracle.summarize(F, X=X, rows_per_partition=1000)
    m = oracle.summarizer_metrics(F, ref)
    np.testing.assert_array_equal(summ.std, m["std"])
    np.testing.assert_array_equal(lab.histogram, np.bincount(y.astype(int)).astype(float))
    inv_std = np.array([1.0 / s if s != 0 else 0.0 for s in summ.std])
    standardize_(blk, inv_std)
    np.testing.assert_array_equal(blk.X.cpu().numpy(), X * inv_std[None, :])
    # CSR: values(k) *= scale(indices(k))
    rp = np.arange(0, 3 * 4 + 1, 4, dtype=np.int64)
    ci = np.array([0, 3, 7, 15, 1, 2, 3, 4, 0, 5, 9, 10], np.int32)
    v = rng.normal(size=12)
    sblk = DeviceInstanceBlock.from_numpy(np.zeros(3), None, csr=(rp, ci, v), numFeatures=F,
                                          device=cuda)
    standardize_(sblk, inv_std)
    np.testing.assert_array_equal(sblk.values.cpu().numpy(), v * inv_std[ci])
