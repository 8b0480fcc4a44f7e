"""Pin the Summarizer restatement (oracle/: SummarizerBuffer.add/merge/metrics,
MultiClassSummarizer) against the reference's SummarizerSuite known answers
(tests/golden/summarizer_known_answers.json).  CPU only."""
import json
import os

import numpy as np
import pytest

import oracle

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden",
                                   "summarizer_known_answers.json")))


def _add(st, F, row, w):
    if isinstance(row, dict):
        size, pairs = row["sparse"]
        assert size == F
        oracle.summarizer_add(st, F, idx=[p[0] for p in pairs], val=[p[1] for p in pairs],
                              weight=w)
    else:
        oracle.summarizer_add(st, F, x=row, weight=w)


def _buffer(case, weighted):
    rows = case["rows"]
    F = len(rows[0]) if not isinstance(rows[0], dict) else rows[0]["sparse"][0]
    ws = case["weights"] if weighted else [1.0] * len(rows)
    split = case.get("split")
    if split is None:
        st = oracle.summarizer_new(F)
        for r, w in zip(rows, ws):
            _add(st, F, r, w)
        return F, st
    a, b = oracle.summarizer_new(F), oracle.summarizer_new(F)
    for r, w in zip(rows[:split], ws[:split]):
        _add(a, F, r, w)
    for r, w in zip(rows[split:], ws[split:]):
        _add(b, F, r, w)
    return F, oracle.summarizer_merge(F, a, b)


@pytest.mark.parametrize("case", GOLD["cases"], ids=lambda c: c["name"])
def test_summarizer_known_answers(case):
    for mode in ("weighted", "unweighted"):
        if mode not in case:
            continue
        F, st = _buffer(case, mode == "weighted")
        m = oracle.summarizer_metrics(F, st)
        for key, want in case[mode].items():
            got = m["count"] if key == "count" else m["numNonzeros" if key == "numNonZeros" else key]
            np.testing.assert_allclose(got, want, rtol=0, atol=case["abs_tol"], err_msg=key)


def test_zero_variance_merge_spark_21818():
    """SummarizerSuite.scala:468-484: merged single-row buffers, variance >= 0."""
    bufs = []
    for w in (0.7, 0.4, 0.5, 0.4):
        st = oracle.summarizer_new(1)
        oracle.summarizer_add(st, 1, x=[3.0], weight=w)
        bufs.append(st)
    acc = bufs[0]
    for b in bufs[1:]:
        oracle.summarizer_merge(1, acc, b)
    assert oracle.summarizer_metrics(1, acc)["variance"][0] >= 0.0


def test_negative_weight_flag():
    st = oracle.summarizer_new(2)
    oracle.summarizer_add(st, 2, x=[1.0, 2.0], weight=-1.0)
    assert st[2 * 8 + 3] == 1.0 and st[2 * 8 + 4] == -1.0


def test_label_summarizer_semantics():
    g = GOLD["labels"]
    hist, inv, nc = oracle.label_summarize(np.array(g["y"]), np.array(g["w"]), 3)
    np.testing.assert_array_equal(hist, g["histogram"])
    assert inv == g["countInvalid"] and nc == g["numClasses"]
