"""LIBSVM input: the native parser (csrc/libsvm.cpp via
cycloneml_amd.mlutils) against the restatement of MLUtils.parseLibSVMFile /
parseLibSVMRecord / computeNumFeatures (oracle.parse_libsvm), bit-exact, on
the reference's own data files (tests/golden/*.txt, copied from
data/mllib/) and on edge cases; the device upload and KMeansExample from the
file are GPU tests."""
import os

import numpy as np
import pytest

import oracle

GOLD = os.path.join(os.path.dirname(__file__), "golden")
FILES = ["sample_kmeans_data.txt", "sample_libsvm_data.txt", "iris_libsvm.txt"]


def _same(a, b):
    la, (ra, ca, va), na = a
    lb, (rb, cb, vb), nb = b
    assert na == nb
    assert np.array_equal(la, lb) and np.array_equal(ra, rb) and np.array_equal(ca, cb)
    assert np.array_equal(va.view(np.int64), vb.view(np.int64))   # bitwise


@pytest.mark.parametrize("name", FILES)
def test_reference_files_bit_exact(name):
    from cycloneml_amd import mlutils
    path = os.path.join(GOLD, name)
    want = oracle.parse_libsvm(open(path).read())
    _same(mlutils.parseLibSVMFile(path), want)
    _same(mlutils.parseLibSVM(open(path, "rb").read(), nthreads=3), want)


def test_known_shapes():
    from cycloneml_amd import mlutils
    labels, (rp, ci, v), nf = mlutils.parseLibSVMFile(os.path.join(GOLD, "sample_kmeans_data.txt"))
    assert nf == 3 and list(labels) == [0, 1, 2, 3, 4, 5] and list(rp) == [0, 3, 6, 9, 12, 15, 18]
    _, (rp, _, _), nf = mlutils.parseLibSVMFile(os.path.join(GOLD, "sample_libsvm_data.txt"))
    assert nf == 692 and rp.size == 101           # the classic 100 x 692 sample
    labels, _, nf = mlutils.parseLibSVMFile(os.path.join(GOLD, "iris_libsvm.txt"))
    assert nf == 4 and labels.size == 150 and set(labels) == {0.0, 1.0, 2.0}


def test_edge_cases_match_restatement():
    from cycloneml_amd import mlutils
    text = ("# comment\n\n   \n1.5 3:2.5  7:-1e-3\t\r\n"
            "0\n-2 1:NaN 2:Infinity 4:-Infinity\n  +3 10:0x1.8p1 11:1d 12:2.5f\n")
    got = mlutils.parseLibSVM(text)
    labels, (rp, ci, v), nf = got
    assert list(labels) == [1.5, 0.0, -2.0, 3.0] and list(rp) == [0, 2, 2, 5, 8] and nf == 12
    assert np.isnan(v[2]) and v[3] == np.inf and v[4] == -np.inf and v[5] == 3.0
    ref = oracle.parse_libsvm(text.replace("NaN", "nan").replace("Infinity", "inf")
                              .replace("0x1.8p1", "3.0").replace("1d", "1").replace("2.5f", "2.5"))
    assert np.array_equal(ref[0], labels) and np.array_equal(ref[1][1], ci)
    # explicit numFeatures and an empty input
    assert mlutils.parseLibSVM(text, numFeatures=40)[2] == 40
    l0, (r0, c0, v0), n0 = mlutils.parseLibSVM("")
    assert l0.size == 0 and list(r0) == [0] and c0.size == 0 and n0 == 1


@pytest.mark.parametrize("bad,msg", [
    ("1 3:1 2:1", "indices should be one-based and in ascending order; found current=1, "
                  "previous=2; line=\"1 3:1 2:1\""),
    ("1 2:1 2:3", "found current=1, previous=1"),
    ("1 0:1", "found current=-1, previous=-1"),
    ("x 1:1", "For input string"),
    ("1 a:1", "For input string"),
    ("1 1:inf", "For input string"),
])
def test_errors(bad, msg):
    from cycloneml_amd import _native as N, mlutils
    with pytest.raises(N.IllegalArgumentException, match="requirement failed") as e:
        mlutils.parseLibSVM("0 1:1\n" + bad + "\n")
    assert msg in str(e.value)
    if "ascending" in msg:
        with pytest.raises(ValueError, match="ascending"):
            oracle.parse_libsvm(bad)


def test_parallel_parse_large_text_equals_sequential():
    """> 1 MiB of text takes the multi-threaded path; rows stay in file order."""
    from cycloneml_amd import mlutils
    rng = np.random.default_rng(0)
    lines = []
    for r in range(20000):
        k = int(rng.integers(0, 12))
        cols = np.sort(rng.choice(5000, size=k, replace=False)) + 1
        lines.append(f"{r % 7} " + " ".join(f"{c}:{rng.normal():.17g}" for c in cols))
    text = "\n".join(lines) + "\n"
    assert len(text) > (1 << 20)
    _same(mlutils.parseLibSVM(text, nthreads=8), mlutils.parseLibSVM(text, nthreads=1))
    _same(mlutils.parseLibSVM(text, nthreads=8), oracle.parse_libsvm(text))


@pytest.mark.gpu
def test_kmeans_example_from_file_on_device(cuda):
    """KMeansExample end to end from data/mllib/sample_kmeans_data.txt: the
    file parsed and uploaded as device CSR (loadLibSVMFile), the device Lloyd
    loop from rows 0 and 3, then KMeansModel.predict / computeCost on the same
    device rows: clusters {0,1,2} / {3,4,5}, centers (0.1,..) / (9.1,..),
    per-row costs bit-exact vs the restatement."""
    from cycloneml_amd import mlutils
    from cycloneml_amd.clustering import KMeans, KMeansModel
    path = os.path.join(GOLD, "sample_kmeans_data.txt")
    blk = mlutils.loadLibSVMFile(path, device=cuda)
    assert blk.numFeatures == 3 and blk.size == 6
    labels, csr, _ = oracle.parse_libsvm(open(path).read())
    assert np.array_equal(blk.labels.cpu().numpy(), labels)
    assert np.array_equal(blk.values.cpu().numpy(), csr[2])
    dense = np.zeros((6, 3))
    for r in range(6):
        dense[r, csr[1][csr[0][r]:csr[0][r + 1]]] = csr[2][csr[0][r]:csr[0][r + 1]]
    km = KMeans(k=2, maxIterations=20, epsilon=1e-4).setInitialModel(KMeansModel(dense[[0, 3]]))
    model = km.run_csr(blk.rowptr, blk.colidx, blk.values, blk.numFeatures)
    np.testing.assert_allclose(sorted(model.clusterCenters.tolist()),
                               [[0.1, 0.1, 0.1], [9.1, 9.1, 9.1]], atol=1e-12)
    p = model.predict_csr(blk.rowptr, blk.colidx, blk.values).cpu().numpy()
    assert p[0] == p[1] == p[2] and p[3] == p[4] == p[5] and p[0] != p[3]
    C = model.clusterCenters
    _, want, s = oracle.point_costs_sparse(csr, oracle.row_norms_csr(csr[0], csr[2]), C,
                                           oracle.row_norms(C))
    _, got = model.pointCosts_csr(blk.rowptr, blk.colidx, blk.values)
    assert np.array_equal(got.cpu().numpy(), want)
    assert model.computeCost_csr(blk.rowptr, blk.colidx, blk.values) == pytest.approx(s,
                                                                                      rel=1e-12)


@pytest.mark.gpu
def test_libsvm_binary_lr_on_device(cuda):
    """sample_libsvm_data.txt (100 x 692, the reference's LR example input) as a
    device CSR block through BinaryLogisticBlockAggregator vs the restatement."""
    from cycloneml_amd import mlutils
    from cycloneml_amd.optim import BinaryLogisticBlockAggregator
    path = os.path.join(GOLD, "sample_libsvm_data.txt")
    blk = mlutils.loadLibSVMFile(path, device=cuda)
    labels, csr, F = oracle.parse_libsvm(open(path).read())
    coef = np.random.default_rng(1).normal(size=F + 1) * 1e-3
    st = dict(grad=np.zeros(F + 1), loss=0.0, weight=0.0)
    oracle.binary_logistic_add(dict(labels=labels, weights=None, rowptr=csr[0], colidx=csr[1],
                                    values=csr[2], F=F), coef, True, False, None, st)
    agg = BinaryLogisticBlockAggregator(np.ones(F), None, True, False, coef, device=cuda).add(blk)
    g = agg.gradientSumArray.cpu().numpy()
    np.testing.assert_allclose(g, st["grad"], rtol=1e-10, atol=1e-10 * np.abs(st["grad"]).max())
    assert float(agg._loss_sum.item()) == pytest.approx(st["loss"], rel=1e-10)


@pytest.mark.parametrize("bad,msg", [
    ("1 3", 'For input string: "3" (index)'),          # no ':' (the reference: split(':')(1))
    ("1 3:", 'For input string: "" (value)'),
    ("1 :3", 'For input string: "" (index)'),
    ("1 1: 2", 'For input string: "" (value)'),
    ("1 99999999999:1", 'For input string: "99999999999" (index)'),   # past Int
    ("1 2147483648:1", 'For input string: "2147483648" (index)'),
    ("1 -5:1", "found current=-6, previous=-1"),
    ("1 1:-0x", 'For input string: "-0x" (value)'),
])
def test_malformed_lines(bad, msg):
    """parseLibSVMRecord's failures on malformed items (MLUtils.scala:129-151:
    item.split(':'), toInt, toDouble, the ascending-index require) come back
    as the reference's exception text; nothing reads past the line."""
    from cycloneml_amd import _native as N, mlutils
    with pytest.raises(N.IllegalArgumentException, match="requirement failed") as e:
        mlutils.parseLibSVM("0 1:1\n" + bad + "\n2 1:3\n")
    assert msg in str(e.value)


def test_overlong_numbers_and_extra_fields():
    """Java's toDouble of a decimal beyond the double range is Infinity (not an
    error), a 5,000-digit mantissa included; an item "1:1:2" keeps fields 0
    and 1 (split(':')); a 400-digit label parses as well."""
    from cycloneml_amd import mlutils
    text = ("1 1:1e999\n1 1:" + "1" * 5000 + "\n1 1:1:2\n1" + "0" * 400 + " 1:1\n"
            "1 1:1  2:2 \n")
    labels, (rp, ci, v), nf = mlutils.parseLibSVM(text)
    assert list(rp) == [0, 1, 2, 3, 4, 6] and nf == 2
    assert v[0] == np.inf and v[1] == np.inf and v[2] == 1.0 and np.isinf(labels[3])
    assert list(ci) == [0, 0, 0, 0, 0, 1]


def test_garbage_never_crashes():
    """Random bytes (digits, ':', signs, exponents, whitespace, NUL and
    non-ASCII) line by line: every line either parses or raises the
    reference's IllegalArgumentException -- the parser stays inside its
    buffer (tools/asan_cpu.sh runs this under AddressSanitizer)."""
    from cycloneml_amd import _native as N, mlutils
    rng = np.random.default_rng(7)
    alphabet = np.frombuffer(b"0123456789:: +-.eE\tabxX\x00\xff\r9", dtype=np.uint8)
    ok = bad = 0
    for i in range(3000):
        line = bytes(rng.choice(alphabet, size=int(rng.integers(0, 40)))).replace(b"\n", b" ")
        try:
            mlutils.parseLibSVM(b"0 1:1\n" + line + b"\n", nthreads=1 + i % 3)
            ok += 1
        except N.IllegalArgumentException:
            bad += 1
    assert ok + bad == 3000 and bad > 0
