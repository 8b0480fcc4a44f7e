"""GPU parity: logistic block aggregators (binary dense / CSR, multinomial
dense) vs the CPU restatement, through the C ABI.  Bar: fp64 gradient and
loss within 1e-10 relative (north_star)."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


def _rel_close(got, ref, rtol=1e-10):
    got, ref = np.asarray(got), np.asarray(ref)
    scale = max(np.abs(ref).max(), 1e-300)
    np.testing.assert_allclose(got, ref, rtol=rtol, atol=rtol * scale)


def _make(n, F, sparse, rng, classes=2, nnz=None, weighted=True, zero_w=False):
    if sparse:
        nnz = nnz or max(1, F // 8)
        rp = [0]
        ci, vv = [], []
        for _ in range(n):
            k = int(rng.integers(0, min(F, 2 * nnz) + 1))
            cols = np.sort(rng.choice(F, size=k, replace=False))
            ci += list(cols)
            vv += list(rng.uniform(-1, 1, size=k))
            rp.append(len(ci))
        csr = (np.array(rp, dtype=np.int64), np.array(ci, dtype=np.int32), np.array(vv))
        X = None
    else:
        X = rng.normal(size=(n, F))
        csr = None
    labels = rng.integers(0, classes, size=n).astype(np.float64)
    w = rng.uniform(0.1, 2.0, size=n) if weighted else None
    if zero_w and w is not None:
        w[::7] = 0.0
    return X, csr, labels, w


def _oracle_block(X, csr, labels, w, F):
    if csr is not None:
        return dict(labels=labels, weights=w, rowptr=csr[0], colidx=csr[1], values=csr[2], F=F)
    return dict(labels=labels, weights=w, X=X)


@pytest.mark.parametrize("sparse", [False, True, "csc", "tiles"])
@pytest.mark.parametrize("fi,fwm", [(False, False), (True, False), (True, True)])
@pytest.mark.parametrize("n,F", [(1, 3), (257, 17), (3000, 64), (2000, 300)])
def test_binary_vs_oracle(cuda, sparse, fi, fwm, n, F):
    from cycloneml_amd.optim import BinaryLogisticBlockAggregator, DeviceInstanceBlock
    rng = np.random.default_rng(n * 7 + F + bool(sparse))
    X, csr, labels, w = _make(n, F, bool(sparse), rng, zero_w=True)
    coef = rng.normal(size=F + (1 if fi else 0)) * 0.5
    sm = rng.normal(size=F) * 0.1 if fwm else None
    st = dict(grad=np.zeros(coef.size), loss=0.0, weight=0.0)
    oracle.binary_logistic_add(_oracle_block(X, csr, labels, w, F), coef, fi, fwm, sm, st)
    blk = DeviceInstanceBlock.from_numpy(labels, w, X=X, csr=csr, numFeatures=F, device=cuda)
    if sparse in ("csc", "tiles"):
        blk.prepare(layout=sparse)
    agg = BinaryLogisticBlockAggregator(np.ones(F), sm, fi, fwm, coef, device=cuda).add(blk)
    _rel_close(agg.gradientSumArray.cpu().numpy(), st["grad"])
    assert abs(agg.weight - st["weight"]) <= 1e-12 * st["weight"]
    assert abs(float(agg._loss_sum.item()) - st["loss"]) <= 1e-10 * abs(st["loss"])


@pytest.mark.parametrize("fi,fwm", [(False, False), (True, False), (True, True)])
@pytest.mark.parametrize("n,F,C", [(1, 2, 3), (300, 5, 3), (2000, 64, 10), (1500, 100, 17),
                                   (5000, 512, 100), (700, 33, 128),
                                   # several 256-row tiles per workgroup: the DMA
                                   # ring and label slots across tile boundaries
                                   (200_003, 5, 3), (140_000, 16, 10), (70_001, 40, 17)])
def test_multinomial_vs_oracle(cuda, fi, fwm, n, F, C):
    from cycloneml_amd.optim import DeviceInstanceBlock, MultinomialLogisticBlockAggregator
    rng = np.random.default_rng(n + F * 3 + C)
    X, _, labels, w = _make(n, F, False, rng, classes=C, zero_w=True)
    coef = rng.normal(size=C * F + (C if fi else 0)) * (1.0 / np.sqrt(F))
    sm = rng.normal(size=F) * 0.1 if fwm else None
    st = dict(grad=np.zeros(coef.size), loss=0.0, weight=0.0)
    oracle.multinomial_logistic_add(dict(labels=labels, weights=w, X=X), coef, C, fi, fwm, sm, st)
    blk = DeviceInstanceBlock.from_numpy(labels, w, X=X, device=cuda)
    agg = MultinomialLogisticBlockAggregator(np.ones(F), sm, fi, fwm, coef, device=cuda).add(blk)
    _rel_close(agg.gradientSumArray.cpu().numpy(), st["grad"])
    assert abs(agg.weight - st["weight"]) <= 1e-12 * st["weight"]
    assert abs(float(agg._loss_sum.item()) - st["loss"]) <= 1e-10 * abs(st["loss"])


@pytest.mark.parametrize("fi,fwm", [(False, False), (True, False), (True, True)])
@pytest.mark.parametrize("n,F,C", [(1, 3, 2), (300, 20, 3), (2000, 64, 10), (1500, 300, 100),
                                   (600, 50, 130)])
def test_multinomial_csr_vs_oracle(cuda, fi, fwm, n, F, C):
    """Sparse InstanceBlocks through the multinomial aggregator (:122 sparse
    gemm, :156-162 sparse gradient): margins by row, gradient over the CSC copy."""
    from cycloneml_amd.optim import DeviceInstanceBlock, MultinomialLogisticBlockAggregator
    rng = np.random.default_rng(n + F * 5 + C)
    _, csr, labels, w = _make(n, F, True, rng, classes=C, zero_w=True)
    coef = rng.normal(size=C * F + (C if fi else 0)) * (1.0 / np.sqrt(F))
    sm = rng.normal(size=F) * 0.1 if fwm else None
    st = dict(grad=np.zeros(coef.size), loss=0.0, weight=0.0)
    oracle.multinomial_logistic_add(_oracle_block(None, csr, labels, w, F), coef, C, fi, fwm, sm,
                                    st)
    blk = DeviceInstanceBlock.from_numpy(labels, w, csr=csr, numFeatures=F, device=cuda)
    agg = MultinomialLogisticBlockAggregator(np.ones(F), sm, fi, fwm, coef, device=cuda).add(blk)
    _rel_close(agg.gradientSumArray.cpu().numpy(), st["grad"])
    assert abs(agg.weight - st["weight"]) <= 1e-12 * max(st["weight"], 1e-300)
    assert abs(float(agg._loss_sum.item()) - st["loss"]) <= 1e-10 * max(abs(st["loss"]), 1e-300)


def test_aggregator_requires(cuda):
    from cycloneml_amd import _native as N
    from cycloneml_amd.optim import BinaryLogisticBlockAggregator, DeviceInstanceBlock
    with pytest.raises(N.IllegalArgumentException, match="should not center"):
        BinaryLogisticBlockAggregator(np.ones(2), np.zeros(2), False, True, np.ones(2),
                                      device=cuda)
    agg = BinaryLogisticBlockAggregator(np.ones(2), np.zeros(2), True, True, np.ones(3),
                                        device=cuda)
    blk = DeviceInstanceBlock.from_numpy(np.ones(1), np.ones(1), X=np.ones((1, 1)), device=cuda)
    with pytest.raises(N.IllegalArgumentException, match="Dimensions mismatch"):
        agg.add(blk)
    blk = DeviceInstanceBlock.from_numpy(np.ones(1), -np.ones(1), X=np.ones((1, 2)), device=cuda)
    with pytest.raises(N.IllegalArgumentException, match="has to be >= 0.0"):
        agg.add(blk)
    with pytest.raises(N.IllegalArgumentException, match="effective number"):
        BinaryLogisticBlockAggregator(np.ones(2), None, False, False, np.ones(2),
                                      device=cuda).gradient


def test_rdd_loss_function(cuda):
    from cycloneml_amd.optim import (BinaryLogisticBlockAggregator, DeviceInstanceBlock,
                                     L2Regularization, RDDLossFunction)
    rng = np.random.default_rng(5)
    F = 20
    X, _, labels, w = _make(1000, F, False, rng)
    blocks = [DeviceInstanceBlock.from_numpy(labels[:400], w[:400], X=X[:400], device=cuda),
              DeviceInstanceBlock.from_numpy(labels[400:], w[400:], X=X[400:], device=cuda)]
    coef = rng.normal(size=F + 1)
    fn = RDDLossFunction(blocks, lambda c: BinaryLogisticBlockAggregator(
        np.ones(F), None, True, False, c, device=cuda),
        L2Regularization(0.1, lambda j: j < F))
    loss, grad = fn.calculate(coef)
    st = dict(grad=np.zeros(F + 1), loss=0.0, weight=0.0)
    oracle.binary_logistic_add(dict(labels=labels, weights=w, X=X), coef, True, False, None, st)
    reg = 0.5 * 0.1 * (coef[:F] ** 2).sum()
    assert abs(loss - (st["loss"] / st["weight"] + reg)) <= 1e-10 * abs(loss)
    exp = st["grad"] / st["weight"]
    exp[:F] += 0.1 * coef[:F]
    _rel_close(grad, exp)


def _config5_rows(n, F, k, seed, cuda):
    """BASELINE configs[4] row shape (bench.py's generator): k distinct
    sorted columns per row, one per F/k band, values U(0, 1)."""
    import torch
    g = torch.Generator(device=cuda).manual_seed(seed)
    band = F // k
    cols = torch.empty(n * k, dtype=torch.int32, device=cuda)
    vals = torch.empty(n * k, dtype=torch.float64, device=cuda)
    step = 1 << 20
    for s in range(0, n, step):
        e = min(n, s + step)
        c = (torch.arange(k, device=cuda) * band).unsqueeze(0) + \
            torch.randint(0, band, (e - s, k), generator=g, device=cuda)
        cols[s * k:e * k] = c.to(torch.int32).reshape(-1)
        vals[s * k:e * k] = torch.rand((e - s) * k, generator=g, device=cuda, dtype=torch.float64)
    rowptr = torch.arange(0, n * k + 1, k, device=cuda, dtype=torch.int64)
    labels = (torch.rand(n, generator=g, device=cuda) < 0.5).to(torch.float64)
    return rowptr, cols, vals, labels


def test_sparse_config5_csc_path(cuda):
    """Config 5 row shape on a 1M-row shard through the CSR + CSC path: a row
    subset equals the oracle, the CSC gradient equals the atomic one within
    1e-10 and is bitwise reproducible."""
    from cycloneml_amd.optim import BinaryLogisticBlockAggregator, DeviceInstanceBlock
    import torch
    n, F, k = 1_000_000, 1_000_000, 64
    rowptr, cols, vals, labels = _config5_rows(n, F, k, 2, cuda)
    coef = torch.randn(F + 1, generator=torch.Generator(device=cuda).manual_seed(3), device=cuda,
                       dtype=torch.float64) * 0.01
    sm = np.random.default_rng(4).uniform(0, 1, F) * 0.5
    blk = DeviceInstanceBlock(labels, None, rowptr=rowptr, colidx=cols, values=vals,
                              numFeatures=F)
    agg = BinaryLogisticBlockAggregator(np.ones(F), sm, True, True, coef, device=cuda).add(blk)
    blk.prepare()
    a3 = BinaryLogisticBlockAggregator(np.ones(F), sm, True, True, coef, device=cuda).add(blk)
    a4 = BinaryLogisticBlockAggregator(np.ones(F), sm, True, True, coef, device=cuda).add(blk)
    g3 = a3.gradientSumArray.cpu().numpy()
    _rel_close(g3, agg.gradientSumArray.cpu().numpy(), rtol=1e-10)
    assert np.array_equal(g3, a4.gradientSumArray.cpu().numpy())
    m = 20000
    st = dict(grad=np.zeros(F + 1), loss=0.0, weight=0.0)
    oracle.binary_logistic_add(dict(labels=labels[:m].cpu().numpy(), weights=None,
                                    rowptr=rowptr[:m + 1].cpu().numpy(),
                                    colidx=cols[:m * k].cpu().numpy(),
                                    values=vals[:m * k].cpu().numpy(), F=F),
                               coef.cpu().numpy(), True, True, sm, st)
    sub = DeviceInstanceBlock(labels[:m], None, rowptr=rowptr[:m + 1], colidx=cols[:m * k],
                              values=vals[:m * k], numFeatures=F).prepare()
    a5 = BinaryLogisticBlockAggregator(np.ones(F), sm, True, True, coef, device=cuda).add(sub)
    _rel_close(a5.gradientSumArray.cpu().numpy(), st["grad"])


@pytest.mark.timeout(900)
def test_sparse_config5_full_size(cuda):
    """BASELINE config 5 at the size bench.py times, on the rows it times:
    200M rows x 1M features, 64 nonzeros per row (12.8G nonzeros, past 2^32,
    154 GB of tiles layout), generated by bench.lr_sparse_chunks and appended
    chunk by chunk with the CSR freed, fitIntercept => fitWithMean with the
    bench's synthetic scaledMean, U(0, 0.014) per feature -- the scale of
    mean / std for these rows, not computed from them
    (BinaryLogisticBlockAggregator.scala:81-145).  Checks:
    (1) bitwise reproducible; (2) the layout's FIRST and LAST 40,000 rows --
    the last ones at nonzero offsets above 2^32 -- equal the restatement
    within 1e-10, selected inside the full 200M-row layout by a weight mask
    (zero-weight rows add nothing, :107-125); (3) linearity: the whole
    layout's state equals the sum of two unequal parts' (120M + 80M rows,
    rebuilt from the same seeds) within 1e-12."""
    import os
    import sys
    import torch
    from cycloneml_amd.optim import (BinaryLogisticBlockAggregator, DeviceInstanceBlock,
                                     SparseTiles)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from conftest import heartbeat
    n, F, k = 200_000_000, 1_000_000, 64
    sub_m = 40_000
    coef = np.random.default_rng(4).normal(size=F + 1) * 0.01
    sm = np.random.default_rng(5).uniform(0.0, 0.014, F)
    sm_dev = torch.as_tensor(sm, device=cuda)

    def run(t, lab, w=None):
        blk = DeviceInstanceBlock(lab, w, tiles=t, numFeatures=F)
        return BinaryLogisticBlockAggregator(np.ones(F), sm_dev, True, True, coef,
                                             device=cuda).add(blk)._state.cpu().numpy()

    def host_rows(rp, ci, vv, lb, lo, hi):
        a, b = int(rp[lo]), int(rp[hi])
        return ((rp[lo:hi + 1] - a).cpu().numpy(), ci[a:b].cpu().numpy(),
                vv[a:b].cpu().numpy(), lb[lo:hi].cpu().numpy())

    whole = SparseTiles(F, n, n * k)
    labels = torch.empty(n, dtype=torch.float64, device=cuda)
    head = tail = None
    for s, e, rp, ci, vv, yc in bench.lr_sparse_chunks(n, cuda, 0, F, k):
        labels[s:e] = yc
        whole.append(rp, ci, vv)
        if s == 0:
            head = host_rows(rp, ci, vv, yc, 0, sub_m)
        if e == n:
            tail = host_rows(rp, ci, vv, yc, e - s - sub_m, e - s)
        if s % (64 * bench.LR_SPARSE_CHUNK) == 0:
            heartbeat(f"config5 whole layout: {e} rows")
        del rp, ci, vv, yc
    assert whole.rows == n and whole.nnz == n * k and whole.nnz > 2 ** 32
    full = run(whole, labels)
    assert np.array_equal(full, run(whole, labels))
    assert full[F + 2] == n
    for lo, rows in ((0, head), (n - sub_m, tail)):
        w = torch.zeros(n, dtype=torch.float64, device=cuda)
        w[lo:lo + sub_m] = 1.0
        got = run(whole, labels, w)
        del w
        rp, ci, vv, lb = rows
        st = dict(grad=np.zeros(F + 1), loss=0.0, weight=0.0)
        oracle.binary_logistic_add(dict(labels=lb, weights=None, rowptr=rp, colidx=ci,
                                        values=vv, F=F), coef, True, True, sm, st)
        _rel_close(got[:F + 1], st["grad"])
        assert abs(got[F + 1] - st["loss"]) <= 1e-10 * abs(st["loss"])
        assert got[F + 2] == sub_m
        heartbeat(f"config5 rows {lo}.. vs the restatement: ok")
    del whole
    torch.cuda.empty_cache()
    cut = 229 * bench.LR_SPARSE_CHUNK                  # 120,061,952 rows: unequal parts
    h1, h2 = SparseTiles(F, cut, cut * k), SparseTiles(F, n - cut, (n - cut) * k)
    for s, e, rp, ci, vv, yc in bench.lr_sparse_chunks(n, cuda, 0, F, k):
        assert torch.equal(yc, labels[s:e])            # the same rows again
        (h1 if s < cut else h2).append(rp, ci, vv)
        if s % (64 * bench.LR_SPARSE_CHUNK) == 0:
            heartbeat(f"config5 parts: {e} rows")
        del rp, ci, vv, yc
    parts = run(h1, labels[:cut]) + run(h2, labels[cut:])
    _rel_close(full, parts, rtol=1e-12)


@pytest.mark.parametrize("fmt", ["wide", "compact"])
@pytest.mark.parametrize("fi,fwm", [(True, False), (True, True), (False, False)])
@pytest.mark.parametrize("n,F,nnz", [(700, 600_000, 40), (300, 1_100_000, 150), (50, 300_000, 1),
                                     (20_000, 30_000, 25), (9000, 8192, 300),
                                     (40_000, 1_000_000, 64), (5000, 100, 10), (3000, 3, 2)])
def test_binary_tiles_vs_oracle(cuda, fmt, fi, fwm, n, F, nnz):
    """The row-block x column-chunk layout: many column chunks (F up to 1.1M
    = 538 chunks of 2048, 68 gradient workgroups of 8 chunks), several row
    blocks and super blocks (40000 rows = 20 row blocks of 2048 = 3 margin
    super blocks of 8), empty rows, zero weights, rows spanning every chunk,
    long runs (9000 rows of ~300 nonzeros over 8 chunks: the batched tail
    path), and narrow F (100 and 3 columns: chunks of 64, most waves without
    a chunk); in both entry formats (wide: 32-bit ids; compact: 16-bit
    column + row step, filler entries for the rows' gaps of 31 or more --
    most of these shapes need fillers); equals the restatement
    within 1e-10, the loss bit for bit-ish (same summation order), and is
    bitwise reproducible run to run."""
    from cycloneml_amd.optim import BinaryLogisticBlockAggregator, DeviceInstanceBlock
    rng = np.random.default_rng(n + F // 1000 + nnz)
    X, csr, labels, w = _make(n, F, True, rng, nnz=nnz, zero_w=True)
    coef = rng.normal(size=F + (1 if fi else 0)) * 0.5
    sm = rng.normal(size=F) * 0.1 if fwm else None
    st = dict(grad=np.zeros(coef.size), loss=0.0, weight=0.0)
    oracle.binary_logistic_add(_oracle_block(X, csr, labels, w, F), coef, fi, fwm, sm, st)
    blk = DeviceInstanceBlock.from_numpy(labels, w, X=None, csr=csr, numFeatures=F, device=cuda)
    blk.prepare(layout="tiles", tiles_format=fmt).release_csr()
    assert blk.tiles.rows == n and blk.tiles.nnz == csr[1].size and blk.tiles.format == fmt
    assert (blk.tiles.entries == blk.tiles.nnz) == (fmt == "wide" or blk.tiles.entries == 0 or
                                                   blk.tiles.entries == blk.tiles.nnz)
    agg = BinaryLogisticBlockAggregator(np.ones(F), sm, fi, fwm, coef, device=cuda).add(blk)
    _rel_close(agg.gradientSumArray.cpu().numpy(), st["grad"])
    assert abs(agg.weight - st["weight"]) <= 1e-12 * st["weight"]
    assert abs(float(agg._loss_sum.item()) - st["loss"]) <= 1e-12 * abs(st["loss"])
    again = BinaryLogisticBlockAggregator(np.ones(F), sm, fi, fwm, coef, device=cuda).add(blk)
    assert np.array_equal(agg._state.cpu().numpy(), again._state.cpu().numpy())


@pytest.mark.parametrize("n,F,nnz", [(40_000, 1_000_000, 64), (9000, 8192, 300), (700, 600_000, 40),
                                     (6000, 50_000, 3)])
def test_tiles_compact_equals_wide(cuda, n, F, nnz):
    """The compact entries hold the same nonzeros in the same order as the
    wide ones (the fillers only move the row), so both passes add the same
    products in the same order: the aggregator state is the same bits in
    both formats, for every aggregator kind the layout serves."""
    import torch
    from cycloneml_amd.optim import (BinaryLogisticBlockAggregator, DeviceInstanceBlock,
                                     HingeBlockAggregator, SparseTiles)
    rng = np.random.default_rng(n + nnz)
    X, csr, labels, w = _make(n, F, True, rng, nnz=nnz, zero_w=True)
    rp, ci, vv = (torch.as_tensor(a, device=cuda) for a in csr)
    lab = torch.as_tensor(labels, device=cuda)
    wt = torch.as_tensor(w, device=cuda)
    coef = rng.normal(size=F + 1) * 0.3
    sm = rng.normal(size=F) * 0.1
    states = []
    for fmt in ("wide", "compact"):
        t = SparseTiles.from_csr(rp, ci, vv, F, format=fmt)
        assert t.format == fmt and t.nnz == ci.numel() and t.entries >= t.nnz
        blk = DeviceInstanceBlock(lab, wt, tiles=t, numFeatures=F)
        b = BinaryLogisticBlockAggregator(np.ones(F), torch.as_tensor(sm, device=cuda), True,
                                          True, coef, device=cuda).add(blk)
        h = HingeBlockAggregator(np.ones(F), torch.as_tensor(sm, device=cuda), True, coef,
                                 device=cuda).add(blk)
        states.append((b._state.cpu().numpy(), h._state.cpu().numpy()))
    assert np.array_equal(states[0][0], states[1][0])
    assert np.array_equal(states[0][1], states[1][1])


def test_tiles_format_choice_and_requires(cuda):
    """CYC_TILES_AUTO: the first append with nonzeros picks compact for dense
    enough segments (config 5's shape: 64 of 1M columns per row) and wide for
    sparse ones (2 nonzeros per row over 1M columns: row gaps of ~500 would
    need ~16 fillers per nonzero); the format is fixed before the first
    append only; a compact layout whose fillers exceed its allowance fails
    with a message naming the wide format."""
    import torch
    from cycloneml_amd import _native as N
    from cycloneml_amd.optim import SparseTiles
    rng = np.random.default_rng(21)
    X, csr, labels, w = _make(8192, 1_000_000, True, rng, nnz=64)
    rp, ci, vv = (torch.as_tensor(a, device=cuda) for a in csr)
    t = SparseTiles(1_000_000, 8192, ci.numel())
    assert t.format == "auto"
    t.append(rp, ci, vv)
    assert t.format == "compact" and t.nnz == ci.numel() and t.nnz < t.entries < 1.05 * t.nnz
    with pytest.raises(N.IllegalArgumentException, match="before the first append"):
        N.check(t._lib.cyc_tiles_set_format(t.handle, 1))
    X, csr, labels, w = _make(4096, 1_000_000, True, rng, nnz=2)
    rp, ci, vv = (torch.as_tensor(a, device=cuda) for a in csr)
    t = SparseTiles.from_csr(rp, ci, vv, 1_000_000)
    assert t.format == "wide" and t.entries == t.nnz
    def every(gap, blocks):
        n = gap * 2048 * blocks                        # a nonzero in every gap-th row
        nz = np.zeros(n, dtype=np.int64)
        nz[::gap] = 1
        rpx = torch.as_tensor(np.concatenate([[0], np.cumsum(nz)]), device=cuda)
        cix = torch.zeros(int(nz.sum()), dtype=torch.int32, device=cuda)
        return n, rpx, cix, torch.ones(cix.numel(), dtype=torch.float64, device=cuda)
    # gaps of 40 rows: one filler per nonzero (~53,000), inside the allowance
    # of 53,248 / 16 + 65,536
    n, rpx, cix, vvx = every(40, 26)
    big = SparseTiles(10, n, cix.numel(), format="compact")
    big.append(rpx, cix, vvx)
    assert 1.9 * big.nnz < big.entries < 2 * big.nnz
    # gaps of 80: two fillers per nonzero, past it
    n, rpx, cix, vvx = every(80, 26)
    over = SparseTiles(10, n, cix.numel(), format="compact")
    with pytest.raises(N.IllegalArgumentException, match="CYC_TILES_WIDE"):
        over.append(rpx, cix, vvx)
    with pytest.raises(ValueError):
        SparseTiles(10, 1, 1, format="narrow")


def test_tiles_appends_and_requires(cuda):
    """Appending whole row blocks in pieces builds the same layout as one
    append; a partial row block seals the layout; SparseVector's index
    requires (ml/linalg/Vectors.scala:617-625) come back with the reference's
    text; capacity and dimension checks."""
    import torch
    from cycloneml_amd import _native as N
    from cycloneml_amd.optim import (BinaryLogisticBlockAggregator, DeviceInstanceBlock,
                                     SparseTiles)
    rng = np.random.default_rng(9)
    n, F = 3 * 8192 + 100, 20_000
    X, csr, labels, w = _make(n, F, True, rng, nnz=12)
    rp, ci, vv = (torch.as_tensor(a, device=cuda) for a in csr)
    coef = rng.normal(size=F + 1) * 0.3
    one = SparseTiles.from_csr(rp, ci, vv, F)
    parts = SparseTiles(F, n, ci.numel())
    for a, b in [(0, 8192), (8192, 3 * 8192), (3 * 8192, n)]:
        q0, q1 = int(csr[0][a]), int(csr[0][b])    # rowptr of any base
        parts.append(rp[a:b + 1], ci[q0:q1], vv[q0:q1])
    with pytest.raises(N.IllegalArgumentException, match="partial row block"):
        parts.append(rp[:2], ci, vv)
    lab = torch.as_tensor(labels, device=cuda)
    res = []
    for t in (one, parts):
        blk = DeviceInstanceBlock(lab, None, tiles=t, numFeatures=F)
        res.append(BinaryLogisticBlockAggregator(np.ones(F), None, True, False, coef,
                                                 device=cuda).add(blk)._state.cpu().numpy())
    assert np.array_equal(res[0], res[1])

    def bad(rows, msg):
        rpb = torch.as_tensor(np.array([0] + list(np.cumsum([len(r) for r in rows])),
                                       dtype=np.int64), device=cuda)
        cib = torch.as_tensor(np.array(sum(rows, []), dtype=np.int32), device=cuda)
        vvb = torch.ones(cib.numel(), dtype=torch.float64, device=cuda)
        with pytest.raises(N.IllegalArgumentException) as e:
            SparseTiles.from_csr(rpb, cib, vvb, 10)
        assert str(e.value) == "requirement failed: " + msg
    bad([[0, 1], [2, -1, 3]], "Index -1 follows 2 and is not strictly increasing")
    bad([[0], [-3, 4]], "Found negative index: -3.")
    bad([[1, 1]], "Index 1 follows 1 and is not strictly increasing")
    bad([[], [3, 9], [2, 10]], "Index 10 out of bounds for vector of size 10")
    with pytest.raises(N.IllegalArgumentException, match="exceeds the capacity"):
        SparseTiles(F, 10, 1000).append(rp[:12], ci, vv)
    blk = DeviceInstanceBlock(lab, None, tiles=one, numFeatures=F)
    with pytest.raises(N.IllegalArgumentException, match="Dimensions mismatch"):
        BinaryLogisticBlockAggregator(np.ones(F + 1), None, True, False, np.zeros(F + 2),
                                      device=cuda).add(blk)


@pytest.mark.parametrize("sparse", [False, True, "csc", "tiles"])
@pytest.mark.parametrize("fi", [False, True])
@pytest.mark.parametrize("n,F", [(1, 3), (257, 17), (3000, 64), (2000, 300)])
def test_hinge_vs_oracle(cuda, sparse, fi, n, F):
    """HingeBlockAggregator (LinearSVC) on the binary kernels
    with the hinge epilogue vs the restatement (orc_hinge_add), 1e-10."""
    from cycloneml_amd.optim import DeviceInstanceBlock, HingeBlockAggregator
    rng = np.random.default_rng(n * 11 + F + bool(sparse))
    X, csr, labels, w = _make(n, F, bool(sparse), rng, zero_w=True)
    coef = rng.normal(size=F + (1 if fi else 0)) * 0.5
    sm = rng.normal(size=F) * 0.1 if fi else None
    st = dict(grad=np.zeros(coef.size), loss=0.0, weight=0.0)
    oracle.hinge_add(_oracle_block(X, csr, labels, w, F), coef, fi, sm, st)
    blk = DeviceInstanceBlock.from_numpy(labels, w, X=X, csr=csr, numFeatures=F, device=cuda)
    if sparse in ("csc", "tiles"):
        blk.prepare(layout=sparse)
    agg = HingeBlockAggregator(np.ones(F), sm, fi, coef, device=cuda).add(blk)
    _rel_close(agg.gradientSumArray.cpu().numpy(), st["grad"])
    assert abs(agg.weight - st["weight"]) <= 1e-12 * st["weight"]
    assert abs(float(agg._loss_sum.item()) - st["loss"]) <= 1e-10 * max(abs(st["loss"]), 1e-300)


def test_hinge_tiles_large_f_and_plan_kinds(cuda):
    """numFeatures = 600K (74 column tiles) with the hinge epilogue; a hinge
    plan refuses the logistic entry point and vice versa."""
    import ctypes
    from cycloneml_amd import _native as N
    from cycloneml_amd.optim import DeviceInstanceBlock, HingeBlockAggregator
    rng = np.random.default_rng(5)
    n, F = 500, 600_000
    X, csr, labels, w = _make(n, F, True, rng, nnz=30, zero_w=True)
    coef = rng.normal(size=F + 1) * 0.5
    sm = rng.normal(size=F) * 0.1
    st = dict(grad=np.zeros(coef.size), loss=0.0, weight=0.0)
    oracle.hinge_add(_oracle_block(X, csr, labels, w, F), coef, True, sm, st)
    blk = DeviceInstanceBlock.from_numpy(labels, w, X=None, csr=csr, numFeatures=F, device=cuda)
    blk.prepare(layout="tiles")
    agg = HingeBlockAggregator(np.ones(F), sm, True, coef, device=cuda).add(blk)
    _rel_close(agg.gradientSumArray.cpu().numpy(), st["grad"])
    assert abs(float(agg._loss_sum.item()) - st["loss"]) <= 1e-10 * abs(st["loss"])
    lib = N.load()
    h = ctypes.c_void_p()
    N.check(lib.cyc_hinge_plan_create(4, 0, ctypes.byref(h)))
    rc = lib.cyc_binary_logistic_add_dense_dev(h, None, None, None, 1, None, None, None, None,
                                               None, None)
    assert rc != 0 and b"not a binary logistic plan" in lib.cyc_last_error()
    lib.cyc_logistic_plan_destroy(h)


@pytest.mark.parametrize("sparse", [False, True, "csc", "tiles"])
@pytest.mark.parametrize("fi", [False, True])
@pytest.mark.parametrize("n,F", [(1, 3), (257, 17), (3000, 64), (2000, 300)])
def test_least_squares_vs_oracle(cuda, sparse, fi, n, F):
    """LeastSquaresBlockAggregator (LinearRegression) on the binary
    kernels with the squared-error epilogue vs the restatement, 1e-10; one
    constant feature (inverseStd 0) exercises effectiveCoef."""
    from cycloneml_amd.optim import DeviceInstanceBlock, LeastSquaresBlockAggregator
    rng = np.random.default_rng(n * 13 + F + bool(sparse))
    X, csr, _, w = _make(n, F, bool(sparse), rng, zero_w=True)
    labels = rng.normal(size=n) * 2.0 + 0.5
    coef = rng.normal(size=F) * 0.5
    inv = rng.uniform(0.5, 2.0, size=F)
    inv[F // 2] = 0.0
    sm = rng.normal(size=F) * 0.1 if fi else None
    ystd, ymean = 1.7, 0.3
    st = dict(grad=np.zeros(F), loss=0.0, weight=0.0)
    oracle.least_squares_add(_oracle_block(X, csr, labels, w, F), coef, inv, fi, ystd, ymean, sm,
                             st)
    blk = DeviceInstanceBlock.from_numpy(labels, w, X=X, csr=csr, numFeatures=F, device=cuda)
    if sparse in ("csc", "tiles"):
        blk.prepare(layout=sparse)
    agg = LeastSquaresBlockAggregator(inv, sm, fi, ystd, ymean, coef, device=cuda).add(blk)
    _rel_close(agg.gradientSumArray.cpu().numpy(), st["grad"])
    assert abs(agg.weight - st["weight"]) <= 1e-12 * st["weight"]
    assert abs(float(agg._loss_sum.item()) - st["loss"]) <= 1e-10 * abs(st["loss"])


def test_least_squares_requires(cuda):
    from cycloneml_amd import _native as N
    from cycloneml_amd.optim import LeastSquaresBlockAggregator
    with pytest.raises(N.IllegalArgumentException, match="label standard"):
        LeastSquaresBlockAggregator(np.ones(3), None, False, 0.0, 0.0, np.zeros(3), device=cuda)


@pytest.mark.parametrize("sparse", [False, True, "csc", "tiles"])
@pytest.mark.parametrize("fi", [False, True])
@pytest.mark.parametrize("n,F", [(1, 3), (257, 17), (3000, 64), (2000, 300)])
def test_huber_vs_oracle(cuda, sparse, fi, n, F):
    """HuberBlockAggregator (LinearRegression loss "huber") on the
    binary kernels with the Huber epilogue vs the restatement, 1e-10; sigma
    chosen so both the quadratic and the linear branch occur."""
    from cycloneml_amd.optim import DeviceInstanceBlock, HuberBlockAggregator
    rng = np.random.default_rng(n * 17 + F + bool(sparse))
    X, csr, _, w = _make(n, F, bool(sparse), rng, zero_w=True)
    labels = rng.normal(size=n) * 2.0
    params = np.concatenate([rng.normal(size=F) * 0.3, [0.4] if fi else [], [0.9]])
    sm = rng.normal(size=F) * 0.1 if fi else None
    st = dict(grad=np.zeros(params.size), loss=0.0, weight=0.0)
    oracle.huber_add(_oracle_block(X, csr, labels, w, F), params, fi, 1.35, sm, st)
    blk = DeviceInstanceBlock.from_numpy(labels, w, X=X, csr=csr, numFeatures=F, device=cuda)
    if sparse in ("csc", "tiles"):
        blk.prepare(layout=sparse)
    agg = HuberBlockAggregator(np.ones(F), sm, fi, 1.35, params, device=cuda).add(blk)
    _rel_close(agg.gradientSumArray.cpu().numpy(), st["grad"])
    assert abs(agg.weight - st["weight"]) <= 1e-12 * st["weight"]
    assert abs(float(agg._loss_sum.item()) - st["loss"]) <= 1e-10 * abs(st["loss"])


@pytest.mark.parametrize("sparse", [False, True, "csc", "tiles"])
@pytest.mark.parametrize("fi", [False, True])
@pytest.mark.parametrize("n,F", [(1, 3), (257, 17), (3000, 64), (2000, 300)])
def test_aft_vs_oracle(cuda, sparse, fi, n, F):
    """AFTBlockAggregator (AFTSurvivalRegression) on the binary
    kernels with the survival epilogue vs the restatement, 1e-10; censors in
    the weights slot, as the reference keeps them."""
    from cycloneml_amd.optim import AFTBlockAggregator, DeviceInstanceBlock
    rng = np.random.default_rng(n * 19 + F + bool(sparse))
    X, csr, _, _ = _make(n, F, bool(sparse), rng)
    labels = rng.exponential(2.0, size=n) + 1e-3
    cens = (rng.uniform(size=n) < 0.6).astype(np.float64)
    coef = np.concatenate([rng.normal(size=F) * 0.1, [0.3 if fi else 0.0], [0.2]])
    sm = rng.normal(size=F) * 0.1 if fi else None
    st = dict(grad=np.zeros(coef.size), loss=0.0, weight=0.0)
    oracle.aft_add(_oracle_block(X, csr, labels, cens, F), coef, fi, sm, st)
    blk = DeviceInstanceBlock.from_numpy(labels, cens, X=X, csr=csr, numFeatures=F, device=cuda)
    if sparse in ("csc", "tiles"):
        blk.prepare(layout=sparse)
    agg = AFTBlockAggregator(sm, fi, coef, device=cuda).add(blk)
    _rel_close(agg.gradientSumArray.cpu().numpy(), st["grad"])
    assert agg.weight == st["weight"] == n
    assert abs(float(agg._loss_sum.item()) - st["loss"]) <= 1e-10 * abs(st["loss"])


def test_aft_requires_positive_labels(cuda):
    from cycloneml_amd import _native as N
    from cycloneml_amd.optim import AFTBlockAggregator, DeviceInstanceBlock
    blk = DeviceInstanceBlock.from_numpy(np.array([1.0, 0.0]), None, X=np.ones((2, 2)),
                                         device=cuda)
    with pytest.raises(N.IllegalArgumentException, match="greater than 0"):
        AFTBlockAggregator(None, False, np.zeros(4), device=cuda).add(blk)


@pytest.mark.timeout(600)
def test_multinomial_bench_shard(cuda):
    """bench.py's lr_multi shard at its benched size, on the rows it times
    (bench.lr_multi_data: the full configs[3], 50M x 512, C = 100, labels from
    softmax(X W), fitIntercept + fitWithMean with scaledMean = mean / std as
    the bench sets it; the first rows of the same stream if the device has
    less free memory), with the bench's coefficients: several 8M-row launch
    chunks and the 32-bit buffer-descriptor caps.  The whole shard's state
    equals the sum of two unequal parts' (chunk boundaries differ) within
    1e-11, and the first and the last 5000 rows equal the restatement within
    1e-10."""
    import os
    import sys
    import torch
    from cycloneml_amd.optim import DeviceInstanceBlock, MultinomialLogisticBlockAggregator
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    F, C = 512, 100
    import gc
    gc.collect()
    torch.cuda.empty_cache()
    free, _ = torch.cuda.mem_get_info(cuda)
    n = int(min(50_000_000, (free - (24 << 30)) // (8 * F)))
    X, y, sm_dev = bench.lr_multi_data(n, cuda, 0, F, C)
    sm = sm_dev.cpu().numpy()
    coef = np.random.default_rng(3).normal(size=C * F + C) * 0.01    # bench's coef

    def run(a, b):
        blk = DeviceInstanceBlock(y[a:b], None, X=X[a:b])
        return MultinomialLogisticBlockAggregator(np.ones(F), sm_dev, True, True, coef,
                                                  device=cuda).add(blk)._state.cpu().numpy()
    full = run(0, n)
    cut = 19_000_001
    _rel_close(run(0, cut) + run(cut, n), full, rtol=1e-11)
    m = 5000
    for a in (0, n - m):
        st = dict(grad=np.zeros(coef.size), loss=0.0, weight=0.0)
        oracle.multinomial_logistic_add(dict(labels=y[a:a + m].cpu().numpy(), weights=None,
                                             X=X[a:a + m].cpu().numpy()), coef, C, True, True, sm,
                                        st)
        part = run(a, a + m)
        _rel_close(part[:coef.size], st["grad"])
        assert abs(part[coef.size] - st["loss"]) <= 1e-10 * abs(st["loss"])


def test_softmax_exp_vs_libm(cuda):
    """The softmax exponential of the dense multinomial margins (exp_neg,
    cyc_softmax_exp_dev) against the host libm over [-750, 0]: within 4 ulp
    where e^x is normal; where it is subnormal (below -708.4: the result
    rounded onto the subnormal grid) within 2 units of 2^-1074 or 1e-12
    relative; 0 below -746 and at -inf, 1 at -0.0, NaN kept."""
    import torch
    from cycloneml_amd import _native as N
    rng = np.random.default_rng(12)
    x = np.concatenate([np.linspace(-750.0, 0.0, 2_000_001), -rng.exponential(3.0, 500_000),
                        -rng.uniform(700.0, 750.0, 200_000), [-0.0, -np.inf, np.nan, -708.0,
                                                              -708.4, -745.1, -746.0, -1e-300]])
    xd = torch.as_tensor(x, device=cuda)
    out = torch.empty_like(xd)
    N.check(N.load().cyc_softmax_exp_dev(N.ptr(xd), x.size, N.ptr(out), None))
    got = out.cpu().numpy()
    ref = np.exp(x)
    fin = np.isfinite(x)
    normal = fin & (ref >= np.finfo(np.float64).tiny)
    ulps = np.abs(got[normal] - ref[normal]) / np.spacing(ref[normal])
    assert ulps.max() <= 4.0, ulps.max()
    sub = fin & ~normal
    err = np.abs(got[sub] - ref[sub])
    assert np.all(err <= np.maximum(2 * 2.0 ** -1074, 1e-12 * ref[sub]))
    assert np.all(got[fin & (x < -746.0)] == 0.0)
    assert got[-8 + 0] == 1.0 and got[-7] == 0.0 and np.isnan(got[-6])
    assert got[-1] == 1.0


def test_multinomial_margin_spread_past_708(cuda):
    """Margins spread by more than 708 within a row, so softmax terms fall
    into the subnormal range and below it (Utils.softmax, ml/impl/Utils.scala:
    108-135): rows whose label's probability is subnormal keep a finite loss
    term, as the reference's Math.exp gives; the state matches the
    restatement within 1e-10."""
    from cycloneml_amd.optim import DeviceInstanceBlock, MultinomialLogisticBlockAggregator
    rng = np.random.default_rng(21)
    n, F, C = 3000, 4, 6
    X = rng.normal(size=(n, F))
    X[:, 0] = rng.uniform(0.96, 1.02, size=n)
    coef = np.zeros(C * F + C)                     # linear C x F column-major, then intercepts
    coef[0 * C + 1] = 720.0                        # class 1 leads by ~690..737
    coef[0 * C + 2] = -30.0                        # class 2: terms below -746 (exactly 0)
    coef[1 * C + 3] = 0.5                          # class 3 within +-2.5
    # labels never class 2 (a zero probability's log is -inf in both); the
    # others' probabilities are subnormal for about half the rows
    labels = rng.choice([0, 1, 3, 4, 5], size=n).astype(np.float64)
    for fi in (False, True):
        c = coef if fi else coef[:C * F]
        st = dict(grad=np.zeros(c.size), loss=0.0, weight=0.0)
        oracle.multinomial_logistic_add(dict(labels=labels, weights=None, X=X), c, C, fi, False,
                                        None, st)
        assert np.isfinite(st["loss"])
        blk = DeviceInstanceBlock.from_numpy(labels, None, X=X, device=cuda)
        agg = MultinomialLogisticBlockAggregator(np.ones(F), None, fi, False, c,
                                                 device=cuda).add(blk)
        _rel_close(agg.gradientSumArray.cpu().numpy(), st["grad"])
        loss = float(agg._loss_sum.item())
        assert np.isfinite(loss) and abs(loss - st["loss"]) <= 1e-10 * abs(st["loss"])


def test_tiles_auto_demotes_to_wide(cuda):
    """CYC_TILES_AUTO decides at the first append; a later append whose rows
    are too sparse for the compact format's filler allowance (a dense head of
    config 5's shape, then a tail with a nonzero every 80th row over 26 row
    blocks: two fillers per nonzero) turns the whole layout wide
    (tiles.hip demote_to_wide) instead of failing, and the aggregator state
    is the same bits as a layout built wide from the start.  An explicitly
    compact layout still fails such an append with the message naming the
    wide format -- and is left as it was before the append."""
    import torch
    from cycloneml_amd import _native as N
    from cycloneml_amd.optim import (BinaryLogisticBlockAggregator, DeviceInstanceBlock,
                                     SparseTiles)
    F = 1_000_000
    rng = np.random.default_rng(33)
    _, (rph, cih, vvh), _, _ = _make(8192, F, True, rng, nnz=64)
    gap, blocks = 80, 26
    nt = gap * 2048 * blocks
    nzt = np.zeros(nt, dtype=np.int64)
    nzt[::gap] = 1
    rpt = np.concatenate([[0], np.cumsum(nzt)])
    cit = rng.integers(0, F, size=int(nzt.sum())).astype(np.int32)
    vvt = rng.uniform(-1, 1, size=cit.size)
    n = 8192 + nt
    rp = np.concatenate([rph, rpt[1:] + rph[-1]])
    ci, vv = np.concatenate([cih, cit]), np.concatenate([vvh, vvt])
    labels = rng.integers(0, 2, size=n).astype(np.float64)
    w = rng.uniform(0.1, 2.0, size=n)
    dev = lambda a: torch.as_tensor(a, device=cuda)
    auto = SparseTiles(F, n, ci.size)
    auto.append(dev(rph), dev(cih), dev(vvh))
    assert auto.format == "compact"
    auto.append(dev(rpt), dev(cit), dev(vvt))
    assert auto.format == "wide" and auto.nnz == ci.size and auto.entries == auto.nnz
    wide = SparseTiles.from_csr(dev(rp), dev(ci), dev(vv), F, format="wide")
    coef = rng.normal(size=F + 1) * 0.3
    sm = dev(rng.normal(size=F) * 0.1)
    states = []
    for t in (auto, wide):
        blk = DeviceInstanceBlock(dev(labels), dev(w), tiles=t, numFeatures=F)
        b = BinaryLogisticBlockAggregator(np.ones(F), sm, True, True, coef, device=cuda).add(blk)
        states.append(b._state.cpu().numpy())
    assert np.array_equal(states[0], states[1])
    comp = SparseTiles(F, n, ci.size, format="compact")
    comp.append(dev(rph), dev(cih), dev(vvh))
    nnz0, ent0 = comp.nnz, comp.entries
    with pytest.raises(N.IllegalArgumentException, match="CYC_TILES_WIDE"):
        comp.append(dev(rpt), dev(cit), dev(vvt))
    assert (comp.format, comp.nnz, comp.entries) == ("compact", nnz0, ent0)
