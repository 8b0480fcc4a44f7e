"""GPU tests of the aggregation step.

- libcyclone's C-ABI communicator over RCCL (cyc_comm_*, include/cyclone.h)
  at world size 1 (the GPU box has one GPU; RCCL refuses two ranks on one
  device): every entry point, device and host forms, and its argument checks.
- two rank processes on the one GPU joined by a gloo group: each rank runs
  the DEVICE kernels on its shard (KMeans accumulate, multinomial / sparse
  binary logistic aggregators, Gramian), the partials meet in the all-reduce
  (parallel.allreduce_) and the merged result must equal the single-process
  restatement over all rows -- the path bench.py --gpus N runs with RCCL.
"""
import ctypes
import os
import socket
import sys

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_comm_world_one(cuda):
    import torch
    from cycloneml_amd import _native as N
    from cycloneml_amd.parallel import Communicator
    uid = Communicator.unique_id()
    assert len(uid) == 128
    comm = Communicator(uid, 0, 1, cuda.index or 0)
    try:
        rng = np.random.default_rng(0)
        x = rng.normal(size=1001)
        t = torch.from_numpy(x.copy()).to(cuda)
        comm.allreduce_sum_(t)
        comm.allreduce_max_(t)
        comm.broadcast_(t, 0)
        g = comm.allgather(t)
        torch.cuda.synchronize()
        assert np.array_equal(t.cpu().numpy(), x)
        assert g.shape == (1, 1001) and np.array_equal(g[0].cpu().numpy(), x)
        # host forms (the resident-dataset layer's outputs are host arrays)
        L = N.load()
        h = x.copy()
        N.check(L.cyc_allreduce_sum(comm.handle, h.ctypes.data, h.size))
        N.check(L.cyc_broadcast(comm.handle, h.ctypes.data, h.size, 0))
        assert np.array_equal(h, x)
        r, w = ctypes.c_int32(), ctypes.c_int32()
        N.check(L.cyc_comm_rank(comm.handle, ctypes.byref(r), ctypes.byref(w)))
        assert (r.value, w.value) == (0, 1)
        with pytest.raises(N.IllegalArgumentException, match="count must be nonnegative"):
            N.check(L.cyc_allreduce_sum_dev(comm.handle, N.ptr(t), -1, None))
        with pytest.raises(N.IllegalArgumentException, match="root must be a rank"):
            N.check(L.cyc_broadcast_dev(comm.handle, N.ptr(t), t.numel(), 1, None))
        with pytest.raises(N.IllegalArgumentException, match="contiguous fp64"):
            comm.allreduce_sum_(t.float())
    finally:
        comm.close()
    with pytest.raises(N.IllegalArgumentException, match="rank must be in"):
        Communicator(uid, 1, 1, 0)


# ----------------------------------------------------- two ranks, one GPU

def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, fn, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, fn(rank, world)))
    except Exception as e:  # surface failures to the parent
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def _run(fn, world=2):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        out = dict(q.get(timeout=150) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    return out


def _kmeans_rank(rank, world):
    import torch
    from cycloneml_amd import parallel
    from cycloneml_amd.clustering import KMeansPlan, row_norms
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(0)
    n, d, k = 40_001, 64, 33
    X = rng.normal(size=(n, d)) + rng.integers(0, 6, size=(n, 1)) * 3.0
    C = X[:k].copy()
    a, b = parallel.shard_bounds(n, rank, world)
    Xd = torch.from_numpy(X[a:b].copy()).to(dev)
    Cd = torch.from_numpy(C.copy() if rank == 0 else np.zeros_like(C)).to(dev)
    parallel.broadcast_(Cd)                       # bcCenters
    xn, cn = row_norms(Xd), row_norms(Cd)
    plan = KMeansPlan(d, k, b - a)
    buf = torch.zeros(k * d + k + 1, dtype=torch.float64, device=dev)
    sums, wsum, cost = buf[:k * d], buf[k * d:k * d + k], buf[k * d + k:]
    asg = torch.empty(b - a, dtype=torch.int32, device=dev)
    plan.accumulate(Xd, xn, None, Cd, cn, sums, wsum, cost, asg, rows=plan.rows(Xd))
    parallel.allreduce_(buf)                      # reduceByKey + costAccum
    conv = torch.zeros(1, dtype=torch.int32, device=dev)
    plan.update(Cd, cn, sums, wsum, 1e-4, conv)
    torch.cuda.synchronize()
    ref = oracle.kmeans_iteration(X, oracle.row_norms(X), None, C, oracle.row_norms(C),
                                  num_partitions=2)
    return bool(np.array_equal(asg.cpu().numpy(), ref["assign"][a:b])
                and np.array_equal(wsum.cpu().numpy(), ref["wsum"])
                and np.allclose(Cd.cpu().numpy(), ref["centers"], rtol=1e-12, atol=1e-12)
                and abs(cost.item() - ref["cost"]) <= 1e-12 * ref["cost"])


def _kmeans_carried_rank(rank, world):
    """Eight Lloyd iterations on row shards with each rank's carried state on
    (bounds, neighbourhoods, incremental sums: k > 96, d <= 256), the state
    merged by the collective every iteration: every iteration equals the
    restatement over the whole data on the same centers (the shard's
    assignments exactly, weights exactly, sums within 1e-10, cost 1e-12)."""
    import torch
    from cycloneml_amd import parallel
    from cycloneml_amd.clustering import KMeansPlan, row_norms
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(7)
    n, d, k = 60_001, 64, 130
    X = rng.normal(scale=3.0, size=(k, d))[rng.integers(0, k, n)] + rng.normal(size=(n, d))
    a, b = parallel.shard_bounds(n, rank, world)
    Xd = torch.from_numpy(X[a:b].copy()).to(dev)
    Cd = torch.from_numpy(X[:k].copy()).to(dev)
    parallel.broadcast_(Cd)
    xn, cn = row_norms(Xd), row_norms(Cd)
    plan = KMeansPlan(d, k, b - a)
    rows = plan.rows(Xd)
    buf = torch.zeros(k * d + k + 1, dtype=torch.float64, device=dev)
    sums, wsum, cost = buf[:k * d], buf[k * d:k * d + k], buf[k * d + k:]
    asg = torch.empty(b - a, dtype=torch.int32, device=dev)
    conv = torch.zeros(1, dtype=torch.int32, device=dev)
    ok = True
    for it in range(8):
        C = Cd.cpu().numpy()
        buf.zero_()
        plan.accumulate(Xd, None, None, Cd, cn, sums, wsum, cost, asg, rows=rows)
        parallel.allreduce_(buf)
        if it in (0, 3, 7):
            ref = oracle.kmeans_iteration(X, oracle.row_norms(X), None, C, oracle.row_norms(C),
                                          num_partitions=2)
            S = sums.cpu().numpy().reshape(k, d)
            ok = ok and bool(np.array_equal(asg.cpu().numpy(), ref["assign"][a:b])
                             and np.array_equal(wsum.cpu().numpy(), ref["wsum"])
                             and np.allclose(S, ref["sums"], rtol=1e-10,
                                             atol=1e-10 * np.abs(ref["sums"]).max())
                             and abs(cost.item() - ref["cost"]) <= 1e-12 * ref["cost"])
        plan.update(Cd, cn, sums, wsum, 1e-4, conv)
    torch.cuda.synchronize()
    calls, _ = rows.bounds_info()
    inc, _ = rows.incremental_info()
    return bool(ok and calls == 8 and inc >= 1)


def _lr_rank(rank, world):
    import torch
    from cycloneml_amd import parallel
    from cycloneml_amd.optim import (BinaryLogisticBlockAggregator, DeviceInstanceBlock,
                                     MultinomialLogisticBlockAggregator, RDDLossFunction)
    rng = np.random.default_rng(1)
    n, F, Cn = 3001, 40, 7
    X = rng.normal(size=(n, F))
    y = rng.integers(0, Cn, size=n).astype(float)
    w = rng.uniform(0.5, 1.5, size=n)
    coef = rng.normal(size=Cn * F + Cn) * 0.1
    mean = rng.normal(size=F) * 0.1
    a, b = parallel.shard_bounds(n, rank, world)
    blk = DeviceInstanceBlock.from_numpy(y[a:b], w[a:b], X=X[a:b], device="cuda:0")
    fn = RDDLossFunction([blk], lambda c: MultinomialLogisticBlockAggregator(
        np.ones(F), mean, True, True, c, device="cuda:0"))
    loss, grad = fn.calculate(coef)
    st = dict(grad=np.zeros(coef.size), loss=0.0, weight=0.0)
    oracle.multinomial_logistic_add(dict(labels=y, weights=w, X=X), coef, Cn, True, True, mean,
                                    st)
    ok_m = (abs(loss - st["loss"] / st["weight"]) <= 1e-10 * abs(loss)
            and np.allclose(grad, st["grad"] / st["weight"], rtol=1e-10, atol=1e-14))
    # sparse binary with fitWithMean (per-row CSR, CSC gradient pass)
    rows = [np.sort(rng.choice(F, size=rng.integers(1, 9), replace=False)) for _ in range(n)]
    rowptr = np.concatenate([[0], np.cumsum([len(r) for r in rows])]).astype(np.int64)
    colidx = np.concatenate(rows).astype(np.int32)
    vals = rng.uniform(0.1, 2.0, size=colidx.size)
    yb = (rng.uniform(size=n) < 0.4).astype(float)
    cb = rng.normal(size=F + 1) * 0.2
    lo, hi = rowptr[a], rowptr[b]
    blk2 = DeviceInstanceBlock.from_numpy(yb[a:b], w[a:b],
                                          csr=(rowptr[a:b + 1] - lo, colidx[lo:hi], vals[lo:hi]),
                                          numFeatures=F, device="cuda:0")
    blk2.prepare()
    fn2 = RDDLossFunction([blk2], lambda c: BinaryLogisticBlockAggregator(
        np.ones(F), mean, True, True, c, device="cuda:0"))
    loss2, grad2 = fn2.calculate(cb)
    st2 = dict(grad=np.zeros(F + 1), loss=0.0, weight=0.0)
    oracle.binary_logistic_add(dict(labels=yb, weights=w, rowptr=rowptr, colidx=colidx,
                                    values=vals, F=F), cb, True, True, mean, st2)
    ok_b = (abs(loss2 - st2["loss"] / st2["weight"]) <= 1e-10 * abs(loss2)
            and np.allclose(grad2, st2["grad"] / st2["weight"], rtol=1e-10, atol=1e-14))
    return bool(ok_m and ok_b)


def _gramian_rank(rank, world):
    import torch
    from cycloneml_amd import parallel
    from cycloneml_amd.linalg import GramianPlan
    rng = np.random.default_rng(2)
    n, p = 5003, 96
    X = rng.uniform(size=(n, p))
    a, b = parallel.shard_bounds(n, rank, world)
    U = torch.zeros(p * (p + 1) // 2, dtype=torch.float64, device="cuda:0")
    GramianPlan(p).accumulate(torch.from_numpy(X[a:b].copy()).to("cuda:0"), U)
    parallel.allreduce_(U)
    return bool(np.allclose(U.cpu().numpy(), oracle.gramian_partition(X), rtol=1e-12))


def _covariance_rank(rank, world):
    """RowMatrix.computeCovariance over two ranks' shards: the form chosen from
    merged moments (the same on both ranks), the fused column sums and the
    syrk all-reduced.  Rank 1's leading rows are far off centre while rank
    0's are not: the merged leading-row moments and the whole matrix decide
    together."""
    import torch
    from cycloneml_amd import parallel
    from cycloneml_amd.linalg import RowMatrix
    rng = np.random.default_rng(9)
    n, p = 6001, 40
    far = rng.normal(size=(n, p)) * 1e-3 + 1e5
    far[:16] = rng.normal(size=(16, p))    # rank 0's leading rows near the origin
    # uncentred on both ranks; then the 16-row samples (one centred, one far
    # off) pass the bound together, the whole matrix does not: centred syrk
    cases = [rng.normal(size=(n, p)) + 2.0, far]
    ok = True
    forms = []
    for X in cases:
        a, b = parallel.shard_bounds(n, rank, world)
        mat = RowMatrix(torch.from_numpy(X[a:b].copy()).to("cuda:0"))
        mat.COV_SAMPLE_ROWS = 16
        cov = mat.computeCovariance()
        U = oracle.gramian_partition(X, X.sum(0) / n)
        ref = np.asarray(oracle.triu_to_full(p, U)).reshape(p, p).T / (n - 1.0)
        ok = ok and bool(np.allclose(cov, ref, rtol=1e-10, atol=1e-10 * np.abs(ref).max()))
        forms.append((mat.lastCovarianceForm, tuple(mat.lastCovariancePasses)))
    mine = parallel.allgather_object(forms)
    return bool(ok and [f for f, _ in forms] == ["uncentred", "centred"] and
                forms[1][1][-2:] == ("syrk + column sums", "centred syrk") and
                all(f == forms for f in mine))


def _init_reference(X, dev, part_starts, shard_rows, k, s, mode):
    """The host composition of KMeans.initRandom / initKMeansParallel over all
    partitions (numbered in rank order), with sumCosts the rank-order sum of
    the ranks' device sums (the all-reduce)."""
    import torch
    from cycloneml_amd.kmeans_init import take_sample_indices
    n = X.shape[0]
    lens = np.diff(part_starts)
    if mode == "random":
        return X[take_sample_indices(lens, k, s)]
    cands = [X[take_sample_indices(lens, 1, s)[0]]]
    new = np.array(cands)
    costs = np.full(n, np.inf)
    for step in range(2):
        _, pc, _ = oracle.point_costs(X, oracle.row_norms(X), new, oracle.row_norms(new))
        costs = np.minimum(pc, costs)
        total = 0.0
        for a, b in shard_rows:
            total += float(torch.from_numpy(costs[a:b].copy()).to(dev).sum().item())
        mask = oracle.kmeans_parallel_sample(costs, part_starts, 0, s, step, k, total)
        new = X[mask.astype(bool)]
        cands.extend(new)
    uniq = []
    for c in cands:
        if not any(np.array_equal(c, u) for u in uniq):
            uniq.append(c)
    uniq = np.array(uniq)
    if uniq.shape[0] <= k:
        return uniq
    a_, _, _ = oracle.point_costs(X, oracle.row_norms(X), uniq, oracle.row_norms(uniq))
    wts = np.bincount(a_, minlength=uniq.shape[0]).astype(np.float64)
    return oracle.local_kmeans_pp(uniq, wts, k, 30, 0)


def _kmeans_init_rank(rank, world):
    """k-means|| and random initialisation across two ranks
    (KMeans.scala:354-432): each rank holds a shard split into its own Spark
    partitions; the initial centers on every rank equal the one-driver
    composition over all partitions, and the Lloyd run from them matches a
    single-process run from those centers."""
    import torch
    from cycloneml_amd import parallel
    from cycloneml_amd.clustering import KMeans, KMeansModel, xorshift_next_int
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(5)
    n, d, k = 4001, 8, 5
    X = rng.normal(size=(n, d)) + rng.integers(0, 5, size=(n, 1)) * 4.0
    shard_rows = [parallel.shard_bounds(n, r, world) for r in range(world)]
    local_parts = [[0, 700, 2001], [0, 333, 999, 1400, 2000]]
    glob = [0]
    for r in range(world):
        glob += [shard_rows[r][0] + v for v in local_parts[r][1:]]
    a, b = shard_rows[rank]
    assert local_parts[rank][-1] == b - a
    Xd = torch.from_numpy(X[a:b].copy()).to(dev)
    ok = True
    for mode in ("k-means||", "random"):
        km = KMeans(k=k, maxIterations=20).setSeed(31).setInitializationMode(mode)
        C0 = km.initial_centers(Xd, partition_starts=local_parts[rank])
        ref = _init_reference(X, dev, np.array(glob, dtype=np.int64), shard_rows, k,
                              xorshift_next_int(31), mode)
        ok = ok and C0.shape == ref.shape and bool(np.array_equal(C0, ref))
        m = km.run(Xd, partition_starts=local_parts[rank])
        single = KMeans(k=C0.shape[0], maxIterations=20).setInitialModel(
            KMeansModel(C0)).run(torch.from_numpy(X).to(dev))
        ok = ok and bool(np.allclose(m.clusterCenters, single.clusterCenters, rtol=1e-12,
                                     atol=1e-12))
    return ok


def _kmeans_init_csr_rank(rank, world):
    """k-means|| over CSR shards on two ranks: the initial centers on every
    rank equal the one-driver composition over the CSR restatement."""
    import torch
    from cycloneml_amd import parallel
    from cycloneml_amd.clustering import KMeans, xorshift_next_int
    from cycloneml_amd.kmeans_init import take_sample_indices
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(9)
    n, d, k = 2001, 30, 4
    X = np.zeros((n, d))
    for i in range(n):
        c = rng.integers(0, 4)
        cols = np.unique(np.concatenate([rng.choice(d, size=5, replace=False), [c * 7]]))
        X[i, cols] = rng.normal(size=cols.size) + (cols // 7 == c) * 4.0

    def csr(rows):
        nz = rows != 0.0
        rp = np.concatenate([[0], np.cumsum(nz.sum(1))]).astype(np.int64)
        r, c = np.nonzero(nz)
        return rp, c.astype(np.int32), rows[r, c]

    shard_rows = [parallel.shard_bounds(n, r, world) for r in range(world)]
    local_parts = [[0, 400, 1001], [0, 999, 1000]]
    glob = np.array([0, 400, 1001, 2000, 2001], dtype=np.int64)
    a, b = shard_rows[rank]
    mine = [torch.from_numpy(v).to(dev) for v in csr(X[a:b])]
    km = KMeans(k=k, maxIterations=5).setSeed(3)
    C0 = km.initial_centers_csr(*mine, d, partition_starts=local_parts[rank])
    # the one-driver composition
    full = csr(X)
    xn = oracle.row_norms_csr(full[0], full[2])
    s = xorshift_next_int(3)
    cands = [X[take_sample_indices(np.diff(glob), 1, s)[0]]]
    new = np.array(cands)
    costs = np.full(n, np.inf)
    for step in range(2):
        _, pc, _ = oracle.point_costs_sparse(full, xn, new, oracle.row_norms(new))
        costs = np.minimum(pc, costs)
        total = 0.0
        for lo, hi in shard_rows:
            total += float(torch.from_numpy(costs[lo:hi].copy()).to(dev).sum().item())
        mask = oracle.kmeans_parallel_sample(costs, glob, 0, s, step, k, total)
        new = X[mask.astype(bool)]
        cands.extend(new)
    uniq = []
    for c in cands:
        if not any(np.array_equal(c, u) for u in uniq):
            uniq.append(c)
    uniq = np.array(uniq)
    if uniq.shape[0] > k:
        asg, _, _ = oracle.point_costs_sparse(full, xn, uniq, oracle.row_norms(uniq))
        wts = np.bincount(asg, minlength=uniq.shape[0]).astype(np.float64)
        cc = csr(uniq)
        cn = oracle.row_norms_csr(cc[0], cc[2])
        ref = oracle.local_kmeans_pp(
            uniq, wts, k, 30, 0,
            closest=lambda C: oracle.point_costs_sparse(cc, cn, C, oracle.row_norms(C))[:2])
    else:
        ref = uniq
    return C0.shape == ref.shape and bool(np.array_equal(C0, ref))


def _silhouette_rank(rank, world):
    """ClusteringEvaluator over two row shards: the cluster statistics and
    the two score sums all-reduced (aggregateByKey's combOp, overallScore's
    sums), the score equal to the one-partition restatement's."""
    import torch
    from cycloneml_amd import parallel
    from cycloneml_amd.evaluation import ClusteringEvaluator
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(7)
    n, d, k = 30_001, 24, 7
    C = rng.normal(size=(k, d)) * 3.0
    p = rng.integers(0, k, size=n).astype(np.int32)
    X = C[p] + rng.normal(size=(n, d))
    w = rng.random(n) * 2.0
    a, b = parallel.shard_bounds(n, rank, world)
    ok = True
    for measure, cos in (("squaredEuclidean", False), ("cosine", True)):
        ev = ClusteringEvaluator(distanceMeasure=measure)
        s = ev.evaluate(torch.from_numpy(X[a:b].copy()).to(dev),
                        torch.from_numpy(p[a:b].copy()).to(dev),
                        torch.from_numpy(w[a:b].copy()).to(dev))
        ref, _ = oracle.silhouette(X, p, k, w, cosine=cos)
        ok = ok and abs(s - ref) <= 1e-12 * abs(ref)
    # a bad weight on rank 1's shard only: both ranks raise the same
    # IllegalArgumentException (checkNonNegativeWeight) and neither is left
    # in the statistics all-reduce
    from cycloneml_amd import _native as N
    wb = w[a:b].copy()
    if rank == 1:
        wb[5] = -2.5
    try:
        ClusteringEvaluator().evaluate(torch.from_numpy(X[a:b].copy()).to(dev),
                                       torch.from_numpy(p[a:b].copy()).to(dev),
                                       torch.from_numpy(wb).to(dev))
        ok = False
    except N.IllegalArgumentException as e:
        ok = ok and str(e) == ("requirement failed: illegal weight value: -2.5. weight must be "
                               ">= 0.0.")
    t = torch.ones(1, dtype=torch.float64, device=dev)
    parallel.allreduce_(t)
    return bool(ok and t.item() == 2.0)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("fn", [_kmeans_rank, _kmeans_carried_rank, _lr_rank, _gramian_rank,
                                _covariance_rank,
                                _kmeans_init_rank, _kmeans_init_csr_rank, _silhouette_rank])
def test_two_ranks_device_kernels_meet_the_collective(fn):
    out = _run(fn)
    assert out == {0: True, 1: True}, out
