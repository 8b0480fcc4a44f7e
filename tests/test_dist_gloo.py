"""Multi-process (world_size 2, gloo on CPU) tests of the N>1 path: row
sharding + the single all-reduce merge (cycloneml_amd/parallel.py) that
replaces treeAggregate / reduceByKey.  The per-shard partial that the GPU
kernels compute is produced here by the CPU restatement (oracle) so the
merge and update logic runs without a device; results must match the
single-process reference on all rows."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


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
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, fn(rank, world)))
    except Exception as e:  # surface failures to the parent
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def _run(fn, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    return out


def _kmeans_rank(rank, world):
    import oracle
    from cycloneml_amd import parallel
    rng = np.random.default_rng(0)
    n, d, k = 3001, 12, 7
    X = rng.normal(size=(n, d)) + rng.integers(0, 4, size=(n, 1)) * 3.0
    C = X[:k].copy()
    Ct = torch.from_numpy(C.copy()) if rank == 0 else torch.zeros(k, d, dtype=torch.float64)
    parallel.broadcast_(Ct)
    C = Ct.numpy().copy()
    cn = oracle.row_norms(C)
    a, b = parallel.shard_bounds(n, rank, world)
    Xs = X[a:b]
    stats = oracle.kmeans_stats(C)
    assign, dist_, sums, wsum, cost = oracle.kmeans_partition(Xs, oracle.row_norms(Xs), None, C,
                                                              cn, stats)
    buf = torch.from_numpy(np.concatenate([sums.ravel(), wsum, [cost]]))
    parallel.allreduce_(buf)
    sums2 = buf[:k * d].numpy().reshape(k, d)
    wsum2 = buf[k * d:k * d + k].numpy()
    C2, cn2 = C.copy(), cn.copy()
    oracle.update_centers(C2, cn2, sums2, wsum2)
    ref = oracle.kmeans_iteration(X, oracle.row_norms(X), None, C, cn)
    ok_assign = np.array_equal(assign, ref["assign"][a:b])
    ok_c = np.allclose(C2, ref["centers"], rtol=1e-12, atol=1e-12)
    ok_w = np.array_equal(wsum2, ref["wsum"])
    ok_cost = abs(buf[-1].item() - ref["cost"]) <= 1e-12 * ref["cost"]
    return ok_assign and ok_c and ok_w and ok_cost


def _aggregator_rank(rank, world):
    import oracle
    from cycloneml_amd.optim import DifferentiableLossAggregator
    rng = np.random.default_rng(1)
    n, F = 999, 9
    X = rng.normal(size=(n, F))
    y = (rng.uniform(size=n) < 0.4).astype(float)
    w = rng.uniform(0.5, 1.5, size=n)
    coef = rng.normal(size=F + 1)
    from cycloneml_amd import parallel
    a, b = parallel.shard_bounds(n, rank, world)
    st = dict(grad=np.zeros(F + 1), loss=0.0, weight=0.0)
    oracle.binary_logistic_add(dict(labels=y[a:b], weights=w[a:b], X=X[a:b]), coef, True, False,
                               None, st)
    agg = DifferentiableLossAggregator()
    agg.dim = F + 1
    agg._init_state("cpu")
    agg._state[:F + 1] = torch.from_numpy(st["grad"])
    agg._state[F + 1] = st["loss"]
    agg._state[F + 2] = st["weight"]
    agg.allreduce()
    ref = dict(grad=np.zeros(F + 1), loss=0.0, weight=0.0)
    oracle.binary_logistic_add(dict(labels=y, weights=w, X=X), coef, True, False, None, ref)
    return (np.allclose(agg.gradient, ref["grad"] / ref["weight"], rtol=1e-12)
            and abs(agg.loss - ref["loss"] / ref["weight"]) <= 1e-12 * abs(agg.loss))


def _gramian_rank(rank, world):
    import oracle
    from cycloneml_amd import parallel
    rng = np.random.default_rng(2)
    X = rng.uniform(size=(501, 6))
    a, b = parallel.shard_bounds(501, rank, world)
    U = torch.from_numpy(oracle.gramian_partition(X[a:b]))
    parallel.allreduce_(U)
    return bool(np.allclose(U.numpy(), oracle.gramian_partition(X), rtol=1e-13))


def _init_shards_rank(rank, world):
    """The host side of the multi-rank k-means|| / random initialisation
    (kmeans_init._Shards): the partitions numbered in rank order, the rows at
    global sampled positions gathered from their owners, collect() in rank
    order, and takeSample over the global partition lengths."""
    from cycloneml_amd import parallel
    from cycloneml_amd.kmeans_init import _Shards, take_sample_indices
    n, d = 901, 3
    X = np.arange(n * d, dtype=np.float64).reshape(n, d)
    a, b = parallel.shard_bounds(n, rank, world)
    parts = [[0, 100, 451], [0, 0, 200, 450]][rank]
    sh = _Shards(parts)
    ok = sh.lens == [100, 351, 0, 200, 250] and sh.first_partition == (0, 2)[rank]
    ok = ok and sh.row_offset == a and sh.rows == b - a
    pos = take_sample_indices(sh.lens, 37, 99)
    got = sh.rows_at(torch.from_numpy(X[a:b].copy()), pos)
    ok = ok and np.array_equal(got, X[pos])
    got2 = sh.rows_of(lambda loc: X[a:b][loc], pos, d)      # the CSR shards' gather
    ok = ok and np.array_equal(got2, X[pos])
    cat = sh.concat(X[a:b][::100])
    return bool(ok and np.array_equal(cat, np.concatenate([X[0:451][::100], X[451:][::100]])))


@pytest.mark.parametrize("fn", [_kmeans_rank, _aggregator_rank, _gramian_rank,
                                _init_shards_rank])
def test_two_rank_merge(fn):
    out = _run(fn)
    assert out == {0: True, 1: True}, out


def test_shard_bounds_cover_rows():
    from cycloneml_amd.parallel import shard_bounds
    for n in (0, 1, 7, 10_000_001):
        for w in (1, 2, 3, 8):
            b = [shard_bounds(n, r, w) for r in range(w)]
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(b[i][1] == b[i + 1][0] for i in range(w - 1))
            assert max(e - s for s, e in b) - min(e - s for s, e in b) <= 1


def _bench_rows_rank(rank, world):
    """bench.py's strong-scaling split at world size 2: every rank's rows of
    configs 3-5 summed over the ranks (one all-reduce, as the bench's
    max_over_ranks) equal the job's rows, and the uncapped totals are the
    BASELINE configs' rows; KMeans config 2 stays 10M per GPU (weak)."""
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    import bench
    ok = True
    for name in bench.ORDER:
        n, mode, total = bench.rows_per_gpu(name, "auto", world, rank)
        t = torch.tensor([n], dtype=torch.int64)
        dist.all_reduce(t)
        ok = ok and int(t.item()) == total
        if name == "kmeans":
            ok = ok and mode == "weak" and n == 10_000_000
        else:
            ok = ok and mode == "strong"
            if name not in ("gramian", "pca"):   # 100M rows of 1024 exceed 2 x 30M resident
                ok = ok and total == bench.CONFIG_ROWS[name]
    return bool(ok)


def _agree_rank(rank, world):
    """parallel.agree: a check that fails on ONE shard only (a bad weight on
    rank 1, checkNonNegativeWeight's message) raises the same exception on
    every rank before the next collective -- the all-reduce after it is
    never entered by one rank alone; a check passing everywhere returns its
    value.  And dense_cluster_ids numbers every rank's distinct ids."""
    from cycloneml_amd import _native as N
    from cycloneml_amd import parallel
    from cycloneml_amd.evaluation import dense_cluster_ids
    msg = "requirement failed: illegal weight value: -1.0. weight must be >= 0.0."

    def check():
        if rank == 1:
            raise N.IllegalArgumentException(msg)
        return rank

    ok = False
    try:
        parallel.agree(check)
    except N.IllegalArgumentException as e:
        ok = str(e) == msg
    t = torch.ones(1, dtype=torch.float64)
    parallel.allreduce_(t)                        # both ranks reach the next collective
    ok = ok and t.item() == 2.0 and parallel.agree(lambda: rank * 10) == rank * 10
    # a JavaAssertionError on rank 0 wins over rank 1's require
    try:
        parallel.agree(lambda: (_ for _ in ()).throw(
            N.JavaAssertionError("assertion failed: a") if rank == 0 else
            N.IllegalArgumentException("requirement failed: b")))
        ok = False
    except N.JavaAssertionError as e:
        ok = ok and str(e) == "assertion failed: a"
    mine = torch.tensor([[5, -3, 5], [1_000_000, 5, 7]][rank])
    ids, K = dense_cluster_ids(mine)
    want = [[1, 0, 1], [3, 1, 2]][rank]
    ok = bool(ok and K == 4 and ids.tolist() == want and ids.dtype == torch.int32)
    # NaN predictions (rank 1 only) are ONE cluster, numbered after every
    # other key, as Spark's grouping of the double column keys them
    nan = float("nan")
    mine = torch.tensor([[5.0, -3.0], [nan, 7.0, nan]][rank], dtype=torch.float64)
    ids, K = dense_cluster_ids(mine)
    want = [[1, 0], [3, 2, 3]][rank]
    return bool(ok and K == 4 and ids.tolist() == want)


def test_agree_two_ranks():
    assert _run(_agree_rank) == {0: True, 1: True}


class _HostComm:
    """A host stand-in for parallel.Communicator: records what init() hands it."""
    ID_BYTES = 128

    @staticmethod
    def unique_id():
        return bytes(range(128))

    def __init__(self, uid, rank, world, device):
        self.uid, self.rank, self.world_size, self.device = uid, rank, world, device


def _rendezvous_rank(rank, world):
    """bench.py --gpus N's control plane: torch.distributed on gloo carries
    rank 0's RCCL id to every rank (a host tensor), and each rank builds ONE
    communicator from it with its own rank and device (parallel.init); a
    second init returns the same one."""
    import torch
    sys.path.insert(0, ROOT)
    import bench
    from cycloneml_amd import parallel
    ok = bench.DIST_BACKEND == "gloo" and torch.distributed.get_backend() == "gloo"
    try:
        c = parallel.init(torch.device("cuda", rank), communicator=_HostComm)
        ok = ok and isinstance(c, _HostComm) and c.uid == bytes(range(128))
        ok = ok and (c.rank, c.world_size, c.device) == (rank, world, rank)
        ok = ok and parallel.init(torch.device("cuda", rank), communicator=_HostComm) is c
        ok = ok and parallel.communicator() is c
    finally:
        parallel._comm = None
    return bool(ok)


def test_rendezvous_one_communicator_two_ranks():
    assert _run(_rendezvous_rank) == {0: True, 1: True}


def test_bench_has_no_nccl_process_group():
    """The only RCCL communicator per GPU is libcyclone's (cyc_comm):
    bench.py's torch.distributed group is gloo."""
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert 'init_process_group("nccl"' not in src and "init_process_group(DIST_BACKEND)" in src


def test_bench_strong_split_two_ranks():
    assert _run(_bench_rows_rank) == {0: True, 1: True}


def test_bench_rows_per_gpu_table():
    """The split of BASELINE's totals for N = 1..8 (bench.py --scaling auto)."""
    sys.path.insert(0, ROOT)
    import bench
    for world in (1, 2, 4, 8):
        for name in bench.ORDER:
            per = [bench.rows_per_gpu(name, "auto", world, r) for r in range(world)]
            assert all(p[2] == per[0][2] for p in per)
            assert sum(p[0] for p in per) == per[0][2]
            assert max(p[0] for p in per) <= bench.MAX_RESIDENT_ROWS[name]
    assert bench.rows_per_gpu("gramian", "auto", 1, 0) == (30_000_000, "strong", 30_000_000)
    assert bench.rows_per_gpu("gramian", "auto", 4, 3) == (25_000_000, "strong", 100_000_000)
    assert bench.rows_per_gpu("lr_sparse", "auto", 8, 7) == (25_000_000, "strong", 200_000_000)
    assert bench.rows_per_gpu("lr_multi", "auto", 8, 0) == (6_250_000, "strong", 50_000_000)
    assert bench.rows_per_gpu("kmeans", "auto", 8, 5) == (10_000_000, "weak", 80_000_000)
    assert bench.rows_per_gpu("lr_sparse", "weak", 2, 1) == (200_000_000, "weak", 400_000_000)
