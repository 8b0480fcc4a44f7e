"""KMeans initialisation: the driver side of "random" and "k-means||"
(mllib/clustering/KMeans.scala:354-432) over a device-resident shard.

The reference runs these on the driver (RDD.takeSample, LocalKMeans) and the
executors (the k-means|| cost passes and draws).  Here the executor passes run
on the device (KMeansModel.pointCosts, KMeans.parallelSample) and the driver
logic is restated on the host with the JVM's generators:
  - java.util.Random (takeSample, PartitionwiseSampledRDD, LocalKMeans);
  - XORShiftRandom (core/.../util/random/XORShiftRandom.scala), its seed hash
    from libcyclone (cyc_xorshift_hash_seed);
  - RDD.takeSample (core/.../rdd/RDD.scala:612-650) with
    SamplingUtils.computeFractionForSampleSize / BinomialBounds
    (core/.../util/random/SamplingUtils.scala:98-168), BernoulliSampler and
    GapSampling (core/.../util/random/RandomSampler.scala:144-176, 240-275),
    Utils.randomizeInPlace (core/.../util/Utils.scala:990-998);
  - LocalKMeans.kMeansPlusPlus (mllib/clustering/LocalKMeans.scala:35-134),
    whose findClosest passes run on the device (bit-exact).
GapSampling's log(u) / log1p(-f) use the host libm; Java's may differ in the
last ulp, which moves a gap only when the quotient sits within an ulp of an
integer.
"""
from __future__ import annotations

import math

import numpy as np

from . import _native as N

_M32 = 0xFFFFFFFF
_M48 = (1 << 48) - 1
_M64 = (1 << 64) - 1


def _i32(v: int) -> int:
    v &= _M32
    return v - (1 << 32) if v >= 1 << 31 else v


def _i64(v: int) -> int:
    v &= _M64
    return v - (1 << 64) if v >= 1 << 63 else v


class JavaRandom:
    """java.util.Random (the 48-bit LCG); scala.util.Random delegates to it."""

    def __init__(self, seed: int):
        self.set_seed(seed)

    def set_seed(self, seed: int):
        self._s = (int(seed) ^ 0x5DEECE66D) & _M48

    def next(self, bits: int) -> int:
        self._s = (self._s * 0x5DEECE66D + 0xB) & _M48
        return _i32(self._s >> (48 - bits))

    def next_int(self, bound: int | None = None) -> int:
        if bound is None:
            return self.next(32)
        if bound <= 0:
            raise ValueError("bound must be positive")
        r = self.next(31)
        m = bound - 1
        if bound & m == 0:                         # a power of two
            return _i32((bound * r) >> 31)
        u = r
        while True:
            r = u % bound
            if _i32(u - r + m) >= 0:
                return r
            u = self.next(31)

    def next_long(self) -> int:
        return _i64((self.next(32) << 32) + self.next(32))

    def next_double(self) -> float:
        return ((self.next(26) << 27) + self.next(27)) * (1.0 / (1 << 53))


class XORShiftRandom(JavaRandom):
    """org.apache.spark.util.random.XORShiftRandom: java.util.Random's
    nextInt / nextDouble over the xorshift next(bits)."""

    def set_seed(self, seed: int):
        self._s = int(N.load().cyc_xorshift_hash_seed(_i64(int(seed)))) & _M64

    def next(self, bits: int) -> int:
        x = self._s
        x ^= (x << 21) & _M64
        x ^= x >> 35
        x ^= (x << 4) & _M64
        self._s = x
        return _i32(x & ((1 << bits) - 1))


def _to_int(x: float) -> int:
    """Scala Double.toInt: toward zero, NaN -> 0, saturating."""
    if x != x:
        return 0
    if x >= 2147483647.0:
        return 2147483647
    if x <= -2147483648.0:
        return -2147483648
    return int(x)


def _bernoulli_positions(m: int, fraction: float, seed: int):
    """BernoulliSampler(fraction) seeded with `seed` over m items: the kept
    positions (RandomSampler.scala:144-176; GapSampling :240-275)."""
    rng = XORShiftRandom(seed)
    if fraction <= 0.0 or m == 0:
        return []
    if fraction >= 1.0:
        return list(range(m))
    if fraction <= 0.4:                          # defaultMaxGapSamplingFraction
        lnq = math.log1p(-fraction)

        def advance():
            u = max(rng.next_double(), 5e-11)    # rngEpsilon
            return _to_int(math.log(u) / lnq)

        out = []
        pos = advance()
        while pos < m:
            out.append(pos)
            pos += advance() + 1
        return out
    return [i for i in range(m) if rng.next_double() <= fraction]


def _fraction_for_sample_size(num: int, total: int) -> float:
    """SamplingUtils.computeFractionForSampleSize without replacement."""
    fraction = float(num) / total
    gamma = -math.log(1e-4) / total
    return min(1.0, max(1e-10, fraction + gamma + math.sqrt(gamma * gamma + 2 * gamma * fraction)))


def _randomize_in_place(arr: list, rand: JavaRandom) -> list:
    for i in range(len(arr) - 1, 0, -1):
        j = rand.next_int(i + 1)
        arr[i], arr[j] = arr[j], arr[i]
    return arr


def take_sample_indices(partition_lengths, num: int, seed: int) -> list:
    """RDD.takeSample(withReplacement = false, num, seed) over partitions of
    the given lengths: the sampled items' global positions (partition order,
    then within the partition), in the order takeSample returns them."""
    lens = [int(v) for v in partition_lengths]
    starts = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    total = int(starts[-1])
    if num == 0 or total == 0:
        return []
    rand = JavaRandom(seed)
    if num >= total:
        return _randomize_in_place(list(range(total)), rand)
    fraction = _fraction_for_sample_size(num, total)

    def sample(s):
        pr = JavaRandom(s)                       # PartitionwiseSampledRDD.getPartitions
        out = []
        for p, m in enumerate(lens):
            ps = pr.next_long()
            out.extend(int(starts[p]) + i for i in _bernoulli_positions(m, fraction, ps))
        return out

    samples = sample(rand.next_int())
    while len(samples) < num:
        samples = sample(rand.next_int())
    return _randomize_in_place(samples, rand)[:num]


def _distinct_rows(rows: np.ndarray) -> np.ndarray:
    """`.map(_.vector).distinct` (Scala Seq.distinct): first occurrences in
    order, vectors equal as Vector.equals compares them -- element by
    element with `!=` on doubles (mllib Vectors.equals), so -0.0 equals 0.0
    and a vector holding a NaN equals nothing, not even another copy of
    itself (Scala's HashSet tests `==`, i.e. equals, not identity)."""
    seen, keep = set(), []
    for i in range(rows.shape[0]):
        if np.isnan(rows[i]).any():
            keep.append(i)
            continue
        key = (rows[i] + 0.0).tobytes()          # -0.0 + 0.0 = +0.0
        if key not in seen:
            seen.add(key)
            keep.append(i)
    return rows[keep]


def _sqdist_to(points: np.ndarray, c: np.ndarray) -> np.ndarray:
    """Vectors.sqdist(point, c) for every point, each sum in index order."""
    s = np.zeros(points.shape[0])
    for j in range(points.shape[1]):
        t = points[:, j] - c[j]
        s = s + t * t
    return s


def local_kmeans_pp(points: np.ndarray, weights: np.ndarray, k: int, max_iterations: int,
                    seed: int, device, closest=None) -> np.ndarray:
    """LocalKMeans.kMeansPlusPlus (LocalKMeans.scala:35-134) with the
    Euclidean measure; the Lloyd rounds' findClosest (without statistics)
    on the device, bit-exact.  points: dense rows.  closest(C) -> (index,
    cost) host arrays of every point against centers C, for points that are
    sparse in the reference (fastSquaredDistance's norm-trick branch, also
    for the seeding costs: one center); default the dense rows themselves
    (Vectors.sqdist)."""
    import torch
    from .clustering import KMeansModel
    points = np.ascontiguousarray(points, dtype=np.float64)
    weights = np.asarray(weights, dtype=np.float64)
    m, d = points.shape
    rand = JavaRandom(seed)
    if closest is None:
        pd = torch.from_numpy(points).to(device)

        def closest(C):
            idx, c = KMeansModel(C).pointCosts(pd)
            return idx.cpu().numpy().astype(np.int64), c.cpu().numpy()

        def cost_to(c):
            return _sqdist_to(points, c)
    else:
        def cost_to(c):
            return closest(c[None, :])[1]

    def pick_weighted():
        r = rand.next_double() * _seq_sum(weights)
        i, cur = 0, 0.0
        while i < m and cur < r:
            cur += weights[i]
            i += 1
        return points[i - 1]

    centers = np.empty((k, d))
    centers[0] = pick_weighted()
    cost = cost_to(centers[0])
    for i in range(1, k):
        total = _seq_sum(cost * weights)
        r = rand.next_double() * total
        cum, j = 0.0, 0
        while j < m and cum < r:
            cum += weights[j] * cost[j]
            j += 1
        centers[i] = points[0] if j == 0 else points[j - 1]
        cost = np.minimum(cost_to(centers[i]), cost)
    old = np.full(m, -1, dtype=np.int64)
    iteration, moved = 0, True
    while moved and iteration < max_iterations:
        moved = False
        idx, _ = closest(centers)
        idx = np.asarray(idx, dtype=np.int64)
        counts = np.zeros(k)
        sums = np.zeros((k, d))
        for p in range(m):
            if weights[p] != 0.0:                # netlib daxpy: da == 0 returns
                sums[idx[p]] = sums[idx[p]] + weights[p] * points[p]
            counts[idx[p]] += weights[p]
        if np.any(idx != old):
            moved = True
            old = idx
        for j in range(k):
            if counts[j] == 0.0:
                centers[j] = points[rand.next_int(m)]
            else:
                centers[j] = (1.0 / counts[j]) * sums[j]
        iteration += 1
    return centers


def _seq_sum(a) -> float:
    s = 0.0
    for v in np.asarray(a, dtype=np.float64).tolist():
        s += v
    return s


class _Shards:
    """The Spark partitions of every rank's shard, numbered in rank order
    (rank r's partitions follow rank r-1's), and the rank's place in them."""

    def __init__(self, partition_starts):
        from . import parallel
        starts = np.asarray(partition_starts, dtype=np.int64)
        self.local_starts = starts
        lens = [int(v) for v in np.diff(starts)]
        every = parallel.allgather_object(lens)
        rank = parallel.world()[0]
        self.lens = [m for r in every for m in r]
        self.first_partition = sum(len(r) for r in every[:rank])
        self.row_offset = sum(sum(r) for r in every[:rank])
        self.rows = int(starts[-1])

    def rows_at(self, X, positions) -> np.ndarray:
        """The rows at global positions (any order), gathered from the ranks
        that hold them."""
        from . import parallel
        pos = np.asarray(positions, dtype=np.int64)
        mine = np.nonzero((pos >= self.row_offset) & (pos < self.row_offset + self.rows))[0]
        local = X[torch_index(pos[mine] - self.row_offset, X.device)].cpu().numpy() \
            if mine.size else None
        out = np.empty((pos.size, int(X.shape[1])))
        for got in parallel.allgather_object((mine, local)):
            if got[0].size:
                out[got[0]] = got[1]
        return out

    def rows_of(self, gather, positions, d: int) -> np.ndarray:
        """rows_at with a gather(local row indices) -> dense host rows."""
        from . import parallel
        pos = np.asarray(positions, dtype=np.int64)
        mine = np.nonzero((pos >= self.row_offset) & (pos < self.row_offset + self.rows))[0]
        local = gather(pos[mine] - self.row_offset) if mine.size else None
        out = np.empty((pos.size, d))
        for got in parallel.allgather_object((mine, local)):
            if got[0].size:
                out[got[0]] = got[1]
        return out

    def concat(self, rows: np.ndarray) -> np.ndarray:
        """`collect()` of per-partition results: every rank's rows in rank
        (= partition) order."""
        from . import parallel
        parts = parallel.allgather_object(rows)
        return np.concatenate(parts) if parts else rows


def torch_index(idx, device):
    import torch
    return torch.from_numpy(np.ascontiguousarray(idx, dtype=np.int64)).to(device)


def init_random(X, k: int, seed: int, partition_starts) -> np.ndarray:
    """KMeans.initRandom (KMeans.scala:354-358)."""
    from .clustering import xorshift_next_int
    sh = _Shards(partition_starts)
    idx = take_sample_indices(sh.lens, k, xorshift_next_int(seed))
    rows = sh.rows_at(X, idx) if idx else np.empty((0, X.shape[1]))
    return _distinct_rows(rows)


def init_kmeans_parallel(X, k: int, seed: int, steps: int, partition_starts,
                         distanceMeasure: str = "euclidean", xnorm=None) -> np.ndarray:
    """KMeans.initKMeansParallel (KMeans.scala:370-432) over the ranks'
    shards: the cost passes, the draws and the candidate counts on each
    rank's device, the sums and counts merged across ranks, the sampling of
    the first center and LocalKMeans on the host (identically on every
    rank, as the reference's driver)."""
    import torch
    from . import parallel
    from .clustering import KMeans, KMeansModel, xorshift_next_int
    sh = _Shards(partition_starts)
    s = xorshift_next_int(seed)
    first = take_sample_indices(sh.lens, 1, s)
    if not first:
        raise N.IllegalArgumentException("requirement failed: No samples available from data")
    centers = [sh.rows_at(X, first)[0]]
    new = np.array(centers)
    costs = None
    total = 0.0
    for step in range(steps):
        if new.shape[0] > 0:       # no new centers: every min(pointCost, cost) is the cost
            costs, total = KMeans.updateParallelCosts(X, new, costs, xnorm=xnorm,
                                                      distanceMeasure=distanceMeasure)
        mask = KMeans.parallelSample(costs, total, s, step, k, sh.local_starts,
                                     sh.first_partition)
        new = sh.concat(X[mask.bool()].cpu().numpy())
        centers.extend(list(new))
    distinct = _distinct_rows(np.array(centers))
    if distinct.shape[0] <= k:
        return distinct
    idx, _ = KMeansModel(distinct, distanceMeasure=distanceMeasure).pointCosts(X, xnorm)
    counts = torch.bincount(idx.long(), minlength=distinct.shape[0]).cpu().numpy()
    counts = np.sum(parallel.allgather_object(counts), axis=0)     # countByValue
    return local_kmeans_pp(distinct, counts.astype(np.float64), k, 30, 0, X.device)


# --------------------------------------------------------------- CSR shards

def csr_rows_dense(rowptr, colidx, values, d: int, rows) -> np.ndarray:
    """Rows of a device CSR shard as dense host rows (a SparseVector's
    toDense; explicit zeros and missing entries both 0.0)."""
    import torch
    rows = torch.as_tensor(np.asarray(rows, dtype=np.int64), device=values.device)
    m = int(rows.numel())
    out = torch.zeros((m, d), dtype=torch.float64, device=values.device)
    if m:
        st, en = rowptr[rows], rowptr[rows + 1]
        lens = en - st
        tot = int(lens.sum().item())
        if tot:
            rid = torch.repeat_interleave(torch.arange(m, device=values.device), lens)
            first = torch.cumsum(lens, 0) - lens
            flat = torch.arange(tot, device=values.device) - first[rid] + st[rid]
            out[rid, colidx[flat].long()] = values[flat]
    return out.cpu().numpy()


def _csr_of_dense(rows: np.ndarray, device):
    """Device CSR of dense rows (their nonzeros)."""
    import torch
    nz = rows != 0.0
    rowptr = np.concatenate([[0], np.cumsum(nz.sum(1))]).astype(np.int64)
    r, c = np.nonzero(nz)
    return (torch.from_numpy(rowptr).to(device),
            torch.from_numpy(c.astype(np.int32)).to(device),
            torch.from_numpy(np.ascontiguousarray(rows[r, c])).to(device))


def init_random_csr(rowptr, colidx, values, d: int, k: int, seed: int,
                    partition_starts) -> np.ndarray:
    """KMeans.initRandom over sparse points (centers dense)."""
    from .clustering import xorshift_next_int
    sh = _Shards(partition_starts)
    idx = take_sample_indices(sh.lens, k, xorshift_next_int(seed))
    return _distinct_rows(sh.rows_of(lambda loc: csr_rows_dense(rowptr, colidx, values, d, loc),
                                     idx, d))


def init_kmeans_parallel_csr(rowptr, colidx, values, d: int, k: int, seed: int, steps: int,
                             partition_starts, xnorm=None,
                             distanceMeasure: str = "euclidean") -> np.ndarray:
    """KMeans.initKMeansParallel (KMeans.scala:370-432) over sparse points:
    as init_kmeans_parallel, the cost passes fastSquaredDistance(center,
    sparse point) on the device (cyc_kmeans_point_cost_csr_dev; dot(sparse,
    sparse) of the reference equals dot(sparse, dense) here, the centers'
    absent entries adding zeros), LocalKMeans over the sparse candidates."""
    import torch
    from . import parallel
    from .clustering import KMeans, KMeansModel, row_norms_csr, xorshift_next_int
    sh = _Shards(partition_starts)
    gather = lambda loc: csr_rows_dense(rowptr, colidx, values, d, loc)   # noqa: E731
    if xnorm is None:
        xnorm = row_norms_csr(rowptr, values)
    s = xorshift_next_int(seed)
    first = take_sample_indices(sh.lens, 1, s)
    if not first:
        raise N.IllegalArgumentException("requirement failed: No samples available from data")
    centers = [sh.rows_of(gather, first, d)[0]]
    new = np.array(centers)
    costs = None
    total = 0.0
    for step in range(steps):
        if new.shape[0] > 0:
            _, c = KMeansModel(new, distanceMeasure=distanceMeasure).pointCosts_csr(
                rowptr, colidx, values, xnorm)
            costs = c if costs is None else torch.minimum(c, costs)
            tot = costs.sum().reshape(1) if costs.numel() else torch.zeros(
                1, dtype=torch.float64, device=values.device)
            parallel.allreduce_(tot)
            total = float(tot.item())
        mask = KMeans.parallelSample(costs, total, s, step, k, sh.local_starts,
                                     sh.first_partition)
        new = sh.concat(gather(torch.nonzero(mask).flatten().cpu().numpy()))
        centers.extend(list(new))
    distinct = _distinct_rows(np.array(centers))
    if distinct.shape[0] <= k:
        return distinct
    idx, _ = KMeansModel(distinct, distanceMeasure=distanceMeasure).pointCosts_csr(
        rowptr, colidx, values, xnorm)
    counts = torch.bincount(idx.long(), minlength=distinct.shape[0]).cpu().numpy()
    counts = np.sum(parallel.allgather_object(counts), axis=0)     # countByValue
    # LocalKMeans is Euclidean whatever the run's measure (LocalKMeans.scala:49)
    cand = _csr_of_dense(distinct, values.device)
    cand_norm = row_norms_csr(cand[0], cand[2])

    def closest(C):
        a, c = KMeansModel(np.asarray(C)).pointCosts_csr(*cand, cand_norm)
        return a.cpu().numpy().astype(np.int64), c.cpu().numpy()

    return local_kmeans_pp(distinct, counts.astype(np.float64), k, 30, 0, values.device,
                           closest=closest)
