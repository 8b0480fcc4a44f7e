"""The aggregation step across GPUs.

The reference merges per-partition results with RDD.treeAggregate /
reduceByKey + collectAsMap and a DoubleAccumulator (core/.../rdd/RDD.scala:
1210-1269, PairRDDFunctions.scala:322, KMeans.scala:308-311), and ships the
model with TorrentBroadcast.  Here every GPU is one process holding a
contiguous shard of the rows (its Spark partitions); each iteration the
ranks all-reduce ONE flat fp64 buffer of aggregator state over RCCL
(torch.distributed backend "nccl") and broadcast the model once at start.
There is no other exchange on the data path.  The same functions run on the
gloo backend for the CPU multi-process tests.
"""
from __future__ import annotations


def _dist():
    import torch
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        return torch.distributed
    return None


def world():
    d = _dist()
    return (d.get_rank(), d.get_world_size()) if d else (0, 1)


def shard_bounds(n: int, rank: int, world_size: int):
    """Contiguous row range of `rank` (balanced to within one row)."""
    q, r = divmod(n, world_size)
    start = rank * q + min(rank, r)
    return start, start + q + (1 if rank < r else 0)


def allreduce_(buf, group=None):
    """Sum `buf` (a flat fp64 tensor of aggregator state) over all ranks in
    place.  One collective per iteration replaces treeAggregate's tree of
    shuffles and the driver fold."""
    d = _dist()
    if d is not None and d.get_world_size() > 1:
        d.all_reduce(buf, group=group)
    return buf


def broadcast_(t, src=0, group=None):
    """TorrentBroadcast of the model (centers / coefficients) from `src`."""
    d = _dist()
    if d is not None and d.get_world_size() > 1:
        d.broadcast(t, src, group=group)
    return t


def max_over_ranks(x: float, device=None) -> float:
    import torch
    d = _dist()
    if d is None or d.get_world_size() == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    d.all_reduce(t, op=d.ReduceOp.MAX)
    return float(t.item())
