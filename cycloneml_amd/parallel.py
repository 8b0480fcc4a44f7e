"""The aggregation step across GPUs.

The reference merges per-partition results with RDD.treeAggregate /
reduceByKey + collectAsMap and a DoubleAccumulator (core/.../rdd/RDD.scala:
1210-1269, PairRDDFunctions.scala:322, KMeans.scala:308-311), and ships the
model with TorrentBroadcast.  Here every GPU is one process holding a
contiguous shard of the rows (its Spark partitions); each iteration the
ranks all-reduce ONE flat fp64 buffer of aggregator state and broadcast the
model once at start.  There is no other exchange on the data path.

On GPUs the collective is libcyclone's own C-ABI communicator over RCCL
(`Communicator`, cyc_comm_* in include/cyclone.h -- the same entry points a
JVM executor-per-GPU binds), created by `init()` once torch.distributed is
up.  torch.distributed itself runs on gloo (host only: the rendezvous, the
128-byte RCCL id, barriers and small host gathers), so each GPU holds ONE
RCCL communicator.  Without `init()` (the CPU multi-process tests, the
two-ranks-on-one-GPU device tests) the same functions use the gloo group.
"""
from __future__ import annotations

import ctypes

_comm = None          # the process's Communicator (RCCL), once init() ran


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


class Communicator:
    """RAII wrapper of cyc_comm: one RCCL communicator per process (GPU)."""

    ID_BYTES = 128

    @staticmethod
    def unique_id() -> bytes:
        from . import _native as N
        buf = ctypes.create_string_buffer(Communicator.ID_BYTES)
        N.check(N.load().cyc_comm_unique_id(buf))
        return buf.raw

    def __init__(self, uid: bytes, rank: int, world_size: int, device: int):
        from . import _native as N
        if len(uid) != self.ID_BYTES:
            raise N.IllegalArgumentException(
                f"requirement failed: the RCCL id has {self.ID_BYTES} bytes, got {len(uid)}")
        self._N = N
        self._lib = N.load()
        h = ctypes.c_void_p()
        N.check(self._lib.cyc_comm_init(uid, int(rank), int(world_size), int(device),
                                        ctypes.byref(h)))
        self.handle = h
        self.rank, self.world_size, self.device = int(rank), int(world_size), int(device)

    def close(self):
        if getattr(self, "handle", None):
            self._lib.cyc_comm_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, t):
        import torch
        if t.dtype != torch.float64 or not t.is_cuda or not t.is_contiguous():
            raise self._N.IllegalArgumentException(
                "requirement failed: the collective takes a contiguous fp64 device tensor")

    def allreduce_sum_(self, t, stream=None):
        self._check(t)
        self._N.check(self._lib.cyc_allreduce_sum_dev(self.handle, self._N.ptr(t), t.numel(),
                                                      self._N.stream_handle(stream)))
        return t

    def allreduce_max_(self, t, stream=None):
        self._check(t)
        self._N.check(self._lib.cyc_allreduce_max_dev(self.handle, self._N.ptr(t), t.numel(),
                                                      self._N.stream_handle(stream)))
        return t

    def broadcast_(self, t, root=0, stream=None):
        self._check(t)
        self._N.check(self._lib.cyc_broadcast_dev(self.handle, self._N.ptr(t), t.numel(),
                                                  int(root), self._N.stream_handle(stream)))
        return t

    def allgather(self, t, out=None, stream=None):
        """out[r] = rank r's t (shape (world, *t.shape))."""
        import torch
        self._check(t)
        if out is None:
            out = torch.empty((self.world_size,) + tuple(t.shape), dtype=t.dtype,
                              device=t.device)
        self._N.check(self._lib.cyc_allgather_dev(self.handle, self._N.ptr(t), self._N.ptr(out),
                                                  t.numel(), self._N.stream_handle(stream)))
        return out


def init(device=None, communicator=Communicator):
    """Create the process's RCCL communicator (one per GPU) from the running
    torch.distributed group, which only carries rank 0's 128-byte RCCL id to
    every rank (a host tensor over gloo -- bench.py's group -- or a device
    tensor over an "nccl" group).  A no-op for world size 1.  `communicator`
    is the class built from (id, rank, world, device index) -- the tests of
    the rendezvous pass a host stand-in.  Returns it, or None."""
    global _comm
    import torch
    d = _dist()
    if d is None or d.get_world_size() == 1:
        return None
    if _comm is not None:
        return _comm
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else device
    uid = torch.zeros(communicator.ID_BYTES, dtype=torch.uint8,
                      device=dev if d.get_backend() == "nccl" else "cpu")
    if d.get_rank() == 0:
        uid.copy_(torch.frombuffer(bytearray(communicator.unique_id()), dtype=torch.uint8))
    d.broadcast(uid, 0)
    _comm = communicator(bytes(uid.cpu().numpy().tobytes()), d.get_rank(), d.get_world_size(),
                         dev.index if dev.index is not None else torch.cuda.current_device())
    return _comm


def shutdown():
    global _comm
    if _comm is not None:
        _comm.close()
        _comm = None


def communicator():
    return _comm


def allreduce_(buf, group=None):
    """Sum `buf` (a flat fp64 tensor of aggregator state) over all ranks in
    place.  One collective per iteration replaces treeAggregate's tree of
    shuffles and the driver fold."""
    import torch
    if _comm is not None and group is None and buf.dtype == torch.float64 and buf.is_cuda:
        return _comm.allreduce_sum_(buf)
    d = _dist()
    if d is not None and d.get_world_size() > 1:
        d.all_reduce(buf, group=group)
    return buf


def broadcast_(t, src=0, group=None):
    """TorrentBroadcast of the model (centers / coefficients) from `src`."""
    import torch
    if _comm is not None and group is None and t.dtype == torch.float64 and t.is_cuda:
        return _comm.broadcast_(t, src)
    d = _dist()
    if d is not None and d.get_world_size() > 1:
        d.broadcast(t, src, group=group)
    return t


def allgather_object(obj) -> list:
    """Every rank's `obj` in rank order (the driver's `collect()` of small
    host data: partition lengths, sampled candidate rows, counts)."""
    d = _dist()
    if d is None or d.get_world_size() == 1:
        return [obj]
    out = [None] * d.get_world_size()
    d.all_gather_object(out, obj)
    return out


def agree(fn):
    """Run fn() on every rank and agree on failure before any collective that
    depends on it: when fn raised on some rank, every rank raises the lowest
    such rank's error (same class for the reference's require / assert, same
    message) -- a failing Spark task fails the whole job with one exception,
    where a lone raising rank would leave the others blocked in the next
    all-reduce.  Returns fn()'s result."""
    from . import _native as N
    err, out = None, None
    try:
        out = fn()
    except Exception as e:  # every rank must reach the gather below
        err = e
    d = _dist()
    if d is None or d.get_world_size() == 1:
        if err is not None:
            raise err
        return out
    mine = None if err is None else (type(err).__name__, str(err))
    first = next((g for g in allgather_object(mine) if g is not None), None)
    if first is None:
        return out
    if err is not None and mine == first:
        raise err
    kinds = {"IllegalArgumentException": N.IllegalArgumentException,
             "JavaAssertionError": N.JavaAssertionError}
    raise kinds.get(first[0], RuntimeError)(first[1])


def max_over_ranks(x: float, device=None) -> float:
    import torch
    d = _dist()
    if d is None or d.get_world_size() == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    if _comm is not None and t.is_cuda:
        _comm.allreduce_max_(t)
    else:
        d.all_reduce(t, op=d.ReduceOp.MAX)
    return float(t.item())
