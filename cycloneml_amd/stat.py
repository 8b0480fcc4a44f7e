"""Device-resident Summarizer pre-pass (org.apache.spark.ml.stat on MI355X).

Mirrors, over device-resident rows (a DeviceInstanceBlock or a dense tensor):
  SummarizerBuffer              ml/stat/Summarizer.scala:428-770
  MultiClassSummarizer          ml/stat/MultiClassSummarizer.scala:30-98
  getClassificationSummarizers  Summarizer.scala:228-241, the first pass of
                                LogisticRegression.train (:511-516)
  standardize_                  the StandardScaler transform of trainImpl
                                (LogisticRegression.scala:957-965,
                                StandardScaler.scala:261-283)
The arithmetic runs in libcyclone (csrc/summarizer.hip); this module holds the
device buffers and reads the metrics back.  A shard is cut into partitions
(`rows_per_partition` dense rows, or the CSC copy's row blocks for CSR); the
partition buffers merge in order, and across ranks the finished buffers are
all-gathered and merged in rank order (treeAggregate's combOp) -- merge is not
a sum, so it is not an all-reduce.
"""
from __future__ import annotations

import math

import numpy as np

from . import _native as N

FIELDS = 8
SCALARS = 5
DEFAULT_ROWS_PER_PARTITION = 1 << 15
METRICS = ("mean", "variance", "std", "sum", "numNonzeros", "max", "min", "normL2", "normL1")


def _torch():
    import torch
    return torch


def _jstr(x: float) -> str:
    """Scala's Double.toString, for the require messages."""
    if math.isnan(x):
        return "NaN"
    if math.isinf(x):
        return "Infinity" if x > 0 else "-Infinity"
    return repr(float(x))


def _require(cond, msg):
    if not cond:
        raise N.IllegalArgumentException("requirement failed: " + msg)


def _dist():
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return dist
    except Exception:
        pass
    return None


class SummarizerBuffer:
    """A finished SummarizerBuffer in HBM (8 x F state + 5 scalars)."""

    def __init__(self, buf, numFeatures: int):
        self.buf = buf
        self.n = int(numFeatures)
        self._scal = None
        self._met = None

    @staticmethod
    def _empty(F, device):
        torch = _torch()
        return torch.empty(FIELDS * F + SCALARS, dtype=torch.float64, device=device)

    @classmethod
    def of_dense(cls, X, weights=None, rows_per_partition=DEFAULT_ROWS_PER_PARTITION,
                 stream=None):
        n, F = int(X.shape[0]), int(X.shape[1])
        buf = cls._empty(F, X.device)
        N.check(N.load().cyc_summarizer_dense_dev(N.ptr(X), N.ptr(weights), n, F,
                                                  int(rows_per_partition), N.ptr(buf),
                                                  N.stream_handle(stream)))
        return cls(buf, F)

    @classmethod
    def of_block(cls, block, rows_per_partition=DEFAULT_ROWS_PER_PARTITION, stream=None):
        """Dense blocks: partitions of rows_per_partition rows.  CSR blocks:
        the row blocks of the block's CSC copy (built here if missing)."""
        if not block.is_sparse:
            return cls.of_dense(block.X, block.weights, rows_per_partition, stream)
        block.prepare(stream)
        buf = cls._empty(block.numFeatures, block.labels.device)
        N.check(N.load().cyc_summarizer_csr_dev(block.csc, N.ptr(block.weights), N.ptr(buf),
                                                N.stream_handle(stream)))
        return cls(buf, block.numFeatures)

    def merge(self, other: "SummarizerBuffer", stream=None) -> "SummarizerBuffer":
        """this.merge(other) (:562-617) as a new buffer."""
        _require(self.n == other.n, "Dimensions mismatch when merging with another "
                 f"summarizer. Expecting {self.n} but got {other.n}.")
        torch = _torch()
        both = torch.stack([self.buf, other.buf])
        out = self._empty(self.n, self.buf.device)
        N.check(N.load().cyc_summarizer_merge_dev(self.n, N.ptr(both), 2, N.ptr(out),
                                                  N.stream_handle(stream)))
        return SummarizerBuffer(out, self.n)

    def allgather_merge(self, group=None) -> "SummarizerBuffer":
        """The ranks' buffers merged in rank order (treeAggregate's combOp)."""
        dist = _dist()
        if dist is None or dist.get_world_size(group) == 1:
            return self
        torch = _torch()
        ws = dist.get_world_size(group)
        parts = [torch.empty_like(self.buf) for _ in range(ws)]
        dist.all_gather(parts, self.buf, group=group)
        stacked = torch.stack(parts)
        out = self._empty(self.n, self.buf.device)
        N.check(N.load().cyc_summarizer_merge_dev(self.n, N.ptr(stacked), ws, N.ptr(out),
                                                  N.stream_handle()))
        return SummarizerBuffer(out, self.n)

    # -- metrics -------------------------------------------------------------
    def _scalars(self):
        if self._scal is None:
            s = self.buf[FIELDS * self.n:].cpu().numpy()
            if s[3] != 0.0:
                raise N.IllegalArgumentException(
                    f"requirement failed: sample weight, {_jstr(s[4])} has to be >= 0.0")
            self._scal = s
        return self._scal

    def _metrics(self):
        if self._met is None:
            torch = _torch()
            out = torch.empty(9 * self.n, dtype=torch.float64, device=self.buf.device)
            N.check(N.load().cyc_summarizer_metrics_dev(self.n, N.ptr(self.buf), N.ptr(out),
                                                        N.stream_handle()))
            self._met = out.cpu().numpy().reshape(9, self.n)
        return self._met

    def _weighted(self, name):
        _require(self._scalars()[1] > 0, "Nothing has been added to this summarizer.")
        return self._metrics()[METRICS.index(name)].copy()

    @property
    def count(self) -> int:
        return int(self._scalars()[0])

    @property
    def weightSum(self) -> float:
        return float(self._scalars()[1])

    @property
    def mean(self):
        return self._weighted("mean")

    @property
    def variance(self):
        return self._weighted("variance")

    @property
    def std(self):
        return self._weighted("std")

    @property
    def sum(self):
        return self._weighted("sum")

    @property
    def numNonzeros(self):
        _require(self.count > 0, "Nothing has been added to this summarizer.")
        return self._metrics()[METRICS.index("numNonzeros")].copy()

    @property
    def max(self):
        return self._weighted("max")

    @property
    def min(self):
        return self._weighted("min")

    @property
    def normL2(self):
        return self._weighted("normL2")

    @property
    def normL1(self):
        return self._weighted("normL1")


class MultiClassSummarizer:
    """MultiClassSummarizer (MultiClassSummarizer.scala:30-98) of device labels."""

    MAX_CLASSES = 8192

    def __init__(self, histogram, invalid: int):
        self._hist = np.asarray(histogram, dtype=np.float64)
        self._invalid = int(invalid)

    @classmethod
    def of_labels(cls, labels, weights=None, rows_per_partition=DEFAULT_ROWS_PER_PARTITION,
                  max_classes=1024, stream=None):
        torch = _torch()
        lib = N.load()
        dev = labels.device
        n = int(labels.shape[0])
        inv = torch.zeros(1, dtype=torch.int64, device=dev)
        mx = torch.zeros(1, dtype=torch.int32, device=dev)
        maxc = int(max_classes)
        while True:
            hist = torch.empty(maxc, dtype=torch.float64, device=dev)
            N.check(lib.cyc_label_summarizer_dev(N.ptr(labels), N.ptr(weights), n,
                                                 int(rows_per_partition), maxc, N.ptr(hist),
                                                 N.ptr(inv), N.ptr(mx), N.stream_handle(stream)))
            m = int(mx.item())
            if m < maxc:
                break
            if m + 1 > cls.MAX_CLASSES:
                raise N.CycloneError(N.CYC_ERR_UNSUPPORTED,
                                     f"more than {cls.MAX_CLASSES} classes on the device path")
            maxc = m + 1
        return cls(hist[:m + 1].cpu().numpy(), int(inv.item()))

    def merge(self, other: "MultiClassSummarizer") -> "MultiClassSummarizer":
        """merge (:66-79): per-class weight sums add up, invalid counts add up."""
        n = max(len(self._hist), len(other._hist))
        h = np.zeros(n)
        h[:len(self._hist)] += self._hist
        h[:len(other._hist)] += other._hist
        return MultiClassSummarizer(h, self._invalid + other._invalid)

    def allgather_merge(self, group=None) -> "MultiClassSummarizer":
        dist = _dist()
        if dist is None or dist.get_world_size(group) == 1:
            return self
        parts = [None] * dist.get_world_size(group)
        dist.all_gather_object(parts, (self._hist.tolist(), self._invalid), group=group)
        acc = MultiClassSummarizer(np.array(parts[0][0]), parts[0][1])
        for h, i in parts[1:]:
            acc = acc.merge(MultiClassSummarizer(np.array(h), i))
        return acc

    @property
    def countInvalid(self) -> int:
        return self._invalid

    @property
    def numClasses(self) -> int:
        return len(self._hist)

    @property
    def histogram(self):
        return self._hist.copy()


def getClassificationSummarizers(blocks, rows_per_partition=DEFAULT_ROWS_PER_PARTITION,
                                 group=None):
    """(SummarizerBuffer, MultiClassSummarizer) over the shard's blocks, merged
    in block order and then across ranks (Summarizer.scala:228-241)."""
    summ = lab = None
    for b in blocks:
        s = SummarizerBuffer.of_block(b, rows_per_partition)
        m = MultiClassSummarizer.of_labels(b.labels, b.weights, rows_per_partition)
        summ = s if summ is None else summ.merge(s)
        lab = m if lab is None else lab.merge(m)
    return summ.allgather_merge(group), lab.allgather_merge(group)


def standardize_(block, inverseStd, stream=None):
    """In-place StandardScaler transform with scale = inverseStd and no shift
    (LogisticRegression.scala:962-965): dense values(i) *= scale(i), CSR
    values(k) *= scale(indices(k)).  A CSC copy built before is dropped."""
    torch = _torch()
    dev = block.labels.device
    s = torch.as_tensor(np.ascontiguousarray(inverseStd, dtype=np.float64), device=dev)
    _require(int(s.shape[0]) == block.numFeatures, "scale size must equal numFeatures")
    lib = N.load()
    if block.is_sparse:
        N.check(lib.cyc_scale_columns_csr_dev(N.ptr(block.colidx), N.ptr(block.values),
                                              int(block.values.shape[0]), N.ptr(s),
                                              N.stream_handle(stream)))
        block.drop_derived()
    else:
        N.check(lib.cyc_scale_columns_dense_dev(N.ptr(block.X), block.size, block.numFeatures,
                                                N.ptr(s), N.stream_handle(stream)))
    return block
