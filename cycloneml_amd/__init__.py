"""cycloneml_amd -- MI355X (gfx950) backend for the MLlib linear-algebra hot
path of wmeddie/CycloneML: KMeans findClosest/cluster sums, the logistic
block aggregators, RowMatrix Gramian/covariance, and the treeAggregate merge
as an RCCL all-reduce.  Kernels live in libcyclone.so (csrc/, C ABI in
include/cyclone.h); these modules mirror the reference's Scala interfaces.
"""
__version__ = "0.1.0"

from . import _native  # noqa: F401  (loads nothing until first use)
