"""Process-wide knobs of this build ("Config / flags").

The reference's own parameters keep their names and meaning on the classes
that mirror it (maxBlockSizeInMB, aggregationDepth, maxIter, tol, ...).  Two
environment knobs are this build's own:

- ``CYCLONE_DEVICES``: a comma list of device ordinals for this node's ranks.
  The rank with ``LOCAL_RANK`` i uses the i-th entry; the default is
  ``LOCAL_RANK`` itself, one process per GPU.
- ``CYCLONE_STRICT_PARITY=1``: every KMeans call recomputes from scratch: no
  carried bounds, neighbourhood re-checks or incremental cluster sums
  (libcyclone reads the variable itself, as ``CYC_KMEANS_BOUNDS=0`` /
  ``CYC_KMEANS_NBR=0`` / ``CYC_KMEANS_INCR=0`` would).  RowMatrix.computeCovariance always takes the centred syrk.
  Assignments and costs are bit-exact either way.  Strict mode makes the
  sums and the covariance independent of the fit's history and of the form
  choice.

Block sizes: the reference's knob is ``maxBlockSizeInMB`` (InstanceBlock,
``ml/param/shared/sharedParams.scala:570``); ``optim.blokify`` honours it.
"""
import os


def strict_parity() -> bool:
    return os.environ.get("CYCLONE_STRICT_PARITY", "0") not in ("", "0")


def devices():
    """The ordinals CYCLONE_DEVICES lists (None: unset)."""
    v = os.environ.get("CYCLONE_DEVICES", "").strip()
    if not v:
        return None
    out = [int(x) for x in v.split(",") if x.strip()]
    if not out or any(d < 0 for d in out):
        raise ValueError(f"CYCLONE_DEVICES must list device ordinals, got {v!r}")
    return out


def device_for_local_rank(local_rank: int) -> int:
    """The device ordinal rank LOCAL_RANK = local_rank uses."""
    devs = devices()
    if devs is None:
        return int(local_rank)
    if not 0 <= local_rank < len(devs):
        raise ValueError(f"LOCAL_RANK {local_rank} has no entry in CYCLONE_DEVICES={devs}")
    return devs[local_rank]
