#!/usr/bin/env python3
"""Does a second read of the sparse tiles layout come from the Infinity Cache?

Builds config 5's rows (bench.lr_sparse_chunks) at several shard sizes and
times repeated BinaryLogisticBlockAggregator evaluations: per launch of
k_tiles_margin / k_tiles_grad, ns per 1000 rows.  Shards of <= ~200 MB of
layout stay resident in the 256 MiB Infinity Cache across evaluations; the
large ones stream from HBM.  Prints one JSON line per size."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import bench
    from cycloneml_amd import _native as N
    from cycloneml_amd.optim import (BinaryLogisticBlockAggregator, DeviceInstanceBlock,
                                     SparseTiles)
    dev = torch.device("cuda", 0)
    F, k = 1_000_000, 64
    sizes = [int(s) for s in (sys.argv[1:] or ["65536", "131072", "262144", "1048576",
                                                 "8388608"])]
    coef = np.random.default_rng(4).normal(size=F + 1) * 0.01
    sm = torch.as_tensor(np.random.default_rng(5).uniform(0.0, 0.014, F), device=dev)
    for n in sizes:
        tiles = SparseTiles(F, n, n * k)
        y = torch.empty(n, dtype=torch.float64, device=dev)
        for s, e, rp, ci, vv, yc in bench.lr_sparse_chunks(n, dev, 0, F, k):
            y[s:e] = yc
            tiles.append(rp, ci, vv)
        blk = DeviceInstanceBlock(y, None, tiles=tiles, numFeatures=F)
        agg = lambda: BinaryLogisticBlockAggregator(np.ones(F), sm, True, True, coef,
                                                    device=dev).add(blk)
        for _ in range(3):
            agg()
        torch.cuda.synchronize()
        N.profile_enable(True)
        for kn in ("k_tiles_margin", "k_tiles_grad"):
            N.profile_query(kn)
        reps = max(5, min(200, int(2e8 // n)))
        t0 = time.perf_counter()
        for _ in range(reps):
            agg()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        out = {"lib": os.environ.get("PROBE_LIB", "in-tree"), "rows": n,
               "layout_MB": tiles.nbytes / 1e6, "reps": reps,
               "eval_us": el / reps * 1e6}
        for kn in ("k_tiles_margin", "k_tiles_grad"):
            ms, cnt = N.profile_query(kn)
            us = ms / max(cnt, 1) * 1e3
            out[kn + "_us"] = us
            out[kn + "_GBps"] = tiles.nbytes / (us * 1e-6) / 1e9
        N.profile_enable(False)
        print(json.dumps(out), flush=True)
        del blk, tiles, y
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
