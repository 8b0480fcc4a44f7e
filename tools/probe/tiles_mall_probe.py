#!/usr/bin/env python3
"""Does a second read of the sparse tiles layout come from the Infinity Cache?

Round 4 timed both passes of the BinaryLogisticBlockAggregator on layouts of
config 5's rows at 65K-67M rows: a layout small enough for the 256 MiB
Infinity Cache gave each workgroup only ~32 steps and a few workgroups, so
launch and ramp decided.  Round 6 measures at FULL occupancy with hundreds of
steps per workgroup: the library built with tiles.hip's probe bit 64
(tools/bin/mall/libcyclone.so, loaded through CYC_LIB_DIR) runs the margin
pass on one workgroup per CU, each taking CYC_TILES_REPS super blocks modulo
the layout's, and the gradient pass walking its row range CYC_TILES_REPS
times.  So a ~150 MB layout (resident) and a multi-GB one (streamed from HBM)
are compared per STEP (one segment per wave, one barrier): if a cached step
is not faster, a windowed single-read evaluation cannot pay.

usage: CYC_LIB_DIR=tools/bin/mall python tools/probe/tiles_mall_probe.py \\
           ROWS:MARGIN_REPS:GRAD_REPS ...
Prints one JSON line per case."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

NB = 6                      # tiles.hip CYC_TILES_NB
MW = 8                      # row blocks per margin super block
ROW_BLOCK = 2048


def main():
    import numpy as np
    import torch
    import bench
    from cycloneml_amd import _native as N
    from cycloneml_amd.optim import (BinaryLogisticBlockAggregator, DeviceInstanceBlock,
                                     SparseTiles)
    dev = torch.device("cuda", 0)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    F, k = 1_000_000, 64
    T = -(-F // 2046)
    Tp = -(-T // NB) * NB
    cases = sys.argv[1:] or ["229376:2:20", "16777216:4:1"]
    coef = np.random.default_rng(4).normal(size=F + 1) * 0.01
    sm = torch.as_tensor(np.random.default_rng(5).uniform(0.0, 0.014, F), device=dev)
    for case in cases:
        n, mreps, greps = (int(x) for x in case.split(":"))
        tiles = SparseTiles(F, n, n * k)
        y = torch.empty(n, dtype=torch.float64, device=dev)
        for s, e, rp, ci, vv, yc in bench.lr_sparse_chunks(n, dev, 0, F, k):
            y[s:e] = yc
            tiles.append(rp, ci, vv)
        blk = DeviceInstanceBlock(y, None, tiles=tiles, numFeatures=F)
        nRB = -(-n // ROW_BLOCK)
        sts = -(-T // 8)
        ranges = max(1, min(nRB, cus // sts))
        span = nRB // ranges
        out = {"lib": os.environ.get("CYC_LIB_DIR", "in-tree"), "rows": n,
               "layout_MB": tiles.nbytes / 1e6, "format": tiles.format, "cus": cus}
        for kn, reps in (("k_tiles_margin", mreps), ("k_tiles_grad", greps)):
            os.environ["CYC_TILES_REPS"] = str(reps)
            agg = lambda: BinaryLogisticBlockAggregator(np.ones(F), sm, True, True, coef,
                                                        device=dev).add(blk)
            for _ in range(2):
                agg()
            torch.cuda.synchronize()
            N.profile_enable(True)
            N.profile_query(kn)
            t0 = time.perf_counter()
            R = 5
            for _ in range(R):
                agg()
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            ms, cnt = N.profile_query(kn)
            N.profile_enable(False)
            us = ms / max(cnt, 1) * 1e3
            if kn == "k_tiles_margin":
                steps = reps * Tp                                   # per workgroup
                bytes_read = tiles.nbytes * reps * cus / max(-(-nRB // MW), 1)
            else:
                steps = -(-span * reps // NB) * NB
                bytes_read = tiles.nbytes * reps
            out[kn] = {"reps": reps, "us_per_launch": us, "steps_per_workgroup": steps,
                       "us_per_step": us / steps, "eval_ms": el / R * 1e3,
                       "GBps_of_layout_reads": bytes_read / (us * 1e-6) / 1e9}
        print(json.dumps(out), flush=True)
        del blk, tiles, y
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
