#!/usr/bin/env python3
"""One KMeans fit (bench.py's config 2, from setInitialModel) and nothing
else, for a kernel trace of its iterations (tools/km_fit_trace.sh)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

if __name__ == "__main__":
    import torch
    import bench
    dev = torch.device("cuda", 0)
    wl = bench.KMeansWorkload(10_000_000, dev, 0)
    torch.cuda.synchronize()
    print(wl.fit_once()["iteration_ms"], flush=True)
