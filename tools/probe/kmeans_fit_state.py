#!/usr/bin/env python3
"""Per-iteration carried state of one KMeans fit (bench.py's config 2, from
setInitialModel): bounded calls / screened rows, re-checked rows, and
incremental calls / moved rows, cumulative after each iteration
(CYC_KMEANS_FIT_TRACE=1).  Diagnostics only."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
os.environ["CYC_KMEANS_FIT_TRACE"] = "1"

if __name__ == "__main__":
    import torch
    import bench
    from cycloneml_amd.clustering import KMeans, KMeansModel
    dev = torch.device("cuda", 0)
    X = bench.kmeans_data(10_000_000, dev, 0)
    km = KMeans(k=1024, maxIterations=20, epsilon=1e-4)
    km.setInitialModel(KMeansModel(X[:1024].cpu().numpy()))
    km.run(X)
    prev = None
    for i, t in enumerate(km.lastFitInfo["per_iteration"]):
        row = {"iteration": i + 1, "screened": t["bounds"][1], "rechecked": t["rechecked"],
               "incremental": t["incremental"][0], "moved": t["incremental"][1]}
        if prev:
            row = {k: (v - prev[k] if k != "iteration" else v) for k, v in row.items()}
        prev = {"iteration": 0, "screened": t["bounds"][1], "rechecked": t["rechecked"],
                "incremental": t["incremental"][0], "moved": t["incremental"][1]}
        print(json.dumps(row), flush=True)
