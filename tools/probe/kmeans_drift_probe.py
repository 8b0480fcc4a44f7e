#!/usr/bin/env python3
"""Center drift per Lloyd iteration on bench.py's KMeans config (10M x 256,
k = 1024, initial centers rows 0..k-1): for iterations 1..25, the largest
and the quantiles of |c_j(t+1) - c_j(t)|, and the fraction of rows whose
one-limb-screen certification margin would survive that drift (from the
fp64 distances of a 200K-row sample: the gap between the best and second
best distance against twice the largest drift), and the fraction of the
sample whose closest center changed since the previous iteration (what an
incremental cluster-sum update would have to touch).  One JSON line per
iteration."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from cycloneml_amd.clustering import KMeansPlan, row_norms
    dev = torch.device("cuda", 0)
    n, d, k = 10_000_000, 256, 1024
    X = bench.kmeans_data(n, dev, 0, d, k)
    C = X[:k].clone()
    cn = row_norms(C)
    xn = row_norms(X)
    plan = KMeansPlan(d, k, n)
    rows = plan.rows(X)
    buf = torch.zeros(k * d + k + 1, dtype=torch.float64, device=dev)
    conv = torch.zeros(1, dtype=torch.int32, device=dev)
    S = X[:: n // 200_000][:200_000]
    prev = None
    for it in range(1, 26):
        # the sample's best / second-best distances to the current centers
        D = torch.cdist(S, C)                       # fp64 distances
        two = torch.topk(D, 2, dim=1, largest=False).values
        gap = (two[:, 1] - two[:, 0])
        best = torch.argmin(D, dim=1)
        moved = float((best != prev).double().mean()) if prev is not None else 1.0
        prev = best
        Cold = C.clone()
        buf.zero_()
        plan.accumulate(X, xn, None, C, cn, buf[:k * d], buf[k * d:k * d + k], buf[k * d + k:],
                        rows=rows)
        plan.update(C, cn, buf[:k * d], buf[k * d:k * d + k], 1e-4, conv)
        drift = (C - Cold).norm(dim=1)
        q = torch.quantile(drift, torch.tensor([0.5, 0.9, 0.99], dtype=torch.float64,
                                               device=dev)).tolist()
        dmax = float(drift.max())
        surv = {f"gap>{m}x": float((gap > m * dmax).double().mean()) for m in (2, 4, 8)}
        print(json.dumps({"iteration": it, "drift_max": dmax, "drift_q50_q90_q99": q,
                          "gap_q10_q50": torch.quantile(gap, torch.tensor(
                              [0.1, 0.5], dtype=torch.float64, device=dev)).tolist(),
                          "moved": moved, **surv}), flush=True)


if __name__ == "__main__":
    main()
