#!/usr/bin/env python3
"""Where a KMeans fit's first iteration goes (bench.py's rows, config 2):
the cached norms, the plan, the row image, then each Lloyd iteration, each
timed between device synchronisations; twice in one process (the second fit
finds the device allocator warm)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from cycloneml_amd.clustering import KMeansPlan, row_norms
    dev = torch.device("cuda", 0)
    n, d, k = 10_000_000, 256, 1024
    X = bench.kmeans_data(n, dev, 0, d, k)
    C0 = X[:k].clone()
    for fit in range(2):
        t = {}
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        xn = row_norms(X)
        torch.cuda.synchronize()
        t["norms"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        p = KMeansPlan(d, k, n)
        torch.cuda.synchronize()
        t["plan"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        rows = p.rows(X)
        torch.cuda.synchronize()
        t["image"] = time.perf_counter() - t0
        C = C0.clone()
        cn = row_norms(C)
        buf = torch.zeros(k * d + k + 1, dtype=torch.float64, device=dev)
        sums, wsum, cost = buf[:k * d], buf[k * d:k * d + k], buf[k * d + k:]
        conv = torch.zeros(1, dtype=torch.int32, device=dev)
        its = []
        for it in range(20):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            buf.zero_()
            p.accumulate(X, xn, None, C, cn, sums, wsum, cost, rows=rows)
            p.update(C, cn, sums, wsum, 1e-4, conv)
            conv.item()
            its.append(round((time.perf_counter() - t0) * 1e3, 3))
        out = {k_: round(v * 1e3, 3) for k_, v in t.items()}
        out["fit"] = fit
        out["iterations_ms"] = its
        out["total_ms"] = round(sum(out[k_] for k_ in ("norms", "plan", "image")) + sum(its), 3)
        print(json.dumps(out), flush=True)
        rows.close()
        p.close()


if __name__ == "__main__":
    main()
