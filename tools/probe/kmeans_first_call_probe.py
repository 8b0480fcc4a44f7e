#!/usr/bin/env python3
"""Host time of each KMeansPlan.accumulate call (enqueue only) vs the
iteration's wall time, for the first iterations of a fit: where the first
iteration's extra milliseconds go (allocations, pinned host buffers, syncs)."""
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
    xn = row_norms(X)
    for fit in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        p = KMeansPlan(d, k, n)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        rows = p.rows(X)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"fit {fit}: plan {1e3 * (t1 - t0):.3f} ms, rows {1e3 * (t2 - t1):.3f} ms", flush=True)
        C = C0.clone()
        cn = row_norms(C)
        buf = torch.zeros(k * d + k + 1, dtype=torch.float64, device=dev)
        sums, wsum, cost = buf[:k * d], buf[k * d:k * d + k], buf[k * d + k:]
        conv = torch.zeros(1, dtype=torch.int32, device=dev)
        for it in range(4):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            buf.zero_()
            p.accumulate(X, xn, None, C, cn, sums, wsum, cost, rows=rows)
            t1 = time.perf_counter()
            p.update(C, cn, sums, wsum, 1e-4, conv)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            print(f"fit {fit} it {it}: accumulate host {1e3 * (t1 - t0):.3f} ms, wall {1e3 * (t2 - t0):.3f} ms",
                  flush=True)
        rows.close()
        p.close()


if __name__ == "__main__":
    main()
