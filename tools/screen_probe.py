"""Time the KMeans screen kernels against k at a fixed row count (bench data
shape, d = 256): separates the one-limb pass's per-center-tile cost from its
per-row-group cost.  Usage: python tools/screen_probe.py [n] [k ...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402
from cycloneml_amd import _native as N  # noqa: E402
from cycloneml_amd.clustering import KMeansPlan, row_norms  # noqa: E402

KERNELS = ("k_kmeans_screen1", "k_kmeans_refine2", "k_kmeans_screen2", "k_kmeans_cands",
           "k_kmeans_screen3", "k_kmeans_compact", "k_chunk_sums")


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4_000_000
    ks = [int(a) for a in sys.argv[2:]] or [256, 512, 1024, 2048]
    dev = torch.device("cuda:0")
    d = 256
    for k in ks:
        X = bench.kmeans_data(n, dev, 0, d=d, k=k)
        C = X[:k].clone()
        cnorm = row_norms(C)
        xnorm = row_norms(X)
        plan = KMeansPlan(d, k, n)
        rows = plan.rows(X)
        buf = torch.zeros(k * d + k + 1, dtype=torch.float64, device=dev)
        conv = torch.zeros(1, dtype=torch.int32, device=dev)

        def step():
            buf.zero_()
            sums, wsum, cost = buf[:k * d], buf[k * d:k * d + k], buf[k * d + k:]
            plan.accumulate(X, xnorm, None, C, cnorm, sums, wsum, cost, rows=rows)
            plan.update(C, cnorm, sums, wsum, 1e-4, conv)

        for _ in range(3):
            step()
        torch.cuda.synchronize()
        N.profile_enable(True)
        for kn in KERNELS:
            N.profile_query(kn)
        steps = 5
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        prof = {kn: N.profile_query(kn) for kn in KERNELS}
        N.profile_enable(False)
        line = " ".join(f"{kn[9:]}={prof[kn][0] / steps:.3f}" for kn in KERNELS if prof[kn][1])
        print(f"n={n} k={k} {line} refine={plan.last_refine()}", flush=True)
        del X, C, rows, plan, buf
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
