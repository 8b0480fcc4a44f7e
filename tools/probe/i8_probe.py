#!/usr/bin/env python3
"""Tier counts of the i8 screen on small synthetic shapes (diagnostic)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    from cycloneml_amd.clustering import KMeansPlan, row_norms
    dev = torch.device("cuda:0")
    os.environ["CYC_KMEANS_ASSIGN"] = "2"
    for n, d, k in [(1000, 96, 1), (1000, 96, 5), (1000, 64, 1), (1000, 128, 1), (1000, 96, 40),
                    (1000, 32, 1), (1000, 256, 1), (1000, 256, 2)]:
        rng = np.random.default_rng(n + 5 * d + k)
        true_c = rng.normal(scale=4.0, size=(k, d))
        X = true_c[rng.integers(0, k, n)] + rng.normal(size=(n, d))
        C = true_c + rng.normal(scale=0.1, size=true_c.shape)
        Xd, Cd = torch.from_numpy(X).to(dev), torch.from_numpy(C).to(dev)
        xn, cn = row_norms(Xd), row_norms(Cd)
        p = KMeansPlan(d, k, n)
        p.stats(Cd)
        rows = p.rows(Xd)
        a = torch.empty(n, dtype=torch.int32, device=dev)
        c = torch.empty(n, dtype=torch.float64, device=dev)
        ne = p.assign(Xd, xn, Cd, cn, a, c, count_exact=True, rows=rows)
        print(n, d, k, "tier2 rows", p.last_tiers()[0], "exact", ne, flush=True)


if __name__ == "__main__":
    main()
