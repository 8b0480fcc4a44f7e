#!/usr/bin/env python3
"""A/B the KMeans assign kernel variants in ONE process (interleaved rounds),
on the BASELINE config 2 shape; checks the variants agree bit for bit.
usage: python tools/kmeans_ab.py [rows]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from cycloneml_amd import _native as N
    from cycloneml_amd.clustering import KMeansPlan, row_norms
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    d, k = 256, 1024
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(1234)
    true_c = torch.randn(k, d, generator=g, device=dev, dtype=torch.float64) * 4.0
    X = torch.empty(n, d, dtype=torch.float64, device=dev)
    for s in range(0, n, 1 << 20):
        e = min(n, s + (1 << 20))
        lab = torch.randint(0, k, (e - s,), generator=g, device=dev)
        X[s:e] = true_c[lab] + torch.randn(e - s, d, generator=g, device=dev, dtype=torch.float64)
    xn = row_norms(X)
    C = X[:k].clone()
    cn = row_norms(C)
    plans = {}
    only = os.environ.get("AB_ONLY")
    variants = os.environ.get("AB_VARIANTS", "3,8").split(",")
    rows = {}
    for v in ((only,) if only else variants):
        # "8": fp64 screen plan + the i8 row image in front of it
        os.environ["CYC_KMEANS_ASSIGN"] = "2" if v == "8" else v
        plans[v] = KMeansPlan(d, k, n)
        plans[v].stats(C)
        rows[v] = plans[v].rows(X) if v == "8" else None
    outs = {v: (torch.empty(n, dtype=torch.int32, device=dev),
                torch.empty(n, dtype=torch.float64, device=dev)) for v in plans}
    N.profile_enable(True)
    res = {v: [] for v in plans}
    for rnd in range(4):
        for v, p in plans.items():
            N.profile_query("k_kmeans_assign")
            N.profile_query("k_kmeans_assign_fp64")
            nex = p.assign(X, xn, C, cn, *outs[v], count_exact=True, rows=rows[v])
            torch.cuda.synchronize()
            ms, cnt = N.profile_query("k_kmeans_assign")
            ms2, _ = N.profile_query("k_kmeans_assign_fp64")
            if rnd > 0:
                res[v].append(ms + ms2)
            t2, _ = p.last_tiers()
            print(f"round {rnd} variant {v}: {ms:.2f} ms + fp64 tier {ms2:.2f} ms, "
                  f"fp64-screen rows {t2}, exact-path rows {nex}", flush=True)
    for v in res:
        best = min(res[v])
        print(f"variant {v}: best {best:.2f} ms = {2.0 * k * d * n / best / 1e9:.1f} "
              "fp64-equivalent TFLOP/s")
    real = [v for v in plans if v in ("1", "2", "3", "8")]
    if only or len(real) < 2:
        return
    same = all(torch.equal(outs[real[0]][i], outs[v][i]) for v in real[1:] for i in range(2))
    print(f"variants {real} bit-identical:", same)
    sys.exit(0 if same else 1)


if __name__ == "__main__":
    main()
