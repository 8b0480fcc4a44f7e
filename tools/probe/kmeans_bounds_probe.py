#!/usr/bin/env python3
"""How many rows could carried bounds keep?  One fit on bench.py's KMeans
rows (config 2, setInitialModel = rows 0..1023) through KMeansPlan.accumulate
with the library's carried bounds (kmeans_i8.hpp Bounds); per iteration:
  lib_screened   rows the library screened (cyc_kmeans_rows_bounds_info)
  exact_kept     on a fixed sample (every 50th row), the fraction EXACT
                 Hamerly bounds would keep: ub = |x - c_w|, lb = the second
                 smallest distance, both exact at a row's last screen, moved
                 by the same drift rule (ub += d_w, lb -= max_{c != w} d_c)
                 and tested with the same 2^-29 slack
  gap_lt_drift   sample rows whose one-step gap lb - ub < d_w + max d
Prints one JSON line per iteration (profiles/r06_kmeans_bounds_probe.jsonl)."""
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
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    X = bench.kmeans_data(n, dev, 0, d, k)
    C = X[:k].clone()
    xn, cn = row_norms(X), row_norms(C)
    p = KMeansPlan(d, k, n)
    rows = p.rows(X)
    conv = torch.zeros(1, dtype=torch.int32, device=dev)
    buf = torch.zeros(k * d + k + 1, dtype=torch.float64, device=dev)
    sums, wsum, cost = buf[:k * d], buf[k * d:k * d + k], buf[k * d + k:]
    S = X[::50].clone()
    ss = (S * S).sum(1)
    ub = lb = None
    Cprev = None
    last = (0, 0)
    for it in range(iters):
        # exact distances of the sample to the current centers
        D = (ss[:, None] + (C * C).sum(1)[None, :] - 2.0 * S @ C.T).clamp_min(0)
        top = torch.topk(D, 2, dim=1, largest=False)
        d1, d2 = top.values[:, 0].sqrt(), top.values[:, 1].sqrt()
        w = top.indices[:, 0]
        out = {"iteration": it + 1}
        if Cprev is not None:
            delta = (C - Cprev).norm(dim=1)
            dv, di = torch.topk(delta, 2)
            dmax = torch.where(w == di[0], dv[1], dv[0])
            U = ub + delta[w_prev]
            L = lb - dmax
            tau = 2.0 ** -29 * (ss + (C * C).sum(1).max())
            keep = (L > 0) & (L * L - U * U > tau) & (w == w_prev)
            out.update({"exact_kept": float(keep.float().mean()),
                        "max_drift": float(dv[0]),
                        "gap_lt_drift": float(((d2_prev - d1_prev) < (delta[w_prev] + dv[0])).float().mean())})
            ub = torch.where(keep, U, d1)
            lb = torch.where(keep, L, d2)
        else:
            ub, lb = d1, d2
        w_prev, d1_prev, d2_prev = w, d1, d2
        Cprev = C.clone()
        buf.zero_()
        p.accumulate(X, xn, None, C, cn, sums, wsum, cost, rows=rows)
        p.update(C, cn, sums, wsum, 1e-4, conv)
        calls, scr = rows.bounds_info()
        out["lib_screened"] = scr - last[1]
        out["lib_kept"] = 1.0 - (scr - last[1]) / n
        last = (calls, scr)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
