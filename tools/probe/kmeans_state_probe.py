#!/usr/bin/env python3
"""Where the rows of one steady-state KMeans step go (bench.py's config 2
fit): with CYC_KMEANS_DUMP set, kmeans.hip dumps the carried-bounds state of
bounded call CYC_KMEANS_DUMP_CALL (after the filter, and after the
re-check); this script runs the bench's steps and tabulates the dumps.
Diagnostics only.  usage: python tools/probe/kmeans_state_probe.py [calls]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
out = os.path.join(ROOT, "gpurun_out", "kmdump")
os.makedirs(out, exist_ok=True)
os.environ["CYC_KMEANS_DUMP"] = out
os.environ.setdefault("CYC_KMEANS_DUMP_CALL", "10")


def qs(x, q):
    import numpy as np
    return [float(v) for v in np.quantile(x, q)] if len(x) else None


def main():
    import numpy as np
    import torch
    import bench
    dev = torch.device("cuda", 0)
    wl = bench.KMeansWorkload(10_000_000, dev, 0)
    for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 12):
        wl.step()
    torch.cuda.synchronize()
    f = lambda n, t: np.fromfile(os.path.join(out, n), dtype=t)
    s0, s1 = f("state_filter", np.uint8), f("state_rc", np.uint8)
    bnd = f("bnd", np.float32).reshape(-1, 2)
    a = f("assign", np.int32)
    R, delta = f("nbrR", np.float32), f("delta", np.float64)
    joint = {f"{i}->{j}": int(((s0 == i) & (s1 == j)).sum()) for i in range(4) for j in range(4)
             if ((s0 == i) & (s1 == j)).any()}
    res = {"call": int(os.environ["CYC_KMEANS_DUMP_CALL"]), "joint": joint}
    m1 = s0 == 1
    ub = bnd[m1, 0].astype(np.float64)
    res["state1_no_bound"] = int((ub < 0).sum())
    U = ub + delta[a[m1]]
    Ra = R[a[m1]].astype(np.float64)
    ok = ub >= 0
    q = Ra[ok] / np.maximum(U[ok], 1e-30)
    res["state1_R_over_U_quantiles"] = qs(q, [0.05, 0.25, 0.5, 0.75, 0.95])
    res["state1_U_quantiles"] = qs(U[ok], [0.05, 0.5, 0.95])
    res["nbrR_quantiles"] = qs(R, [0.05, 0.25, 0.5, 0.75, 0.95])
    res["kept_ub_quantiles"] = qs(bnd[s0 == 0, 0], [0.05, 0.5, 0.95])
    res["max_drift"] = float(delta.max())
    # failed re-checks (2 or 3 -> 1): their moved bounds
    for st in (2, 3):
        mf = (s0 == st) & (s1 == 1)
        if mf.any():
            u = bnd[mf, 0].astype(np.float64) + delta[a[mf]]
            res[f"failed{st}_R_over_U_quantiles"] = qs(R[a[mf]] / np.maximum(u, 1e-30),
                                                       [0.05, 0.5, 0.95])
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
