#!/usr/bin/env python3
"""Row counts of the KMeans screen's tiers on bench.py's config (10M x 256,
k = 1024) after W Lloyd iterations: the one-limb pass's listed rows, the
full two-limb pass's rows, the refinement's candidate-union size, the fp64
candidate pass's rows, the three-limb pass's rows, and the rows left to the
fp64 screen / exact loop.  One JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    dev = torch.device("cuda", 0)
    wl = bench.KMeansWorkload(10_000_000, dev, 0)
    for _ in range(int(os.environ.get("ITERS", "8"))):
        wl.step()
    assign = torch.empty(wl.n, dtype=torch.int32, device=dev)
    cost = torch.empty(wl.n, dtype=torch.float64, device=dev)
    n_exact = wl.plan.assign(wl.X, wl.xnorm, wl.C, wl.cnorm, assign, cost, count_exact=True,
                             rows=wl.rows)
    listed, full, union = wl.plan.last_refine()
    print(json.dumps({"listed_by_one_limb": listed, "full_two_limb": full,
                      "refine_union_centers": union,
                      "candidate_pass": wl.plan.last_candidates(),
                      "three_limb": wl.plan.last_screen(),
                      "fp64_screen_exact": wl.plan.last_tiers(), "exact": n_exact}), flush=True)


if __name__ == "__main__":
    main()
