#!/usr/bin/env python3
"""bench.py -- rows/s per training iteration on MI355X (BASELINE.json metric).

Default workload (BASELINE.json configs[1]): KMeans k=1024 on synthetic dense
fp64 10M x 256, one Lloyd iteration per step (KMeans.scala:275-334: statistics,
findClosest for every row, per-cluster sums/weights/cost, merge, centroid
update).  With --gpus N (launched one process per GPU by torch.distributed.run)
every rank holds its own 10M-row shard in HBM (weak scaling) and the merge is
one RCCL all-reduce of [sums | weights | cost] per iteration.

Prints ONE JSON line on rank 0.  `roofline` is for the dominant kernel (the
fp64-MFMA assign kernel), timed with HIP events on its own stream inside the
timed region; `cpu_baseline` is the CPU restatement (oracle/, a C port of the
reference loops) run on a bounded sample on this host's cores.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP64_PEAK_TFLOPS = 78.6   # MI355X fp64 (vector = matrix) spec, BASELINE.md section 2
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md chip table (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="kmeans", choices=["kmeans"])
    ap.add_argument("--rows", type=int, default=10_000_000, help="rows per GPU")
    ap.add_argument("--dim", type=int, default=256)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="target CPU time of the cpu_baseline sample (0 disables)")
    return ap.parse_args()


def pmc_traffic(name):
    """HBM bytes per launch of `name` from the committed rocprofv3 --pmc summary
    (profiles/*_pmc.json written by tools/pmc_summary.py), else None."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json")))
    for f in reversed(files):
        try:
            d = json.load(open(f))
            if name in d:
                return d[name].get("hbm_bytes_per_launch")
        except Exception:
            continue
    return None


def cpu_baseline_kmeans(Xs, C, seconds):
    """Time the CPU restatement (oracle.kmeans_iteration) on a bounded sample,
    rows split into one Spark-like partition per thread (local[N])."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(os.cpu_count() or 1, 16)
    xn = oracle.row_norms(Xs)
    cn = oracle.row_norms(C)
    # calibrate on a small slice, then size the sample for ~`seconds`
    m = min(2000, Xs.shape[0])
    t0 = time.perf_counter()
    oracle.kmeans_iteration(Xs[:m], xn[:m], None, C, cn, num_partitions=1)
    t1 = time.perf_counter() - t0
    stats_t0 = time.perf_counter()
    oracle.kmeans_stats(C)
    t_stats = time.perf_counter() - stats_t0
    per_row = max((t1 - t_stats) / m, 1e-9)
    rows = int(min(Xs.shape[0], max(threads * 1000, seconds * threads / per_row)))
    rows = max(rows - rows % threads, threads)
    t0 = time.perf_counter()
    oracle.kmeans_iteration(Xs[:rows], xn[:rows], None, C, cn, num_partitions=threads,
                            threads=threads)
    el = time.perf_counter() - t0
    return {"value": rows / el, "unit": "rows/s", "cores": threads, "kind": "port",
            "sample": f"{rows} rows of the same synthetic 256-dim data, same k=1024 centers, "
                      f"one Lloyd iteration (stats+findClosest+sums+merge+update), "
                      f"{threads} partitions on {threads} threads, {el:.1f} s"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from cycloneml_amd import _native as N
    from cycloneml_amd.clustering import KMeansPlan, row_norms
    N.load()

    n, d, k = args.rows, args.dim, args.k
    # Synthetic data (BASELINE config 2 / SURVEY 8d): 1024 true centers
    # ~ N(0, 4^2) per dim + point noise N(0, 1); generated on device with
    # torch's Philox generator (seeded), resident in HBM before timing.
    g = torch.Generator(device=dev).manual_seed(1234)
    true_c = torch.randn(k, d, generator=g, device=dev, dtype=torch.float64) * 4.0
    gr = torch.Generator(device=dev).manual_seed(1000 + rank)
    X = torch.empty(n, d, dtype=torch.float64, device=dev)
    chunk = 1 << 20
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        lab = torch.randint(0, k, (e - s,), generator=gr, device=dev)
        X[s:e] = true_c[lab] + torch.randn(e - s, d, generator=gr, device=dev,
                                           dtype=torch.float64)
    del true_c
    xnorm = row_norms(X)
    C0 = X[:k].clone()                     # setInitialModel semantics: rows 0..k-1
    if world > 1:
        dist.broadcast(C0, 0)
    C = C0.clone()
    cnorm = row_norms(C)
    plan = KMeansPlan(d, k, n)
    buf = torch.zeros(k * d + k + 1, dtype=torch.float64, device=dev)
    sums, wsum, cost_sum = buf[:k * d], buf[k * d:k * d + k], buf[k * d + k:]
    conv = torch.zeros(1, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream()

    def step():
        buf.zero_()
        plan.accumulate(X, xnorm, None, C, cnorm, sums, wsum, cost_sum, stream=stream)
        if world > 1:
            dist.all_reduce(buf)
        plan.update(C, cnorm, sums, wsum, 1e-4, conv, stream=stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    plan.set_timing(True)
    plan.get_timing()  # reset
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    assign_ms, launches = plan.get_timing()
    plan.set_timing(False)
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    total_rows = n * world * args.steps
    value = total_rows / el
    avg_launch_s = (assign_ms / max(launches, 1)) / 1e3
    flops_per_launch = 2.0 * k * d * n
    achieved = flops_per_launch / avg_launch_s / 1e12 if launches else None
    traffic = pmc_traffic("k_kmeans_assign")

    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        import numpy as np
        m = min(n, 400_000)
        Xs = X[:m].cpu().numpy()
        cpu = cpu_baseline_kmeans(np.ascontiguousarray(Xs), C0.cpu().numpy(), args.cpu_seconds)

    if rank == 0:
        line = {
            "metric": "rows/s per training iteration (KMeans Lloyd iteration)",
            "value": value,
            "unit": "rows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": el / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (torch Philox, seeded): 1024 Gaussian centers sd 4 + N(0,1) noise",
            "config": {"workload": "KMeans k=1024 Lloyd iteration, dense fp64 "
                                   f"{n} x {d} rows per GPU (BASELINE configs[1])",
                       "rows_per_gpu": n, "dim": d, "k": k,
                       "parallelism": f"dp{world} (row shards, RCCL all-reduce merge)"},
            "roofline": {"kernel": "k_kmeans_assign", "bound": "mfma",
                         "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": (achieved / FP64_PEAK_TFLOPS) if achieved else None,
                         "traffic": traffic,
                         "avg_launch_ms": avg_launch_s * 1e3, "launches": launches,
                         "flops_per_launch": flops_per_launch},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
