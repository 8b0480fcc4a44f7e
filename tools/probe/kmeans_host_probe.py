"""Where the host stands during bench.py's KMeans steps: per step, the host
time of each call (zero_, accumulate, all-reduce, update) and the GPU time
of the step, so a step whose host side is slower than its GPU side shows.

usage (GPU box): python tools/probe/kmeans_host_probe.py [steps]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))


def main():
    import torch
    import bench
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda:0")
    wl = bench.KMeansWorkload(10_000_000, dev, 0)
    for _ in range(3):
        wl.step()
    torch.cuda.synchronize()
    k, d = wl.k, wl.d
    rec = []
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    t_all = time.perf_counter()
    ev[0].record()
    for i in range(steps):
        buf = wl.buf
        sums, wsum, cost = buf[:k * d], buf[k * d:k * d + k], buf[k * d + k:]
        t0 = time.perf_counter()
        buf.zero_()
        t1 = time.perf_counter()
        wl.plan.accumulate(wl.X, wl.xnorm, None, wl.C, wl.cnorm, sums, wsum, cost, rows=wl.rows)
        t2 = time.perf_counter()
        # did the GPU already finish this call's work when the host got back?
        e = torch.cuda.Event()
        e.record()
        done = e.query()
        tail_us = -1.0
        if i == steps - 1:   # how much of this call's GPU work was left at the return
            ts = time.perf_counter()
            e.synchronize()
            tail_us = (time.perf_counter() - ts) * 1e6
        wl.parallel.allreduce_(buf)
        t3 = time.perf_counter()
        wl.plan.update(wl.C, wl.cnorm, sums, wsum, 1e-4, wl.conv)
        t4 = time.perf_counter()
        ev[i + 1].record()
        rec.append({"zero_us": (t1 - t0) * 1e6, "accumulate_us": (t2 - t1) * 1e6,
                    "allreduce_us": (t3 - t2) * 1e6, "update_us": (t4 - t3) * 1e6,
                    "gpu_done_at_return": int(done), "gpu_left_at_return_us": tail_us})
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t_all) * 1e3 / steps
    for i, r in enumerate(rec):
        r["gpu_ms"] = ev[i].elapsed_time(ev[i + 1])
        print(json.dumps({k2: round(v, 1) if k2 != "gpu_ms" else round(v, 3) for k2, v in r.items()}))
    print(json.dumps({"wall_ms_per_step": round(wall, 3)}))


if __name__ == "__main__":
    main()
