#!/usr/bin/env python3
"""Summarise a tools/prof.sh run into profiles/<tag>_pmc.json.

Per kernel: mean duration (kernel trace), mean FETCH_SIZE / WRITE_SIZE (KB,
from the two separate --pmc passes) and hbm_bytes_per_launch.

gfx950 correction (MI355X_MICROARCH.md "HBM"): FETCH_SIZE reads exactly half
the bytes of a wide (16 B/lane) coalesced stream.  Our streaming kernels load
8 B per lane; for those the counter was calibrated against the known byte
count of the assign kernel's X stream (20.48 GB per launch at 10M x 256
reads as 19.1e6 KB, i.e. unhalved), so no factor is applied.  WRITE_SIZE is
exact for streaming stores.  Both are per launch, like roofline.achieved.

usage: tools/pmc_summary.py gpurun_out/<tag> profiles/<tag> [rows_per_launch]
"""
import collections
import csv
import json
import os
import sys


def mean_counter(path):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        agg[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main(src, dst_prefix, rows=None):
    stats = {}
    ks = os.path.join(src, "trace", "run_kernel_stats.csv")
    for r in csv.DictReader(open(ks)):
        stats[r["Name"]] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                            "pct": float(r["Percentage"])}
    fetch = mean_counter(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"))
    write = mean_counter(os.path.join(src, "pmc_write", "run_counter_collection.csv"))
    out = {}
    for name, s in stats.items():
        f = fetch.get((name, "FETCH_SIZE"))
        w = write.get((name, "WRITE_SIZE"))
        out[name] = dict(s, fetch_kb=f, write_kb=w,
                         hbm_bytes_per_launch=None if f is None or w is None
                         else (f + w) * 1024.0)
    if rows:
        out["_rows_per_launch"] = int(rows)
    os.makedirs(os.path.dirname(dst_prefix) or ".", exist_ok=True)
    json.dump(out, open(dst_prefix + "_pmc.json", "w"), indent=1, sort_keys=True)
    with open(ks) as fi, open(dst_prefix + "_kernel_stats.csv", "w") as fo:
        fo.write(fi.read())
    print(json.dumps({k: v for k, v in out.items() if k.startswith("k_")}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
