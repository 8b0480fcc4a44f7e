#!/usr/bin/env python3
"""Per-iteration kernel time of a KMeans fit from a rocprofv3 kernel trace:
iterations split at each launch of MARK (default k_inc_moved, one per Lloyd
call); per iteration the busy time, span and the top kernels.
usage: fit_trace_summary.py <kernel_trace.csv> [MARK] [TOP]"""
import collections
import csv
import sys

path = sys.argv[1]
mark = sys.argv[2] if len(sys.argv) > 2 else "k_inc_moved"
top = int(sys.argv[3]) if len(sys.argv) > 3 else 8
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [0] + [i for i, r in enumerate(rows) if mark in r["Kernel_Name"]]
idx.append(len(rows))
for it in range(len(idx) - 1):
    if idx[it + 1] <= idx[it]:
        continue
    seg = rows[idx[it]:idx[it + 1]]
    t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
    acc = collections.Counter()
    for r in seg:
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        acc[name[:60]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    busy = sum(acc.values())
    print(f"segment {it} (to mark {it + 1}): span {(t1 - t0) / 1e3:.0f} us, busy {busy:.0f} us, {len(seg)} launches")
    for name, us in acc.most_common(top):
        print(f"   {us:9.1f}  {name}")
