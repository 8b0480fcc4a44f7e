#!/usr/bin/env python3
"""The bench line's dominant kernel against a rocprofv3 kernel trace of the
same command: the kernel's launches in trace order, the timed ones picked
as launches [skip, skip + steps) (warm-up launches first), their average
beside the line's avg_launch_ms.
usage: agree_summary.py <kernel_trace.csv> <bench.json> <kernel> <skip> <steps>"""
import csv
import json
import sys

trace, bench, kern, skip, steps = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), int(sys.argv[5])
rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows
     if kern + "<" in r["Kernel_Name"] or r["Kernel_Name"].split("(")[0].endswith(kern)]
line = json.loads(open(bench).read().strip().splitlines()[-1])
roof = line["roofline"]
timed = d[skip:skip + steps]
print(f"kernel {kern}: {len(d)} launches in the trace (warm-up, timed, after-clock passes, the fit)")
print(f"trace, launches [{skip}, {skip + steps}): avg {sum(timed) / len(timed):.1f} us "
      f"(min {min(timed):.1f}, max {max(timed):.1f})")
print(f"bench line under the profiler: {roof['kernel']} avg_launch_ms {roof['avg_launch_ms'] * 1e3:.1f} us, "
      f"ms_per_step {line['ms_per_step']:.3f}, value {line['value'] / 1e6:.1f} M rows/s")
print(f"all launches: avg {sum(d) / len(d):.1f} us")
