#!/usr/bin/env python3
"""Summary of a KMeans bench line: rate, step, priced / diag kernels, the
carried-bounds and incremental-sums counters, the fit."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(round(d["value"] / 1e6, 1), "M rows/s", round(d["ms_per_step"], 3), "ms", r["kernel"],
      round(r["frac"], 3), "step_frac", round(r.get("step_frac") or 0, 3))
print({k: round(v, 3) for k, v in r["kernels_ms_per_step"].items()})
print({k: round(v, 3) for k, v in r["diag_kernels_ms_per_step"].items()})
for key in ("incremental_sums", "carried_bounds"):
    print(key, {k: v for k, v in r.get(key, {}).items() if k != "note"})
f = d.get("fit", {})
print("fit", round(f.get("fit_ms", 0), 1), f.get("iteration_ms"))
print("cpu", (d.get("cpu_baseline") or {}).get("value"))
