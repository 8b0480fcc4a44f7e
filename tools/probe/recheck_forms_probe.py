#!/usr/bin/env python3
"""Determinism of the carried-state counters: the re-check forms test's
child (tests/test_kmeans_gpu.py _RECHECK_CHILD) run twice per form, its
per-iteration (screened, re-checked) counters and assignments compared."""
import ast
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
src = open(os.path.join(ROOT, "tests", "test_kmeans_gpu.py")).read()
child = next(n.value.value for n in ast.parse(src).body
             if isinstance(n, ast.Assign) and n.targets[0].id == "_RECHECK_CHILD")
d, k, n = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (256, 300, 80000)
out = {}
for tag, form in (("a0", "0"), ("b0", "0"), ("a1", "1"), ("b1", "1")):
    f = os.path.join(ROOT, "gpurun_out", f"rfp_{tag}.npy")
    env = dict(os.environ, CYC_KMEANS_RECHECK=form)
    r = subprocess.run([sys.executable, "-c", child, f, str(d), str(k), str(n)], env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    out[tag] = (np.load(f), r.stdout.split())
    os.remove(f)
    print(tag, " ".join(out[tag][1]), flush=True)
for x, y in (("a0", "b0"), ("a1", "b1"), ("a0", "a1")):
    print(x, y, "assign equal:", bool((out[x][0] == out[y][0]).all()),
          "counters equal:", out[x][1] == out[y][1])
