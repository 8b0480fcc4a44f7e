#!/usr/bin/env python3
"""One iteration's kernel timeline from a rocprofv3 --kernel-trace CSV: the
launches between two consecutive starts of the kernel matching MARK
(default: the one-limb KMeans pass) -- the pair ending at the BACK-th last
start (default 2: the last full iteration before whatever follows the timed
loop) -- with start / end / duration in microseconds and the idle gap before
each launch.

usage: tools/trace_timeline.py <run_kernel_trace.csv> [MARK] [BACK]
"""
import csv
import sys


def main():
    path = sys.argv[1]
    mark = sys.argv[2] if len(sys.argv) > 2 else "k_screen32<8, 4, 1, false>"
    back = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if mark in r["Kernel_Name"]]
    if len(idx) < back + 1:
        sys.exit(f"fewer than {back + 1} launches match {mark!r}")
    i0, i1 = idx[-back - 1], idx[-back]
    t0 = int(rows[i0]["Start_Timestamp"])
    prev_end = t0
    busy = 0.0
    for r in rows[i0:i1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} "
              f"gap {max(0, s - prev_end) / 1e3:6.1f}  {name[:80]}")
        busy += (e - s) / 1e3
        prev_end = max(prev_end, e)
    total = (int(rows[i1]["Start_Timestamp"]) - t0) / 1e3
    print(f"iteration {total:.1f} us, {i1 - i0} launches, kernel time {busy:.1f} us")


if __name__ == "__main__":
    main()
