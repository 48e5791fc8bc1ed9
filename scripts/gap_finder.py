#!/usr/bin/env python3
"""Idle gaps of the GPU in a rocprofv3 csv trace (kernels + memory copies):
prints every gap longer than --min-us with the activity just before / after.

    python scripts/gap_finder.py run_kernel_trace.csv [--copies run_memory_copy_trace.csv] [--min-us 500]
"""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument("kernels")
ap.add_argument("--copies")
ap.add_argument("--min-us", type=float, default=500.0)
ap.add_argument("--ctx", type=int, default=4)
a = ap.parse_args()
ev = []
for r in csv.DictReader(open(a.kernels)):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]))
if a.copies:
    for r in csv.DictReader(open(a.copies)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r.get("Direction", "")))
ev.sort()
end = ev[0][1]
for i in range(1, len(ev)):
    gap = ev[i][0] - end
    if gap > a.min_us * 1e3:
        print(f"gap {gap / 1e3:.0f} us before event {i}:")
        for j in range(max(0, i - a.ctx), min(len(ev), i + a.ctx)):
            s, e, n = ev[j]
            print(f"   {'>' if j == i else ' '} {(s - ev[i][0]) / 1e3:10.1f} {(e - s) / 1e3:8.1f}  {n}")
    end = max(end, ev[i][1])
