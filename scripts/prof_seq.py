#!/usr/bin/env python3
"""Print the kernel sequence of one training step from a rocprofv3 kernel
trace (start offset, duration, grid, workgroup, kernel), delimited by a
once-per-step marker kernel.

  python scripts/prof_seq.py gpurun_out/prof/run_kernel_trace.csv [--marker k_auc] [--back 2]
"""
import argparse
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="k_auc")
    ap.add_argument("--back", type=int, default=2, help="which step from the end")
    args = ap.parse_args()
    with open(args.trace) as f:
        rows = list(csv.DictReader(f))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if args.marker in r["Kernel_Name"]]
    lo, hi = marks[-args.back - 1] + 1, marks[-args.back] + 1
    t0 = int(rows[lo]["Start_Timestamp"])
    for r in rows[lo:hi]:
        name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")
        name = re.sub(r"\(.*", "", name)[:90]
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        grid = r.get("Grid_Size_X", r.get("Grid_Size", ""))
        wg = r.get("Workgroup_Size_X", r.get("Workgroup_Size", ""))
        print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}us grid={grid!s:>8} wg={wg!s:>4} {name}")


if __name__ == "__main__":
    main()
