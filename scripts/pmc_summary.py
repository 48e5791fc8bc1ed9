#!/usr/bin/env python3
"""Per-kernel PMC summary of a rocprofv3 --pmc run (counter_collection.csv):
mean counter value per dispatch over the last N dispatches of each pbx::
kernel, with its mean duration and the implied DRAM-side bandwidth when
FETCH_SIZE / WRITE_SIZE (KB) are present.  usage: pmc_summary.py csv [csv ...]"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    name = name.replace("pbx::(anonymous namespace)::", "pbx::").replace("void ", "")
    return re.sub(r"\(.*", "", name)


def main(paths, last=20):
    vals = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(dict)
    for p in paths:
        with open(p) as f:
            for r in csv.DictReader(f):
                k = short(r["Kernel_Name"])
                if not k.startswith("pbx::"):
                    continue
                d = int(r["Dispatch_Id"])
                vals[k][r["Counter_Name"]].append((d, float(r["Counter_Value"])))
                dur[k][d] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
    names = sorted({c for k in vals for c in vals[k]})
    print(f"{'kernel':34s} {'us':>7s} " + " ".join(f"{c:>14s}" for c in names) + "  GB/s(fetch+write)")
    rows = []
    for k in vals:
        ds = sorted(dur[k])[-last:]
        us = sum(dur[k][d] for d in ds) / len(ds)
        means = {}
        for c in names:
            xs = [v for d, v in vals[k].get(c, []) if d in set(ds)]
            means[c] = sum(xs) / len(xs) if xs else float("nan")
        kb = sum(means.get(c, 0.0) for c in ("FETCH_SIZE", "WRITE_SIZE") if means.get(c) == means.get(c))
        rows.append((us, k, means, kb * 1024 / (us * 1e-6) / 1e9 if us else 0.0))
    for us, k, means, bw in sorted(rows, reverse=True):
        print(f"{k:34s} {us:7.1f} " + " ".join(f"{means[c]:14.1f}" for c in names) + f"  {bw:8.0f}")


if __name__ == "__main__":
    main(sys.argv[1:])
