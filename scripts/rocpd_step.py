#!/usr/bin/env python3
"""Per-step kernel table of a rocprofv3 kernel-trace database (rocpd
SQLite): the last K steps, steps delimited by a once-per-step kernel.

    python scripts/rocpd_step.py run_results.db [--marker adam] [--steps 40] [--top 30]
"""
import argparse
import re
import sqlite3
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--marker", default="adam")
ap.add_argument("--steps", type=int, default=40)
ap.add_argument("--top", type=int, default=40)
a = ap.parse_args()
c = sqlite3.connect(a.db)
rows = list(c.execute("select name, start, end, grid_x, grid_y, grid_z, workgroup_x from kernels order by start"))
marks = [i for i, r in enumerate(rows) if a.marker in r[0].lower()]
per = marks[-1] - marks[-2]
rows = rows[len(rows) - per * a.steps:]
agg = defaultdict(list)
for n, s, e, gx, gy, gz, wx in rows:
    m = re.search(r"::(k_\w+(<[^()]*>)?)\(", n) or re.search(r"(\w*elementwise\w*|__amd\w+|\w+Functor)", n)
    agg[((m.group(1) if m else n[:40])[:48], gx // max(wx, 1), gy, gz)].append((e - s) / 1e3)
tot = sum(sum(v) for v in agg.values()) / a.steps
print(f"{per} dispatches/step, {tot:.1f} us GPU/step (last {a.steps} steps)")
print(f"{'us/step':>8} {'n/step':>6} {'us/call':>8}  kernel (grid)")
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[: a.top]:
    print(f"{sum(v) / a.steps:8.2f} {len(v) / a.steps:6.2f} {sum(v) / len(v):8.2f}  {k[0]} {k[1:]}")
