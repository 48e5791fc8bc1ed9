#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 SQLite (rocpd) result over the last
N dispatches-per-step window:  python scripts/rocpd_summary.py run_results.db [--steps K]"""
import argparse
import sqlite3
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--steps", type=int, default=0, help="divide totals by K timed steps (per-step view)")
ap.add_argument("--last", type=int, default=0, help="only the last N dispatches")
a = ap.parse_args()
c = sqlite3.connect(a.db)
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name_col = "name" if "name" in cols else ("kernel_name" if "kernel_name" in cols else cols[0])
rows = list(c.execute(f"select {name_col}, start, end from kernels order by start"))
if a.last:
    rows = rows[-a.last:]
agg = defaultdict(lambda: [0, 0.0])
for n, s, e in rows:
    agg[n][0] += 1
    agg[n][1] += (e - s) / 1e3
tot = sum(v[1] for v in agg.values())
div = a.steps or 1
print(f"{len(rows)} dispatches, {tot:.1f} us total" + (f", {tot / div:.1f} us/step" if a.steps else ""))
for n, (k, us) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    short = n if len(n) < 90 else n[:87] + "..."
    print(f"{us / div:9.2f} us  {k / div:7.2f}x  {100 * us / tot:5.1f}%  {short}")
