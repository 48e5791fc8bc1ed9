"""Per-kernel mean durations in the two largest dense runs of kernels of a
rocprofv3 kernel trace (e.g. a bench measured twice in one process)."""
import csv
import glob
import sys
from collections import defaultdict

path = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = []
with open(path) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
# split at gaps > 50 ms into phases
phases, cur = [], [rows[0]]
for r in rows[1:]:
    if r[0] - cur[-1][1] > 50_000_000:
        phases.append(cur)
        cur = []
    cur.append(r)
phases.append(cur)
print("phases:", [(len(p), round((p[-1][1] - p[0][0]) / 1e6, 1)) for p in phases])
big = sorted(sorted(phases, key=len)[-6:], key=lambda p: p[0][0])
names = sorted({r[2][:60] for p in big for r in p})
stats = []
for p in big:
    d = defaultdict(list)
    for s, e, n in p:
        d[n[:60]].append(e - s)
    stats.append(d)
print("%-60s " % "kernel" + " ".join("%14s" % ("ph%d n/us" % i) for i in range(len(big))))
for n in names:
    cells = []
    for d in stats:
        v = d.get(n)
        cells.append("%6d %7.1f" % (len(v), sum(v) / len(v) / 1e3) if v else "%14s" % "-")
    print("%-60s " % n + " ".join(cells))
for i, p in enumerate(big):
    busy = sum(e - s for s, e, _ in p)
    print("phase %d: kernels %d span %.1f ms busy %.1f ms" % (i, len(p), (p[-1][1] - p[0][0]) / 1e6, busy / 1e6))
