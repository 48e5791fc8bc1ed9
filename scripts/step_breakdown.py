"""Per-step kernel breakdown of a rocprofv3 kernel trace: the last --steps
training steps (delimited by an anchor kernel, default the tower forward),
average time per kernel name and the launch count per step."""
import argparse
import collections
import csv

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--anchor", default="k_tower_fwd")
ap.add_argument("--steps", type=int, default=10)
ap.add_argument("--copies", default=None, help="rocprofv3 memory_copy_trace.csv: shown in the timeline")
a = ap.parse_args()
rows = list(csv.DictReader(open(a.trace)))
copies = []
if a.copies:
    try:
        for r in csv.DictReader(open(a.copies)):
            copies.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                           "copy " + r.get("Direction", "?") + " " + r.get("Size", r.get("Bytes", "")) + "B"))
    except OSError:
        copies = []
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if a.anchor in r["Kernel_Name"]]
idx = idx[-(a.steps + 1):]
agg = collections.defaultdict(float)
cnt = collections.Counter()
busy = 0.0
for s, e in zip(idx[:-1], idx[1:]):
    for r in rows[s:e]:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        n = r["Kernel_Name"].replace("pbx::(anonymous namespace)::", "").replace("void ", "").split("(")[0][:60]
        agg[n] += d
        cnt[n] += 1
        busy += d
n = len(idx) - 1
span = (int(rows[idx[-1]]["Start_Timestamp"]) - int(rows[idx[0]]["Start_Timestamp"])) / 1e3 / n
print(f"steps={n} wall/step={span:.1f}us kernel-busy/step={busy / n:.1f}us launches/step={sum(cnt.values()) / n:.1f}")
for k, v in sorted(agg.items(), key=lambda kv: -kv[1]):
    print(f"{k:60s} {cnt[k] / n:5.1f}x {v / n:8.1f}us")

# timeline of the last full step: start offset / duration per kernel (gaps show
# launch latency, overlap shows the side streams)
s, e = idx[-2], idx[-1]
t0 = int(rows[s]["Start_Timestamp"])
# include the kernels of the same step launched before the anchor
prev = idx[-3] if len(idx) >= 3 else s
print("\ntimeline (us from the anchor of the last step; negative = before it):")
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
       r["Kernel_Name"].replace("pbx::(anonymous namespace)::", "").replace("void ", "").split("(")[0][:50])
      for r in rows[prev:e]]
lo, hi = ev[0][0], int(rows[e]["Start_Timestamp"])
ev += [c for c in copies if lo <= c[0] < hi]
for b0, b1, n in sorted(ev):
    st = (b0 - t0) / 1e3
    d = (b1 - b0) / 1e3
    if st > -200:
        print(f"  {st:8.1f} {st + d:8.1f} {d:7.1f}  {n}")
