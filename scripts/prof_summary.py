#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace over the last N training steps.

A step is delimited by a marker kernel that runs exactly once per step
(default: the AUC histogram kernel).  Reports per-kernel time per step, GPU
busy time per step and the wall span per step (gaps = launch/host overhead).

  python scripts/prof_summary.py gpurun_out/prof/run_kernel_trace.csv --steps 15
"""
import argparse
import collections
import csv
import re


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"\(.*", "", name)
    if name.startswith("Cijk_"):
        return "hipBLASLt GEMM " + name.split("_MT")[1].split("_")[0] if "_MT" in name else "hipBLASLt GEMM"
    if "rocprim" in name:
        m = re.search(r"wrapped_(\w+?)_config", name)
        return "rocprim::" + (m.group(1) if m else "kernel")
    if "at::native" in name:
        m = re.search(r"at::native::(?:\(anonymous namespace\)::)?(\w+)", name)
        f = re.search(r"(\w+Functor\w*|\w+_kernel\w*)", name[20:])
        return "aten::" + (m.group(1) if m else "") + ("/" + f.group(1) if f else "")
    return name[:80]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--marker", default="k_auc")
    args = ap.parse_args()
    rows = []
    with open(args.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if args.marker in r[2]]
    if len(marks) < args.steps + 1:
        raise SystemExit(f"only {len(marks)} marker kernels")
    lo, hi = marks[-args.steps - 1] + 1, marks[-1] + 1
    win = rows[lo:hi]
    per = collections.defaultdict(lambda: [0, 0])
    busy = 0
    for s, e, n in win:
        k = short(n)
        per[k][0] += e - s
        per[k][1] += 1
        busy += e - s
    span = win[-1][1] - win[0][0]
    n = args.steps
    print(f"steps={n}  wall span/step={span / n / 1e3:.1f} us  GPU busy/step={busy / n / 1e3:.1f} us  "
          f"kernels/step={len(win) / n:.1f}")
    print(f"{'kernel':70s} {'us/step':>9s} {'calls/step':>10s} {'%busy':>6s}")
    for k, (t, c) in sorted(per.items(), key=lambda x: -x[1][0]):
        print(f"{k:70s} {t / n / 1e3:9.1f} {c / n:10.1f} {100 * t / busy:6.1f}")


if __name__ == "__main__":
    main()
