#!/usr/bin/env python3
"""Per-step kernel timeline of a rocprofv3 --kernel-trace database (the
``*_results.db`` it writes): steps are delimited by a marker kernel that runs
once per training step (default: the fp32 tower forward), the last ``--steps``
of them are analysed.

Per step: wall, GPU busy (union over all queues), idle.  Per kernel: mean
time per step, and its *exposed* time -- the part of its run during which no
other kernel was running, i.e. what it adds to the step when nothing hides it
(a critical-path proxy).

    python scripts/prof/step_timeline.py gpurun_out/prof_bench/bench_results.db --marker k_t32_fwd --steps 100
"""
import argparse
import sqlite3
from collections import defaultdict


def short(name: str) -> str:
    n = name.replace("pbx::(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0][:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="k_t32_fwd")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--timeline", action="store_true",
                    help="also list every kernel of the last step (us from its marker launch)")
    ap.add_argument("--which", type=int, default=1, help="with --timeline: the k-th last step")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end, queue_id from kernels order by start").fetchall()
    marks = [s for (n, s, e, q) in rows if a.marker in n]
    if len(marks) < a.steps + 1:
        raise SystemExit(f"only {len(marks)} marker kernels")
    t0, t1 = marks[-a.steps - 1], marks[-1]
    steps = a.steps
    ks = [(short(n), max(s, t0), min(e, t1), q) for (n, s, e, q) in rows if e > t0 and s < t1]
    # sweep: busy union and exposed (sole-running) time per kernel
    ev = []
    for i, (n, s, e, q) in enumerate(ks):
        ev.append((s, 1, i))
        ev.append((e, -1, i))
    ev.sort()
    running = set()
    busy = 0
    exposed = defaultdict(float)
    last = t0
    for t, d, i in ev:
        if running:
            busy += t - last
            if len(running) == 1:
                exposed[ks[next(iter(running))][0]] += t - last
        last = t
        if d > 0:
            running.add(i)
        else:
            running.discard(i)
    tot = defaultdict(float)
    cnt = defaultdict(int)
    for n, s, e, q in ks:
        tot[n] += e - s
        cnt[n] += 1
    wall = (t1 - t0) / steps / 1e3
    print(f"# {steps} steps between '{a.marker}' launches: wall {wall:.1f} us/step, GPU busy "
          f"{busy / steps / 1e3:.1f} us/step, idle {(t1 - t0 - busy) / steps / 1e3:.1f} us/step")
    print(f"| kernel | calls/step | us/step | exposed us/step |")
    print(f"|---|---|---|---|")
    for n in sorted(tot, key=lambda k: -exposed[k] - 1e-3 * tot[k])[:a.top]:
        print(f"| {n} | {cnt[n] / steps:.2f} | {tot[n] / steps / 1e3:.1f} | {exposed[n] / steps / 1e3:.1f} |")
    if a.timeline:
        a0, a1 = marks[-a.which - 1], marks[-a.which]
        print(f"\ntimeline of the last step (us from its '{a.marker}' start; queue id)")
        for n, s, e, q in rows:
            if e > a0 - 200_000 and s < a1:
                print(f"  {(s - a0) / 1e3:8.1f} {(e - a0) / 1e3:8.1f} {(e - s) / 1e3:6.1f}  q{q}  {short(n)}")


if __name__ == "__main__":
    main()
