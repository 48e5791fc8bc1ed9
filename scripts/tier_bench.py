#!/usr/bin/env python3
"""BASELINE config 4 shape: the graph-captured fp32 DeepFM step (bench.py's
CtrTrainStep) trained pass by pass over a feature space much larger than the
HBM table, through the HBM <- host <- SSD tiers:

* every pass's batches are generated on the GPU before timing (synthetic
  Criteo-shaped, power-law ids) and fed to the captured step device-to-device;
* FeedPass of pass p+1 stages its working set (host probe, SSD reload, gather,
  H2D, insert into the second GPU table) in the background while pass p trains;
* EndPass exports the live table and writes it back (D2H, host scatter, pass
  stamps, SSD spill of the oldest passes beyond ``--host-cap`` rows) in the
  background while pass p+1 trains;
* ``--mode hbm`` trains the same passes from one all-in-HBM table for the
  reference point.

Per pass (stderr): begin/train/end times and whether the background staging /
write-back finished inside the training window.  One JSON line on stdout.

    python scripts/tier_bench.py --mode tiered --passes 5 --steps 1000 \\
        --features 1e9 --hbm-cap 6e7 --host-cap 1e8 --ssd /tmp/pbx_ssd
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from paddlebox_amd.data.synthetic import CriteoSynth  # noqa: E402
from paddlebox_amd.ps.box_wrapper import BoxWrapper  # noqa: E402
from paddlebox_amd.runtime.ctr_step import CtrTrainStep  # noqa: E402
from paddlebox_amd.runtime.graph_step import GraphedTrainStep, pack_batch  # noqa: E402


def log(msg):
    print(msg, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--passes", type=int, default=5)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--features", type=float, default=1e9)
    ap.add_argument("--hbm-cap", type=float, default=6e7)
    ap.add_argument("--host-cap", type=float, default=0, help="host-tier rows before the oldest passes spill to SSD")
    ap.add_argument("--ssd", type=str, default="")
    ap.add_argument("--mode", choices=("tiered", "hbm"), default="tiered")
    ap.add_argument("--spill-unseen", type=float, default=-1.0,
                    help="also spill host rows unseen for >= this many days (-1: off)")
    ap.add_argument("--precision", choices=("fp32", "bf16"), default="fp32")
    ap.add_argument("--no-retain", action="store_true",
                    help="write back / restage every row at each pass boundary (no GPU retention of next-pass rows)")
    ap.add_argument("--graph-steps", type=int, default=4,
                    help="training steps per captured graph (bench.py's headline step: 4)")
    ap.add_argument("--pipeline", choices=("on", "off"), default="on",
                    help="pipelined front (bench.py's headline step: on)")
    ap.add_argument("--headline-ms", type=float, default=0.0,
                    help="bench.py's ms/step on the same box: the steady ratio is also reported against it")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    synth = CriteoSynth(total_features=int(args.features), alpha=1.05, seed=7, device=str(dev))
    S = synth.S
    box = BoxWrapper(8, device=dev)
    box.cfg.tier.spill_unseen_days = args.spill_unseen
    box.cfg.tier.ssd_spill_threshold = int(args.host_cap)
    # hbm mode: a table sized for every key the passes touch
    cap = int(args.hbm_cap) if args.mode == "tiered" else int(args.hbm_cap) * args.passes
    box.initialize_gpu_and_load_model(slot_vector=list(range(1, S + 1)), max_keys=args.batch * S, capacity=cap,
                                      mode=args.mode, ssd_path=(args.ssd or None) if args.mode == "tiered" else None)
    if box.tier is not None:
        box.tier.retain = not args.no_retain
    t0 = time.perf_counter()
    passes = []
    for p in range(args.passes):
        passes.append([pack_batch(synth.batch(args.batch), device=dev) for _ in range(args.steps)])
    keys = [torch.cat([b.keys for b in bs]) for bs in passes]
    torch.cuda.synchronize()
    log(f"[tier] generated {args.passes} x {args.steps} batches in {time.perf_counter() - t0:.1f} s")
    torch.manual_seed(0)
    step = CtrTrainStep(box.engine, "deepfm", args.precision, num_slots=S, hidden=(400, 400, 400))
    rows, bg = [], []
    K = max(1, int(args.graph_steps))
    if args.steps % K:
        raise SystemExit("--steps must be a multiple of --graph-steps")
    pipe = ((lambda b, j: step.prefetch(b, j), step.set_next, box.engine.clear_prefetch)
            if args.pipeline == "on" else None)
    if pipe is not None:
        box.engine.ensure_pull_ring(3 * K)
    t_all = time.perf_counter()
    box.feed_pass(keys[0])
    g = None
    for p in range(args.passes):
        st0 = dict(box.tier.stats) if box.tier is not None else {}
        t0 = time.perf_counter()
        box.begin_pass()
        t1 = time.perf_counter()
        if p + 1 < args.passes:
            box.feed_pass(keys[p + 1])  # staged in the background while this pass trains
        t2 = time.perf_counter()
        bs = passes[p]
        if g is None:
            # capture once (the live table never moves); the warm steps train
            # the first K batches (so every pass trains whole graphs after it)
            g = GraphedTrainStep(step.train_step, bs[0], dev, warmup=0, warm_batches=bs[:K], n_buffers=3 if pipe else 2,
                                 pipeline=pipe, steps_per_graph=K, join_each_step=not step.adam_overlap)
            first = K
        else:
            # the activation rewrote the live table: every buffer set is
            # pooled again before its replay
            g.invalidate_prefetch()
            first = 0
        groups = [bs[i:i + K] if K > 1 else bs[i] for i in range(first, len(bs), K)]
        ahead = 2 if pipe is not None else 1
        for a in range(min(ahead, len(groups))):
            g.load(a % g.n, groups[a])
        for q in range(len(groups)):
            g.run(q % g.n)
            if q + ahead < len(groups):  # never past the pass: the next pass's rows are not live yet
                g.load((q + ahead) % g.n, groups[q + ahead])
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        # did the background work of this window finish while the pass trained?
        stage_done = box.tier is None or box.tier._stage_thread is None or not box.tier._stage_thread.is_alive()
        wb_done = box.tier is None or box.tier._wb_thread is None or not box.tier._wb_thread.is_alive()
        box.end_pass()
        t4 = time.perf_counter()
        st1 = dict(box.tier.stats) if box.tier is not None else {}
        d = {k: st1[k] - st0.get(k, 0) for k in st1}
        r = dict(pass_id=p, begin_pass_ms=(t1 - t0) * 1e3, feed_call_ms=(t2 - t1) * 1e3, train_ms=(t3 - t2) * 1e3,
                 end_pass_ms=(t4 - t3) * 1e3, live_rows=box.engine.table.size(),
                 stage_done_in_pass=stage_done, writeback_done_in_pass=wb_done,
                 host_rows=box.host.size() if box.host is not None else 0,
                 ssd_rows=len(box.ssd) if box.ssd is not None else 0)
        r.update({f"d_{k}": v for k, v in d.items()})
        rows.append(r)
        log("[tier] " + json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items()}))
    if box.tier is not None:
        box.tier.wait_writeback()
    wall = time.perf_counter() - t_all
    st = dict(box.tier.stats) if box.tier is not None else {}
    steady = rows[1:] if len(rows) > 1 else rows
    mid = rows[1:-1] if len(rows) > 2 else steady
    mid_wall = sum(r["begin_pass_ms"] + r["feed_call_ms"] + r["train_ms"] + r["end_pass_ms"] for r in mid) / 1e3
    mid_train = sum(r["train_ms"] for r in mid) / 1e3
    train_s = sum(r["train_ms"] for r in rows) / 1e3
    out = {
        "mode": args.mode, "precision": args.precision, "passes": args.passes, "steps_per_pass": args.steps,
        "batch": args.batch, "features": int(args.features), "hbm_cap_rows": cap, "host_cap_rows": int(args.host_cap),
        "wall_s": round(wall, 3), "samples_per_s": round(args.passes * args.steps * args.batch / wall, 1),
        "train_only_samples_per_s": round(args.passes * args.steps * args.batch / train_s, 1),
        "train_ms_per_step": round(sum(r["train_ms"] for r in steady) / (len(steady) * args.steps), 4),
        # steady state: passes 1 .. N-2 (pass 0 pays the first staging and the
        # graph capture, the last one the final full write-back), each pass's
        # main-thread wall = begin + feed call + train + end
        "steady_passes": len(mid),
        "steady_samples_per_s": round(len(mid) * args.steps * args.batch / max(mid_wall, 1e-9), 1),
        "steady_train_only_samples_per_s": round(len(mid) * args.steps * args.batch / max(mid_train, 1e-9), 1),
        "steady_ratio": round(mid_train / max(mid_wall, 1e-9), 4),
        "begin_pass_ms_mean": round(sum(r["begin_pass_ms"] for r in steady) / len(steady), 2),
        "end_pass_ms_mean": round(sum(r["end_pass_ms"] for r in steady) / len(steady), 2),
        "live_rows_mean": int(sum(r["live_rows"] for r in rows) / len(rows)),
        "host_rows": box.host.size() if box.host is not None else 0,
        "ssd_rows": len(box.ssd) if box.ssd is not None else 0,
        "stage_hidden_passes": sum(1 for r in rows if r["stage_done_in_pass"]),
        "writeback_hidden_passes": sum(1 for r in rows if r["writeback_done_in_pass"]),
        "tier_stats": {k: (round(v, 3) if isinstance(v, float) else v) for k, v in st.items()},
        "ssd_direct_io": bool(box.ssd.direct_io) if box.ssd is not None else None,
        "retain": bool(box.tier.retain) if box.tier is not None else None,
        "steps_per_graph": K, "pipelined_front": pipe is not None,
    }
    if args.headline_ms > 0:
        # against bench.py's headline step (its ms/step on this box): the
        # whole-pass wall of the steady passes vs the same steps at that rate
        out["headline_ms_per_step"] = args.headline_ms
        out["steady_ratio_vs_headline"] = round(len(mid) * args.steps * args.headline_ms / 1e3 / max(mid_wall, 1e-9), 4)
        out["train_ratio_vs_headline"] = round(args.headline_ms / max(out["train_ms_per_step"], 1e-9), 4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
