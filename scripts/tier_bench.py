#!/usr/bin/env python3
"""Scaled-down tiered-store run (BASELINE config 4 shape): DeepFM passes over
a feature space larger than the HBM cap, HBM <- host (<- SSD) staging of the
next pass overlapped with training, write-back overlapped with the next pass.
Prints per-pass timings and the tier statistics (stderr) and one JSON line.

    python scripts/tier_bench.py --passes 6 --steps 40 --features 5e7 --hbm-cap 4e6 [--ssd DIR]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from paddlebox_amd.data.synthetic import CriteoSynth  # noqa: E402
from paddlebox_amd.models.deepfm import DeepFM  # noqa: E402
from paddlebox_amd.parallel.dense import DenseArena, FlatAdam  # noqa: E402
from paddlebox_amd.ps.box_wrapper import BoxWrapper  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--passes", type=int, default=6)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--features", type=float, default=5e7)
    ap.add_argument("--hbm-cap", type=float, default=4e6)
    ap.add_argument("--ssd", type=str, default="")
    ap.add_argument("--mode", choices=("tiered", "hbm"), default="tiered")
    ap.add_argument("--spill-unseen", type=float, default=1.0,
                    help="write-back spills host rows unseen for >= this many days to SSD (0: every written-back row)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    synth = CriteoSynth(total_features=int(args.features), alpha=1.05, seed=7, device=str(dev))
    S = synth.S
    cap = int(args.hbm_cap) if args.mode == "tiered" else int(args.features)
    box = BoxWrapper(8, device=dev)
    box.cfg.tier.spill_unseen_days = args.spill_unseen
    box.initialize_gpu_and_load_model(slot_vector=list(range(1, S + 1)), max_keys=args.batch * S, capacity=cap,
                                      mode=args.mode, ssd_path=args.ssd or None)
    model = DeepFM(box.engine, num_slots=S, dense_dim=13, hidden=(400, 400, 400)).to(dev)
    arena = DenseArena(model.parameters(), dev)
    opt = FlatAdam(arena, lr=1e-3, clear_grad=True).fuse(mlps=[model.mlp], data_norms=[model.dn])
    one = torch.ones((), device=dev)
    passes = [[synth.batch(args.batch) for _ in range(args.steps)] for _ in range(args.passes)]
    keys = [torch.cat([b.keys for b in bs]) for bs in passes]
    t_all = time.perf_counter()
    box.feed_pass(keys[0])
    rows = []
    for p in range(args.passes):
        t0 = time.perf_counter()
        box.begin_pass()
        t1 = time.perf_counter()
        if p + 1 < args.passes:
            box.feed_pass(keys[p + 1])  # staged in the background while this pass trains
        t2 = time.perf_counter()
        for b in passes[p]:
            loss, _ = model(b)
            loss.backward(one)
            opt.step()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        box.end_pass()
        t4 = time.perf_counter()
        rows.append(dict(pass_id=p, begin_pass_ms=(t1 - t0) * 1e3, feed_call_ms=(t2 - t1) * 1e3,
                         train_ms=(t3 - t2) * 1e3, end_pass_ms=(t4 - t3) * 1e3,
                         live_rows=box.engine.table.size()))
        print("[tier]", json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in rows[-1].items()}),
              file=sys.stderr, flush=True)
    if box.tier is not None:
        box.tier.wait_writeback()
    wall = time.perf_counter() - t_all
    st = dict(box.tier.stats) if box.tier is not None else {}
    out = {
        "mode": args.mode, "passes": args.passes, "steps_per_pass": args.steps, "batch": args.batch,
        "features": int(args.features), "hbm_cap_rows": cap, "wall_s": round(wall, 3),
        "samples_per_s": round(args.passes * args.steps * args.batch / wall, 1),
        "train_ms_mean": round(sum(r["train_ms"] for r in rows[1:]) / max(1, len(rows) - 1), 2),
        "begin_pass_ms_mean": round(sum(r["begin_pass_ms"] for r in rows[1:]) / max(1, len(rows) - 1), 2),
        "end_pass_ms_mean": round(sum(r["end_pass_ms"] for r in rows[1:]) / max(1, len(rows) - 1), 2),
        "host_rows": box.host.size() if box.host is not None else 0,
        "ssd_rows": len(box.ssd) if box.ssd is not None else 0,
        "tier_stats": {k: (round(v, 3) if isinstance(v, float) else v) for k, v in st.items()},
        # staging of pass p+1 and write-back of pass p-1 run during pass p's training:
        # the part of their time the training hid
        "stage_s_total": round(st.get("stage_s", 0.0), 3),
        "train_s_total": round(sum(r["train_ms"] for r in rows) / 1e3, 3),
        "ssd_direct_io": bool(box.ssd.direct_io) if box.ssd is not None else None,
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
