#!/usr/bin/env python3
"""The fluid / BoxPS user path at the headline config: the canonical
PaddleBox program (pull_box_sparse -> fused_seqpool_cvm -> concat(dense) ->
data_norm -> fc 400-400-400 -> fc 1 -> sigmoid log-loss, Adam) over 26
Criteo-shaped slots + 13 dense, batch 8192, trained with
exe.train_from_dataset on an in-memory PadBoxSlotDataset (text lines parsed
by the native loader).  Prints one JSON line with samples/s of a steady-state
pass (stderr: per-pass stats).

    python scripts/bench_fluid.py [--batches 200] [--passes 3] [--no-graph]
        [--features 1e9] [--no-prefill] [--fc-precision fp32|bf16]
        [--steps-per-graph K] [--no-pipeline]

The table is pre-populated with all --features features (as bench.py does:
random-init rows, as if a base model was loaded), so the fluid step runs
against the same 1e9-row HBM table as the headline.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import paddlebox_amd.fluid as fluid  # noqa: E402
from paddlebox_amd.data.synthetic import CriteoSynth  # noqa: E402

S, DENSE = 26, 13


def build(hidden):
    main, startup = fluid.Program(), fluid.Program()
    with fluid.program_guard(main, startup), fluid.unique_name.guard():
        label = fluid.layers.data("label", shape=[1], dtype="int64")
        slots = [fluid.layers.data(f"slot{i}", shape=[1], dtype="int64", lod_level=1) for i in range(S)]
        dense = fluid.layers.data("dense", shape=[DENSE], dtype="float32")
        show = fluid.layers.fill_constant_batch_size_like(label, shape=[-1, 1], dtype="float32", value=1.0)
        click = fluid.layers.cast(label, "float32")
        cvm = fluid.layers.concat([show, click], axis=1)
        embs = fluid.layers._pull_box_sparse(slots, size=11)
        pooled = fluid.contrib.layers.fused_seqpool_cvm(embs, "sum", cvm)
        x = fluid.layers.concat(pooled + [dense], axis=1)
        x = fluid.layers.data_norm(x, name="dn")
        h = x
        for i, n in enumerate(hidden):
            h = fluid.layers.fc(h, n, act="relu", name=f"fc{i}")
        logit = fluid.layers.fc(h, 1, name="out")
        pred = fluid.layers.sigmoid(logit)
        loss = fluid.layers.reduce_mean(fluid.layers.sigmoid_cross_entropy_with_logits(logit, click))
        fluid.optimizer.BoxPSOptimizer(fluid.optimizer.Adam(learning_rate=1e-3)).minimize(loss)
    return main, startup, slots, label, dense, pred, loss


def lines_from(synth, B, n):
    """Text instances ("1 label | len ids... per slot | 13 dense") of n batches."""
    out = []
    for _ in range(n):
        b = synth.batch(B)
        keys = b.keys.cpu().numpy()
        lod = b.lod.cpu().numpy().reshape(S, B + 1)
        dense = b.dense.cpu().numpy()
        label = b.label.cpu().numpy().astype(np.int64)
        for i in range(B):
            toks = ["1", str(int(label[i]))]
            for s in range(S):
                a, e = lod[s, i], lod[s, i + 1]
                toks.append(str(e - a))
                toks.extend(str(int(k)) for k in keys[a:e])
            toks.append(str(DENSE))
            toks.extend(f"{v:.4g}" for v in dense[i])
            out.append(" ".join(toks))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--batches", type=int, default=200,
                    help="batches per pass (a pass of 40 measured 0.40 ms/step: its start / end costs over few steps)")
    ap.add_argument("--passes", type=int, default=3)
    ap.add_argument("--features", type=float, default=1e9)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-prefill", action="store_true")
    ap.add_argument("--fc-precision", choices=("fp32", "bf16"), default="fp32")
    ap.add_argument("--steps-per-graph", type=int, default=0)
    ap.add_argument("--no-pipeline", action="store_true")
    args = ap.parse_args()
    from paddlebox_amd.utils.flags import set_flags

    set_flags({"FLAGS_padbox_fc_precision": args.fc_precision,
               "FLAGS_padbox_train_steps_per_graph": args.steps_per_graph,
               "FLAGS_padbox_pipelined_front": not args.no_pipeline})
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    t0 = time.time()
    synth = CriteoSynth(total_features=int(args.features), alpha=1.05, seed=11, device=str(dev))
    lines = lines_from(synth, args.batch, args.batches)
    print(f"[fluid] generated {len(lines)} lines in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    box = fluid.core.BoxWrapper(8, device="cuda:0", new=True)
    cap = int(args.features) if not args.no_prefill else 20_000_000
    box.initialize_gpu_and_load_model(slot_vector=list(range(S)), max_keys=args.batch * S, capacity=cap)
    if not args.no_prefill:
        from paddlebox_amd.ops import reference as ref

        t2 = time.time()
        for chunk in synth.all_keys_chunks(1 << 26):
            box.engine.insert_local_mixed(ref.mix64(chunk), init_embedx=True)
        torch.cuda.synchronize()
        print(f"[fluid] prefilled {box.engine.table.size()} features "
              f"({box.engine.table.memory_bytes() / 2**30:.1f} GiB) in {time.time() - t2:.1f}s", file=sys.stderr,
              flush=True)
    main_p, startup, slots, label, dense, pred, loss = build((400, 400, 400))
    main_p._pipeline_opt = dict(main_p._pipeline_opt or {}, use_graph=not args.no_graph)
    exe = fluid.Executor(fluid.CUDAPlace(0))
    exe.run(startup)
    ds = fluid.DatasetFactory().create_dataset("PadBoxSlotDataset")
    ds.set_use_var([label] + slots + [dense])
    ds.set_batch_size(args.batch)
    ds.disable_shuffle()
    t1 = time.time()
    ds.add_lines(lines)
    print(f"[fluid] parsed {len(ds)} instances in {time.time() - t1:.1f}s", file=sys.stderr, flush=True)
    box.init_metric("AucCalculator", "auc", label.name, pred.name, bucket_size=100000)
    boxps = fluid.core.BoxPS(ds)
    box.feed_pass(ds)
    stats = []
    for p in range(args.passes):
        boxps.begin_pass()
        st = exe.train_from_dataset(main_p, ds, fetch_list=[loss], print_period=10 ** 9)
        boxps.end_pass()
        stats.append(st)
        print("[fluid] pass", p, json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in st.items()}),
              file=sys.stderr, flush=True)
    last = stats[-1]
    out = {"metric": "samples/sec, fluid train_from_dataset (canonical PaddleBox DeepFM-style program)",
           "value": round(last["ins_per_sec"], 1), "unit": "samples/s", "n_gpus": 1,
           "ms_per_step": round(last["seconds"] / max(1, last["batches"]) * 1e3, 4),
           "batches": last["batches"], "batch": args.batch, "graph": not args.no_graph,
           "graph_replays": last.get("graph_replays", 0), "auc": box.get_metric_msg("auc")[0],
           "fc_precision": args.fc_precision, "steps_per_graph": last.get("steps_per_graph", 1),
           "pipelined_front": last.get("pipelined_front", False), "table_rows": box.engine.table.size(),
           "step_s": round(last.get("step", 0.0), 4),
           "adam_overlap": bool(getattr(exe.sessions_for(main_p)[0], "side_adam", False))}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
