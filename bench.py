#!/usr/bin/env python3
"""Headline benchmark: samples/sec (whole node) for Criteo-1TB-shape DeepFM.

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W

One process per GPU (RCCL over xGMI).  Config (BASELINE.json "DeepFM
Criteo-1TB-shape"): 26 sparse slots over a 1e9-feature space (Criteo-1TB
per-slot cardinalities scaled to 1B, power-law id popularity), 13 dense
features, 8-dim embedx (+show/click/embed_w = 11-wide pull records), sparse
Adagrad in the GPU parameter server, DeepFM (FM + data_norm + MLP 400-400-400)
with the MLP at fp32 precision (fp32 storage and accumulation, every product as
three bf16 MFMAs on hi + lo halves: finer than the TF32 math the reference's
fp32 fc runs on by default) and fused Adam; the same run also times the
exact-fp32 tower (fp32 MFMA products) and DCN-V2 (BASELINE config 5) as
secondaries in ``config``.  The feature table is pre-populated with
all 1e9 features (random-init weights, as if a base model was loaded) and
sharded across GPUs by hash; keys are exchanged with all-to-all each step.
Weak scaling: the per-GPU batch is fixed.  Each timed step = a device-to-device
copy of the step's batch into the captured graph's inputs (the pass's
synthetic batches are HBM-resident, ``--inputs hbm``, default; ``--inputs
host`` copies it H2D from pinned host memory instead) + pull + forward +
backward + sparse push/Adagrad + dense all-reduce + Adam.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# the package (and its HIP extension) is imported inside main(), after the
# launcher decision: a parent that spawns one rank per GPU never loads it

METRIC = "samples/sec (whole node) on Criteo-1TB-shape DeepFM"
METRIC_DCN = "samples/sec (whole node) on Criteo-1TB-shape DCN-V2 (BASELINE config 5)"


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


def _free_port() -> int:
    import socket

    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _visible_gpus() -> int:
    # device_count() does not initialise the HIP runtime on this image
    return torch.cuda.device_count()


def launch_ranks(argv, n: int, dry: bool) -> int:
    """``bench.py --gpus N`` started without a launcher: run one rank per GPU
    (torch.distributed.run over 127.0.0.1) as CHILD processes of this parent,
    which never touches the GPU itself, relay their output (rank 0 prints the
    JSON line) and exit with the worst child return code.  Reference: one
    worker per device, boxps_trainer.cc:53-79."""
    import subprocess

    if not dry and "--same-gpu" not in argv:  # the same-GPU rehearsal runs every rank on cuda:0
        have = _visible_gpus()
        if n > have:
            print(f"[bench] --gpus {n} but only {have} GPU(s) visible: refusing to measure fewer GPUs than asked",
                  file=sys.stderr, flush=True)
            return 3
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py")] + list(argv)
    env = dict(os.environ)
    env["PBX_BENCH_LAUNCHER"] = "bench.py-spawn"
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    print(f"[bench] launching {n} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True, bufsize=1)
    for line in p.stdout:
        sys.stdout.write(line)
        sys.stdout.flush()
    return p.wait()


def dry_run(args, world, rank):
    """CPU rehearsal of the launcher contract (gloo): every rank joins the
    group, the rank count is all-reduced and rank 0 prints the JSON line with
    ``config.ranks_seen``.  No GPU, no model: tests the plumbing only."""
    one = torch.ones(1)
    if "WORLD_SIZE" in os.environ:
        dist.init_process_group("gloo", init_method="env://")
        dist.all_reduce(one)
        dist.barrier()
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "samples/s", "n_gpus": world,
                          "steps": args.steps, "warmup": args.warmup, "dry_run": True,
                          "config": {"ranks_seen": int(one.item()),
                                     "launcher": os.environ.get("PBX_BENCH_LAUNCHER", "external")}}), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()




def graph_steps_for(steps: int, warmup: int, requested: int = 0, world: int = 1) -> int:
    """Steps per captured graph: every timed and warmup step still runs in
    full; only the graph-launch boundary (and the wait on the batch copy) is
    paid once per K steps instead of once per step.  requested -1 (default):
    4, else 2, else 1 -- the largest that divides the timed steps (the warmup
    is rounded up to whole graphs; K = 4 vs 2: 0.362-0.364 vs ~0.368 ms/step
    over 200 steps, profiles/r4_input_stall.txt)."""
    if requested < 0:
        # multi-rank: 2 (the same-GPU 2-rank rehearsal ran 1.43 ms/step at
        # K = 2 and 2.51 at K = 4; K = 2 is the validated multi-rank form)
        if world == 1 and steps % 4 == 0:
            return 4
        return 2 if steps % 2 == 0 else 1
    if requested > 0:
        if steps % requested:
            raise SystemExit(f"--graph-steps {requested} must divide --steps {steps}")
        return requested
    for k in range(8, 0, -1):
        if steps % k == 0 and warmup % k == 0:
            return k
    return 1


def _build_summary() -> dict:
    """Provenance of the loaded gfx950 libraries (build stamp vs this tree's sources)."""
    from paddlebox_amd import _native

    bi = _native.build_info()
    st = bi["stamp"] or {}
    return {"sources": st.get("sources"), "sources_match_tree": bi["matches_tree"], "hipcc": st.get("hipcc"),
            "built_at": st.get("built_at")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--batch-per-gpu", type=int, default=8192)
    ap.add_argument("--total-features", type=float, default=1e9)
    ap.add_argument("--alpha", type=float, default=1.05)
    ap.add_argument("--num-batches", type=int, default=128,
                    help="distinct synthetic batches cycled (enough that the model does not memorise them)")
    ap.add_argument("--no-prefill", action="store_true")
    ap.add_argument("--hidden", type=str, default="400,400,400")
    ap.add_argument("--graph", dest="graph", action="store_true", default=True,
                    help="capture the train step into HIP graphs (default)")
    ap.add_argument("--no-graph", dest="graph", action="store_false")
    ap.add_argument("--diag-windows", type=int, default=0,
                    help="after the measurement, time this many more K-step windows (stderr only)")
    ap.add_argument("--graph-steps", type=int, default=-1,
                    help="training steps per captured HIP graph (0 = auto: the largest k <= 8 dividing both --steps "
                         "and --warmup).  Default -1: 4 on one rank when it divides --steps, else 2 when it "
                         "does, else 1 (multi-rank: 2); see graph_steps_for")
    ap.add_argument("--graph-warm", type=int, default=32,
                    help="load+replay cycles run right after capture (runtime warm-up, part of graph setup)")
    ap.add_argument("--trace-steps", type=int, default=0,
                    help="before warmup, print per-step host time of load / replay for this many steps (stderr)")
    ap.add_argument("--host-diag", action="store_true",
                    help="after the measurement, split host time into replay / H2D load (stderr only)")
    ap.add_argument("--mlp-dtype", choices=("bf16", "fp32", "fp32x3"), default="fp32x3",
                    help="fp32x3 (default headline): fp32 operands / accumulation with every product as three "
                         "bf16 MFMAs on hi + lo halves (tower_x3.hip) -- finer than the TF32 math the reference's "
                         "fp32 fc runs on by default (gpu_context.cc:65-67,580-588); fp32: exact fp32 products "
                         "(tower32.hip, v_mfma_f32_16x16x4_f32); bf16: the bf16 MFMA tower"),
    ap.add_argument("--secondary-dtype", choices=("auto", "fp32", "fp32x3", "bf16", "none"), default="auto",
                    help="after the headline measurement, time the same K steps at this MLP precision in the same "
                         "run and report it in config (auto: the other precision when the headline is DeepFM on "
                         "one GPU)")
    ap.add_argument("--secondary-dcn", choices=("auto", "on", "off"), default="auto",
                    help="also time DCN-V2 (BASELINE config 5, bf16 MLP) in the same run over the same sparse "
                         "engine and report it in config (auto: on for the one-GPU DeepFM headline)")
    ap.add_argument("--model", choices=("deepfm", "dcn_v2"), default="deepfm",
                    help="deepfm = the headline config; dcn_v2 = BASELINE config 5 (cross layers on the MFMA GEMM)")
    ap.add_argument("--cross-layers", type=int, default=3)
    ap.add_argument("--pipeline", choices=("auto", "on", "off"), default="auto",
                    help="pipelined pull with the whole sparse front: each graph pools the next batch (dedup + "
                         "seqpool) right after its sparse push, under its dW GEMM (3 batch buffers).  auto: on for "
                         "the fp32 DeepFM step (0.399 vs 0.417 ms, same box), off for the bf16 / DCN-V2 steps, "
                         "whose shorter dW hides less of it (0.244 vs 0.241, 0.397 vs 0.386)")
    ap.add_argument("--prefetch", dest="prefetch", action="store_true", default=False,
                    help="pipelined pull: batch i+1's dedup + probe on a side stream beside batch i's dense "
                         "work (measured slower on one MI355X: 0.356 vs 0.281 ms/step, see "
                         "profiles/r2_bench_prefetch.txt)")
    ap.add_argument("--no-prefetch", dest="prefetch", action="store_false")
    ap.add_argument("--dense", choices=("ipc", "rccl"), default="ipc",
                    help="multi-rank dense gradient all-reduce: the in-house IPC mesh (xGMI peer writes, "
                         "two-phase; self-tested, falls back to RCCL) or RCCL")
    ap.add_argument("--sparse-exchange", choices=("ipc", "rccl"), default="ipc",
                    help="multi-rank sparse key/value/grad exchange: IPC mesh (self-tested, falls back to RCCL) "
                         "or RCCL all_to_all")
    ap.add_argument("--same-gpu", action="store_true",
                    help="rehearsal: every rank on cuda:0 with a gloo control plane (all in-step collectives "
                         "then run on the IPC meshes); exercises the N-GPU step on one GPU")
    ap.add_argument("--force-collectives", action="store_true",
                    help="run the multi-GPU exchange/all-reduce path even on 1 rank (rehearsal)")
    ap.add_argument("--dedup", choices=("on", "off"), default="on",
                    help="FLAGS_enable_pullpush_dedup_keys: off = single-shard step without a key dedup "
                         "(per-occurrence probe + leader-elected push merge)")
    ap.add_argument("--inputs", choices=("host", "hbm"), default="hbm",
                    help="hbm (default): the pass's packed batches are kept in HBM and each step copies its batch "
                         "into the graph inputs device-to-device; host: a pinned host-to-device DMA per step, whose "
                         "hipMemcpyAsync blocks the launching thread 7-19 ms once early in a fresh timing window "
                         "(20-step windows measured 0.69-1.10 vs 0.40 ms/step, profiles/r4_input_stall.txt)")
    ap.add_argument("--gc-off", type=int, default=1,
                    help="1: Python's cyclic GC disabled inside the timed window (collected just before)")
    ap.add_argument("--trace-timed", action="store_true",
                    help="diagnostics: host time of every replay inside the timed window")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU/gloo rehearsal of the multi-rank launch (no GPU, no model); prints ranks_seen")
    args = ap.parse_args()
    if args.force_collectives:
        os.environ["PBX_FORCE_COLLECTIVES"] = "1"

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher around us: start one rank per GPU ourselves
        sys.exit(launch_ranks(sys.argv[1:], args.gpus, args.dry_run))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        return dry_run(args, world, rank)
    if world != args.gpus and rank == 0:
        log(rank, f"[bench] note: --gpus {args.gpus} but the launcher started {world} ranks; measuring {world}")
    launcher = os.environ.get("PBX_BENCH_LAUNCHER", "torchrun" if "WORLD_SIZE" in os.environ else "single")

    from paddlebox_amd.data.synthetic import CriteoSynth
    from paddlebox_amd.ops import reference as ref
    from paddlebox_amd.runtime.ctr_step import CtrTrainStep
    from paddlebox_amd.ps.config import PSConfig
    from paddlebox_amd.ps.sparse_engine import SparseEngine

    if args.same_gpu:
        # all ranks' spinning IPC collectives share one GPU's workgroup slots:
        # together they hold at most half the CUs, so a peer's whole-CU kernels
        # (the x3 tower: 104 KB LDS and 2 x 237 VGPRs per SIMD per workgroup)
        # still find CUs to run on while the others spin (with 256 // W blocks
        # per rank the 4-rank rehearsal hit the IPC spin bound)
        os.environ.setdefault("PBX_IPC_MAX_BLOCKS", str(max(8, min(64, 128 // max(1, world)))))
    gpu_index = 0 if args.same_gpu else local_rank
    torch.cuda.set_device(gpu_index)
    device = torch.device("cuda", gpu_index)
    multi = world > 1 or args.force_collectives
    ranks_seen = 1
    # control-plane tensors live where the backend wants them
    cdev = torch.device("cpu") if args.same_gpu else device
    if multi:
        if args.same_gpu:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=device)
        seen = torch.ones(1, device=cdev)
        dist.all_reduce(seen)
        ranks_seen = int(seen.item())

    B = args.batch_per_gpu
    total = int(args.total_features)
    synth = CriteoSynth(total_features=total, alpha=args.alpha, seed=1000 + rank, device=str(device))
    S = synth.S
    cfg = PSConfig(embedx_dim=8)

    # "load into memory": the pass's batches live in pinned host memory; every
    # step copies its batch H2D (one DMA) on a side stream, overlapped
    from paddlebox_amd.runtime.graph_step import pack_batch

    host_batches = [pack_batch(synth.batch(B).to("cpu"), pin=True) for _ in range(args.num_batches)]
    # sparse work per step: distinct keys per batch (U) over key occurrences (L)
    u_per_batch = [int(torch.unique(hb.keys.to(device)).numel()) for hb in host_batches]
    l_per_batch = int(host_batches[0].keys.numel())
    u_over_l = sum(u_per_batch) / (len(u_per_batch) * l_per_batch)
    xcap = None
    if multi:
        # the pass is known before it is trained (BoxPS feed pass): size the key
        # exchange exactly by distinct keys per owner, max over batches and ranks
        from paddlebox_amd.ps.sparse_engine import exchange_capacity_for

        xc = torch.tensor([exchange_capacity_for([hb.keys.to(device) for hb in host_batches], world)], device=cdev)
        dist.all_reduce(xc, op=dist.ReduceOp.MAX)
        xcap = int(xc.item())
        log(rank, f"[bench] key exchange capacity {xcap} per peer (heuristic bound would be "
                  f"{int(math.ceil(B * S / world * 1.25)) + 64})")
    engine = SparseEngine(cfg, max_keys=B * S, device=device, capacity=synth.total_features,
                          slot_ids=[float(s + 1) for s in range(S)], auto_insert=args.no_prefill,
                          exchange_capacity=xcap, exchange=args.sparse_exchange, dedup=args.dedup == "on",
                          pull_ring=(3 * graph_steps_for(args.steps, args.warmup, args.graph_steps, world)
                                     if args.pipeline != "off" else 2))

    t0 = time.time()
    if not args.no_prefill:
        n_ins = 0
        for chunk in synth.all_keys_chunks(1 << 26):
            h = ref.mix64(chunk)
            if world > 1:
                h = h[ref.owner_of(h, world) == rank]
            engine.insert_local_mixed(h, init_embedx=True)
            n_ins += h.numel()
        torch.cuda.synchronize()
        log(rank, f"[bench] prefilled {n_ins} features on rank0 (table size {engine.table.size()}, "
                  f"{engine.table.memory_bytes() / 2**30:.1f} GiB) in {time.time() - t0:.1f}s")

    def measure(mlp_dtype: str, primary: bool, model_name: str = args.model):
        """Build the model at this MLP precision over the shared sparse engine,
        capture the step, run W warmup + K timed steps; returns the timings."""
        hidden = tuple(int(x) for x in args.hidden.split(","))
        dcn = model_name == "dcn_v2"
        # nothing a previous measurement prepared steers this one's capture, and
        # the pull slots' occurrence rows are all -1 again (a pipelined run
        # leaves rows there, which a split pull must not read as occurrences)
        engine.clear_prefetch(reset_rows=True)
        if dcn and mlp_dtype in ("fp32", "fp32x3"):
            raise SystemExit("DCN-V2 (BASELINE config 5) is a bf16-MLP config: run it with --mlp-dtype bf16")
        auc_table = torch.zeros(2 * 1_000_000, dtype=torch.float64, device=device)
        auc_stats = torch.zeros(5, dtype=torch.float64, device=device)
        # the model, dense arena + fused Adam, the dense all-reduce (IPC mesh
        # launched from the tower's dense-grads hook, RCCL fallback) and the
        # data_norm statistics in the gradient bucket: runtime/ctr_step.py
        # the pipelined front (next batch pooled after the push): fp32 DeepFM by
        # default; multi-rank it runs the sharded pull with its IPC exchanges
        # inside the graphs and pairs with the dW GEMM + IPC dense all-reduce
        # on the side stream (rehearsal 0.526 -> 0.434 ms/step with both,
        # either alone no faster: profiles/r4_sharded_pipeline_ab.txt);
        # PBX_SHARDED_PIPELINE=0 turns the multi-rank form off
        # and DCN-V2 on one rank, with the next batch's dedup after the head
        # backward (CtrTrainStep's default there, profiles/r6_dcn_split_ab.txt)
        # bf16 DeepFM on one rank too: 0.2161 / 0.2165 vs 0.2188 / 0.2199
        # ms/step without it (profiles/r6_pipeline_bf16_split_ab.txt)
        want_pipe = args.pipeline == "on" or (args.pipeline == "auto" and (
            (mlp_dtype in ("fp32", "fp32x3") and not dcn) or (not multi)))
        pipe_ok = args.graph and engine.can_prefetch_pull() and (
            not engine.sharded or os.environ.get("PBX_SHARDED_PIPELINE", "1") == "1")
        use_pipe = want_pipe and pipe_ok and not (args.prefetch and engine.can_prefetch())
        # (not in the same-GPU rehearsal: its W processes' spinning collectives
        # share one GPU's CU slots, and two concurrent meshes per process ran
        # into the IPC wait bound there)
        set_ov = (use_pipe and engine.sharded and not args.same_gpu
                  and "PBX_OVERLAP_DW_IPC" not in os.environ)
        if set_ov:
            os.environ["PBX_OVERLAP_DW_IPC"] = "1"  # read by CtrTrainStep's constructor only
        step = CtrTrainStep(engine, model_name, mlp_dtype, num_slots=S, dense_dim=13, hidden=hidden,
                            cross_layers=args.cross_layers, multi=multi, dense=args.dense, same_gpu=args.same_gpu,
                            fused_auc=(auc_table, auc_stats), log=lambda m: log(rank, "[bench] dense " + m))
        if set_ov:
            del os.environ["PBX_OVERLAP_DW_IPC"]
        model, opt, arena, sync, ipc, fused = step.model, step.opt, step.arena, step.sync, step.ipc, step.fused

        # every pinned batch buffer is streamed to the device once up front so the
        # timed steps do not pay the driver's first-touch cost of a pinned range
        scratch = torch.empty_like(host_batches[0]._flat, device=device)
        for hb in host_batches:
            scratch.copy_(hb._flat, non_blocking=True)
        torch.cuda.synchronize()
        del scratch
        from paddlebox_amd.runtime.streams import side_stream

        copy_stream = side_stream(device, "graph_copy")
        train_step = step.train_step

        nb = len(host_batches)
        # every measurement (headline and same-run secondaries) takes K steps
        # per graph over the same engine (tests/test_gpu_pipeline.py: a
        # pipelined K = 4 program followed by a plain K = 2 one)
        K = graph_steps_for(args.steps, args.warmup, args.graph_steps, world)
        graphed = None
        if args.graph:
            try:
                from paddlebox_amd.runtime.graph_step import GraphedTrainStep

                pre = (engine, lambda b: b.keys) if (args.prefetch and engine.can_prefetch()) else None
                pipe = None
                if use_pipe and pre is None:
                    pipe = (lambda b, j: step.prefetch(b, j), step.set_next, engine.clear_prefetch)
                graphed = GraphedTrainStep(train_step, host_batches[0], device, prefetch=pre,
                                           steps_per_graph=K if pre is None else 1,
                                           n_buffers=3 if pipe is not None else 2, pipeline=pipe,
                                           join_each_step=not (step.adam_overlap or step.adam_overlap_multi))
                if args.inputs == "hbm":
                    graphed.stage_inputs(host_batches)
                graphed.warm(host_batches, replays=args.graph_warm)
                log(rank, f"[bench] training step captured into HIP graphs ({args.graph_warm} warm replays)")
            except Exception as e:  # pragma: no cover - depends on runtime
                log(rank, f"[bench] graph capture failed ({e!r}); running eagerly")
                graphed = None
                # no pooling ahead in the eager loop: forget what the capture prepared
                step.set_next(None)
                engine.clear_prefetch()

        if graphed is not None:
            K = graphed.K  # run(i) trains group i: steps i*K .. i*K+K-1

            def group(i):
                return host_batches[i % nb] if K == 1 else [host_batches[(i * K + k) % nb] for k in range(K)]

            # buffers in flight ahead of the replay: graph i of a pipelined
            # step also reads buffer i+1, so its copy is issued a step earlier
            ahead = 2 if graphed.pipeline is not None else 1
            for a in range(ahead):
                graphed.load(a % graphed.n, group(a))

            load_marks = []

            def run(i):
                # launch first, then queue the copy for the set `ahead` replays
                # on: the copy waits (on the device) for the replay that last
                # read that set, so the order changes nothing but the host time
                # in front of this replay's launch
                out = graphed.run(i % graphed.n)
                graphed.load((i + ahead) % graphed.n, group(i + ahead))
                if args.trace_timed:
                    load_marks.append(time.perf_counter())
                return out
        else:
            K = 1

            def fetch(i):
                with torch.cuda.stream(copy_stream):
                    b = host_batches[i % nb].to(device, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(copy_stream)
                return b, ev

            pending = [fetch(0)]

            def run(i):
                b, ev = pending.pop()
                pending.append(fetch(i + 1))
                torch.cuda.current_stream().wait_event(ev)
                for t in (b.keys, b.lod, b.dense, b.label, b.cvm):
                    t.record_stream(torch.cuda.current_stream())
                return train_step(b)

        if primary and args.trace_steps and graphed is not None and K == 1:
            # diagnostics: per-step host time of the H2D load and the replay
            tl, tr = [], []
            for i in range(args.trace_steps):
                t0 = time.perf_counter()
                graphed.load((i + 1) % graphed.n, host_batches[(i + 1) % nb])
                t1 = time.perf_counter()
                graphed.run(i % graphed.n)
                tr.append(time.perf_counter() - t1)
                tl.append(t1 - t0)
            torch.cuda.synchronize()
            log(rank, "[bench] trace load us: " + " ".join(f"{x * 1e6:.0f}" for x in tl))
            log(rank, "[bench] trace run  us: " + " ".join(f"{x * 1e6:.0f}" for x in tr))
        # K divides both counts (graph_steps_for): exactly W warmup and K timed steps
        # warmup in whole graphs: W rounded up to a multiple of K (at most K-1
        # extra untimed steps); the timed steps are exactly K * sg = --steps
        wg, sg = -(-args.warmup // K), args.steps // K
        import gc

        gc.collect()
        for i in range(wg):
            run(i)
        torch.cuda.synchronize()
        if multi:
            dist.barrier()
        torch.cuda.synchronize()
        if graphed is not None:
            graphed.drained()
        import gc

        gcev = []
        if primary and args.trace_timed:
            def _gc_cb(phase, info, _ev=gcev):
                _ev.append((phase, info.get("generation"), time.perf_counter()))
            gc.callbacks.append(_gc_cb)
        # Python's cyclic GC off inside the timed window (as timeit does): a
        # generation-2 pass over the graphs' / model's objects blocks the host
        # for ~10 ms, longer than the few replays it keeps queued.  The
        # collection itself runs before the warmup replays (a collection right
        # before the window idles the GPU for tens of ms first)
        gc_was = gc.isenabled()
        if args.gc_off:
            gc.disable()
        t_start = time.perf_counter()
        loss = None
        tt = [] if (primary and args.trace_timed) else None
        if tt is not None and graphed is not None:
            graphed.trace = []
        for i in range(sg):
            loss = run(wg + i)
            if tt is not None:
                tt.append(time.perf_counter())
        t_enq = time.perf_counter() - t_start
        if gc_was:
            gc.enable()
        if gcev:
            gc.callbacks.pop()
            log(rank, "[bench] gc in timed window: " + " ".join(
                f"{ph[0]}{gen}@{(t - t_start) * 1e6:.0f}" for ph, gen, t in gcev if t >= t_start))
        if tt is not None:
            torch.cuda.synchronize()
            t_end = time.perf_counter()
            marks = [t_start] + tt
            log(rank, "[bench] timed-window host us per replay: "
                + " ".join(f"{(b - a) * 1e6:.0f}" for a, b in zip(marks, marks[1:]))
                + f" | drain {(t_end - marks[-1]) * 1e6:.0f}")
            if graphed is not None and graphed.trace:
                tr = graphed.trace[-len(tt):]
                log(rank, "[bench] timed-window throttle-wait/rest us: "
                    + " ".join(f"{a * 1e6:.0f}/{b * 1e6:.0f}" for a, b in tr))
            lm = load_marks[-len(tt):] if graphed is not None else []
            if lm:
                log(rank, "[bench] timed-window load us: "
                    + " ".join(f"{(l - a) * 1e6:.0f}" for a, l in zip(marks, lm)))
        torch.cuda.synchronize()
        if multi:
            dist.barrier()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t_start
        if multi:
            t = torch.tensor([dt], device=cdev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        log(rank, f"[bench] host enqueue {t_enq / args.steps * 1e3:.4f} ms/step, wall {dt / args.steps * 1e3:.4f} ms/step")
        # diagnostics only (after the measurement): further windows of K steps
        for w in range(args.diag_windows if primary else 0):
            torch.cuda.synchronize()
            t0w = time.perf_counter()
            for i in range(sg):
                run(wg + sg * (w + 1) + i)
            torch.cuda.synchronize()
            log(rank, f"[bench] diag window {w}: {(time.perf_counter() - t0w) / args.steps * 1e3:.4f} ms/step")
        if primary and args.host_diag and graphed is not None and K == 1:
            # where the host time of a step goes: replay alone, H2D load alone, both
            for name, fn in (("replay", lambda i: graphed.graphs[i % 2][0].replay()),
                             ("load", lambda i: graphed.load(i % 2, host_batches[i % nb])),
                             ("load+run", lambda i: run(i))):
                for w in range(3):
                    torch.cuda.synchronize()
                    t0w = time.perf_counter()
                    for i in range(args.steps):
                        fn(i)
                    th = time.perf_counter() - t0w
                    torch.cuda.synchronize()
                    tw = time.perf_counter() - t0w
                    log(rank, f"[bench] host-diag {name} window {w}: host {th / args.steps * 1e3:.4f} "
                              f"wall {tw / args.steps * 1e3:.4f} ms/step")

        # the kernels' index guards (skipped + recorded, never followed) must
        # not have tripped anywhere in this measurement
        engine.check_guards()
        res = dict(dt=dt, t_enq=t_enq, graph_steps=K, loss=float(loss) if loss is not None else float("nan"),
                   auc_stats=auc_stats.clone(), ipc=ipc,
                   prefetch=bool(graphed is not None and graphed.prefetch is not None),
                   pipeline=bool(graphed is not None and graphed.pipeline is not None), fused=fused)
        # free this precision's graphs / model before the next measurement
        del graphed, model, opt, arena, sync, step
        return res

    hidden = tuple(int(x) for x in args.hidden.split(","))
    dcn = args.model == "dcn_v2"
    if dcn and args.mlp_dtype in ("fp32", "fp32x3"):
        args.mlp_dtype = "bf16"  # config 5 names a bf16 MLP
    res = measure(args.mlp_dtype, True)
    dt, t_enq, loss, auc_stats, ipc = res["dt"], res["t_enq"], res["loss"], res["auc_stats"], res["ipc"]
    overflow_1 = engine.check_overflow()
    if ipc is not None:
        ipc.check()
    second = None
    sec_dtype = args.secondary_dtype
    if sec_dtype == "auto":
        # one GPU: the driver's headline run; the N-GPU scaling runs keep one measurement
        # (fp32x3 headline: the exact-fp32 step, so both fp32-class numbers come from one run)
        sec_dtype = ("bf16" if args.mlp_dtype == "fp32" else "fp32") if (not dcn and world == 1) else "none"
    if dcn:
        sec_dtype = "none"

    def _release():
        nonlocal ipc
        if ipc is not None:
            ipc.close()
            ipc = None
        import gc

        gc.collect()
        if os.environ.get("PBX_BENCH_KEEP_CACHE", "0") != "1":
            torch.cuda.empty_cache()

    if sec_dtype != "none" and sec_dtype != args.mlp_dtype:
        # same run, same sparse engine: the other MLP precision's step time
        _release()
        second = measure(sec_dtype, False)
        ipc = second["ipc"]
        log(rank, f"[bench] {sec_dtype} MLP: {second['dt'] / args.steps * 1e3:.4f} ms/step")
    dcn_res = None
    if args.secondary_dcn == "on" or (args.secondary_dcn == "auto" and not dcn and world == 1):
        # BASELINE config 5 (DCN-V2, bf16 MLP) over the same sparse engine
        _release()
        dcn_res = measure("bf16", False, "dcn_v2")
        ipc = dcn_res["ipc"]
        log(rank, f"[bench] DCN-V2: {dcn_res['dt'] / args.steps * 1e3:.4f} ms/step")

    overflow = engine.check_overflow() or overflow_1  # also raises if an IPC exchange timed out
    if ipc is not None:
        ipc.check()
    samples = B * world * args.steps
    value = samples / dt
    if rank == 0:
        st = auc_stats.cpu().tolist()
        log(rank, f"[bench] loss={float(loss):.4f} actual_ctr={st[3] / max(st[4], 1):.4f} "
                  f"pred_ctr={st[2] / max(st[4], 1):.4f} overflow={overflow}")
        out = {
            "metric": METRIC_DCN if dcn else METRIC,
            "value": round(value, 1),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.mlp_dtype,
            "data": "synthetic (Criteo-1TB-shape: 13 dense + 26 sparse slots, 1e9-feature space, "
                    f"power-law alpha={args.alpha}), random-init weights",
            "config": {
                "model": ("DCN-V2 (%d full-rank cross layers + data_norm + MLP %s), embedx_dim=8, sparse Adagrad GPU PS"
                          % (args.cross_layers, args.hidden)) if dcn else
                         ("DeepFM (FM + data_norm + MLP %s), embedx_dim=8, sparse Adagrad GPU PS" % args.hidden),
                "global_batch": B * world,
                "batch_per_gpu": B,
                "seq_len": S,
                "total_features": synth.total_features,
                "parallelism": f"dp{world}+sparse-shard{world}",
                "ranks_seen": ranks_seen,
                "launcher": launcher,
                "dense_allreduce": ("ipc" if ipc is not None else "rccl") if multi else "none",
                "sparse_exchange": engine.exchange_mode,
                "inputs": ("HBM-resident synthetic batches, device-to-device copy into the captured graph inputs every step" if args.inputs == "hbm" else "pinned host batches, host-to-device DMA every step"),
                "same_gpu_rehearsal": bool(args.same_gpu),
                "pipelined_pull": res["prefetch"],
                "pipelined_front": res.get("pipeline", False),
                "steps_per_graph": res.get("graph_steps", 1),
                "key_dedup": bool(engine.dedup),
                "mlp_dtype": args.mlp_dtype,
                **({"mlp_precision": "fp32 activations / weights / accumulation; each fp32 operand carried as bf16 "
                                     "hi + lo halves (16 significant bits) and each product as hi*hi + hi*lo + "
                                     "lo*hi on bf16 MFMA: dot-product error <= ~2^-15 of sum |terms| (tested "
                                     "element-wise at 2^-13 against fp64, tests/test_gpu_tower_x3.py); the "
                                     "reference's fp32 fc runs TF32 by default (11-bit inputs, ~2^-10): "
                                     "paddle/phi/backends/gpu/gpu_context.cc:65-67,580-588"}
                   if args.mlp_dtype == "fp32x3" else {}),
                **({f"{sec_dtype}_ms_per_step": round(second["dt"] / args.steps * 1e3, 4),
                    f"{sec_dtype}_samples_per_s": round(B * world * args.steps / second["dt"], 1),
                    f"{sec_dtype}_mlp": ("exact fp32 products on v_mfma_f32_16x16x4_f32 (the reference fc with "
                                         "FLAGS_enable_cublas_tf32_op_math off)" if sec_dtype == "fp32" else
                                         "fp32x3: fp32 via bf16 hi + lo halves, three MFMA products"
                                         if sec_dtype == "fp32x3" else "bf16 operands on bf16 MFMA, fp32 "
                                         "accumulate") + ", same run, same sparse engine"}
                   if second is not None else {}),
                **({"dcn_v2_ms_per_step": round(dcn_res["dt"] / args.steps * 1e3, 4),
                    "dcn_v2_samples_per_s": round(B * world * args.steps / dcn_res["dt"], 1),
                    "dcn_v2_model": "DCN-V2 (%d full-rank cross layers + data_norm + MLP %s, bf16 MFMA), BASELINE "
                                    "config 5 shape on one GPU, same run, same sparse engine"
                                    % (args.cross_layers, args.hidden)}
                   if dcn_res is not None else {}),
                "native_build": _build_summary(),
                "unique_keys_per_batch": round(sum(u_per_batch) / len(u_per_batch), 1),
                "keys_per_batch": l_per_batch,
                "u_over_l": round(u_over_l, 4),
                "table_hit_rate": 1.0 if not args.no_prefill else None,
            },
        }
        print(json.dumps(out), flush=True)
    if multi:
        dist.barrier()
        torch.cuda.synchronize()
        sys.stdout.flush()
        sys.stderr.flush()
        if ipc is None or engine.exchange_mode != "ipc":
            # the captured graphs hold RCCL work: tearing the communicator
            # down under them can block, so leave the process without it once
            # every rank is done (output is flushed above)
            os._exit(0)
        # no RCCL in the step (IPC meshes): a normal exit, so profilers flush
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
