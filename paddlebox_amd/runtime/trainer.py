"""BoxPS trainer / device worker (dataset-driven training loop).

Reference: ``BoxPSTrainer`` (``fw/boxps_trainer.cc:27-320``) and
``BoxPSWorker`` (``fw/boxps_worker.cc:373-1482``, hot loop ``TrainFiles``
:1278-1357), configured by ``trainer_desc.proto:121-129`` / the Python
``BoxPSWorker._gen_worker_desc`` (``py/fluid/device_worker.py:623-652``).

MI355X design: one process per GPU, so the trainer owns exactly one worker
(the reference's worker-thread-per-GPU becomes a rank; ``thread`` is
accepted and ignored).  Per batch the worker
  1. binds the device batch (prefetched + H2D-copied on a side stream by the
     dataset) to the program's data variables,
  2. runs the lowered program (fused pull/seqpool/CVM, fused MLP, ...),
  3. backward (sparse push + data_norm summaries happen inside it),
  4. dense sync per ``sync_dense_mode`` and the fused optimizer step --
     or, in async mode, pushes the flat gradient to the host
     :class:`AsyncDenseTable` and pulls fresh parameters,
  5. accumulates the registered metrics on the device, dumps fields,
     checks NaN/Inf, and prints ``fetch_info`` every ``print_period``.
"""
from __future__ import annotations

import collections
import os
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch

from ..parallel.dense import join_grad_producers
import torch.distributed as dist

from .. import _native
from ..fluid.executor import ExecContext, Session
from ..fluid.kernels import Ragged
from ..utils import flags as _flags
from ..utils.log import logger

log = logger()

# lowered ops whose kernels are shape-static and free of host syncs: a step made
# only of these can be captured into a HIP graph (the sparse data vars reach
# the engine only through the fused pull, which reads the padded key buffer)
GRAPH_SAFE_OPS = {
    "__pull_seqpool_cvm", "__fused_mlp", "__ctr_tower", "__cvm_show_click", "data_norm", "concat", "cast", "fill_constant_batch_size_like",
    "sigmoid", "sigmoid_cross_entropy_with_logits", "reduce_mean", "relu", "fc", "elementwise_add",
    "elementwise_mul", "elementwise_sub", "scale", "log_loss", "mean", "reduce_sum", "tanh", "softmax",
}

# transpiler-inserted dense-sync ops (run after backward / after the update):
# all device work on the session's communicator, capturable
GRAPH_SAFE_SYNC_OPS = {"coalesce_tensor", "c_allreduce_sum", "scale", "elementwise_sub", "assign", "c_allgather"}


@dataclass
class _GraphBatch:
    """Fixed-shape device batch of the captured step: keys padded with -1 to
    the pass's largest batch, lod, dense slots."""

    keys: torch.Tensor
    lod: torch.Tensor
    dense: torch.Tensor


R_HOST = 4  # pinned host batches per size in flight (host-assembly path)

# sync_dense_mode (boxps_worker.cc:393-395,1191-1258)
SYNC_NONE = 0
SYNC_KSTEP_NODE = 1
SYNC_KSTEP_ALL = 2
SYNC_DATA_NORM = 3


@dataclass
class TrainerDesc:
    async_mode: bool = False
    sync_dense_mode: int = 0
    sync_weight_step: int = 1
    sync_one_ring: bool = False
    param_need_sync: List[str] = field(default_factory=list)
    dump_fields: List[str] = field(default_factory=list)
    dump_fields_path: str = ""
    dump_param: List[str] = field(default_factory=list)
    dump_thread_num: int = 1
    dump_mode: int = 0
    dump_interval: int = 1
    check_nan_var_names: List[str] = field(default_factory=list)
    profile: bool = False

    @staticmethod
    def from_program(program) -> "TrainerDesc":
        d = TrainerDesc()
        po = program._pipeline_opt or {}
        fo = program._fleet_opt or {}
        d.async_mode = bool(po.get("async_mode", False))
        d.sync_dense_mode = int(po.get("sync_dense_mode", 0))
        d.sync_weight_step = max(1, int(po.get("sync_weight_step", 1) or 1))
        d.sync_one_ring = bool(po.get("sync_one_ring", False))
        d.param_need_sync = list(po.get("param_need_sync", []))
        d.dump_thread_num = int(po.get("dump_thread_num", fo.get("dump_thread_num", 1)))
        d.dump_fields = list(fo.get("dump_fields", []))
        d.dump_fields_path = fo.get("dump_fields_path", "")
        d.dump_param = list(fo.get("dump_param", []))
        d.dump_mode = int(fo.get("dump_fields_mode", 1 if fo.get("dump_interval", 1) > 1 else 0))
        d.dump_interval = int(fo.get("dump_interval", 1))
        d.check_nan_var_names = list(fo.get("check_nan_var_names", []))
        return d


class _FetchView(dict):
    """name -> tensor view of an ExecContext env for the metric registry."""

    def __init__(self, ctx: ExecContext, batch):
        super().__init__()
        self.ctx, self.batch = ctx, batch
        self.fused_metrics = ctx.fused_metrics

    def __missing__(self, name):
        if name == "__cmatch_rank__" and self.batch is not None and "cmatch_rank" in self.batch.extra:
            return self.batch.extra["cmatch_rank"]
        v = self.ctx.get(name)
        return v.values if isinstance(v, Ragged) else v

    def __contains__(self, name):
        try:
            self[name]
            return True
        except KeyError:
            return False


class AsyncDense:
    """Async dense mode: params + Adam moments live in the native host table
    (``csrc/host/async_dense.cc``); the GPU keeps a working copy that is
    refreshed from the table before each batch."""

    def __init__(self, session: Session, lr: float, device_num: int = 1, threads: int = 8):
        self.s = session
        self.arenas = session.arenas
        flat = torch.cat([a.flat.detach().cpu() for a in self.arenas]) if self.arenas else torch.zeros(0)
        self.adam_len = flat.numel()
        summ = [t for n, t in session.storage.items() if not isinstance(t, torch.nn.Parameter)
                and n.endswith(("batch_size", "batch_sum", "batch_square_sum"))]
        self.summ = summ
        init = torch.cat([flat] + [t.detach().float().cpu().reshape(-1) for t in summ]) if summ else flat
        lrs = torch.full((self.adam_len,), float(lr))
        self.table = _native.host().AsyncDenseTable(init.contiguous(), self.adam_len, lrs, device_num, threads)
        self.host = torch.empty(init.numel(), dtype=torch.float32).pin_memory() if torch.cuda.is_available() \
            else torch.empty(init.numel(), dtype=torch.float32)
        self.summary_grads: Dict[int, torch.Tensor] = {}

    def pull(self):
        self.table.pull(self.host)
        off = 0
        for a in self.arenas:
            n = a.flat.numel()
            a.flat.data.copy_(self.host[off:off + n], non_blocking=True)
            off += n
        for t in self.summ:
            n = t.numel()
            t.copy_(self.host[off:off + n].view_as(t), non_blocking=True)
            off += n

    def push(self, summary_stats: Optional[List[torch.Tensor]] = None):
        from ..parallel.dense import join_grad_producers

        join_grad_producers()  # .cpu() syncs the compute stream only, not the dW side stream
        parts = [a.grad.detach().float().cpu() for a in self.arenas]
        for i, t in enumerate(self.summ):
            st = summary_stats[i] if summary_stats and i < len(summary_stats) else torch.zeros(t.numel())
            parts.append(st.detach().float().cpu().reshape(-1))
        self.table.push(torch.cat(parts) if parts else torch.zeros(0))

    def finalize(self):
        self.table.finalize()
        self.pull()


class BoxPSWorker:
    def __init__(self, trainer: "BoxPSTrainer"):
        self.t = trainer
        self.s: Session = trainer.session
        self.batches = 0
        self.timers = {"read": 0.0, "step": 0.0, "metric": 0.0, "dump": 0.0}

    def train_files(self) -> Dict[str, float]:
        why = self._graph_blocker()
        if why is None:
            return self._train_files_graphed()
        if self.t.use_graph:
            log.info("train_from_dataset: running eagerly (%s)", why)
        return self._train_files_eager()

    def _graph_blocker(self) -> Optional[str]:
        """None when the step can be captured, else the reason it cannot."""
        t, s = self.t, self.s
        if not t.use_graph:
            return "graph capture disabled"
        if t.profile:
            return "profile mode times every op"
        if s.device.type != "cuda":
            return "not a GPU session"
        if t.infer or t.async_dense is not None:
            return "infer / async dense mode"
        if t.dumper is not None or _flags.get_bool("check_nan_inf"):
            return "dump / nan-inf check need per-step host work"
        ds = t.dataset
        if ds is None or not hasattr(ds, "_native"):
            return "no in-memory slot dataset"
        if ds.rank_offset or ds.parse_ins_id or ds.parse_logkey:
            return "per-batch host extras (rank_offset / ins_id / logkey)"
        if any(sy.mode not in ("none", "grad_allreduce") for sy in s.syncs):
            return "k-step / allgather dense sync keeps host counters"
        eng = t.box.engine if t.box is not None else None
        if eng is None or eng.auto_insert:
            return "engine auto-insert syncs the host"
        role_ops = {op.type for op in s.lowered.backward_ops + s.lowered.optimize_ops}
        bad = sorted(({op.type for op in s.lowered.steps} - GRAPH_SAFE_OPS) | (role_ops - GRAPH_SAFE_SYNC_OPS))
        if bad:
            return f"ops not graph-safe: {bad}"
        return None

    def _train_files_graphed(self) -> Dict[str, float]:
        """TrainFiles with the whole step (forward, backward, sparse push,
        dense sync, optimizer) replayed from a HIP graph per batch size.
        The first two batches of each size run eagerly through the capture
        buffers (real training steps that also warm the lazy state), then the
        step is captured and every further batch is one H2D + one replay
        (reference per-batch op loop: boxps_worker.cc:1278-1357)."""
        from collections import Counter

        from ..data.dataset import SlotBatch
        from .graph_step import GraphedTrainStep, pack_batch

        t, s, ds, box = self.t, self.s, self.t.dataset, self.t.box
        dev = s.device
        nat = ds._native
        plan = ds.prepare_train()
        S = int(nat.num_sparse_slots())
        names, dnames, ddims = nat.sparse_slot_names(), nat.dense_slot_names(), nat.dense_slot_dims()
        Dw = int(nat.dense_width())
        lens = [int(nat.batch_len(b0, c)) for b0, c in plan]
        Lcap = (max(lens + [1]) + 16383) // 16384 * 16384
        # captured steps persist across passes (per session and batch size)
        # while their key buffer covers the pass's largest batch
        cache = s.cache.setdefault("graphs", {})
        if Lcap > box.engine.max_keys:
            log.info("train_from_dataset: batch keys %d exceed engine max_keys; running eagerly", Lcap)
            return self._train_files_eager()
        sizes = Counter(c for _, c in plan)
        graph_B = {B for B, n in sizes.items() if n >= 3}
        label = ds.label_name if ds.label_name in dnames else None
        # the label / cvm extras only feed data variables of those names that
        # are not dense slots (the canonical program builds its cvm from the
        # label with its own ops): otherwise not built, two launches a step less
        if label is not None and not any(v.name in ("label", "cvm") and v.name not in dnames for v in s.data_vars):
            label = None

        def host_buf(B):
            return pack_batch(_GraphBatch(torch.empty(Lcap, dtype=torch.int64),
                                          torch.empty(S * (B + 1), dtype=torch.int64),
                                          torch.empty(B, Dw, dtype=torch.float32)), pin=True)

        def slot_batch(keys, lod, dense, B, lod_host):
            b = SlotBatch(keys, lod, dense, B, S, names, dnames, ddims, lod_host=lod_host)
            if label is not None:
                lab = b.dense_var(label)[:, 0].contiguous()
                b.extra["label"] = lab
                b.extra["cvm"] = torch.stack([torch.ones_like(lab), lab], 1)
            return b

        def step_fn_for(B, lod_host):
            def fn(gb):
                batch = slot_batch(gb.keys, gb.lod, gb.dense, B, lod_host)
                ctx = ExecContext(s, batch, training=True)
                s.feed_batch(ctx, batch)
                s.step(ctx)
                return ctx, batch
            return fn

        def metrics(out):
            if box is not None and box.metrics.metrics:
                box.metrics.add_batch(_FetchView(*out))

        from ..data.device_pass import device_pass_for

        dp = device_pass_for(ds, dev)
        if dp is not None:
            return self._train_device_pass(dp, plan, Lcap, cache, graph_B, S, Dw, slot_batch, step_fn_for, metrics)
        graphs, warm, rings, nused = {}, {}, {}, {}
        for B, (cL, g, rg) in cache.items():
            # the host-assembly loop replays single-step, non-pipelined graphs
            if B in graph_B and cL >= Lcap and g.K == 1 and g.pipeline is None:
                graphs[B], rings[B], nused[B] = g, rg, 0
                if rg is None:  # captured by the device-pass path: no host ring yet
                    rings[B] = [host_buf(B) for _ in range(R_HOST)]
        Lcap = max([Lcap] + [cache[B][0] for B in graphs])
        R = R_HOST  # pinned host batches per size in flight
        # the pass's batch assembly runs on a native thread (csrc/host/
        # batch_assembler.cc) into pinned buffers; ring slots are handed back
        # once their H2D has completed
        cached = set(graphs)
        jobs, meta, slot_ids = [], [], {}
        used = Counter()
        for (b0, c) in plan:
            sid = -1
            if c in graph_B:
                k = used[c]
                used[c] += 1
                if c not in cached and k < 2:
                    hb, tag = host_buf(c), "warm"
                else:
                    r = (k - (0 if c in cached else 2)) % R
                    ring = rings.setdefault(c, [host_buf(c) for _ in range(R)])
                    sid = slot_ids.setdefault((c, r), len(slot_ids))
                    hb, tag = ring[r], "ring"
            else:
                hb, tag = host_buf(c), "eager"
            jobs.append((b0, c, hb.keys, hb.lod, hb.dense, sid))
            meta.append((c, hb, tag, sid))
        asm = _native.host().BatchAssembler(nat, jobs, len(slot_ids))
        pending: "collections.deque" = collections.deque()
        t0 = time.time()
        n_ins = 0
        replays = 0
        asm.start()
        while True:
            i = asm.next()
            if i < 0:
                break
            c, hb, tag, sid = meta[i]
            t_s = time.time()
            if tag == "warm":
                warm.setdefault(c, []).append(hb)
                if len(warm[c]) == 2:
                    g = GraphedTrainStep(step_fn_for(c, warm[c][1].lod.clone()), warm[c][0], dev, warmup=0,
                                         warm_batches=warm[c], on_warm=metrics)
                    graphs[c] = g
                    nused[c] = 0
                    cache[c] = (Lcap, g, rings.setdefault(c, [host_buf(c) for _ in range(R)]))
            elif tag == "ring":
                g = graphs[c]
                j = nused[c] % g.n
                nused[c] += 1
                g.load(j, hb)
                ev = torch.cuda.Event()
                ev.record(g.copy_stream)
                pending.append((sid, ev))
                out = g.run(j)
                replays += 1
                metrics(out)
            else:  # odd-sized batch: eager
                bt = slot_batch(hb.keys.to(dev, non_blocking=True), hb.lod.to(dev, non_blocking=True),
                                hb.dense.to(dev, non_blocking=True), c, hb.lod)
                ctx = ExecContext(s, bt, training=True)
                s.feed_batch(ctx, bt)
                s.step(ctx)
                metrics((ctx, bt))
            while pending and (len(pending) > R - 2 or pending[0][1].query()):
                sid0, ev0 = pending.popleft()
                ev0.synchronize()
                asm.release(sid0)
            self.timers["step"] += time.time() - t_s
            self.batches += 1
            n_ins += c
        self.timers["read"] = asm.build_seconds()
        self.timers["read_wait"] = asm.wait_seconds()
        # a size seen fewer than 3 times (or its warm batches) never captured
        for c, hbs in warm.items():
            if c in graphs:
                continue
            for hb in hbs:
                bt = slot_batch(hb.keys.to(dev), hb.lod.to(dev), hb.dense.to(dev), c, hb.lod)
                ctx = ExecContext(s, bt, training=True)
                s.feed_batch(ctx, bt)
                s.step(ctx)
                metrics((ctx, bt))
        join_grad_producers()
        torch.cuda.synchronize(dev)
        el = time.time() - t0
        return {"batches": self.batches, "instances": n_ins, "seconds": el,
                "ins_per_sec": n_ins / el if el > 0 else 0.0, "graph_replays": replays,
                "graph_sizes": sorted(graphs), **self.timers}

    # metric kinds accumulated by device kernels only (capturable inside a
    # multi-step graph); the others pull predictions to the host per batch
    DEVICE_METRICS = {"AucCalculator", "MaskAucCalculator", "MultiMaskAucCalculator"}

    def _metrics_in_graph(self) -> bool:
        box = self.t.box
        ms = list(box.metrics.metrics.values()) if box is not None else []
        return all(m.method in self.DEVICE_METRICS and not m.sample_scale_var and m.phase == -1 for m in ms)

    def _steps_per_graph(self, metrics_in_graph: bool) -> int:
        """FLAGS_padbox_train_steps_per_graph (0 = auto: 4 on one rank, 2 on
        several -- bench.py's measured choice -- when every metric can be
        accumulated inside the graph, else 1)."""
        k = _flags.get_int("padbox_train_steps_per_graph")
        if k <= 0:
            k = (4 if self.t.world == 1 else 2) if metrics_in_graph else 1
        return k if metrics_in_graph else 1

    def _train_device_pass(self, dp, plan, Lcap, cache, graph_B, S, Dw, slot_batch, step_fn_for, metrics):
        """The graphed TrainFiles over a device-resident pass
        (data/device_pass.py): every batch is assembled by the batch kernels
        on the pass stream straight into the replay's input buffers, so the
        host loop per batch is a few launches + one graph replay.

        The step is the one bench.py times (runtime/graph_step.py):
        * K training steps per captured graph (FLAGS_padbox_train_steps_per_graph,
          metrics accumulated inside the graph);
        * the pipelined front (FLAGS_padbox_pipelined_front): each step pools
          the next batch right after its sparse push, beside the tower's dW
          GEMM, so the next step starts at the dense head.  Buffer sets are
          filled two graphs ahead of their replay (graph j pools set j+1).
        Reference hot loop: boxps_worker.cc:1278-1357."""
        from .graph_step import GraphedTrainStep, pack_batch

        s, dev, box = self.s, self.s.device, self.t.box
        eng = box.engine
        # the fused towers' side work rides in launches the step has anyway
        # (weight re-pack + data_norm update in Adam, AUC in the loss tail);
        # the optimizer is this loop's only weight writer, so one eager
        # re-pack at the pass start covers checkpoint loads between passes
        s.fuse_towers(box.metrics)
        s.repack_towers()
        in_graph = self._metrics_in_graph()
        K = self._steps_per_graph(in_graph)
        pipe_on = _flags.get_bool("padbox_pipelined_front") and s.pipeline_pull_op() is not None
        n_buf = 3 if pipe_on else 2

        def dev_buf(B):
            return pack_batch(_GraphBatch(torch.empty(Lcap, dtype=torch.int64), torch.empty(S * (B + 1), dtype=torch.int64),
                                          torch.empty(B, Dw, dtype=torch.float32)), device=dev)

        def step_for(c, lod_host):
            fn0 = step_fn_for(c, lod_host)

            def fn(gb):
                out = fn0(gb)
                s.fuse_towers(box.metrics)  # host-only: a tower first built by this step (before the capture)
                return out
            if not in_graph:
                return fn

            def fn_m(gb):
                out = fn(gb)
                metrics(out)  # device histogram kernels, captured with the step
                return out
            return fn_m

        def pipe_for(c, lod_host):
            if not pipe_on:
                return None

            def as_batch(buf):
                return slot_batch(buf.keys, buf.lod, buf.dense, c, lod_host)

            return (lambda buf, j: s.prefetch(as_batch(buf), j),
                    lambda buf, j: s.set_next(None if buf is None else as_batch(buf), j),
                    eng.clear_prefetch)

        graphs, warm, state, queue = {}, {}, {}, {}
        for B, (cL, g, _rg) in cache.items():
            if (B in graph_B and cL >= Lcap and g.K == K and (g.pipeline is not None) == pipe_on
                    and getattr(g, "metrics_in_graph", False) == in_graph):
                graphs[B] = g
        Lcap = max([Lcap] + [cache[B][0] for B in graphs])
        t0 = time.time()
        n_ins = replays = 0

        def invalidate_others(c):
            # a step of another size (or an eager one, c = None) changed the
            # table after a graph pooled its next buffer set: that set is
            # pooled again before its replay
            for c2, g2 in graphs.items():
                if c2 != c:
                    g2.invalidate_prefetch()

        def run_one(c):
            nonlocal replays
            g, st = graphs[c], state[c]
            out = g.run(st[1] % g.n)
            st[1] += 1
            replays += g.K
            if not in_graph:
                metrics(out)
            invalidate_others(c)

        def fill_group(c, grp):
            g, st = graphs[c], state.setdefault(c, [0, 0])
            fns = [lambda buf, b0=b0, c=c: dp.assemble(b0, c, buf.keys, buf.lod, buf.dense) for b0 in grp]
            g.fill(st[0] % g.n, fns if g.K > 1 else fns[0], dp.stream)
            st[0] += 1
            lag = 2 if g.pipeline is not None else 1  # graph j pools set j+1: fill it first
            while st[0] - st[1] >= lag:
                run_one(c)

        def eager(db, c):
            bt = slot_batch(db.keys, db.lod, db.dense, c, db.lod.cpu())
            ctx = ExecContext(s, bt, training=True)
            s.feed_batch(ctx, bt)
            s.step(ctx)
            metrics((ctx, bt))
            invalidate_others(None)

        def drain(c):
            # everything of size c still pending, in plan order: its filled
            # buffer sets, then the batches short of a whole graph and the
            # warm-up batches (eagerly) -- before a batch of another size runs,
            # so the pass trains in the plan's order (sparse and Adam updates
            # are order-dependent)
            st = state.get(c)
            if c in graphs and st is not None:
                while st[1] < st[0]:
                    run_one(c)
            for b0 in queue.pop(c, []):
                db = dev_buf(c)
                dp.assemble_sync(b0, c, db.keys, db.lod, db.dense)
                eager(db, c)
            for db in warm.pop(c, []):
                eager(db, c)

        last_c = None
        for (b0, c) in plan:
            t_s = time.time()
            if last_c is not None and c != last_c:
                drain(last_c)
            last_c = c
            if c in graphs:
                q = queue.setdefault(c, [])
                q.append(b0)
                if len(q) == graphs[c].K:
                    fill_group(c, list(q))
                    q.clear()
            else:
                db = dev_buf(c)
                dp.assemble_sync(b0, c, db.keys, db.lod, db.dense)
                if c in graph_B:
                    warm.setdefault(c, []).append(db)
                    if len(warm[c]) == 2:
                        lh = db.lod.cpu()
                        if pipe_on:
                            eng.ensure_pull_ring(n_buf * K)
                        # the overlapped Adam of a step may run on under the next
                        # step of the same graph (that step's forward joins it)
                        g = GraphedTrainStep(step_for(c, lh), warm[c][0], dev, warmup=0, warm_batches=warm[c],
                                             on_warm=None if in_graph else metrics, n_buffers=n_buf,
                                             pipeline=pipe_for(c, lh), steps_per_graph=K,
                                             join_each_step=not s.side_adam)
                        g.metrics_in_graph = in_graph
                        invalidate_others(c)
                        graphs[c] = g
                        cache[c] = (Lcap, g, None)
                        del warm[c]
                else:
                    eager(db, c)
            self.timers["step"] += time.time() - t_s
            self.batches += 1
            n_ins += c
        # the graphs' filled sets not yet replayed, then the batches short of a
        # whole graph and the sizes seen once (never captured) run eagerly
        for c, g in graphs.items():
            st = state.get(c, [0, 0])
            while st[1] < st[0]:
                run_one(c)
        for c, q in queue.items():
            for b0 in q:
                db = dev_buf(c)
                dp.assemble_sync(b0, c, db.keys, db.lod, db.dense)
                eager(db, c)
        for c, dbs in warm.items():
            for db in dbs:
                eager(db, c)
        join_grad_producers()  # the last step's side-stream update (overlapped Adam) and its pre-head event
        torch.cuda.synchronize(dev)
        if dp.overflowed():
            raise RuntimeError("device batch assembly: a batch had more keys than the captured key buffer")
        eng.check_guards()
        el = time.time() - t0
        return {"batches": self.batches, "instances": n_ins, "seconds": el,
                "ins_per_sec": n_ins / el if el > 0 else 0.0, "graph_replays": replays,
                "graph_sizes": sorted(graphs), "device_pass": True, "steps_per_graph": K,
                "pipelined_front": pipe_on, **self.timers}

    def _train_files_eager(self) -> Dict[str, float]:
        t = self.t
        s = self.s
        if t.profile and s.op_profiler is None:
            from .op_profiler import OpProfiler

            s.op_profiler = OpProfiler(s.device)
        try:
            stats = self._train_files_eager_loop()
        finally:
            prof, s.op_profiler = s.op_profiler, None
        if prof is not None:
            stats["op_profile"] = prof.report()
            log.info("per-op profile (%d batches):\n%s", self.batches, prof.format())
        return stats

    def _train_files_eager_loop(self) -> Dict[str, float]:
        t = self.t
        s = self.s
        box = t.box
        if box is not None:
            s.fuse_towers(box.metrics, optimizer=False)  # keep a fused-tower AUC bound to the current metric
        ds = t.dataset
        dev = s.device
        desc = t.desc
        plan_batches = ds.batches(dev) if ds is not None else iter(())
        t0 = time.time()
        last = time.time()
        n_ins = 0
        for batch in plan_batches:
            t_read = time.time()
            self.timers["read"] += t_read - last
            ctx = ExecContext(s, batch, training=not t.infer)
            s.feed_batch(ctx, batch)
            if t.async_dense is not None:
                t.async_dense.pull()
            if t.infer:
                with torch.no_grad():
                    s.forward(ctx)
            elif t.async_dense is not None:
                s.forward(ctx)
                loss = ctx.get(s.program._optimize["loss"])
                for a in s.arenas:
                    a.zero_grad()
                (loss.values if isinstance(loss, Ragged) else loss).float().sum().backward()
                t.async_dense.push()
            else:
                s.step(ctx)
                self._dense_sync_extra()
            t_step = time.time()
            self.timers["step"] += t_step - t_read
            if box is not None and box.metrics.metrics:
                box.metrics.add_batch(_FetchView(ctx, batch))
            t_met = time.time()
            self.timers["metric"] += t_met - t_step
            if t.dumper is not None and desc.dump_fields:
                self._dump(ctx, batch)
            self.timers["dump"] += time.time() - t_met
            if _flags.get_bool("check_nan_inf"):
                self._check_nan_inf(ctx)
            self.batches += 1
            n_ins += batch.B
            if t.fetch_list and t.print_period > 0 and self.batches % t.print_period == 0:
                self._print_fetch(ctx)
            last = time.time()
        if dev.type == "cuda":
            join_grad_producers()
            torch.cuda.synchronize(dev)
        el = time.time() - t0
        return {"batches": self.batches, "instances": n_ins, "seconds": el,
                "ins_per_sec": n_ins / el if el > 0 else 0.0, **self.timers}

    def _dense_sync_extra(self):
        """sync_dense_mode 3: average only the data_norm summaries every k steps."""
        t = self.t
        if t.desc.sync_dense_mode != SYNC_DATA_NORM or t.world <= 1:
            return
        if self.batches % t.desc.sync_weight_step != 0:
            return
        summ = [v for n, v in self.s.storage.items() if not isinstance(v, torch.nn.Parameter)
                and n.endswith(("batch_size", "batch_sum", "batch_square_sum"))]
        if summ:
            flat = torch.cat([v.reshape(-1) for v in summ])
            dist.all_reduce(flat, group=t.group)
            flat.mul_(1.0 / t.world)
            off = 0
            for v in summ:
                v.copy_(flat[off:off + v.numel()].view_as(v))
                off += v.numel()

    def _dump(self, ctx, batch):
        t = self.t
        names, mats = [], []
        for f in t.desc.dump_fields:
            try:
                v = ctx.get(f)
            except KeyError:
                continue
            v = v.values if isinstance(v, Ragged) else v
            if v.dim() == 0 or v.shape[0] != batch.B:
                continue
            names.append(f)
            mats.append(v.detach().float().reshape(batch.B, -1))
        if not names:
            return
        lineids = batch.extra.get("ins_ids") if isinstance(batch.extra.get("ins_ids"), list) else None
        if lineids is None:
            lineids = [str(self.batches * batch.B + i) for i in range(batch.B)]
        t.dumper.dump_fields(lineids, names, mats, t.desc.dump_mode, t.desc.dump_interval,
                             _flags.get_bool("lineid_have_extend_info"))

    def _check_nan_inf(self, ctx):
        for name, v in ctx.env.items():
            v = v.values if isinstance(v, Ragged) else v
            if isinstance(v, torch.Tensor) and v.is_floating_point():
                if not bool(torch.isfinite(v).all()):
                    raise FloatingPointError(f"NaN/Inf detected in variable '{name}' at batch {self.batches}")

    def _print_fetch(self, ctx):
        t = self.t
        parts = []
        for i, f in enumerate(t.fetch_list):
            name = f if isinstance(f, str) else f.name
            info = t.fetch_info[i] if t.fetch_info and i < len(t.fetch_info) else name
            v = ctx.get(name)
            v = v.values if isinstance(v, Ragged) else v
            parts.append(f"{info}: {v.detach().float().mean().item():.6f}")
        log.info("batch %d  %s", self.batches, "  ".join(parts))


class BoxPSTrainer:
    def __init__(self, executor, program, scope, dataset, infer=False, debug=False, fetch_list=None,
                 fetch_info=None, print_period=100, fetch_handler=None):
        from ..ps.box_wrapper import BoxWrapper

        self.exe = executor
        self.program = program
        self.scope = scope
        self.dataset = dataset
        self.infer = infer
        self.debug = debug
        self.fetch_list = list(fetch_list or [])
        self.fetch_info = list(fetch_info or [])
        self.print_period = print_period
        self.fetch_handler = fetch_handler
        self.desc = TrainerDesc.from_program(program)
        # HIP-graph capture of the step (default on GPU; _pipeline_opt
        # {"use_graph": False} or FLAGS_padbox_use_graph=0 turn it off)
        po = program._pipeline_opt or {}
        try:
            flag = _flags.get("padbox_use_graph")
        except Exception:
            flag = None
        self.use_graph = bool(po.get("use_graph", True)) and str(flag).lower() not in ("0", "false")
        self.box = BoxWrapper._instance
        self.group = getattr(dataset, "group", None)
        ready = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(self.group) if ready else 1
        self.rank = dist.get_rank(self.group) if ready else 0
        sync_mode, k = self._sync_policy()
        names = [f if isinstance(f, str) else f.name for f in self.fetch_list]
        names += [f for f in self.desc.dump_fields]
        if self.box is not None:
            for m in self.box.metrics.metrics.values():
                names += [m.label_var, m.pred_var] + [x for x in (m.mask_var, m.cmatch_rank_var, m.uid_var) if x]
                names += m.pred_list + m.mask_list
        self.session = executor._session(program, scope, names, sync_mode=sync_mode, sync_k=k,
                                          group=self.group)
        self.async_dense = None
        if self.desc.async_mode and not infer and program._optimize is not None:
            spec = program._optimize["optimizer"].spec()
            self.async_dense = AsyncDense(self.session, spec["lr"], device_num=1,
                                          threads=int(os.environ.get("PBX_ASYNC_DENSE_THREADS", "8")))
        self.dumper = None
        if self.desc.dump_fields and self.desc.dump_fields_path:
            dev_id = self.session.device.index or 0
            ddir = os.path.join(self.desc.dump_fields_path, f"rank{self.rank:03d}")
            os.makedirs(ddir, exist_ok=True)
            self.dumper = _native.host().DumpWriter(ddir, dev_id, max(1, self.desc.dump_thread_num))
        # profile mode (reference TrainFilesWithProfiler, entered with
        # train_from_dataset(debug=True) or TrainerDesc.profile): per-op times
        self.profile = bool(debug or self.desc.profile)
        if self.session.device.type == "cuda" and _flags.get_bool("enable_binding_train_cpu"):
            from .affinity import bind_worker

            lr = int(os.environ.get("LOCAL_RANK", "0"))
            lw = int(os.environ.get("LOCAL_WORLD_SIZE", "1"))
            bind_worker(self.session.device, lr, lw)
        self.worker = BoxPSWorker(self)

    def _sync_policy(self):
        d = self.desc
        if self.world <= 1:
            return "none", 1
        if getattr(self.program, "_collective", None):
            return None, 1  # the transpiler / fleet strategy decides (Session._build_optimizer)
        if d.sync_dense_mode in (SYNC_KSTEP_ALL,):
            return "kstep", d.sync_weight_step
        if d.sync_dense_mode == SYNC_KSTEP_NODE:
            # reference SyncParam returns early on one node; across nodes the
            # k-step parameter average is hierarchical (node reduce-scatter,
            # cross-node shard all-reduce, node all-gather)
            local = int(os.environ.get("LOCAL_WORLD_SIZE", self.world))
            if local <= 0 or self.world <= local:
                return "none", 1
            return "kstep_node", d.sync_weight_step
        if d.sync_dense_mode == SYNC_DATA_NORM:
            return "none", 1
        return "grad_allreduce", 1

    def run(self):
        stats = self.worker.train_files()
        if self.async_dense is not None:
            self.async_dense.finalize()
        if self.dumper is not None:
            if self.desc.dump_param:
                ts = [self.session.logical[n] for n in self.desc.dump_param if n in self.session.logical]
                self.dumper.dump_params(self.worker.batches, [n for n in self.desc.dump_param
                                                              if n in self.session.logical], ts)
            self.dumper.flush()
        if self.debug:
            log.info("trainer stats: %s", stats)
        return stats


def create_trainer(executor, program, scope, dataset, **kw) -> BoxPSTrainer:
    """TrainerFactory: every program runs on the BoxPS trainer (the reference
    picks it from ``program._pipeline_opt['trainer']``)."""
    return BoxPSTrainer(executor, program, scope, dataset, **kw)
