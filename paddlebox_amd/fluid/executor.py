"""Executor: runs fluid programs on one MI355X (one process per GPU).

``Executor.run`` executes a program on a feed dict; ``train_from_dataset`` /
``infer_from_dataset`` hand the program to the BoxPS trainer
(``paddlebox_amd/runtime/trainer.py``), mirroring
``py/fluid/executor.py:1787-1936`` -> ``core.Executor.run_from_dataset`` ->
``BoxPSTrainer``/``BoxPSWorker`` (``fw/boxps_trainer.cc``, ``fw/boxps_worker.cc``).

A :class:`Session` is the per-(program, scope) compiled state: the lowered
step list, the dense parameter arena + fused optimizer, and the dense sync
policy.  It is created lazily and cached on the executor.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Sequence

import os
import warnings

import numpy as np
import torch
import torch.distributed as dist

from ..utils.log import logger
from ..parallel.dense import join_grad_producers, DenseArena, DenseSync, FlatAdagrad, FlatAdam, FlatMomentum, FlatSGD
from .framework import (LoDTensor, Parameter, Program, Scope, Variable, default_main_program,
                        default_startup_program, global_scope, to_device, torch_dtype)
from .kernels import KERNELS, LazyRagged, Ragged
from .lowering import Lowered, lower


def _box():
    from ..ps.box_wrapper import BoxWrapper

    return BoxWrapper._instance


log = logger()


class ExecContext:
    """Per-run variable environment handed to the kernels."""

    def __init__(self, session: "Session", batch=None, training: bool = True, B: int = 0):
        self.s = session
        self.env: Dict[str, Any] = {}
        self.batch = batch
        self.training = training
        self.B = B
        # metrics a kernel already accumulated for this batch (the fused
        # tower's AUC histogram): the registry skips them
        self.fused_metrics = set()

    # session passthroughs
    @property
    def device(self):
        return self.s.device

    @property
    def scope(self) -> Scope:
        return self.s.scope

    @property
    def generator(self):
        return self.s.generator

    @property
    def generator_dev(self):
        return self.s.generator_dev

    @property
    def group(self):
        return self.s.group

    @property
    def box(self):
        b = _box()
        if b is None:
            raise RuntimeError("BoxWrapper is not initialised (fluid.core.BoxWrapper(...) + "
                               "initialize_gpu_and_load_model) but the program uses BoxPS ops")
        return b

    @property
    def engine(self):
        e = self.box.engine
        if e is None:
            raise RuntimeError("BoxWrapper.initialize_gpu_and_load_model() has not been called")
        return e

    @property
    def cache(self) -> dict:
        return self.s.cache

    def get(self, v):
        name = v if isinstance(v, str) else v.name
        if name in self.env:
            return self.env[name]
        if name in self.s.logical:
            return self.s.logical[name]
        if name in self.s.scope:
            return self.s.scope.get(name)
        raise KeyError(f"variable '{name}' has no value (not fed / not computed)")

    def set(self, v, val):
        self.env[v if isinstance(v, str) else v.name] = val

    def param(self, v) -> torch.Tensor:
        return self.get(v)

    def storage(self, v) -> torch.Tensor:
        return self.s.storage[v if isinstance(v, str) else v.name]


def _make_opt(spec: dict, arena: DenseArena, lr_mult: float = 1.0):
    t = spec["type"]
    lr = spec["lr"] * lr_mult
    if t == "adam":
        # the update kernel also zeroes the gradients (no separate fill per step)
        return FlatAdam(arena, lr, spec.get("beta1", 0.9), spec.get("beta2", 0.999), spec.get("epsilon", 1e-8),
                        clear_grad=arena.flat.is_cuda)
    if t == "adamw":
        return FlatAdam(arena, lr, spec.get("beta1", 0.9), spec.get("beta2", 0.999), spec.get("epsilon", 1e-8),
                        spec.get("weight_decay", 0.01))
    if t == "momentum":
        return FlatMomentum(arena, lr, spec.get("momentum", 0.9), spec.get("use_nesterov", False))
    if t == "adagrad":
        return FlatAdagrad(arena, lr, spec.get("epsilon", 1e-6), spec.get("initial_accumulator_value", 0.0))
    return FlatSGD(arena, lr)


def _side_adam_hook(sess, opt, tower):
    """The tower's dense-grads hook for Session._side_adam, holding the
    session and tower weakly (no tower <-> hook reference cycle)."""
    import weakref

    sr, tr = weakref.ref(sess), weakref.ref(tower)

    def hook():
        s, t = sr(), tr()
        if s is not None and t is not None:
            s._side_adam(opt, t)
    return hook


class Session:
    def __init__(self, program: Program, scope: Scope, device: torch.device, fetch_names=(), group=None,
                 sync_mode: Optional[str] = None, sync_k: int = 1, fuse: bool = True):
        self.program = program
        self.scope = scope
        self.device = device
        self.group = group
        self.cache: dict = {}
        self.generator = torch.Generator().manual_seed(program.random_seed or 0)
        self.generator_dev = None
        self.training = program._optimize is not None and not program._is_test
        box = _box()
        cvm_off = 2
        self.lowered: Lowered = lower(program, fetch_names, gpu=device.type == "cuda", engine_cvm_offset=cvm_off,
                                      fuse=fuse)
        self._dump_program(device)
        self.storage: Dict[str, torch.Tensor] = {}
        self.logical: Dict[str, torch.Tensor] = {}
        self._materialize()
        self.arenas: List[DenseArena] = []
        self.opts = []
        self.syncs: List[DenseSync] = []
        if self.training:
            self._build_optimizer(sync_mode, sync_k)
        self.data_vars = [v for v in program.global_block().vars.values() if v.is_data]
        self.box = box
        self._one = None
        self.op_profiler = None  # runtime.op_profiler.OpProfiler in the trainer's profile mode
        # pipelined front (graphed train loop): (batch, pull slot) pooled right
        # after this step's sparse push, so the next step starts at the dense head
        self._next = None
        self._side_stepped = set()  # optimizers the tower hook already stepped this step
        self.side_adam = False  # a tower's update runs on its dW side stream (no join at the step end)

    def close(self):
        """Release the session's IPC mesh (each session's mesh stayed
        registered and mapped forever): unregistered when it is the group's
        current one, then closed.  A mesh shared from another session is left
        to its owner."""
        ipc, self.ipc = getattr(self, "ipc", None), None
        if ipc is None or not getattr(self, "_owns_ipc", False):
            return
        from ..parallel.comm import group_mesh, register_group_mesh

        if group_mesh(self.group) is ipc:
            register_group_mesh(self.group, None)
        for s in self.syncs:
            if getattr(s, "ipc", None) is ipc:
                s.ipc = None
        ipc.close()
        self._owns_ipc = False

    # -------------------------------------------------------------- pipelined front
    def pipeline_pull_op(self):
        """The program's single fused pull op when the pipelined front applies
        (a GPU engine that can prepare pulls, the pull's dense columns are data
        variables of the batch), else None."""
        pulls = [op for op in self.lowered.steps if op.type == "__pull_seqpool_cvm"]
        eng = getattr(self.box, "engine", None) if self.box is not None else None
        if len(pulls) != 1 or eng is None or not eng.can_prefetch_pull() or not self.training:
            return None
        data = {v.name for v in self.data_vars}
        if any(v.name not in data for v in pulls[0].inputs.get("Dense", [])):
            return None
        return pulls[0]

    def fuse_towers(self, metrics=None, optimizer: bool = True):
        """Fold each fused tower's per-step side work into launches the step
        already has (the form bench.py times, runtime/ctr_step.py): the
        tower weight re-pack and the data_norm summary update into the fused
        Adam launch of the arena holding the tower, and an AucCalculator over
        the tower's prediction / label into the tower's loss tail.  For
        loops where the optimizer is the only writer of the weights between
        steps (the graphed train loop re-packs at each pass start)."""
        from ..parallel.dense import FlatAdam

        for key, t in list(self.cache.items()):
            if not (isinstance(key, tuple) and key and key[0] == "tower"):
                continue
            if optimizer and not getattr(t, "_opt_fused", False) and self.training:
                for a, o in zip(self.arenas, self.opts):
                    fs = a.flat.untyped_storage().data_ptr()
                    if isinstance(o, FlatAdam) and all(w.untyped_storage().data_ptr() == fs for w in t.mlp.w):
                        side = self._adam_overlap_ok(a, o, t)
                        # overlapped: the data_norm update stays in the tower's
                        # dense tail, ahead of the side-stream Adam
                        o.fuse(mlps=list(o._fuse_mlps) + [t.mlp],
                               data_norms=list(o._fuse_dns) + ([t.dn] if t.dn is not None and not side else []))
                        if side:
                            if t.dn is not None:
                                t.dn.fused_update = False
                            t.on_dense_grads = _side_adam_hook(self, o, t)
                            self.side_adam = True
                        # the packed copy predates the last (unfused) update:
                        # the next forward packs, later updates re-pack
                        t.mlp.invalidate_pack()
                        t._opt_fused = True
                        break
            if metrics is not None and t.auc is not None and (
                    metrics.metrics.get(getattr(t, "auc_metric", None)) is not getattr(t, "auc_metric_obj", None)):
                t.auc = t.auc_metric = t.auc_metric_obj = None  # the metric was re-registered: bind the new one
            if metrics is not None and t.auc is None:
                pred, labels = getattr(t, "io", (None, ()))
                for name, m in metrics.metrics.items():
                    if (m.method == "AucCalculator" and not m.mask_var and m.phase == -1 and not m.sample_scale_var
                            and m.pred_var == pred and m.label_var in labels
                            and getattr(m, "fused_tower", None) is None):
                        tab, st = metrics._dev_tables(m, self.device)
                        t.auc = (tab, st, None)
                        t.auc_metric, t.auc_metric_obj = name, m
                        m.fused_tower = t
                        break

    def _adam_overlap_ok(self, arena, opt, tower) -> bool:
        """The overlapped optimizer of bench.py's step (CtrTrainStep
        adam_overlap, PBX_ADAM_OVERLAP): one rank, a plain (untranspiled)
        program, and an arena holding only this tower's parameters."""
        if os.environ.get("PBX_ADAM_OVERLAP", "1") != "1":
            return False
        if self.group is not None or getattr(self, "async_dense", None) or not (tower.fp32 or tower.x3):
            return False
        lw = self.lowered
        if lw.backward_ops or lw.optimize_ops:
            return False
        tp = {p.data_ptr() for p in tower._params}
        return all(p.data_ptr() in tp for p in arena.params)

    def _side_adam(self, opt, tower):
        """Tower dense-grads hook (on the dW side stream, after the data_norm
        summary update): mark where the next step's head may start, then the
        fused Adam -- the next forward joins it before the tower reads the
        weights (parallel.dense pre-head events)."""
        from ..parallel.dense import set_pre_head_event

        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        set_pre_head_event(tower.uid, ev)
        opt.step(1.0, join=False)
        self._side_stepped.add(id(opt))

    def repack_towers(self):
        """Eager re-pack of every fused tower workspace (start of a graphed
        pass: a checkpoint load or scope write since the last optimizer step
        is not seen by captured steps that rely on the optimizer's re-pack)."""
        for key, t in list(self.cache.items()):
            if isinstance(key, tuple) and key and key[0] == "tower":
                for tw in t.mlp.tower_workspaces():
                    tw.pack([w.detach() for w in t.mlp.w])

    def set_next(self, batch, slot: int = 0):
        """Batch to pool at the end of each step (None: none)."""
        self._next = None if batch is None else (batch, int(slot))

    def prefetch(self, batch, slot: int) -> bool:
        """Pool ``batch`` for its step now, into pull slot ``slot``."""
        from .kernels import prefetch_pull_op

        op = self.pipeline_pull_op()
        if op is None:
            return False
        ctx = ExecContext(self, batch, training=True)
        self.feed_batch(ctx, batch)
        return prefetch_pull_op(ctx, op, slot)

    # -------------------------------------------------------------- params
    def _materialize(self):
        blk = self.program.global_block()
        opt_params = set(self.program._optimize["params"]) if self.program._optimize else set()
        for p in blk.all_parameters():
            if p.name not in self.scope:
                t = torch.empty([max(1, s) for s in p.shape], dtype=torch_dtype(p.dtype))
                p.initializer(t, self.generator)
                self.scope.set(p.name, t.to(self.device))
            cur = self.scope.get(p.name).to(self.device)
            spec = self.lowered.storage.get(p.name)
            trainable = p.name in opt_params and self.training
            if spec is None or spec.kind == "plain":
                st = cur.reshape(spec.shape) if spec is not None else cur
            elif spec.kind == "t_pad":
                st = torch.zeros(spec.shape, dtype=cur.dtype, device=self.device)
                K, N = spec.logical
                st[:N, :K] = cur.reshape(K, N).t()
            else:  # "pad"
                st = torch.zeros(spec.shape, dtype=cur.dtype, device=self.device)
                st[: spec.logical[0]] = cur.reshape(-1)
            if trainable:
                st = torch.nn.Parameter(st.contiguous())
            self.storage[p.name] = st
        self._refresh_logical()

    def _refresh_logical(self):
        for name, st in self.storage.items():
            spec = self.lowered.storage.get(name)
            if spec is None or spec.kind == "plain":
                lg = st.view(spec.logical) if spec is not None else st
            elif spec.kind == "t_pad":
                K, N = spec.logical
                lg = st[:N, :K].t()
            else:
                lg = st[: spec.logical[0]]
            self.logical[name] = lg
            # scope tensors alias the live storage (np.array(scope var) sees training)
            self.scope._tensors[name] = lg

    def _build_optimizer(self, sync_mode, sync_k):
        spec = self.program._optimize["optimizer"].spec()
        blk = self.program.global_block()
        groups: Dict[float, List[torch.nn.Parameter]] = {}
        for name, st in self.storage.items():
            if isinstance(st, torch.nn.Parameter):
                lr = blk.var(name).optimize_attr.get("learning_rate", 1.0) if isinstance(blk.var(name), Parameter) \
                    else 1.0
                box = _box()
                if box is not None and box.lr_map:
                    for pat, v in box.lr_map.items():
                        if pat in name:
                            lr = v / max(spec["lr"], 1e-30)
                groups.setdefault(lr, []).append(st)
        world = dist.get_world_size(self.group) if dist.is_available() and dist.is_initialized() else 1
        coll = getattr(self.program, "_collective", None) or {}
        sharded = coll.get("mode") == "sharding" and spec["type"] in ("adam", "adamw")
        if coll.get("rewritten"):
            sync_mode, sync_k = "none", 1  # the program's own collective ops sync (transpiler rewrite)
        if sync_mode is None and coll:
            # transpiler / fleet choice (py/fluid/transpiler/collective.py modes)
            sync_mode = {"grad_allreduce": "grad_allreduce", "local_sgd": "local_sgd", "allgather": "allgather",
                         "sharding": "none"}.get(coll.get("mode"), "grad_allreduce")
            sync_k = int(coll.get("k", sync_k))
        if sync_mode is None:
            sync_mode = "grad_allreduce" if world > 1 else "none"
        arenas = [(lr_mult, DenseArena(ps, self.device)) for lr_mult, ps in groups.items()]
        # One process per GPU: the dense gradient all-reduce, the transpiled
        # c_allreduce_sum ops and data_norm sync_stats of this session run on a
        # self-tested IPC mesh of the group (one collective kernel, side
        # stream, graph-capturable), RCCL when the mesh is unavailable
        # (PBX_DENSE_IPC=0 forces RCCL).  Collective: every rank builds it.
        self.ipc = None
        self._owns_ipc = False
        if world > 1 and self.device.type == "cuda" and arenas and os.environ.get("PBX_DENSE_IPC", "1") != "0":
            from ..parallel.comm import group_mesh, register_group_mesh
            from ..runtime.ctr_step import make_ipc_mesh

            nbytes = max(max(a.grad.numel() for _, a in arenas) * 4, 1 << 20)
            live = group_mesh(self.group)
            if live is not None and getattr(live, "slot_bytes", 0) >= nbytes and live.device == self.device:
                # another session's mesh of this group serves this one too (the
                # same decision on every rank: sizes come from the program)
                self.ipc = live
            else:
                self.ipc = make_ipc_mesh(nbytes, self.device, group=self.group,
                                         log=lambda m: log.warning("fluid dense sync: %s", m))
                self._owns_ipc = self.ipc is not None
                if self.ipc is not None:
                    # the group's collectives (c_allreduce_sum, data_norm
                    # sync_stats) use the newest mesh; an older, smaller one
                    # stays alive for the session that owns it
                    register_group_mesh(self.group, self.ipc)
        for lr_mult, arena in arenas:
            self.arenas.append(arena)
            if sharded:
                # ZeRO-1: reduce-scatter grads, Adam on this rank's slice, all-gather params
                from ..parallel.sharding import ShardedFlatAdam

                self.opts.append(ShardedFlatAdam(arena, spec["lr"] * lr_mult, spec.get("beta1", 0.9),
                                                 spec.get("beta2", 0.999), spec.get("epsilon", 1e-8),
                                                 spec.get("weight_decay", 0.0), self.group))
                self.syncs.append(DenseSync(arena, "none", 1, self.group))
                continue
            self.opts.append(_make_opt(spec, arena, lr_mult))
            self.syncs.append(DenseSync(arena, sync_mode, sync_k, self.group,
                                        ipc=self.ipc if sync_mode == "grad_allreduce" else None))
        # arena rebinding moved the storage: re-point logical views
        self._refresh_logical()
        self._restore_optimizer_state_from_scope()

    def on_tower_grads(self, tower):
        """The fused tower's dense gradients (and data_norm statistics) are
        final: start the gradient all-reduce of every arena that holds only
        this tower's parameters on its side stream now, so it overlaps the
        head backward and the sparse push (the reference's dense sync hook,
        box_wrapper.h:686-719, boxps_worker.cc:1216-1236); ``before_step``
        joins it.  Arenas with other parameters sync after the backward."""
        own = getattr(self, "_early_sync", None)
        if own is None:
            tp = {p.data_ptr() for p in tower._params}
            own = self._early_sync = [all(p.data_ptr() in tp for p in a.params) for a in self.arenas]
        for s, early in zip(self.syncs, own):
            if early and s.ipc is not None:
                s.launch()

    # -------------------------------------------------------------- feeding
    def feed_batch(self, ctx: ExecContext, batch):
        """Bind a SlotBatch (dataset / synthetic) to the program's data vars."""
        B = batch.B
        ctx.B = B
        S = batch.S
        lod = batch.lod.view(S, B + 1) if S else None
        lh = batch.lod_host if batch.lod_host is not None else batch.lod.cpu()
        lh = lh.view(S, B + 1) if S else None
        sparse_idx = {n: i for i, n in enumerate(batch.sparse_names)}
        for v in self.data_vars:
            if v.name in sparse_idx:
                s = sparse_idx[v.name]
                a, e = int(lh[s, 0]), int(lh[s, B])
                ctx.set(v, LazyRagged(batch.keys[a:e], lod[s], a, B, s))
            elif v.name in batch.dense_names:
                ctx.set(v, batch.dense_var(v.name))
            elif v.name in batch.extra:
                ctx.set(v, batch.extra[v.name])

    def feed_dict(self, ctx: ExecContext, feed: Dict[str, Any]):
        B = 0
        for name, val in (feed or {}).items():
            v = self.program.global_block().vars.get(name)
            if isinstance(val, LoDTensor):
                t = val.value.to(self.device)
                if val.lod():
                    offs = torch.tensor(val.lod()[-1], dtype=torch.int64, device=self.device)
                    if v is not None and v.dtype == "int64":
                        t = t.reshape(-1)
                    ctx.set(name, Ragged(t, offs, offs.numel() - 1))
                    B = B or offs.numel() - 1
                    continue
            elif isinstance(val, torch.Tensor):
                t = val.to(self.device)
            else:
                arr = np.asarray(val)
                t = torch.as_tensor(arr).to(self.device)
            if v is not None and v.dtype in ("float32",) and t.dtype == torch.float64:
                t = t.float()
            ctx.set(name, t)
            B = B or (t.shape[0] if t.dim() else 1)
        ctx.B = ctx.B or B

    # -------------------------------------------------------------- run
    def _dump_program(self, device):
        """FLAGS_enable_dump_main_program (reference boxps_worker.cc:1163-1189):
        ./device_<id>_ops_<phase>.txt with the lowered op list (after fusion),
        the fusions applied and the parameter storage layout."""
        from ..utils import flags as _fl

        try:
            on = _fl.get_bool("enable_dump_main_program")
        except Exception:
            on = False
        if not on:
            return
        dev = device.index if device.type == "cuda" and device.index is not None else 0
        phase = "train" if self.training else "test"
        lines = [f"# lowered program: {len(self.lowered.steps)} ops, fusions: {self.lowered.fusions}"]
        lines += [f"{i:4d} {l}" for i, l in enumerate(self.lowered.describe().splitlines())]
        lines += [f"storage {n}: {sp.kind} {sp.shape} (logical {sp.logical})" for n, sp in self.lowered.storage.items()]
        with open(f"./device_{dev}_ops_{phase}.txt", "w") as f:
            f.write("\n".join(lines) + "\n")

    def forward(self, ctx: ExecContext):
        prof = self.op_profiler
        if prof is None and self._print_ops():
            for op in self.lowered.steps:
                log.info("op %s: %s -> %s", op.type, op.input_arg_names, op.output_arg_names)
                KERNELS[op.type](ctx, op)
            return
        if prof is None:
            for op in self.lowered.steps:
                KERNELS[op.type](ctx, op)
            return
        for op in self.lowered.steps:
            t0 = prof.begin()
            KERNELS[op.type](ctx, op)
            prof.end(op.type, t0)
            if ctx.training:
                names = op.output_arg_names
                names = names() if callable(names) else names
                prof.watch_grad(op.type + "_grad", [ctx.env[n] for n in names if n in ctx.env])

    def _print_ops(self) -> bool:
        """FLAGS_padbox_enable_print_op_debug: log every op as it runs
        (reference boxps_worker.cc:1304-1307); eager runs only (a captured
        step has no per-op host work)."""
        from ..utils import flags as _fl

        try:
            return _fl.get_bool("padbox_enable_print_op_debug")
        except Exception:
            return False

    def step(self, ctx: ExecContext):
        """forward + backward + dense sync + optimizer (one training batch)."""
        self.forward(ctx)
        if not (self.training and ctx.training):
            return
        prof = self.op_profiler
        t0 = prof.begin() if prof is not None else None
        loss = ctx.get(self.program._optimize["loss"])
        loss = loss.values if isinstance(loss, Ragged) else loss
        for a, o in zip(self.arenas, self.opts):
            if not getattr(o, "clear_grad", False):  # else the update kernel zeroed them last step
                a.zero_grad()
        if loss.dim() == 0 and loss.dtype == torch.float32:
            if self._one is None:
                self._one = torch.ones((), device=loss.device)
            loss.backward(self._one)  # persistent seed: no fill kernel per step
        else:
            loss.float().sum().backward()
        if self._next is not None:
            # the sparse push is on this stream already: pool the next batch
            # now, beside the tower's dW GEMM on its side stream
            self.prefetch(*self._next)
        if prof is not None:
            prof.end("backward (all grad ops + sparse push)", t0)
            t0 = prof.begin()
        lw = self.lowered
        side = self._side_stepped
        if lw.backward_ops or lw.optimize_ops:
            self._transpiled_sync(ctx)
        else:
            for s, o in zip(self.syncs, self.opts):
                if id(o) in side:  # already issued on the dW side stream by the tower's hook
                    s.after_step(o)
                else:
                    s.apply(o)
        if side:
            side.clear()  # the next forward joins the side-stream update
        else:
            join_grad_producers()  # an update issued behind the dW side stream
        if prof is not None:
            prof.end("dense sync + optimizer", t0)

    # ------------------------------------------------ optimizer state (checkpoints)
    def _opt_slots(self):
        """(param name, optimizer, element offset in its arena, storage shape,
        full-arena m, full-arena v) for every trainable parameter with Adam
        state.  ShardedFlatAdam's moments are all-gathered (collective: every
        rank must call this); an optimizer without exportable state warns
        instead of silently dropping it from the checkpoint."""
        from ..parallel.sharding import ShardedFlatAdam

        for a, o in zip(self.arenas, self.opts):
            if isinstance(o, FlatAdam):
                m, v = o.m, o.v
            elif isinstance(o, ShardedFlatAdam):
                m, v = o.gather_moments()
            else:
                if not isinstance(o, FlatSGD):  # SGD has no state to lose
                    warnings.warn(f"optimizer {type(o).__name__} has no exportable state: "
                                  "save_persistables writes the parameters only", RuntimeWarning)
                continue
            base = a.flat.data_ptr()
            for name, st in self.storage.items():
                if isinstance(st, torch.nn.Parameter) and st.untyped_storage().data_ptr() == \
                        a.flat.untyped_storage().data_ptr():
                    yield name, o, (st.data_ptr() - base) // 4, st.shape, m, v

    def optimizer_state(self) -> Dict[str, torch.Tensor]:
        """Adam state under the reference's persistable names
        (``<param>_moment1_0``, ``_moment2_0``, ``_beta1_pow_acc_0``,
        ``_beta2_pow_acc_0``, fluid/optimizer.py AdamOptimizer), in the
        parameters' fluid layout, so save_persistables / load_persistables
        resume training exactly.

        Beta powers: the reference initialises the accumulators to beta and
        multiplies after each update (optimizer.py:2518-2523), so after t steps
        they hold beta^(t+1); FlatAdam's ``pows`` hold beta^t (multiplied
        before use).  The boundary converts both ways."""
        out = {}
        for name, o, off, shape, m, v in self._opt_slots():
            n = int(np.prod(shape))
            out[name + "_moment1_0"] = self._logical_of(name, m[off:off + n].view(shape))
            out[name + "_moment2_0"] = self._logical_of(name, v[off:off + n].view(shape))
            out[name + "_beta1_pow_acc_0"] = o.pows[0:1] * o.b1
            out[name + "_beta2_pow_acc_0"] = o.pows[1:2] * o.b2
        return out

    def load_optimizer_state(self, state: Dict[str, Any], reference_pows: bool = True) -> int:
        """``reference_pows``: the beta-pow accumulators hold beta^(t+1) (the
        reference convention, what optimizer_state writes); False for files
        written before io.save_persistables recorded the convention (beta^t)."""
        from ..parallel.sharding import ShardedFlatAdam

        n_loaded = 0
        touched = {}
        with torch.no_grad():
            for name, o, off, shape, m, v in self._opt_slots():
                n = int(np.prod(shape))
                for suffix, buf in (("_moment1_0", m), ("_moment2_0", v)):
                    if name + suffix in state:
                        dst = self._logical_of(name, buf[off:off + n].view(shape))
                        dst.copy_(torch.as_tensor(state[name + suffix]).reshape(dst.shape).to(dst.device))
                        n_loaded += 1
                        touched[id(o)] = (o, m, v)
                for i, (suffix, beta) in enumerate((("_beta1_pow_acc_0", o.b1), ("_beta2_pow_acc_0", o.b2))):
                    if name + suffix in state:
                        acc = torch.as_tensor(state[name + suffix], dtype=torch.float32).reshape(1)
                        o.pows[i:i + 1].copy_((acc / beta if reference_pows else acc).to(o.pows.device))
            for o, m, v in touched.values():
                if isinstance(o, ShardedFlatAdam):
                    o.scatter_moments(m, v)
        return n_loaded

    def _restore_optimizer_state_from_scope(self):
        """load_persistables before the first run stages Adam state in the
        scope (no session yet); pick it up once the optimizers exist."""
        names = {n for n in self.optimizer_state()}
        staged = {n: self.scope.get(n) for n in names if n in self.scope}
        if staged:
            conv = self.scope.get("@beta_pow_convention@") if "@beta_pow_convention@" in self.scope else None
            self.load_optimizer_state(staged, reference_pows=conv is None or bool(int(conv)))
            self.scope._tensors.pop("@beta_pow_convention@", None)
            for n in staged:  # consumed: a later session must not re-apply a stale checkpoint
                self.scope._tensors.pop(n, None)

    # ------------------------------------------------ transpiled dense sync
    def _logical_of(self, name: str, t: torch.Tensor) -> torch.Tensor:
        """View of a storage-layout tensor (a parameter or its gradient) in
        the fluid (logical) layout -- same mapping as ``_refresh_logical``."""
        spec = self.lowered.storage.get(name)
        if spec is None or spec.kind == "plain":
            return t.view(spec.logical) if spec is not None else t
        if spec.kind == "t_pad":
            K, N = spec.logical
            return t[:N, :K].t()
        return t[: spec.logical[0]]

    def _run_role_ops(self, ctx: ExecContext, ops, bound: Dict[str, torch.Tensor]):
        """Run transpiler ops on ``bound`` tensors, then write every rewritten
        value back in place (kernels are functional; coalesced buffers are
        split back into their member tensors)."""
        for n, t in bound.items():
            ctx.set(n, t)
        ctx.cache["coalesced"] = {}
        for op in ops:
            KERNELS[op.type](ctx, op)
        with torch.no_grad():
            for fused, members in ctx.cache["coalesced"].items():
                val = ctx.env.get(fused)
                if val is None or val.dim() != 1:
                    continue
                off = 0
                for m in members:
                    dst = bound.get(m)
                    if dst is None:
                        continue
                    n = dst.numel()
                    dst.copy_(val[off:off + n].view(dst.shape))
                    off += n
            for n, dst in bound.items():
                val = ctx.env.get(n)
                if val is not None and val is not dst:
                    dst.copy_(val.view(dst.shape) if val.numel() == dst.numel() else val)
            # persistable outputs that are not bound (LocalSGD snapshots) live in the scope
            blk = self.program.global_block()
            for op in ops:
                for n in op.output_arg_names:
                    if n not in bound and blk.has_var(n) and blk.var(n).persistable and n in ctx.env:
                        self.scope.set(n, ctx.env[n].detach().clone())

    def _transpiled_sync(self, ctx: ExecContext):
        """Dense sync carried by the program (GradAllReduce / LocalSGD /
        MultiThread transpilers): backward-role ops on the @GRAD values, the
        optimizer update(s), then optimize-role ops on the parameters."""
        lw = self.lowered
        # the backward-role ops read the gradients: wait for the side streams
        # still producing them (the tower's dW runs beside the sparse push)
        join_grad_producers()
        grads = {}
        for name, st in self.storage.items():
            if isinstance(st, torch.nn.Parameter):
                if st.grad is None:
                    st.grad = torch.zeros_like(st)
                grads[name + "@GRAD"] = self._logical_of(name, st.grad)
        self._run_role_ops(ctx, lw.backward_ops, grads)
        gather = next((op for op in lw.backward_ops if op.type == "c_allgather" and op.attrs.get("per_rank_update")),
                      None)
        if gather is not None:
            # one update per gathered gradient, in rank order (all_gather mode)
            gathered = ctx.get(gather.outputs["Out"][0])
            members = ctx.cache["coalesced"][gather.inputs["X"][0].name]
            per = sum(grads[m].numel() for m in members if m in grads)
            world = max(1, gathered.numel() // max(1, per))
            with torch.no_grad():
                for r in range(world):
                    part, off = gathered[r * per:(r + 1) * per], 0
                    for m in members:
                        g = grads.get(m)
                        if g is None:
                            continue
                        g.copy_(part[off:off + g.numel()].view(g.shape))
                        off += g.numel()
                    for o in self.opts:
                        o.step(1.0 / world)
        else:
            for s, o in zip(self.syncs, self.opts):
                s.apply(o)
        if lw.optimize_ops:
            join_grad_producers()
            params = {name: self.logical[name] for name, st in self.storage.items()
                      if isinstance(st, torch.nn.Parameter)}
            self._run_role_ops(ctx, lw.optimize_ops, params)

    def fetch(self, ctx: ExecContext, fetch_list, return_numpy=True):
        out = []
        for f in fetch_list or []:
            v = ctx.get(f)
            t = v.values if isinstance(v, Ragged) else v
            t = t.detach()
            if return_numpy:
                out.append(t.float().cpu().numpy() if t.dtype == torch.bfloat16 else t.cpu().numpy())
            else:
                out.append(LoDTensor(t))
        return out


class Executor:
    def __init__(self, place=None):
        self.place = place
        self.device = to_device(place)
        self._sessions: Dict[tuple, Session] = {}

    def sessions_for(self, program: Program) -> List[Session]:
        return [s for k, s in self._sessions.items() if k[0] == id(program) and s.training]

    def _session(self, program: Program, scope: Scope, fetch_names=(), **kw) -> Session:
        key = (id(program), program._version, id(scope), tuple(sorted(fetch_names)))
        s = self._sessions.get(key)
        if s is None:
            s = Session(program, scope, self.device, fetch_names, **kw)
            self._sessions = {k: v for k, v in self._sessions.items() if k[0] != id(program)}
            self._sessions[key] = s
        return s

    @staticmethod
    def _is_startup(program: Program) -> bool:
        ops = program.global_block().ops
        # init_param, plus the parameter snapshots a LocalSGD transpile adds
        return bool(ops) and program._optimize is None and all(op.type in ("init_param", "assign") for op in ops) \
            and any(op.type == "init_param" for op in ops)

    def run(self, program: Optional[Program] = None, feed=None, fetch_list=None, feed_var_name="feed",
            fetch_var_name="fetch", scope: Optional[Scope] = None, return_numpy=True, use_program_cache=False,
            **_):
        program = program or default_main_program()
        program = getattr(program, "_program", program)  # CompiledProgram
        scope = scope or global_scope()
        if self._is_startup(program) or not program.global_block().ops:
            ctx = ExecContext(_StartupSession(scope, self.device, program), training=False)
            for op in program.global_block().ops:
                KERNELS[op.type](ctx, op)
            blk = program.global_block()
            for name, val in ctx.env.items():  # persistable outputs (snapshots) live in the scope
                if blk.has_var(name) and blk.var(name).persistable and isinstance(val, torch.Tensor):
                    scope.set(name, val.detach().clone())
            return []
        names = [f if isinstance(f, str) else f.name for f in (fetch_list or [])]
        s = self._session(program, scope, names)
        ctx = ExecContext(s, training=s.training)
        s.feed_dict(ctx, feed)
        s.step(ctx)
        return s.fetch(ctx, names, return_numpy)

    def train_from_dataset(self, program=None, dataset=None, scope=None, thread=0, debug=False, fetch_list=None,
                           fetch_info=None, print_period=100, fetch_handler=None):
        from ..runtime.trainer import create_trainer

        program = getattr(program or default_main_program(), "_program", program or default_main_program())
        trainer = create_trainer(self, program, scope or global_scope(), dataset, infer=False, debug=debug,
                                 fetch_list=fetch_list, fetch_info=fetch_info, print_period=print_period,
                                 fetch_handler=fetch_handler)
        return trainer.run()

    def infer_from_dataset(self, program=None, dataset=None, scope=None, thread=0, debug=False, fetch_list=None,
                           fetch_info=None, print_period=100, fetch_handler=None):
        from ..runtime.trainer import create_trainer

        program = getattr(program or default_main_program(), "_program", program or default_main_program())
        trainer = create_trainer(self, program, scope or global_scope(), dataset, infer=True, debug=debug,
                                 fetch_list=fetch_list, fetch_info=fetch_info, print_period=print_period,
                                 fetch_handler=fetch_handler)
        return trainer.run()

    def close(self):
        for sess in self._sessions.values():
            if hasattr(sess, "close"):
                sess.close()
        self._sessions.clear()


class _StartupSession:
    def __init__(self, scope, device, program):
        self.scope = scope
        self.device = device
        self.generator = torch.Generator().manual_seed(program.random_seed or 0)
        self.generator_dev = None
        self.group = None
        self.cache = {}
        self.logical = {}
        self.storage = {}


class CompiledProgram:
    """Accepted for API compatibility; programs are always lowered/fused."""

    def __init__(self, program_or_graph, build_strategy=None):
        self._program = program_or_graph

    def with_data_parallel(self, loss_name=None, build_strategy=None, exec_strategy=None, share_vars_from=None,
                           places=None):
        return self
