"""Dense-parameter arena + data-parallel sync + fused optimizer.

All dense parameters of a model live in ONE contiguous fp32 buffer and their
gradients in another (the reference packs params for fused sync,
``boxps_worker.cc:481-520`` AllocParamTensor, and ``coalesce_tensor`` for
gradient fusion).  That makes data-parallel sync a single RCCL all-reduce
(one bucket: CTR MLPs are a few MB, well inside the one-shot regime of the
xGMI mesh) and the optimizer a single fused Adam launch.

Sync modes (``trainer_desc.proto:121-129`` / ``boxps_worker.cc:1191-1258``):
  * ``grad_allreduce``  -- all-reduce grads every step (transpiler GradAllReduce)
  * ``kstep``           -- local steps, parameter averaging every k steps
                            (sync_dense_mode 2, DenseKStepALL)
  * ``none``            -- no sync
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional

import torch
import torch.distributed as dist

from .. import _native
from ..ops import reference as ref
from .comm import collective_active


# Side streams still writing dense gradients (the tower's dW GEMM runs there,
# overlapped with the head backward + sparse push).  Anything that reads the
# gradients or rewrites the parameters joins them first.
_GRAD_PRODUCERS: List[torch.cuda.Stream] = []


def add_grad_producer(stream) -> None:
    _GRAD_PRODUCERS.append(stream)


# Overlapped optimizer (CtrTrainStep adam_overlap): the side stream records an
# event once the data_norm summaries are updated (before its Adam); the next
# step's head may start after that event instead of after the whole side
# stream.  Keyed by the tower; any full join makes the events moot.
_PRE_HEAD: Dict[int, "torch.cuda.Event"] = {}


def set_pre_head_event(key: int, ev) -> None:
    _PRE_HEAD[key] = ev


def pop_pre_head_event(key: int):
    return _PRE_HEAD.pop(key, None)


def join_grad_producer_upto_now(stream) -> None:
    """Make the current stream wait for what ``stream`` has queued so far and
    stop tracking it as a gradient producer -- work queued on it afterwards
    (e.g. the next batch's dedup on the dW stream) is not waited for by a
    later ``join_grad_producers``.  Other producers and pre-head events stay."""
    if stream in _GRAD_PRODUCERS:
        ev = torch.cuda.Event()
        ev.record(stream)
        torch.cuda.current_stream(stream.device).wait_event(ev)
        while stream in _GRAD_PRODUCERS:
            _GRAD_PRODUCERS.remove(stream)


def join_grad_producers() -> None:
    """Make the current stream wait for every pending gradient producer."""
    while _GRAD_PRODUCERS:
        s = _GRAD_PRODUCERS.pop()
        torch.cuda.current_stream(s.device).wait_stream(s)
    _PRE_HEAD.clear()


class DenseArena:
    def __init__(self, params: Iterable[torch.nn.Parameter], device: torch.device, extra_grad: int = 0):
        """``extra_grad`` floats are appended to the gradient buffer (not to the
        parameters): values that must be summed across ranks together with the
        gradients -- e.g. data_norm batch statistics -- ride in the same single
        all-reduce instead of a collective of their own (``grad_tail``)."""
        self.params: List[torch.nn.Parameter] = [p for p in params if p.requires_grad]
        n = sum(p.numel() for p in self.params)
        # pad each param to 4 floats so every view is 16-B aligned
        sizes = [(p.numel() + 3) // 4 * 4 for p in self.params]
        total = sum(sizes)
        self.numel = n
        self.flat = torch.zeros(total, device=device)
        self.grad = torch.zeros(total + (int(extra_grad) + 3) // 4 * 4, device=device)
        self._tail = total
        off = 0
        self.views = []
        for p, sz in zip(self.params, sizes):
            v = self.flat[off:off + p.numel()].view_as(p)
            v.copy_(p.data)
            p.data = v
            p.grad = self.grad[off:off + p.numel()].view_as(p)
            self.views.append((off, p.numel()))
            off += sz
        # callbacks run when something other than the optimizer rewrites the
        # fp32 masters (parameter averaging, checkpoint load): derived copies
        # such as the packed bf16 tower weights must be rebuilt
        self.on_modified = []

    def notify_modified(self):
        for f in self.on_modified:
            f()

    def grad_tail(self, n: int) -> torch.Tensor:
        """Reserve n floats of the extra gradient region (summed by the dense
        all-reduce, never touched by the optimizer)."""
        if self._tail + n > self.grad.numel():
            raise ValueError("DenseArena: extra_grad region exhausted")
        v = self.grad[self._tail:self._tail + n]
        self._tail += (n + 3) // 4 * 4
        return v

    @property
    def param_grad(self) -> torch.Tensor:
        """The gradient entries of the parameters (without the extra region)."""
        return self.grad[: self.flat.numel()]

    def zero_grad(self):
        join_grad_producers()
        self.grad.zero_()

    def state_dict(self) -> Dict[str, torch.Tensor]:
        return {"flat": self.flat}


class FlatAdam:
    """Adam over the whole arena in one kernel (Paddle adam semantics)."""

    def __init__(self, arena: DenseArena, lr: float = 1e-3, beta1: float = 0.9, beta2: float = 0.999,
                 epsilon: float = 1e-8, weight_decay: float = 0.0, clear_grad: bool = False):
        self.a = arena
        self.lr, self.b1, self.b2, self.eps, self.wd = lr, beta1, beta2, epsilon, weight_decay
        # clear_grad: the update kernel zeroes the gradient arena after use, so
        # the training step needs no separate zero_grad launch
        self.clear_grad = clear_grad
        self.m = torch.zeros_like(arena.flat)
        self.v = torch.zeros_like(arena.flat)
        # [beta1^t, beta2^t] on the device: advanced by the kernel itself so the
        # step is HIP-graph replayable (no host scalars baked into the graph)
        self.pows = torch.ones(2, dtype=torch.float32, device=arena.flat.device)
        self.ticket = torch.zeros(1, dtype=torch.int32, device=arena.flat.device)
        self._fuse_mlps, self._fuse_dns = [], []

    MAX_PACK_REGIONS = 8  # kernels.h kMaxPackRegions

    def fuse(self, mlps=(), data_norms=()):
        """Let the update kernel also (a) re-pack the bf16 tower copies of
        these MLPs' weights and (b) apply these data_norm layers' summary
        updates from their batch statistics -- one launch per step for the
        whole dense side (csrc/hip/tower.hip k_adam_fused)."""
        if not self.a.flat.is_cuda:
            return self
        self._fuse_mlps = [m for m in mlps if m is not None]
        self._fuse_dns = [d for d in data_norms if d is not None]
        for m in self._fuse_mlps:
            m.packed_by_optimizer = True
        for d in self._fuse_dns:
            d.fused_update = True
        self.a.on_modified.extend(m.invalidate_pack for m in self._fuse_mlps)
        return self

    def _extras(self):
        base = self.a.flat.data_ptr()
        pack = []
        for mlp in self._fuse_mlps:
            if not mlp.packed_by_optimizer:
                continue  # its forward packs (too many workspaces for the launch)
            # the tower packs on its first forward; every batch size's
            # workspace keeps its own packed copy, all re-packed here
            tws = mlp.tower_workspaces() if hasattr(mlp, "tower_workspaces") else (
                [mlp._tw] if mlp._tw is not None else [])
            regs = [((w.data_ptr() - base) // 4,) + tuple(reg) for tw in tws for reg, w in zip(tw.pack_regions(), mlp.w)]
            if len(pack) + len(regs) > self.MAX_PACK_REGIONS:
                # more batch sizes than one launch re-packs: this MLP's forward
                # packs its current workspace from now on (always correct)
                mlp.packed_by_optimizer = False
                mlp.invalidate_pack()
                continue
            pack += regs
        dn = [(d.stats, d.batch_size, d.batch_sum, d.batch_square_sum, d.decay)
              for d in self._fuse_dns if d.training and d.update_norm]
        return pack, dn

    def step(self, grad_scale: float = 1.0, join: bool = True):
        # (issuing the update on the dW side stream instead, beside the sparse
        # push, measured no faster: 0.286 vs 0.280-0.285 ms/step; bench.py
        # PBX_ADAM_ON_SIDE re-measures it).  join=False: the caller is on the
        # stream that produced the gradients
        if join:
            join_grad_producers()
        if self.a.flat.is_cuda:
            pack, dn = self._extras()
            _native.hip().adam_fused(self.a.flat, self.a.param_grad, self.m, self.v, self.pows, self.ticket, self.lr,
                                     self.b1, self.b2, self.eps, grad_scale, self.wd, self.clear_grad, pack, dn)
        else:
            self.pows[0] *= self.b1
            self.pows[1] *= self.b2
            ref.adam_flat(self.a.flat, self.a.param_grad, self.m, self.v, self.lr, self.b1, self.b2, self.eps,
                          float(self.pows[0]), float(self.pows[1]), grad_scale, self.wd)
            if self.clear_grad:
                self.a.param_grad.zero_()

    def state_dict(self):
        return {"m": self.m, "v": self.v, "pows": self.pows}

    def load_state_dict(self, sd):
        self.m.copy_(sd["m"])
        self.v.copy_(sd["v"])
        self.pows.copy_(sd["pows"])


def _flags_get_bool(name: str) -> bool:
    from ..utils import flags as _fl

    try:
        return _fl.get_bool(name)
    except Exception:
        return False


class HierarchicalAllReduce:
    """Node-aware all-reduce: reduce-scatter inside the node (xGMI), all-reduce
    of each shard across nodes between the ranks with the same local index,
    all-gather inside the node.  Nodes are consecutive blocks of
    ``local_size`` ranks (torchrun's LOCAL_WORLD_SIZE).  gloo (CPU tests)
    has no reduce-scatter: the node reduce is an all-reduce there and each
    rank keeps its shard."""

    def __init__(self, group=None, local_size: int = 0):
        import os

        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        ls = int(local_size or os.environ.get("LOCAL_WORLD_SIZE", self.world))
        if ls <= 0 or self.world % ls:
            ls = self.world
        self.local_size = ls
        self.nodes = self.world // ls
        ranks = dist.get_process_group_ranks(group) if group is not None else list(range(self.world))
        self.node_group = self.cross_group = None
        for n in range(self.nodes):  # every rank creates every group (collective new_group)
            g = dist.new_group(ranks[n * ls:(n + 1) * ls])
            if n == self.rank // ls:
                self.node_group = g
        for i in range(ls):
            g = dist.new_group([ranks[n * ls + i] for n in range(self.nodes)])
            if i == self.rank % ls:
                self.cross_group = g
        self.gloo = dist.get_backend(group) == "gloo"

    def allreduce_(self, t: torch.Tensor) -> torch.Tensor:
        ls, li = self.local_size, self.rank % self.local_size
        n = t.numel()
        part = (n + ls - 1) // ls
        flat = t.view(-1)
        pad = part * ls - n
        buf = torch.cat([flat, flat.new_zeros(pad)]) if pad else flat
        shard = buf.new_empty(part)
        if self.gloo:
            tmp = buf.clone()
            dist.all_reduce(tmp, group=self.node_group)
            shard.copy_(tmp[li * part:(li + 1) * part])
        else:
            dist.reduce_scatter_tensor(shard, buf, group=self.node_group)
        if self.nodes > 1:
            dist.all_reduce(shard, group=self.cross_group)
        out = buf if pad else buf.new_empty(buf.numel())
        dist.all_gather_into_tensor(out, shard, group=self.node_group) if not self.gloo else \
            dist.all_gather(list(out.view(ls, part)), shard, group=self.node_group)
        flat.copy_(out[:n])
        return t


class DenseSync:
    """Data-parallel dense synchronisation over RCCL (or gloo on CPU)."""

    def __init__(self, arena: DenseArena, mode: str = "grad_allreduce", k: int = 1, group=None,
                 overlap_group=None, ipc=None):
        """``overlap_group``: a process group of its own (own communicator) on
        which ``launch()`` runs the gradient all-reduce on a side stream, so it
        overlaps the rest of the backward (the sparse push and its key
        all-to-all, which use the default group).  ``ipc``: an
        :class:`~paddlebox_amd.parallel.ipc.IpcMesh` whose one-shot all-reduce
        replaces RCCL's ring for the gradient buffer (intra-node)."""
        self.a = arena
        self.mode = mode
        self.k = max(1, k)
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        self.active = collective_active(group)
        self.steps = 0
        self.overlap_group = overlap_group
        self.ipc = ipc
        self._stream = None
        self._launched = False
        self.hier = HierarchicalAllReduce(group) if mode == "kstep_node" and self.active else None

    def _allreduce_grad(self, group):
        if self.ipc is not None:
            self.ipc.allreduce_(self.a.grad)
        else:
            dist.all_reduce(self.a.grad, group=group)

    def launch(self):
        """Start the gradient all-reduce now, on a side stream (call when the
        dense gradients are final); ``before_step`` joins it."""
        if not (self.active and self.mode == "grad_allreduce") or not self.a.grad.is_cuda:
            return
        join_grad_producers()
        dev = self.a.grad.device
        cur = torch.cuda.current_stream(dev)
        if self._stream is None:
            from ..runtime.streams import side_stream

            self._stream = side_stream(dev, "dense_sync")
        self._stream.wait_stream(cur)
        with torch.cuda.stream(self._stream):
            self._allreduce_grad(self.overlap_group if self.overlap_group is not None else self.group)
        self._launched = True

    def grad_scale(self) -> float:
        return 1.0 / self.world if (self.mode == "grad_allreduce" and self.world > 1) else 1.0

    def before_step(self):
        """Called after backward, before the optimizer.
        FLAGS_enable_dense_nccl_barrier: a barrier before the (eager) dense
        all-reduce, so its timer measures the collective alone
        (box_wrapper.h:711-713)."""
        if self.active and self.mode == "grad_allreduce" and not self._launched and \
                _flags_get_bool("enable_dense_nccl_barrier") and not (torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()):
            dist.barrier(group=self.group)
        if self._launched or (self.active and self.mode == "grad_allreduce"):
            join_grad_producers()
        if self._launched:
            torch.cuda.current_stream(self.a.grad.device).wait_stream(self._stream)
            self._launched = False
            return
        if self.active and self.mode == "grad_allreduce":
            self._allreduce_grad(self.group)

    def apply(self, opt):
        """Sync + optimizer update for one step, every mode.

        ``allgather`` is the transpiler's MultiThread all_gather mode
        (``py/fluid/transpiler/collective.py:499-636``): every rank gathers all
        ranks' gradients and runs one optimizer update per gathered gradient,
        in rank order, so all replicas stay identical."""
        join_grad_producers()
        if self.active and self.mode == "allgather":
            g = self.a.grad
            parts = [torch.empty_like(g) for _ in range(self.world)]
            dist.all_gather(parts, g, group=self.group)
            for p in parts:
                g.copy_(p)
                opt.step(1.0 / self.world)
            self.after_step()
            return
        self.before_step()
        opt.step(self.grad_scale())
        self.after_step(opt)

    def after_step(self, opt=None):
        self.steps += 1
        if self.active and self.mode in ("kstep", "local_sgd", "kstep_node") and self.steps % self.k == 0:
            self.sync_params()
            # FLAGS_enable_sync_dense_moment: average the Adam moments with the
            # parameters (boxps_worker.cc:464-476)
            if opt is not None and _flags_get_bool("enable_sync_dense_moment"):
                for buf in (getattr(opt, "m", None), getattr(opt, "v", None)):
                    if isinstance(buf, torch.Tensor):
                        dist.all_reduce(buf, group=self.group)
                        buf.mul_(1.0 / self.world)

    def sync_params(self):
        """Parameter averaging (boxps_worker.cc:1235-1239: sum then x 1/devices).
        ``kstep_node`` (sync_dense_mode 1 across nodes, :1211-1228): the
        node's GPUs reduce-scatter the parameters, each shard is all-reduced
        with the same shard of every other node, and the node all-gathers
        the result -- the cross-node traffic is 1/local_size of the buffer
        per GPU, in parallel over the node's GPUs."""
        if not self.active:
            return
        if self.mode == "kstep_node" and self.hier is not None:
            self.hier.allreduce_(self.a.flat)
        else:
            dist.all_reduce(self.a.flat, group=self.group)
        self.a.flat.mul_(1.0 / self.world)
        self.a.notify_modified()


class FlatSGD:
    """p -= lr * g over the whole arena (one axpy)."""

    def __init__(self, arena: DenseArena, lr: float = 0.01, weight_decay: float = 0.0):
        self.a, self.lr, self.wd = arena, lr, weight_decay

    def step(self, grad_scale: float = 1.0):
        join_grad_producers()
        g = self.a.grad
        if self.wd:
            self.a.flat.mul_(1.0 - self.lr * self.wd)
        self.a.flat.add_(g, alpha=-self.lr * grad_scale)

    def state_dict(self):
        return {}

    def load_state_dict(self, sd):
        pass


class FlatMomentum:
    def __init__(self, arena: DenseArena, lr: float = 0.01, momentum: float = 0.9, use_nesterov: bool = False):
        self.a, self.lr, self.mu, self.nesterov = arena, lr, momentum, use_nesterov
        self.vel = torch.zeros_like(arena.flat)

    def step(self, grad_scale: float = 1.0):
        join_grad_producers()
        g = self.a.grad if grad_scale == 1.0 else self.a.grad * grad_scale
        self.vel.mul_(self.mu).add_(g)
        upd = g.add(self.vel, alpha=self.mu) if self.nesterov else self.vel
        self.a.flat.add_(upd, alpha=-self.lr)

    def state_dict(self):
        return {"velocity": self.vel}

    def load_state_dict(self, sd):
        self.vel.copy_(sd["velocity"])


class FlatAdagrad:
    def __init__(self, arena: DenseArena, lr: float = 0.01, epsilon: float = 1e-6, initial_accumulator_value=0.0):
        self.a, self.lr, self.eps = arena, lr, epsilon
        self.acc = torch.full_like(arena.flat, float(initial_accumulator_value))

    def step(self, grad_scale: float = 1.0):
        join_grad_producers()
        g = self.a.grad if grad_scale == 1.0 else self.a.grad * grad_scale
        self.acc.addcmul_(g, g)
        self.a.flat.addcdiv_(g, self.acc.sqrt().add_(self.eps), value=-self.lr)

    def state_dict(self):
        return {"moment": self.acc}

    def load_state_dict(self, sd):
        self.acc.copy_(sd["moment"])
