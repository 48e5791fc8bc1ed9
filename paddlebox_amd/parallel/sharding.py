"""ZeRO-1 optimizer-state sharding over the flat dense arena.

Reference behaviour: ``ThreadShardingOptimizer``
(``py/distributed/fleet/meta_optimizers/sharding_optimizer.py:1867-2053``) +
the BoxPS worker's sharding mode (``boxps_worker.cc:601-770,1024-1147``):
each rank keeps optimizer moments only for the parameters it owns, updates
them, and the owners broadcast the new values.

MI355X-first form: the dense params already live in ONE contiguous arena
(``DenseArena``), so ownership is a contiguous 1/world slice of it instead of
a per-parameter assignment.  A step is

    reduce_scatter(grad)  -> this rank's grad slice (sum over ranks)
    Adam on the slice     -> one fused kernel over 1/world of the params
    all_gather(params)    -> every rank has the full updated arena

which moves the same bytes as one all-reduce (RS + AG) but keeps only
1/world of the Adam moments per GPU.  On xGMI both collectives are
per-link-parallel mesh operations inside RCCL.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .. import _native
from ..ops import reference as ref
from .comm import collective_active
from .dense import join_grad_producers, DenseArena


def _backend(group) -> str:
    try:
        return dist.get_backend(group)
    except Exception:  # pragma: no cover
        return "gloo"


def reduce_scatter_flat(out: torch.Tensor, flat: torch.Tensor, group=None):
    """out = (sum over ranks of flat)[rank slice]; len(flat) = world*len(out)."""
    if _backend(group) == "nccl":
        dist.reduce_scatter_tensor(out, flat, group=group)
        return
    tmp = flat.clone()  # gloo has no reduce_scatter: all-reduce then slice
    dist.all_reduce(tmp, group=group)
    r = dist.get_rank(group)
    out.copy_(tmp[r * out.numel():(r + 1) * out.numel()])


def all_gather_flat(flat: torch.Tensor, part: torch.Tensor, group=None):
    if _backend(group) == "nccl":
        dist.all_gather_into_tensor(flat, part, group=group)
        return
    w = dist.get_world_size(group)
    parts = list(flat.view(w, -1).unbind(0))
    dist.all_gather(parts, part.contiguous(), group=group)
    flat.copy_(torch.cat(parts))


class ShardedFlatAdam:
    """Adam whose moments cover only this rank's slice of the arena."""

    def __init__(self, arena: DenseArena, lr: float = 1e-3, beta1: float = 0.9, beta2: float = 0.999,
                 epsilon: float = 1e-8, weight_decay: float = 0.0, group=None):
        self.a = arena
        self.group = group
        self.active = collective_active(group)
        self.world = dist.get_world_size(group) if self.active else 1
        self.rank = dist.get_rank(group) if self.active else 0
        self.lr, self.b1, self.b2, self.eps, self.wd = lr, beta1, beta2, epsilon, weight_decay
        n = arena.flat.numel()
        self.shard = (n + self.world - 1) // self.world
        self.padded = self.shard * self.world
        dev = arena.flat.device
        # arena.flat / arena.grad are padded in place views when sizes differ
        self._pflat = torch.zeros(self.padded, device=dev)
        self._pgrad = torch.zeros(self.padded, device=dev)
        self.m = torch.zeros(self.shard, device=dev)
        self.v = torch.zeros(self.shard, device=dev)
        self.g = torch.zeros(self.shard, device=dev)
        self.pows = torch.ones(2, dtype=torch.float32, device=dev)

    def _slice(self, t: torch.Tensor) -> torch.Tensor:
        return t[self.rank * self.shard:(self.rank + 1) * self.shard]

    def step(self, grad_scale: float = 1.0):
        join_grad_producers()
        n = self.a.flat.numel()
        self._pgrad[:n].copy_(self.a.grad)
        if self.active:
            reduce_scatter_flat(self.g, self._pgrad, self.group)
        else:
            self.g.copy_(self._pgrad)
        self._pflat[:n].copy_(self.a.flat)
        p = self._slice(self._pflat)
        scale = grad_scale / self.world  # mean over ranks, like grad_allreduce
        if p.is_cuda:
            _native.hip().adam_flat(p, self.g, self.m, self.v, self.pows, self.lr, self.b1, self.b2, self.eps,
                                    scale, self.wd, False)
        else:
            self.pows[0] *= self.b1
            self.pows[1] *= self.b2
            ref.adam_flat(p, self.g, self.m, self.v, self.lr, self.b1, self.b2, self.eps, float(self.pows[0]),
                          float(self.pows[1]), scale, self.wd)
        if self.active:
            all_gather_flat(self._pflat, p.clone(), self.group)
        self.a.flat.copy_(self._pflat[:n])

    def gather_moments(self):
        """Full-arena (m, v) assembled from every rank's shard (collective)."""
        n = self.a.flat.numel()
        if not self.active:
            return self.m[:n].clone(), self.v[:n].clone()
        out = []
        for part in (self.m, self.v):
            full = torch.empty(self.padded, device=part.device)
            all_gather_flat(full, part, self.group)
            out.append(full[:n])
        return out[0], out[1]

    def scatter_moments(self, m_full: torch.Tensor, v_full: torch.Tensor):
        """Inverse of gather_moments: keep this rank's slice of full-arena moments."""
        n = self.a.flat.numel()
        for part, full in ((self.m, m_full), (self.v, v_full)):
            pad = torch.zeros(self.padded, device=part.device)
            pad[:n] = full.reshape(-1)[:n].to(part.device)
            part.copy_(self._slice(pad))

    def state_dict(self):
        return {"m": self.m, "v": self.v, "pows": self.pows, "rank": self.rank, "world": self.world}

    def load_state_dict(self, sd):
        self.m.copy_(sd["m"])
        self.v.copy_(sd["v"])
        self.pows.copy_(sd["pows"])
