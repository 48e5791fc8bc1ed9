"""Collective-communication facade for the engine.

``TorchDistComm`` maps onto ``torch.distributed`` (backend ``nccl`` = RCCL on
ROCm over xGMI; ``gloo`` on the CPU).  ``LoopbackGroup`` runs W engine ranks
as threads inside ONE process (on one GPU or the CPU) with an in-memory
exchange: it exercises exactly the sharded code path (key/value/gradient
all-to-all, owner-side merge) without needing W devices -- the single-GPU
stand-in for the multi-GPU xGMI exchange in tests.

Reference collectives replaced: NCCL group calls in ``boxps_worker.cc:1220-1236``
and ``c_mixallgather_op.cc:221-327``; BoxPS's closed GPU<->GPU key routing.
"""
from __future__ import annotations

import os
import threading
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist


class Comm:
    world: int = 1
    rank: int = 0

    def all_to_all_single(self, out: torch.Tensor, inp: torch.Tensor, out_splits: Optional[Sequence[int]] = None,
                          in_splits: Optional[Sequence[int]] = None):
        raise NotImplementedError

    def all_reduce(self, t: torch.Tensor, op: str = "sum"):
        raise NotImplementedError

    def barrier(self):
        pass

    @property
    def backend(self) -> str:
        return "none"


class TorchDistComm(Comm):
    def __init__(self, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)

    def all_to_all_single(self, out, inp, out_splits=None, in_splits=None):
        dist.all_to_all_single(out, inp, None if out_splits is None else list(out_splits),
                               None if in_splits is None else list(in_splits), group=self.group)

    def all_reduce(self, t, op="sum"):
        o = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op]
        dist.all_reduce(t, op=o, group=self.group)

    def barrier(self):
        dist.barrier(group=self.group)

    @property
    def backend(self) -> str:
        return dist.get_backend(self.group)


def force_collectives() -> bool:
    """``PBX_FORCE_COLLECTIVES=1``: run every collective of the multi-GPU path
    (key/value/grad all-to-all, dense all-reduce, data_norm stats) even for a
    world of one rank.  A 1-GPU box rehearses the exact N-GPU step -- RCCL
    calls captured inside the HIP graph included -- this way."""
    return os.environ.get("PBX_FORCE_COLLECTIVES", "0") == "1"


def collective_active(group=None) -> bool:
    """True when collectives over ``group`` must actually run."""
    if not (dist.is_available() and dist.is_initialized()):
        return False
    return dist.get_world_size(group) > 1 or force_collectives()


def default_comm(group=None) -> Optional[Comm]:
    if collective_active(group):
        return TorchDistComm(group)
    return None


class LoopbackGroup:
    """W in-process ranks (threads) with a barrier-synchronised exchange."""

    def __init__(self, world: int):
        self.world = world
        self._barrier = threading.Barrier(world)
        self._slots: List[object] = [None] * world

    def comm(self, rank: int) -> "LoopbackComm":
        return LoopbackComm(self, rank)


class LoopbackComm(Comm):
    def __init__(self, grp: LoopbackGroup, rank: int):
        self.g = grp
        self.world = grp.world
        self.rank = rank

    def _sync(self):
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        self.g._barrier.wait()

    def all_to_all_single(self, out, inp, out_splits=None, in_splits=None):
        W = self.world
        if in_splits is None:
            n = inp.shape[0] // W
            in_splits = [n] * W
        if out_splits is None:
            n = out.shape[0] // W
            out_splits = [n] * W
        self._sync()
        self.g._slots[self.rank] = (inp, list(in_splits))
        self._sync()
        off = 0
        for src in range(W):
            t, splits = self.g._slots[src]
            s0 = sum(splits[:self.rank])
            cnt = splits[self.rank]
            assert cnt == out_splits[src], "loopback all_to_all split mismatch"
            out[off:off + cnt].copy_(t[s0:s0 + cnt])
            off += cnt
        self._sync()

    def all_reduce(self, t, op="sum"):
        self._sync()
        self.g._slots[self.rank] = t.clone()
        self._sync()
        acc = self.g._slots[0].clone()
        for r in range(1, self.world):
            x = self.g._slots[r]
            if op == "sum":
                acc += x
            elif op == "max":
                acc = torch.maximum(acc, x)
            else:
                acc = torch.minimum(acc, x)
        self._sync()
        t.copy_(acc)

    def barrier(self):
        self._sync()

    @property
    def backend(self) -> str:
        return "loopback"


def run_ranks(world: int, fn):
    """Run fn(rank, comm) for W loopback ranks in threads; re-raise errors."""
    grp = LoopbackGroup(world)
    errs: List[BaseException] = []
    outs = [None] * world

    def body(r):
        try:
            outs[r] = fn(r, grp.comm(r))
        except BaseException as e:  # pragma: no cover
            errs.append(e)
            grp._barrier.abort()

    th = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errs:
        raise errs[0]
    return outs


# ------------------------------------------------------------------ dense IPC meshes per group
# A training session that set up a self-tested IPC mesh for its process group
# (fluid Session, runtime.ctr_step) registers it here; the in-step sums of
# that group -- c_allreduce_sum, data_norm sync_stats, the dense gradient
# all-reduce -- then run as one IPC collective kernel instead of an RCCL call.
_GROUP_MESH = {}


def _gkey(group):
    if group is None or (dist.is_available() and group is dist.group.WORLD):
        return None  # the default group under either name
    return id(group)


def register_group_mesh(group, mesh) -> None:
    if mesh is None:
        _GROUP_MESH.pop(_gkey(group), None)
    else:
        _GROUP_MESH[_gkey(group)] = mesh


def group_mesh(group=None):
    return _GROUP_MESH.get(_gkey(group))


def allreduce_sum(t, group=None) -> str:
    """In-place sum of ``t`` over ``group``: the group's IPC mesh when one is
    registered and ``t`` is a contiguous fp32 GPU tensor that fits its slot,
    else torch.distributed.  Returns the transport used ("ipc" / "dist")."""
    m = group_mesh(group)
    if m is not None and t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() and \
            t.numel() * 4 <= m.slot_bytes:
        m.allreduce_(t)
        return "ipc"
    dist.all_reduce(t, group=group)
    return "dist"
