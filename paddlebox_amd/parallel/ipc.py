"""In-house IPC mesh collectives for the GPUs of one node
(``csrc/hip/ipc.hip``): peer-to-peer writes over xGMI into IPC-mapped inboxes,
one kernel per collective, no host synchronisation, graph-capturable.

* ``allreduce_(t)`` -- one-shot all-reduce: every rank writes its whole
  buffer into every peer's inbox and sums the W copies locally.  For the
  ~2 MB dense arena this is one xGMI hop (7 links in parallel on MI355X)
  instead of a 2(W-1)-step ring, which is latency-bound at that size.
* ``exchange(send)`` -- all-to-all of fixed-size slots (the key / value
  exchange of the sharded sparse step with per-peer capacity): slot p of
  ``send`` lands in peer p's inbox; returns this rank's inbox view
  ``[world, slot_bytes]`` (valid until the second-next collective).

Reference: the c_mixallgather / heter_comm peer copies
(``c_mixallgather_op.cc:221-327``, ``heter_comm_inl.h:273-490``); here the
memory handles are exchanged once over the process group and every later
call is a single kernel.  Every rank must issue the same sequence of
collectives (as with RCCL).  A peer that never arrives makes the wait time
out (``error()`` turns true) instead of hanging the GPU.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from .. import _native


class IpcMesh:
    def __init__(self, slot_bytes: int, group=None, device=None, blocks: int = 32):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        if self.world > 8:
            raise ValueError("IpcMesh spans the GPUs of one node (<= 8 ranks)")
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.slot_bytes = (int(slot_bytes) + 15) // 16 * 16
        h = _native.hip()
        W = self.world
        self.inbox = torch.zeros(2 * W * self.slot_bytes, dtype=torch.uint8, device=self.device)
        self.flags = torch.zeros(W, dtype=torch.int64, device=self.device)
        self.state = torch.zeros(4, dtype=torch.int64, device=self.device)
        self.comm = h.IpcComm(self.rank, W, self.slot_bytes, self.state, int(blocks))
        mine = (h.ipc_handle(self.inbox), h.ipc_handle(self.flags))
        allh = [None] * W
        if W > 1:
            dist.all_gather_object(allh, mine, group=group)
        else:
            allh = [mine]
        self._opened = []
        for p in range(W):
            if p == self.rank:
                self.comm.set_peer(p, self.inbox.data_ptr(), self.flags.data_ptr())
                continue
            (ih, io), (fh, fo) = allh[p]
            ip = h.ipc_open(ih, io)
            fp = h.ipc_open(fh, fo)
            self._opened += [ip - io, fp - fo]
            self.comm.set_peer(p, ip, fp)
        torch.cuda.synchronize(self.device)
        if W > 1:
            dist.barrier(group=group)
        self._calls = 0

    def allreduce_(self, t: torch.Tensor, average: bool = False) -> torch.Tensor:
        """In-place sum (or mean) over the ranks of a contiguous f32 tensor."""
        self.comm.allreduce(t, t, 1.0 / self.world if average else 1.0)
        self._calls += 1
        return t

    def exchange(self, send: torch.Tensor) -> torch.Tensor:
        """send: [world, slot_bytes] (any dtype, contiguous); returns the
        received slots as a uint8 view [world, slot_bytes] of the inbox."""
        self.comm.exchange(send)
        self._calls += 1
        par = self._calls & 1  # epoch e = calls, parity e & 1
        W, sb = self.world, self.slot_bytes
        return self.inbox[par * W * sb:(par + 1) * W * sb].view(W, sb)

    def error(self) -> bool:
        return bool(int(self.state[2].item()) != 0)

    def close(self):
        h = _native.hip()
        torch.cuda.synchronize(self.device)
        for p in self._opened:
            h.ipc_close(p)
        self._opened = []
