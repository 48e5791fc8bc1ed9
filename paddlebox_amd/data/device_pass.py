"""Device-resident pass data: the in-memory dataset's record store in HBM and
on-device batch assembly (``csrc/hip/batch_ops.hip``).

The reference assembles every minibatch on CPU threads (``data_feed.cc``
PackBatchTask / ``MiniBatchGpuPack``: per-slot offset scans and key copies,
then one H2D per batch) and keeps the pass in host memory.  An MI355X has
288 GB of HBM: a pass's columnar store (``SlotDataset``'s CSR arrays, ~16 B
per key) fits next to the embedding table, so it is copied once and each
batch is produced by two kernels writing straight into the captured step's
input buffers -- no host work, no per-batch H2D, and the trainer's host loop
is reduced to a launch + a graph replay.  (Measured on one MI355X: host
assembly of a 8192 x 26-slot batch costs 0.44 ms on 8 threads, more than the
whole GPU step.)

The copy is keyed on the native store version (any load / add / shuffle of
records bumps it); the pass order is re-uploaded per training call (it
changes with every local shuffle).  A pass larger than
``padbox_device_pass_max_gb`` (default 64) stays on the host path.
"""
from __future__ import annotations

from typing import Optional

import torch

from .. import _native
from ..utils import flags as _flags


class DevicePass:
    def __init__(self, nat, device):
        self.nat = nat
        self.device = torch.device(device)
        self.version = int(nat.version())
        self.nrec = int(nat.size())
        self.nu = int(nat.num_u64_slots())
        self.nf = int(nat.num_f32_slots())
        self.S = int(nat.num_sparse_slots())
        self.Dw = int(nat.dense_width())
        self.u64, self.uoff, self.f32, self.foff = nat.store_to(str(self.device))
        self.sparse_idx = torch.tensor(list(nat.sparse_slot_u64_index()), dtype=torch.int32, device=self.device)
        self.drefs = nat.dense_refs().to(self.device).contiguous()
        self.order: Optional[torch.Tensor] = None
        self.tot = torch.zeros(max(1, self.S), dtype=torch.int64, device=self.device)
        self.overflow = torch.zeros(1, dtype=torch.int32, device=self.device)
        # every assembly runs on this stream: the slot-total scratch is shared
        self.stream = torch.cuda.Stream(self.device)

    @staticmethod
    def bytes_needed(nat) -> int:
        st_u = int(nat.num_u64_slots())
        st_f = int(nat.num_f32_slots())
        n = int(nat.size())
        # offsets (8 B per record-slot) + values (batch_len of the whole
        # store counts the sparse keys; dense values are a fraction of that)
        return 16 * n * (st_u + st_f) + 8 * int(nat.batch_len(0, n)) if n else 0

    def set_order(self, order: torch.Tensor):
        o = order.to(torch.int64)
        if o.numel() and (int(o.min()) < 0 or int(o.max()) >= self.nrec):
            raise ValueError("DevicePass: pass order refers to records outside the store")
        self.order = o.to(self.device, non_blocking=False).contiguous()

    def assemble(self, begin: int, count: int, keys: torch.Tensor, lod: torch.Tensor, dense: torch.Tensor):
        """Enqueue the build of batch order[begin:begin+count] into device
        buffers on the current stream (callers run it on ``self.stream``):
        keys padded with -1 to ``keys.numel()``."""
        if self.order is None:
            raise RuntimeError("DevicePass.assemble before set_order")
        dense_arg = dense if dense.numel() else torch.empty(0, dtype=torch.float32, device=self.device)
        _native.hip().batch_assemble(self.u64, self.uoff, self.f32, self.foff, self.order, self.sparse_idx,
                                     self.drefs, self.nu, self.nf, self.Dw, self.nrec, begin, count, lod, self.tot,
                                     keys, dense_arg, self.overflow)

    def assemble_sync(self, begin: int, count: int, keys, lod, dense):
        """Assemble on the pass stream, ordered after and before the current
        stream's work (buffers allocated on the current stream)."""
        cur = torch.cuda.current_stream(self.device)
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            self.assemble(begin, count, keys, lod, dense)
        cur.wait_stream(self.stream)

    def overflowed(self) -> bool:
        return bool(int(self.overflow.item()))


def device_pass_for(dataset, device) -> Optional[DevicePass]:
    """The dataset's device copy (created / refreshed as needed), or None when
    the pass does not fit the configured budget or is disabled."""
    nat = dataset._native
    dev = torch.device(device)
    if dev.type != "cuda" or not _flags.get_bool("padbox_device_pass"):
        return None
    cur = getattr(dataset, "_device_pass", None)
    if cur is not None and cur.version == int(nat.version()) and cur.device == dev:
        dp = cur
    else:
        dataset._device_pass = None
        limit = float(_flags.get("padbox_device_pass_max_gb")) * (1 << 30)
        if DevicePass.bytes_needed(nat) > limit:
            return None
        dp = DevicePass(nat, dev)
        dataset._device_pass = dp
    dp.set_order(nat.order())
    return dp
