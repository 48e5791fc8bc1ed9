"""GPU-resident sparse table (one shard per GPU).

Thin Python owner of the native ``GpuTable`` (bucketized two-choice cuckoo
hash, csrc/hip/table.hip).  Keys in the table are ``h = mix64(feasign)``; the
shard a key belongs to is ``owner_of(h, world)`` so every rank holds 1/world of
the feature space (BoxPS shards the feature table across GPUs inside the closed
libbox_ps.so; open analogue ``heter_ps/heter_comm_inl.h:1117-1171``).
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch

from .. import _native
from .config import ShrinkConfig, SparseSGDConfig, row_layout


class GpuSparseTable:
    def __init__(self, dim: int, capacity: int, device: torch.device, stash_cap: int = 4096,
                 load_factor: float = 0.85):
        self.dim = dim
        self.device = torch.device(device)
        self.load_factor = load_factor
        slots = int(math.ceil(max(capacity, 16) / load_factor))
        self._mod = _native.hip()
        with torch.cuda.device(self.device):
            self.t = self._mod.GpuTable(dim, slots, stash_cap, self.device.index or 0)
        self.layout = row_layout(dim)
        self._seed = 0x5EED

    # -- build ------------------------------------------------------------
    def insert_mixed(self, h: torch.Tensor, sgd: SparseSGDConfig, init_embedx: bool = False,
                     n_dev: Optional[torch.Tensor] = None) -> int:
        """Insert unique mixed keys not yet present.  Returns #unplaceable keys."""
        if h.numel() == 0:
            return 0
        self._seed += 1
        fails = self.t.insert(h.contiguous(), n_dev, sgd.to_native(self._mod), self._seed, init_embedx)
        if fails:
            raise RuntimeError(f"GpuSparseTable: {fails} keys could not be placed (table full?)")
        return fails

    def probe(self, h: torch.Tensor, n_dev: Optional[torch.Tensor] = None) -> torch.Tensor:
        return self.t.probe(h, n_dev)

    # -- inspection / IO ---------------------------------------------------
    def size(self) -> int:
        return int(self.t.size())

    @property
    def capacity(self) -> int:
        return int(self.t.capacity)

    @property
    def values(self) -> torch.Tensor:
        return self.t.values

    def export(self, with_values: bool = True) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
        k, v = self.t.export_all(with_values)
        return k, (v if with_values else None)

    def assign(self, h: torch.Tensor, vals: torch.Tensor):
        rows = self.probe(h)
        self.t.assign(rows, vals.contiguous().float())

    def read(self, h: torch.Tensor) -> torch.Tensor:
        rows = self.probe(h)
        out = torch.zeros(h.numel(), self.layout["stride"], device=self.device)
        ok = rows >= 0
        out[ok] = self.t.values[rows[ok]]
        return out

    def clear(self):
        self.t.clear()

    def shrink(self, cfg: ShrinkConfig) -> int:
        return int(self.t.shrink(cfg.to_native(self._mod)))

    def memory_bytes(self) -> int:
        t = self.t
        return t.keys.numel() * 8 + t.values.numel() * 4 + t.fill.numel() * 4
