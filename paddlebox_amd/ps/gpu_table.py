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
    """``codec`` (ps/feature_types.FeatureCodec) selects a non-default row
    layout: the native table then stores ``codec.storage_dim`` embedding words
    plus the codec state, and ``export`` / ``assign`` / ``read`` speak the
    canonical fp32 layout ``row_layout(D + De)`` (+ codec state)."""

    def __init__(self, dim: int, capacity: int, device: torch.device, stash_cap: int = 4096,
                 load_factor: float = 0.85, codec=None):
        self.codec = codec
        self.dim = codec.DX if codec is not None else dim
        self.device = torch.device(device)
        self.load_factor = load_factor
        self.stash_cap = stash_cap
        slots = int(math.ceil(max(capacity, 16) / load_factor))
        self._mod = _native.hip()
        with torch.cuda.device(self.device):
            if codec is None:
                self.t = self._mod.GpuTable(dim, slots, stash_cap, self.device.index or 0)
            else:
                self.t = self._mod.GpuTable(codec.storage_dim, slots, stash_cap, self.device.index or 0, codec.extra)
                assert int(self.t.stride) == codec.raw_stride
        self.layout = row_layout(self.dim)
        self._seed = 0x5EED

    @staticmethod
    def like(other: "GpuSparseTable") -> "GpuSparseTable":
        """An empty table with exactly the geometry of ``other`` (same bucket
        count, stash and row stride), so whole-table copies between them are
        plain device copies."""
        slots = int(other.t.capacity)
        t = GpuSparseTable(other.dim, int(slots * other.load_factor), other.device, other.stash_cap,
                           other.load_factor, other.codec)
        if int(t.t.capacity) != slots:
            raise RuntimeError("GpuSparseTable.like: geometry mismatch")
        return t

    # -- build ------------------------------------------------------------
    def insert_mixed(self, h: torch.Tensor, sgd: SparseSGDConfig, init_embedx: bool = False,
                     n_dev: Optional[torch.Tensor] = None) -> int:
        """Insert unique mixed keys not yet present.  Returns #unplaceable keys."""
        if h.numel() == 0:
            return 0
        self._seed += 1
        if self.codec is not None:
            # the insert zeroes new rows; the codec then writes its state (and
            # the encoded embedding when init_embedx) into exactly those rows
            if n_dev is not None:  # build phase: a host sync is fine here
                h, n_dev = h[:int(n_dev.reshape(-1)[0].item())], None
            h = h.contiguous()
            new = h[self.t.probe(h, None) < 0]
            fails = self.t.insert(h, None, sgd.to_native(self._mod), self._seed, False)
            if new.numel():
                new = new.contiguous()
                rows = self.t.probe(new, None)
                self.t.codec_init(self.codec.native(), rows, new, sgd.to_native(self._mod), self._seed, init_embedx)
        else:
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

    @property
    def rows(self) -> int:
        """Value rows (slots + stash): the index space of a table row."""
        return int(self.t.values.shape[0])

    def export(self, with_values: bool = True) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
        k, v = self.t.export_all(with_values)
        if with_values and self.codec is not None:
            v = self.codec.decode(v)
        return k, (v if with_values else None)

    def assign(self, h: torch.Tensor, vals: torch.Tensor):
        rows = self.probe(h)
        vals = vals.contiguous().float()
        if self.codec is not None:
            vals = self.codec.encode(vals)
        self.t.assign(rows, vals)

    def read(self, h: torch.Tensor) -> torch.Tensor:
        rows = self.probe(h)
        ok = rows >= 0
        if self.codec is not None:
            out = torch.zeros(h.numel(), self.codec.canon_width, device=self.device)
            out[ok] = self.codec.decode(self.t.values[rows[ok]])
            return out
        out = torch.zeros(h.numel(), self.layout["stride"], device=self.device)
        out[ok] = self.t.values[rows[ok]]
        return out

    def clear(self):
        self.t.clear()

    def shrink(self, cfg: ShrinkConfig) -> int:
        return int(self.t.shrink(cfg.to_native(self._mod)))

    def memory_bytes(self) -> int:
        t = self.t
        return t.keys.numel() * 8 + t.values.numel() * 4 + t.fill.numel() * 4
