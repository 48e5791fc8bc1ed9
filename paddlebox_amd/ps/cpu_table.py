"""CPU sparse table: the in-process CPU parameter server (BASELINE config 1).

Backed by the native C++ table in ``_pbx_host`` (csrc/host/cpu_ps.cc) when it
is built, with identical semantics to the GPU table: same row layout
(csrc/common/pbx_common.h), same Adagrad rule.  The reference's CPU "device"
mode of BoxWrapper (``box_wrapper_impl.h:236-342,524-595``,
``box_wrapper_impl.cc:28-188``) is the behaviour reproduced.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from .. import _native
from .config import ShrinkConfig, SparseSGDConfig, row_layout
from ..ops import reference as ref


class CpuSparseTable:
    """Mixed-key -> value-row store on the host."""

    def __init__(self, dim: int, capacity: int = 0, nshards: int = 16):
        self.dim = dim
        self.layout = row_layout(dim)
        self.stride = self.layout["stride"]
        self.device = torch.device("cpu")
        self._native = None
        if _native.host_available():
            self._native = _native.host().CpuTable(dim, nshards)
        else:
            # pure-torch fallback store (sorted keys + value matrix)
            self._keys = torch.empty(0, dtype=torch.int64)
            self._vals = torch.empty(0, self.stride, dtype=torch.float32)
        self._seed = 0x5EED

    # rows are indices into an internal value matrix; -1 = missing
    def probe(self, h: torch.Tensor, n_dev=None) -> torch.Tensor:
        if self._native is not None:
            return self._native.probe(h.contiguous())
        if self._keys.numel() == 0:
            return torch.full((h.numel(),), -1, dtype=torch.int64)
        pos = torch.searchsorted(self._keys, h).clamp(max=self._keys.numel() - 1)
        hit = self._keys[pos] == h
        return torch.where(hit, pos, torch.full_like(pos, -1))

    def insert_mixed(self, h: torch.Tensor, sgd: SparseSGDConfig, init_embedx: bool = False, n_dev=None) -> int:
        h = h[h != -1]
        if h.numel() == 0:
            return 0
        self._seed += 1
        if self._native is not None:
            self._native.insert(h.contiguous(), sgd.initial_range, sgd.mf_initial_range, int(init_embedx), self._seed)
            return 0
        rows = self.probe(h)
        new = torch.unique(h[rows < 0])
        if new.numel() == 0:
            return 0
        v = torch.zeros(new.numel(), self.stride)
        if sgd.initial_range > 0:
            v[:, 2] = (torch.rand(new.numel()) * 2 - 1) * sgd.initial_range
        if init_embedx:
            v[:, 3:3 + self.dim] = torch.rand(new.numel(), self.dim) * sgd.mf_initial_range
            v[:, self.layout["mf_size"]] = 1
        keys = torch.cat([self._keys, new])
        vals = torch.cat([self._vals, v])
        order = torch.argsort(keys)
        self._keys, self._vals = keys[order], vals[order]
        return 0

    def gather_pull(self, rows: torch.Tensor, out_stride: int) -> torch.Tensor:
        P = 3 + self.dim
        out = torch.zeros(rows.numel(), out_stride)
        ok = rows >= 0
        if self._native is not None:
            full = self._native.gather(rows.contiguous())
        else:
            full = torch.zeros(rows.numel(), self.stride)
            full[ok] = self._vals[rows[ok]]
        out[:, :P] = full[:, :P]
        out[~ok] = 0
        return out

    def push_adagrad(self, rows: torch.Tensor, push: torch.Tensor, sgd: SparseSGDConfig):
        ok = rows >= 0
        if not bool(ok.any()):
            return
        if self._native is not None:
            self._native.push_adagrad(rows.contiguous(), push.contiguous().float(), _cfg_list(sgd))
            return
        r = rows[ok]
        self._vals[r] = ref.adagrad_update(self._vals[r], push[ok], self.dim, sgd)

    def size(self) -> int:
        if self._native is not None:
            return int(self._native.size())
        return int(self._keys.numel())

    @property
    def capacity(self) -> int:
        return self.size()

    def export(self, with_values: bool = True) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
        if self._native is not None:
            k, v = self._native.export_all()
            return k, (v if with_values else None)
        return self._keys.clone(), (self._vals.clone() if with_values else None)

    def assign(self, h: torch.Tensor, vals: torch.Tensor):
        rows = self.probe(h)
        ok = rows >= 0
        if self._native is not None:
            self._native.assign(rows.contiguous(), vals.contiguous().float())
            return
        self._vals[rows[ok]] = vals[ok].float()[:, : self.stride]

    def read(self, h: torch.Tensor) -> torch.Tensor:
        rows = self.probe(h)
        if self._native is not None:
            return self._native.gather(rows.contiguous())
        out = torch.zeros(h.numel(), self.stride)
        ok = rows >= 0
        out[ok] = self._vals[rows[ok]]
        return out

    def shrink(self, cfg: ShrinkConfig) -> int:
        if self._native is not None:
            return int(self._native.shrink(cfg.show_click_decay_rate, cfg.delete_threshold,
                                           cfg.delete_after_unseen_days, cfg.nonclk_coeff, cfg.clk_coeff))
        l = self.layout
        v = self._vals
        v[:, 0] *= cfg.show_click_decay_rate
        v[:, 1] *= cfg.show_click_decay_rate
        v[:, l["unseen_days"]] += 1
        score = (v[:, 0] - v[:, 1]) * cfg.nonclk_coeff + v[:, 1] * cfg.clk_coeff
        keep = (score >= cfg.delete_threshold) & (v[:, l["unseen_days"]] <= cfg.delete_after_unseen_days)
        deleted = int((~keep).sum())
        self._keys, self._vals = self._keys[keep], v[keep]
        return deleted

    def clear(self):
        if self._native is not None:
            self._native.clear()
        else:
            self._keys = torch.empty(0, dtype=torch.int64)
            self._vals = torch.empty(0, self.stride, dtype=torch.float32)

    def select_for_save(self, mode: int, f) -> Tuple[torch.Tensor, torch.Tensor]:
        """Native xbox filter (mode 0 base, 1 delta, 2 all); resets delta."""
        return self._native.select_for_save(mode, f)

    def memory_bytes(self) -> int:
        return self.size() * (8 + 4 * self.stride)


def _cfg_list(c: SparseSGDConfig):
    return [c.nonclk_coeff, c.clk_coeff, c.min_bound, c.max_bound, c.learning_rate, c.initial_g2sum,
            c.initial_range, c.mf_create_thresholds, c.mf_learning_rate, c.mf_initial_g2sum, c.mf_initial_range,
            c.mf_min_bound, c.mf_max_bound, c.nodeid_slot, c.feature_learning_rate, float(c.use_feature_lr)]
