"""Sparse feature types of the GPU parameter server.

BoxPS selects a value layout per model (``InitializeGPUAndLoadModel(...,
feature_type, pull_embedx_scale)``, reference box_wrapper.h:650-680): plain
fp32 embedx, int16-quantised embedx read as ``q * pull_embedx_scale``
(``EmbedxQuantOp``, box_wrapper.cu:37-43), an "expand" block pulled next to
embedx for ``pull_box_extended_sparse`` (NNCross / variable, box_wrapper.cu:
146-322) and the SparseAdam row rule (heter_ps/optimizer.cuh.h:147-330).

Here all of them are one *row codec* (csrc/hip/feature_ops.hip): the table
row keeps the standard head and tail fields, the embedding block is stored
per codec, and codec state (expand g2sum, Adam moments and beta powers)
follows the tail.  ``FeatureCodec`` mirrors the native ``make_codec`` field
arithmetic so the layout is known on the host (checkpoint IO converts to and
from the canonical fp32 layout ``row_layout(D + De)`` + codec state), and
``update_ref`` is the torch oracle the GPU tests compare the kernel with.
"""
from __future__ import annotations

from typing import Optional

import torch

from .config import PSConfig, SparseSGDConfig, row_layout

KIND_FP32, KIND_INT16, KIND_ADAM, KIND_VAR = 0, 1, 2, 3


class FeatureCodec:
    def __init__(self, kind: int, D: int, De: int = 0, qscale: float = 1.0, beta1: float = 0.9,
                 beta2: float = 0.999, eps: float = 1e-8):
        if kind not in (KIND_FP32, KIND_INT16, KIND_ADAM, KIND_VAR):
            raise ValueError(f"feature codec kind {kind}")
        if kind == KIND_VAR and De <= 0:
            raise ValueError("the variable feature type needs expand_embed_dim > 0")
        self.kind, self.D, self.De = int(kind), int(D), int(De)
        self.qscale, self.beta1, self.beta2, self.eps = float(qscale), float(beta1), float(beta2), float(eps)
        q = kind == KIND_INT16
        var = kind == KIND_VAR
        # variable: one block of max(D, De) columns; the row's size field says
        # how many are live (0 before creation, then D or De)
        self.Wx = (D + 1) // 2 if q else (max(D, De) if var else D)
        self.We = (De + 1) // 2 if q else (0 if var else De)
        self.storage_dim = self.Wx + self.We
        sl = row_layout(self.storage_dim)
        self.raw = sl
        used = sl["mf_size"] + 1
        self.eg2 = used
        used += 1 if De > 0 and not var else 0
        self.xsz = used
        used += 1 if var else 0
        self.adam = used
        used += 6 + 2 * (D + De) if kind == KIND_ADAM else 0
        self.extra = used - (sl["mf_size"] + 1)
        self.raw_stride = ((sl["mf_size"] + 1 + self.extra) + 3) & ~3 if self.extra else sl["stride"]
        # canonical (IO) layout: fp32 embedx+expand as one block, then the
        # codec state copied verbatim
        self.DX = max(D, De) if var else D + De
        self.canon = row_layout(self.DX)
        self.canon_width = self.canon["stride"] + self.extra
        self._native = None
        self.device = None  # set by the engine (variable slot bitmap lives there)

    @staticmethod
    def from_config(cfg: PSConfig) -> Optional["FeatureCodec"]:
        """The codec a PSConfig asks for, or None for the default fp32 Adagrad
        layout without expand (served by the engine's fused kernels)."""
        opt = getattr(cfg, "sparse_optimizer", "adagrad")
        kind = KIND_ADAM if opt == "adam" else (KIND_INT16 if cfg.feature_type == 1 else KIND_FP32)
        De = int(cfg.expand_embed_dim or 0)
        if cfg.feature_type == 2 and opt != "adam":
            kind = KIND_VAR
        if kind == KIND_FP32 and De == 0 and not getattr(cfg, "force_codec", False):
            return None
        return FeatureCodec(kind, cfg.embedx_dim, De, cfg.pull_embedx_scale, getattr(cfg, "adam_beta1", 0.9),
                            getattr(cfg, "adam_beta2", 0.999), getattr(cfg, "adam_epsilon", 1e-8))

    def native(self):
        if self._native is None:
            from .. import _native

            self._native = _native.hip().Codec(self.kind, self.D, self.De, self.qscale, self.beta1, self.beta2,
                                               self.eps)
            assert self._native.storage_dim == self.storage_dim and self._native.extra == self.extra
            if self.kind == KIND_VAR:
                self._vslots = None
                self.set_expand_slots([])
        return self._native

    def set_expand_slots(self, slot_ids):
        """Variable feature type: the slot ids whose new features are created
        with De columns (the slots pulled into an expand output)."""
        import torch as _t

        ids = [int(s) for s in slot_ids]
        nbits = max([64] + [s + 1 for s in ids])
        bm = _t.zeros((nbits + 31) // 32, dtype=_t.int64)
        for s in ids:
            bm[s >> 5] |= 1 << (s & 31)
        bm = ((bm + (1 << 31)) % (1 << 32) - (1 << 31)).to(_t.int32)  # two's complement words
        dev = getattr(self, "device", None) or _t.device("cuda", _t.cuda.current_device())
        self._vslots = bm.to(dev)
        self._vslot_ids = sorted(set(ids))
        self.native().set_expand_slots(self._vslots)

    # ------------------------------------------------------------ row IO
    _TAIL = ("embed_g2sum", "embedx_g2sum", "delta_score", "slot", "unseen_days", "mf_size")

    def _emb_raw(self, raw: torch.Tensor):
        """(embedx [n, D], expand [n, De]) fp32 views/copies of raw rows
        (variable: the whole block, and an empty second part)."""
        blk = raw[:, 3:3 + self.storage_dim]
        if self.kind == KIND_VAR:
            return blk, blk[:, :0]
        if self.kind == KIND_INT16:
            q = blk.contiguous().view(torch.int16).float() * self.qscale
            return q[:, :self.D], q[:, 2 * self.Wx:2 * self.Wx + self.De]
        return blk[:, :self.D], blk[:, self.Wx:self.Wx + self.De]

    def decode(self, raw: torch.Tensor) -> torch.Tensor:
        """raw table rows [n, raw_stride] -> canonical [n, canon_width]."""
        n = raw.shape[0]
        out = torch.zeros(n, self.canon_width, dtype=torch.float32, device=raw.device)
        out[:, :3] = raw[:, :3]
        ex, ee = self._emb_raw(raw)
        out[:, 3:3 + ex.shape[1]] = ex
        out[:, 3 + ex.shape[1]:3 + self.DX] = ee
        for f in self._TAIL:
            out[:, self.canon[f]] = raw[:, self.raw[f]]
        if self.extra:
            b = self.raw["mf_size"] + 1
            out[:, self.canon["stride"]:] = raw[:, b:b + self.extra]
        return out

    def save_map(self):
        """Column map of ``decode`` for the native streaming saver
        (csrc/hip/ckpt.hip SaveDecode): per canonical column, the stored float
        column (>= 0), -1 for zero, or -2 - e for int16 element e of the
        embedding block (times qscale)."""
        m = [-1] * self.canon_width
        m[0], m[1], m[2] = 0, 1, 2
        for j in range(self.DX):
            if self.kind == KIND_VAR:
                src = 3 + j
            elif self.kind == KIND_INT16:
                src = -2 - (j if j < self.D else 2 * self.Wx + (j - self.D))
            else:
                src = 3 + j if j < self.D else 3 + self.Wx + (j - self.D)
            m[3 + j] = src
        for f in self._TAIL:
            m[self.canon[f]] = self.raw[f]
        b = self.raw["mf_size"] + 1
        for e in range(self.extra):
            m[self.canon["stride"] + e] = b + e
        return m

    def quantize(self, x: torch.Tensor) -> torch.Tensor:
        return torch.clamp(torch.round(x / self.qscale), -32768, 32767)

    def encode(self, canon: torch.Tensor) -> torch.Tensor:
        """canonical rows -> raw table rows (int16 rounding to nearest)."""
        n = canon.shape[0]
        raw = torch.zeros(n, self.raw_stride, dtype=torch.float32, device=canon.device)
        raw[:, :3] = canon[:, :3]
        ex, ee = canon[:, 3:3 + self.D], canon[:, 3 + self.D:3 + self.DX]
        if self.kind == KIND_VAR:
            raw[:, 3:3 + self.DX] = canon[:, 3:3 + self.DX]
        elif self.kind == KIND_INT16:
            q = torch.zeros(n, 2 * self.storage_dim, dtype=torch.int16, device=canon.device)
            q[:, :self.D] = self.quantize(ex).to(torch.int16)
            q[:, 2 * self.Wx:2 * self.Wx + self.De] = self.quantize(ee).to(torch.int16)
            raw[:, 3:3 + self.storage_dim] = q.view(torch.float32)
        else:
            raw[:, 3:3 + self.D] = ex
            raw[:, 3 + self.Wx:3 + self.Wx + self.De] = ee
        for f in self._TAIL:
            raw[:, self.raw[f]] = canon[:, self.canon[f]]
        if self.extra:
            b = self.raw["mf_size"] + 1
            raw[:, b:b + self.extra] = canon[:, self.canon["stride"]:]
        return raw

    # ------------------------------------------------------------ oracle
    def update_ref(self, canon: torch.Tensor, push: torch.Tensor, cfg: SparseSGDConfig) -> torch.Tensor:
        """Torch oracle of k_codec_update on canonical rows of already-created
        features (mf_size != 0; creation draws device randoms).  push rows:
        [slot, show, click, embed_g, embedx_g[D], expand_g[De]]."""
        c, v = self.canon, canon.clone().float()
        D, DX = self.D, self.DX
        slot, gs, gc = push[:, 0], push[:, 1], push[:, 2]
        v[:, c["slot"]] = slot
        v[:, 0] += gs
        v[:, 1] += gc
        v[:, c["delta_score"]] += cfg.nonclk_coeff * (gs - gc) + cfg.clk_coeff * gc
        v[:, c["unseen_days"]] = 0
        scale = torch.where(gs > 0, gs, torch.ones_like(gs))
        x = v[:, 3:3 + DX]
        gx = push[:, 4:4 + DX] / scale.unsqueeze(1)
        sg = push[:, 3] / scale
        if self.kind == KIND_VAR:
            return self._update_var_ref(v, push, cfg, gs, sg, scale, slot)
        if self.kind == KIND_ADAM:
            st = v[:, c["stride"] + (self.adam - self.raw["mf_size"] - 1):]
            b1, b2 = self.beta1, self.beta2
            ratio = cfg.learning_rate * torch.sqrt(1 - st[:, 3]) / (1 - st[:, 2])
            m = b1 * st[:, 0] + (1 - b1) * sg
            s2 = b2 * st[:, 1] + (1 - b2) * sg * sg
            v[:, 2] = (v[:, 2] + ratio * (m / (torch.sqrt(s2) + self.eps))).clamp(cfg.mf_min_bound, cfg.mf_max_bound)
            st[:, 0], st[:, 1] = m, s2
            st[:, 2] *= b1
            st[:, 3] *= b2
            xm, xv, xp = st[:, 4:4 + DX], st[:, 4 + DX:4 + 2 * DX], st[:, 4 + 2 * DX:6 + 2 * DX]
            ratio = (cfg.learning_rate * torch.sqrt(1 - xp[:, 1]) / (1 - xp[:, 0])).unsqueeze(1)
            m = b1 * xm + (1 - b1) * gx
            s2 = b2 * xv + (1 - b2) * gx * gx
            nx = (x + ratio * (m / (torch.sqrt(s2) + self.eps))).clamp(cfg.mf_min_bound, cfg.mf_max_bound)
            xm.copy_(m)
            xv.copy_(s2)
            xp[:, 0] *= b1
            xp[:, 1] *= b2
            v[:, 3:3 + DX] = nx
            v[:, c["stride"] + (self.adam - self.raw["mf_size"] - 1):] = st
            return v
        lr = torch.full_like(gs, cfg.learning_rate)
        mf_lr = torch.full_like(gs, cfg.mf_learning_rate)
        if cfg.use_feature_lr:
            msk = slot != cfg.nodeid_slot
            lr = torch.where(msk, torch.full_like(lr, cfg.feature_learning_rate), lr)
            mf_lr = torch.where(msk, torch.full_like(lr, cfg.feature_learning_rate), mf_lr)
        g2 = v[:, c["embed_g2sum"]]
        ratio = lr * torch.sqrt(cfg.initial_g2sum / (cfg.initial_g2sum + g2))
        v[:, 2] = (v[:, 2] + sg * ratio).clamp(cfg.min_bound, cfg.max_bound)
        v[:, c["embed_g2sum"]] = g2 + sg * sg
        groups = [(0, D, c["embedx_g2sum"])]
        if self.De:
            groups.append((D, self.De, c["stride"] + (self.eg2 - self.raw["mf_size"] - 1)))
        for j0, nj, gi in groups:
            g2x = v[:, gi]
            rx = (mf_lr * torch.sqrt(cfg.mf_initial_g2sum / (cfg.mf_initial_g2sum + g2x))).unsqueeze(1)
            gg = gx[:, j0:j0 + nj]
            nx = (x[:, j0:j0 + nj] + gg * rx).clamp(cfg.mf_min_bound, cfg.mf_max_bound)
            if self.kind == KIND_INT16:
                nx = self.quantize(nx) * self.qscale
            v[:, 3 + j0:3 + j0 + nj] = nx
            v[:, gi] = g2x + (gg * gg).sum(1) / nj
        return v

    def _update_var_ref(self, v, push, cfg, gs, sg, scale, slot):
        c = self.canon
        lr = torch.full_like(gs, cfg.learning_rate)
        mf_lr = torch.full_like(gs, cfg.mf_learning_rate)
        if cfg.use_feature_lr:
            msk = slot != cfg.nodeid_slot
            lr = torch.where(msk, torch.full_like(lr, cfg.feature_learning_rate), lr)
            mf_lr = torch.where(msk, torch.full_like(lr, cfg.feature_learning_rate), mf_lr)
        g2 = v[:, c["embed_g2sum"]]
        ratio = lr * torch.sqrt(cfg.initial_g2sum / (cfg.initial_g2sum + g2))
        v[:, 2] = (v[:, 2] + sg * ratio).clamp(cfg.min_bound, cfg.max_bound)
        v[:, c["embed_g2sum"]] = g2 + sg * sg
        xs = v[:, c["stride"] + (self.xsz - self.raw["mf_size"] - 1)].long()
        live = torch.arange(self.DX, device=v.device).unsqueeze(0) < xs.unsqueeze(1)
        gx = push[:, 4:4 + self.DX] / scale.unsqueeze(1) * live
        g2x = v[:, c["embedx_g2sum"]]
        rx = (mf_lr * torch.sqrt(cfg.mf_initial_g2sum / (cfg.mf_initial_g2sum + g2x))).unsqueeze(1)
        x = v[:, 3:3 + self.DX]
        nx = torch.where(live, (x + gx * rx).clamp(cfg.mf_min_bound, cfg.mf_max_bound), x)
        v[:, 3:3 + self.DX] = nx
        v[:, c["embedx_g2sum"]] = torch.where(xs > 0, g2x + (gx * gx).sum(1) / xs.clamp(min=1), g2x)
        return v

    def memory_per_row(self) -> int:
        return self.raw_stride * 4

    def __repr__(self) -> str:
        names = {0: "fp32-adagrad", 1: "int16-adagrad", 2: "fp32-adam", 3: "variable-adagrad"}
        return (f"FeatureCodec({names[self.kind]}, D={self.D}, De={self.De}, scale={self.qscale:g}, "
                f"row={self.raw_stride * 4}B)")


def quant_scale_for(bound: float) -> float:
    """A pull_embedx_scale that maps [-bound, bound] onto the int16 range."""
    return float(bound) / 32767.0 if bound > 0 else 1.0


__all__ = ["FeatureCodec", "KIND_FP32", "KIND_INT16", "KIND_ADAM", "KIND_VAR", "quant_scale_for"]
