"""DCN-V2 (parallel form) on the PaddleBox sparse stack (BASELINE config 5).

    pull_box_sparse -> fused_seqpool_cvm   one HIP kernel, [pooled | dense]
    x0 = data_norm(x)                      fused head kernel (FM off), bf16,
                                           written into the MLP workspace
    cross:  x_{l+1} = x0 * (W_l x_l + b_l) + x_l      L full-rank layers,
            fp32 state, bf16 MFMA GEMMs with the cross update fused in
            the epilogue (CrossWorkspace, csrc/hip/bindings_cross.cpp)
    deep:   FusedMLP hidden -> 1           MFMA GEMMs, bias+ReLU fused
    logit = deep + w_c . x_L  -> fused sigmoid + logloss

(The parallel DCN-V2 head ``[x_L, h_deep] . w`` is split into the deep
MLP's own output layer plus ``w_c . x_L``.)  Sparse features are updated by
the fused push + sparse Adagrad in the pull's backward, dense parameters by
one fused Adam over the arena.
"""
from __future__ import annotations

from typing import Sequence

import os

import torch
from torch import nn

from .. import _native
from ..ops.ctr import DataNorm, ctr_head, logit_logloss
from ..ops.mlp import FusedMLP, _ensure_grad, pad8
from ..ops.tower import CtrTower
from ..ops.sparse import prefetch_pool_seqpool_cvm_concat, prefetch_seqpool_cvm_concat, pull_seqpool_cvm_concat
from ..ps.sparse_engine import SeqpoolParams, SparseEngine


class _CrossHipFn(torch.autograd.Function):
    """s = x_L . w_c over the cross stack on the GPU.  x0 / x0^T are the MLP
    workspace's bf16 input buffers (X_0 [M, pad64(D)], X_0^T with the ones
    row); parameter gradients accumulate straight into ``p.grad`` (dense-arena
    views); returns d(loss)/d(x0) as bf16 [M, pad64(D)]."""

    @staticmethod
    def forward(ctx, y, yt, mod, w_c, *params):
        xw = mod.workspace(y)
        s = xw.forward(y, [w.detach() for w in mod.w], [b.detach() for b in mod.b], w_c.detach())
        ctx.mod, ctx.y, ctx.yt, ctx.w_c = mod, y, yt, w_c
        ctx.n_params = len(params)
        return s

    @staticmethod
    def backward(ctx, ds):
        mod = ctx.mod
        dy = mod._xw.backward(ctx.y, ctx.yt, ds.float().contiguous(), [_ensure_grad(w) for w in mod.w],
                              [_ensure_grad(b) for b in mod.b], ctx.w_c.detach(), _ensure_grad(ctx.w_c))
        return (dy, None, None, None) + (None,) * ctx.n_params


def cross_logit(y: torch.Tensor, cross: "CrossNetV2", w_c: torch.Tensor,
                yt: torch.Tensor = None) -> torch.Tensor:
    """[M] = CrossNetV2(y[:, :D]) . w_c.  GPU: y / yt are the MLP workspace's
    bf16 X_0 / X_0^T (the HIP cross stack); CPU: fp32 torch."""
    D = w_c.numel()
    if y.is_cuda:
        return _CrossHipFn.apply(y, yt, cross, w_c, *cross.parameters(), w_c)
    yy = y[:, :D].float()
    if yy.shape[1] < D:  # the cross width is the padded tower width
        yy = torch.nn.functional.pad(yy, (0, D - yy.shape[1]))
    return cross(yy) @ w_c


class CrossNetV2(nn.Module):
    """``dim`` (a multiple of 8 on the GPU) is the padded MLP input width;
    features >= ``valid`` are zero padding (their weights start at zero and
    receive zero gradients)."""

    def __init__(self, dim: int, layers: int = 3, valid: int = None):
        super().__init__()
        self.dim = dim
        self._xw = None
        self.w = nn.ParameterList()
        self.b = nn.ParameterList()
        for _ in range(layers):
            v = valid or dim
            w = torch.zeros(dim, dim)
            nn.init.xavier_uniform_(w[:v, :v])
            self.w.append(nn.Parameter(w * 0.1))
            self.b.append(nn.Parameter(torch.zeros(dim)))

    def workspace(self, y: torch.Tensor):
        M, ld = int(y.shape[0]), int(y.shape[1])
        if self._xw is None or self._xw_key != (M, ld, y.device):
            # batch rows per split-K slice of the dW GEMMs (PBX_CROSS_KSPLIT, multiple of 64)
            ks = int(os.environ.get("PBX_CROSS_KSPLIT", "1024"))
            self._xw = _native.hip().CrossWorkspace(M, self.dim, len(self.w), y.device.index or 0, ks)
            self._xw_key = (M, ld, y.device)
            self._xw.set_pack_by_optimizer(self.packed_by_optimizer)
        return self._xw

    # The fused Adam (parallel/dense.py FlatAdam.fuse) re-packs the bf16 copies
    # of the cross weights after each update, as it does the tower's, instead
    # of a k_cross_pack launch in every forward (the FusedMLP interface).
    @property
    def packed_by_optimizer(self) -> bool:
        return bool(self.__dict__.get("_pack_by_opt", False))

    @packed_by_optimizer.setter
    def packed_by_optimizer(self, v: bool):
        self.__dict__["_pack_by_opt"] = bool(v)
        if self._xw is not None:
            self._xw.set_pack_by_optimizer(bool(v))

    def invalidate_pack(self):
        if self._xw is not None:
            self._xw.invalidate_pack()

    def tower_workspaces(self):
        return [self._xw] if self._xw is not None else []

    def forward(self, x0: torch.Tensor) -> torch.Tensor:
        """fp32 reference stack (CPU path and the GPU kernels' oracle)."""
        x = x0
        for w, b in zip(self.w, self.b):
            x = x0 * torch.nn.functional.linear(x, w, b) + x
        return x


class DCNv2(nn.Module):
    def __init__(self, engine: SparseEngine, num_slots: int = 26, dense_dim: int = 13, cross_layers: int = 3,
                 hidden: Sequence[int] = (512, 256), use_data_norm: bool = True, seqpool: SeqpoolParams = None,
                 fused_tower: bool = True):
        super().__init__()
        self.engine = engine
        self.S = num_slots
        self.Dd = dense_dim
        self.sp = seqpool or SeqpoolParams(use_cvm=True, cvm_offset=2)
        self.Eo = self.sp.out_width(engine.E)
        C = self.S * self.Eo + dense_dim
        self.C = C
        self.Cp = pad8(C)
        self.dn = DataNorm(C) if use_data_norm else None
        self.mlp = FusedMLP(C, hidden, 1)
        self.ew_col = 2 if self.sp.use_cvm and not self.sp.clk_filter else (1 if self.sp.use_cvm else 0)
        # the cross stack runs inside the fused tower (csrc/hip/tower.hip
        # head + MLP, cross GEMMs on the normalised input the head writes)
        # when the tower's padded input width is a whole number of 64-wide
        # GEMM k-tiles; otherwise beside the MLP workspace
        k0 = (self.mlp.in_dim + 31) // 32 * 32
        self.use_tower = fused_tower and k0 % 64 == 0 and len(self.mlp.hidden) <= 8
        D = k0 if self.use_tower else self.Cp
        self.cross = CrossNetV2(D, cross_layers, valid=C)
        self.w_c = nn.Parameter(torch.zeros(D))
        self.tower = CtrTower(self.mlp, self.dn, self.S, self.Eo, self.ew_col, 0, use_head_lin=False,
                              cross=(self.cross, self.w_c)) if self.use_tower else None

    def prefetch(self, batch, slot: int) -> bool:
        """Pool the NEXT batch now (after this step's sparse push), so its
        step starts at the data_norm head (ops/sparse.py)."""
        return prefetch_seqpool_cvm_concat(self.engine, batch.keys, batch.lod, batch.B, batch.S, batch.dense, self.sp,
                                           slot)

    def prefetch_pool(self, batch, slot: int) -> bool:
        """The pooling half of prefetch (its dedup issued earlier: engine.prefetch_dedup)."""
        return prefetch_pool_seqpool_cvm_concat(self.engine, batch.keys, batch.lod, batch.B, batch.S, batch.dense,
                                                self.sp, slot)

    def forward(self, batch):
        B, S = batch.B, batch.S
        x = pull_seqpool_cvm_concat(self.engine, batch.keys, batch.lod, B, S, batch.cvm, batch.dense, self.sp)
        if x.is_cuda and self.tower is not None:
            return self.tower(x, batch.label)
        if x.is_cuda:
            ws = self.mlp.workspace(B, x.device)
            y, _ = ctr_head(x, self.dn, S, self.Eo, self.ew_col, 0, self.Cp, ws.x(0), ws.xt(0))
            deep = self.mlp.forward_ws(y)
            cross = cross_logit(y, self.cross, self.w_c, ws.xt(0))
        else:
            y, _ = ctr_head(x, self.dn, S, self.Eo, self.ew_col, 0, self.Cp)
            deep = self.mlp(y)
            cross = cross_logit(y, self.cross, self.w_c)
        return logit_logloss(deep, cross, batch.label)
