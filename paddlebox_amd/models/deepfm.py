"""DeepFM on the PaddleBox sparse stack (headline benchmark model).

Graph (PaddleBox canonical CTR graph, SURVEY Appendix B, plus the FM term):

    pull_box_sparse -> fused_seqpool_cvm   one HIP kernel, written straight
                                           into the [pooled | dense] buffer
    CtrTower (ops/tower.py, csrc/hip/tower.hip), forward = 2 launches:
        k_head_fwd : data_norm(x) -> bf16 MLP input, first order
                     sum_s embed_w(s) + FM over embedx[8]
        k_tower_fwd: MLP 400-400-400 -> 1 on MFMA with activations held in
                     LDS, + (first + FM), sigmoid, logloss, AUC
    backward = k_tower_bwd + k_tower_dw + k_head_bwd

The embedding update happens in the backward of the pull (push_box_sparse
with fused sparse Adagrad); dense params live in one flat arena updated by
one fused Adam launch.
"""
from __future__ import annotations

from typing import Sequence

import torch
from torch import nn

from ..ops.ctr import DataNorm, ctr_head, fm_interaction, logit_logloss
from ..ops.mlp import FusedMLP, pad8
from ..ops.sparse import prefetch_pool_seqpool_cvm_concat, prefetch_seqpool_cvm_concat, pull_seqpool_cvm_concat
from ..ops.tower import CtrTower
from ..ps.sparse_engine import SeqpoolParams, SparseEngine


class _StageWs(torch.autograd.Function):
    """Copy a [B, Cp] bf16 head output into the MLP workspace input (and its
    transpose); gradient = the workspace's dX0 columns."""

    @staticmethod
    def forward(ctx, y, ws, Cp):
        x0 = ws.x(0)
        x0[:, :Cp].copy_(y)
        ws.xt(0)[:Cp, : y.shape[0]].copy_(y.t())
        ctx.Cp = Cp
        return x0.view_as(x0)

    @staticmethod
    def backward(ctx, g):
        return g[:, : ctx.Cp].contiguous(), None, None


class DeepFM(nn.Module):
    def __init__(self, engine: SparseEngine, num_slots: int = 26, dense_dim: int = 13,
                 hidden: Sequence[int] = (400, 400, 400), use_data_norm: bool = True,
                 seqpool: SeqpoolParams = None, compute_dtype=torch.bfloat16):
        super().__init__()
        self.engine = engine
        self.S = num_slots
        self.Dd = dense_dim
        self.sp = seqpool or SeqpoolParams(use_cvm=True, cvm_offset=2)
        self.Eo = self.sp.out_width(engine.E)
        self.D = engine.dim
        C = self.S * self.Eo + dense_dim
        self.in_dim = C
        self.Cp = pad8(C)
        self.dn = DataNorm(C) if use_data_norm else None
        # the global bias is the MLP output layer's bias (b_out)
        self.mlp = FusedMLP(C, hidden, 1)
        self.use_workspace = True
        self.head_into_workspace = True
        # column of embed_w inside each slot block; embedx follow it
        self.ew_col = 2 if self.sp.use_cvm and not self.sp.clk_filter else (1 if self.sp.use_cvm else 0)
        # fused head + MLP + loss (csrc/hip/tower.hip); use_tower=False keeps
        # the per-layer GEMM path (mlp.hip) for comparison
        self.tower = CtrTower(self.mlp, self.dn, self.S, self.Eo, self.ew_col, self.D, use_head_lin=True)
        self.use_tower = True
        # "fp32": the reference's precision (fluid fc = fp32 GEMMs): the
        # exact-fp32 fused tower (tower32.hip, v_mfma_f32_16x16x4_f32); layer
        # widths above its LDS budget fall back to fp32 library GEMMs
        self.precision = "bf16"

    def set_precision(self, precision: str):
        """"bf16", "fp32" (exact fp32 products, tower32.hip) or "fp32x3"
        (fp32 operands as bf16 hi + lo halves, three bf16 MFMA products per
        step, tower_x3.hip: finer than the TF32 math the reference's fp32 fc
        runs on by default, gpu_context.cc:65-67,580-588)."""
        if precision not in ("bf16", "fp32", "fp32x3"):
            raise ValueError(precision)
        x3 = precision == "fp32x3" and self.mlp.tower_x3_ok()
        self.precision = "fp32" if precision == "fp32x3" else precision
        self.tower.x3 = x3
        self.tower.fp32 = self.precision == "fp32" and not x3 and self.mlp.tower_fp32_ok()
        self.mlp.invalidate_pack()

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
        if self.precision == "fp32" and x.is_cuda and not (self.use_tower and (self.tower.fp32 or self.tower.x3)):
            return self._forward_fp32(x, batch.label)
        if self.use_tower or not x.is_cuda:
            return self.tower(x, batch.label)
        if self.use_workspace:
            # the head writes the MLP input (and its transpose) straight into
            # the MLP workspace; the MLP streams it HBM -> LDS by DMA
            ws = self.mlp.workspace(B, x.device)
            if self.head_into_workspace:
                y, lin = ctr_head(x, self.dn, S, self.Eo, self.ew_col, self.D, self.Cp, ws.x(0), ws.xt(0))
            else:
                y0, lin = ctr_head(x, self.dn, S, self.Eo, self.ew_col, self.D, self.Cp)
                y = _StageWs.apply(y0, ws, self.Cp)
            deep = self.mlp.forward_ws(y)
        else:
            y, lin = ctr_head(x, self.dn, S, self.Eo, self.ew_col, self.D, self.Cp)
            deep = self.mlp(y)
        # logit = deep + lin, sigmoid, log-loss and its gradient: one kernel
        loss, pred = logit_logloss(deep, lin, batch.label)
        return loss, pred

    def _forward_fp32(self, x, label):
        y = self.dn(x) if self.dn is not None else x
        lin = x[:, self.ew_col:self.S * self.Eo:self.Eo].sum(1) + fm_interaction(x, self.S, self.D, self.ew_col + 1,
                                                                                 self.Eo)
        deep = self.mlp.forward_fp32(y)
        return logit_logloss(deep, lin, label)
