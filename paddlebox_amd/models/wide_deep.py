"""Wide&Deep on the PaddleBox sparse stack (BASELINE configs 1 and 4).

    pull_box_sparse -> fused_seqpool_cvm      one HIP kernel, [pooled | dense]
    ctr_head (FM disabled)                    wide  = sum_s embed_w(s) (the LR
                                              part lives in the 1-d embed_w of
                                              every feature, updated by sparse
                                              Adagrad in the push)
                                              deep input = data_norm(x), bf16
    deep = FusedMLP hidden -> 1               MFMA GEMMs, bias+ReLU fused
    logit = wide + deep -> fused sigmoid + logloss

Same engine and kernels as DeepFM with the second-order term switched off
(``D = 0`` in the head kernel).
"""
from __future__ import annotations

from typing import Sequence

import torch
from torch import nn

from ..ops.ctr import DataNorm, ctr_head, logit_logloss
from ..ops.mlp import FusedMLP, pad8
from ..ops.sparse import pull_seqpool_cvm_concat
from ..ops.tower import CtrTower
from ..ps.sparse_engine import SeqpoolParams, SparseEngine


class WideDeep(nn.Module):
    def __init__(self, engine: SparseEngine, num_slots: int = 26, dense_dim: int = 13,
                 hidden: Sequence[int] = (512, 256, 128), use_data_norm: bool = True,
                 seqpool: SeqpoolParams = None):
        super().__init__()
        self.engine = engine
        self.S = num_slots
        self.Dd = dense_dim
        self.sp = seqpool or SeqpoolParams(use_cvm=True, cvm_offset=2)
        self.Eo = self.sp.out_width(engine.E)
        C = self.S * self.Eo + dense_dim
        self.in_dim = C
        self.Cp = pad8(C)
        self.dn = DataNorm(C) if use_data_norm else None
        self.mlp = FusedMLP(C, hidden, 1)
        self.ew_col = 2 if self.sp.use_cvm and not self.sp.clk_filter else (1 if self.sp.use_cvm else 0)
        self.tower = CtrTower(self.mlp, self.dn, self.S, self.Eo, self.ew_col, 0, use_head_lin=True)
        self.use_tower = True

    def forward(self, batch):
        B, S = batch.B, batch.S
        x = pull_seqpool_cvm_concat(self.engine, batch.keys, batch.lod, B, S, batch.cvm, batch.dense, self.sp)
        if self.use_tower or not x.is_cuda:
            return self.tower(x, batch.label)
        if x.is_cuda:
            ws = self.mlp.workspace(B, x.device)
            y, wide = ctr_head(x, self.dn, S, self.Eo, self.ew_col, 0, self.Cp, ws.x(0), ws.xt(0))
            deep = self.mlp.forward_ws(y)
        else:
            y, wide = ctr_head(x, self.dn, S, self.Eo, self.ew_col, 0, self.Cp)
            deep = self.mlp(y)
        return logit_logloss(deep, wide, batch.label)
