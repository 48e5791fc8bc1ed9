"""DCN-V2 (parallel form) on the PaddleBox sparse stack (BASELINE config 5).

    pull_box_sparse -> fused_seqpool_cvm   one HIP kernel, [pooled | dense]
    x0 = data_norm(x)                      fused head kernel (FM off), bf16,
                                           written into the MLP workspace
    cross:  x_{l+1} = x0 * (W_l x_l + b_l) + x_l      L full-rank layers,
            fp32 state, bf16 MFMA GEMMs
    deep:   FusedMLP hidden -> 1           MFMA GEMMs, bias+ReLU fused
    logit = deep + w_c . x_L  -> fused sigmoid + logloss

(The parallel DCN-V2 head ``[x_L, h_deep] . w`` is split into the deep
MLP's own output layer plus ``w_c . x_L``.)  Sparse features are updated by
the fused push + sparse Adagrad in the pull's backward, dense parameters by
one fused Adam over the arena.
"""
from __future__ import annotations

from typing import Sequence

import torch
from torch import nn

from ..ops.ctr import DataNorm, ctr_head, logit_logloss
from ..ops.mlp import FusedMLP, pad8
from ..ops.sparse import pull_seqpool_cvm_concat
from ..ps.sparse_engine import SeqpoolParams, SparseEngine


class CrossNetV2(nn.Module):
    def __init__(self, dim: int, layers: int = 3):
        super().__init__()
        self.w = nn.ParameterList()
        self.b = nn.ParameterList()
        for _ in range(layers):
            w = torch.empty(dim, dim)
            nn.init.xavier_uniform_(w)
            self.w.append(nn.Parameter(w * 0.1))
            self.b.append(nn.Parameter(torch.zeros(dim)))

    def forward(self, x0: torch.Tensor) -> torch.Tensor:
        x = x0
        gpu = x0.is_cuda
        for w, b in zip(self.w, self.b):
            if gpu:  # bf16 MFMA GEMM, fp32 accumulate / state
                z = torch.nn.functional.linear(x.to(torch.bfloat16), w.to(torch.bfloat16), b.to(torch.bfloat16))
                z = z.float()
            else:
                z = torch.nn.functional.linear(x, w, b)
            x = x0 * z + x
        return x


class DCNv2(nn.Module):
    def __init__(self, engine: SparseEngine, num_slots: int = 26, dense_dim: int = 13, cross_layers: int = 3,
                 hidden: Sequence[int] = (512, 256), use_data_norm: bool = True, seqpool: SeqpoolParams = None):
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
        self.cross = CrossNetV2(C, cross_layers)
        self.w_c = nn.Parameter(torch.zeros(C))
        self.mlp = FusedMLP(C, hidden, 1)
        self.ew_col = 2 if self.sp.use_cvm and not self.sp.clk_filter else (1 if self.sp.use_cvm else 0)

    def forward(self, batch):
        B, S = batch.B, batch.S
        x = pull_seqpool_cvm_concat(self.engine, batch.keys, batch.lod, B, S, batch.cvm, batch.dense, self.sp)
        if x.is_cuda:
            ws = self.mlp.workspace(B, x.device)
            y, _ = ctr_head(x, self.dn, S, self.Eo, self.ew_col, 0, self.Cp, ws.x(0), ws.xt(0))
            deep = self.mlp.forward_ws(y)
        else:
            y, _ = ctr_head(x, self.dn, S, self.Eo, self.ew_col, 0, self.Cp)
            deep = self.mlp(y)
        xl = self.cross(y[:, : self.C].float())
        return logit_logloss(deep, xl @ self.w_c, batch.label)
