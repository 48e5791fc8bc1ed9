"""DeepFM on the PaddleBox sparse stack (headline benchmark model).

Graph (PaddleBox canonical CTR graph, SURVEY Appendix B, with the FM term):

    pull_box_sparse -> fused_seqpool_cvm  (one fused HIP kernel, written
                                           straight into the concat buffer)
    concat(pooled[S*11], dense[13])       (free: same buffer)
    first order  = sum_s embed_w(s)       (pulled embed_w column)
    second order = FM over embedx[8]      (HIP kernel)
    deep         = data_norm -> MLP 400-400-400 -> 1 (bf16 MFMA GEMMs)
    logit = first + second + deep -> fused sigmoid + logloss (HIP kernel)

The embedding update happens in the backward of the pull (push_box_sparse with
fused sparse Adagrad); dense params use one flat arena + fused Adam.
"""
from __future__ import annotations

from typing import Sequence

import torch
from torch import nn

from ..ops.ctr import DataNorm, fm_interaction, sigmoid_logloss
from ..ops.sparse import pull_seqpool_cvm_concat
from ..ps.sparse_engine import SeqpoolParams, SparseEngine


class MLP(nn.Module):
    def __init__(self, in_dim: int, hidden: Sequence[int], out_dim: int = 1, compute_dtype=torch.bfloat16):
        super().__init__()
        dims = [in_dim] + list(hidden)
        self.layers = nn.ModuleList(nn.Linear(a, b) for a, b in zip(dims[:-1], dims[1:]))
        self.out = nn.Linear(dims[-1], out_dim)
        self.compute_dtype = compute_dtype
        for l in list(self.layers) + [self.out]:
            nn.init.xavier_uniform_(l.weight)
            nn.init.zeros_(l.bias)

    def forward(self, x):
        if x.is_cuda and self.compute_dtype != torch.float32:
            with torch.autocast("cuda", dtype=self.compute_dtype):
                for l in self.layers:
                    x = torch.relu(l(x))
                return self.out(x).float()
        for l in self.layers:
            x = torch.relu(l(x))
        return self.out(x)


class DeepFM(nn.Module):
    def __init__(self, engine: SparseEngine, num_slots: int = 26, dense_dim: int = 13,
                 hidden: Sequence[int] = (400, 400, 400), use_data_norm: bool = True,
                 compute_dtype=torch.bfloat16, seqpool: SeqpoolParams = None):
        super().__init__()
        self.engine = engine
        self.S = num_slots
        self.Dd = dense_dim
        self.sp = seqpool or SeqpoolParams(use_cvm=True, cvm_offset=2)
        self.Eo = self.sp.out_width(engine.E)
        self.D = engine.dim
        C = self.S * self.Eo + dense_dim
        self.in_dim = C
        self.dn = DataNorm(C) if use_data_norm else None
        self.mlp = MLP(C, hidden, 1, compute_dtype)
        self.bias = nn.Parameter(torch.zeros(1))
        # column of embed_w / first embedx inside each slot block
        self.ew_col = 2 if self.sp.use_cvm and not self.sp.clk_filter else (1 if self.sp.use_cvm else 0)

    def forward(self, batch):
        B, S = batch.B, batch.S
        x = pull_seqpool_cvm_concat(self.engine, batch.keys, batch.lod, B, S, batch.cvm, batch.dense, self.sp)
        first = x[:, self.ew_col:S * self.Eo:self.Eo].sum(1)
        second = fm_interaction(x, S, self.D, self.ew_col + 1, self.Eo)
        h = self.dn(x) if self.dn is not None else x
        deep = self.mlp(h).view(-1)
        logit = deep + first + second + self.bias
        loss, pred = sigmoid_logloss(logit, batch.label)
        return loss, pred
