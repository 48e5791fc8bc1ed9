"""Fused MLP on hand-written MFMA GEMMs (csrc/hip/gemm.hip).

Hidden layers ``h = relu(x W^T + b)`` run as one bf16 MFMA GEMM each with the
bias+ReLU epilogue fused; the output layer (1 logit) is a GEMV.  The backward
fuses the ReLU mask into the GEMM operand staging and computes db inside the
dW GEMM (virtual ones column), writing parameter gradients straight into the
dense arena (no per-parameter gradient tensors / add kernels).

CPU tensors use plain fp32 PyTorch (the reference path).
"""
from __future__ import annotations

from typing import List, Sequence

import torch
from torch import nn

from .. import _native


def pad8(n: int) -> int:
    return (n + 7) // 8 * 8


class _FusedMLPFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, mod: "FusedMLP", *params):
        h = _native.hip()
        wb = mod.bf16_weights()
        hs = [x]
        cur = x
        for i, w in enumerate(wb):
            cur = h.linear_fwd(cur, w, mod.b[i], True)
            hs.append(cur)
        out = h.gemv_out(cur, mod.w_out.view(-1), mod.b_out)
        ctx.mod = mod
        ctx.hs = hs
        ctx.wb = wb
        ctx.x_needs_grad = x.requires_grad
        return out

    @staticmethod
    def backward(ctx, dout):
        h = _native.hip()
        mod, hs, wb = ctx.mod, ctx.hs, ctx.wb
        mod.ensure_grads()
        dh = h.gemv_out_bwd(hs[-1], mod.w_out.view(-1), dout.float(), mod.w_out.grad.view(-1), mod.b_out.grad)
        dx = None
        for i in reversed(range(len(wb))):
            need_dx = i > 0 or ctx.x_needs_grad
            dh = h.linear_bwd(dh, hs[i + 1], hs[i], wb[i], mod.w[i].grad, mod.b[i].grad, need_dx, mod.k_split)
        dx = dh if ctx.x_needs_grad else None
        ctx.hs = None
        return (dx, None) + (None,) * (len(mod.w) * 2 + 2)


class FusedMLP(nn.Module):
    def __init__(self, in_dim: int, hidden: Sequence[int], out_dim: int = 1):
        super().__init__()
        if out_dim != 1:
            raise ValueError("FusedMLP output layer is a single logit (CTR)")
        self.in_dim = pad8(in_dim)
        self.hidden = [pad8(h) for h in hidden]
        dims = [self.in_dim] + self.hidden
        self.w = nn.ParameterList()
        self.b = nn.ParameterList()
        for a, b in zip(dims[:-1], dims[1:]):
            w = torch.empty(b, a)
            nn.init.xavier_uniform_(w[:, :in_dim] if a == self.in_dim else w)
            if a == self.in_dim and in_dim < a:
                w[:, in_dim:] = 0
            self.w.append(nn.Parameter(w))
            self.b.append(nn.Parameter(torch.zeros(b)))
        wo = torch.empty(1, dims[-1])
        nn.init.xavier_uniform_(wo)
        self.w_out = nn.Parameter(wo)
        self.b_out = nn.Parameter(torch.zeros(1))
        self._bf16: List[torch.Tensor] = []
        self.k_split = 512

    def bf16_weights(self) -> List[torch.Tensor]:
        h = _native.hip()
        if len(self._bf16) != len(self.w) or any(c.data_ptr() == 0 for c in self._bf16):
            self._bf16 = [torch.empty(w.shape, dtype=torch.bfloat16, device=w.device) for w in self.w]
        for w, c in zip(self.w, self._bf16):
            h.cast_bf16(w.detach(), c)
        return self._bf16

    def ensure_grads(self):
        for p in self.parameters():
            if p.grad is None:
                p.grad = torch.zeros_like(p)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if x.is_cuda:
            if x.dtype != torch.bfloat16:
                x = x.to(torch.bfloat16)
            if x.shape[1] != self.in_dim:
                x = torch.nn.functional.pad(x, (0, self.in_dim - x.shape[1]))
            return _FusedMLPFn.apply(x.contiguous(), self, *self.parameters())
        x = x.float()
        if x.shape[1] != self.in_dim:
            x = torch.nn.functional.pad(x, (0, self.in_dim - x.shape[1]))
        for w, b in zip(self.w, self.b):
            x = torch.relu(x @ w.t() + b)
        return (x @ self.w_out.t() + self.b_out).view(-1)
