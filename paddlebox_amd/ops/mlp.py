"""Fused MLP on hand-written MFMA GEMMs (csrc/hip/gemm.hip).

Hidden layers ``h = relu(x W^T + b)`` run as one bf16 MFMA GEMM each with the
bias+ReLU epilogue fused; the output layer (1 logit) is a GEMV.  The backward
fuses the ReLU mask into the GEMM operand staging and computes db inside the
dW GEMM (virtual ones column), writing parameter gradients straight into the
dense arena (no per-parameter gradient tensors / add kernels).

CPU tensors use plain fp32 PyTorch (the reference path).
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence

import torch
from torch import nn

from .. import _native


def pad32(n: int) -> int:
    return (n + 31) // 32 * 32


def pad8(n: int) -> int:
    return (n + 7) // 8 * 8


def _ensure_grad(p: torch.Tensor):
    if p.grad is None:
        p.grad = torch.zeros_like(p)
    return p.grad


def _bf16_copies(ws: Sequence[torch.Tensor], cache: List[torch.Tensor]) -> List[torch.Tensor]:
    h = _native.hip()
    if len(cache) != len(ws) or any(c.shape != w.shape for c, w in zip(cache, ws)):
        cache[:] = [torch.empty(w.shape, dtype=torch.bfloat16, device=w.device) for w in ws]
    for w, c in zip(ws, cache):
        h.cast_bf16(w.detach(), c)
    return cache


class _MLPFn(torch.autograd.Function):
    """Functional fused MLP: ``len(ws)`` ReLU layers (W: [N, K] fp32 master
    weights, K % 8 == 0) and an optional single-logit GEMV head.  Parameter
    gradients are accumulated straight into ``p.grad`` (dense-arena views);
    returns [M] fp32 logits (head) or the last bf16 hidden [M, N]."""

    @staticmethod
    def forward(ctx, x, ws, bs, w_out, b_out, cache, k_split, *params):
        h = _native.hip()
        wb = _bf16_copies(ws, cache)
        hs = [x]
        cur = x
        for w, b in zip(wb, bs):
            cur = h.linear_fwd(cur, w, b, True)
            hs.append(cur)
        ctx.ws, ctx.bs, ctx.w_out, ctx.b_out = ws, bs, w_out, b_out
        ctx.hs, ctx.wb, ctx.k_split = hs, wb, k_split
        ctx.x_needs_grad = x.requires_grad
        ctx.n_params = len(params)
        if w_out is not None:
            return h.gemv_out(cur, w_out.view(-1), b_out)
        return cur

    @staticmethod
    def backward(ctx, dout):
        h = _native.hip()
        hs, wb = ctx.hs, ctx.wb
        if ctx.w_out is not None:
            dh = h.gemv_out_bwd(hs[-1], ctx.w_out.view(-1), dout.float().contiguous(),
                                _ensure_grad(ctx.w_out).view(-1), _ensure_grad(ctx.b_out))
        else:
            dh = dout.to(torch.bfloat16).contiguous()
        for i in reversed(range(len(wb))):
            need_dx = i > 0 or ctx.x_needs_grad
            dh = h.linear_bwd(dh, hs[i + 1], hs[i], wb[i], _ensure_grad(ctx.ws[i]), _ensure_grad(ctx.bs[i]),
                              need_dx, ctx.k_split)
        ctx.hs = None
        dx = dh if ctx.x_needs_grad else None
        return (dx,) + (None,) * (6 + ctx.n_params)


class _MLPWsFn(torch.autograd.Function):
    """Fused MLP over the persistent MlpWorkspace (csrc/hip/mlp.hip)."""

    @staticmethod
    def forward(ctx, x0, mod, *params):
        ws = mod._ws
        logits = ws.forward(list(mod.w), list(mod.b), mod.w_out.view(-1), mod.b_out)
        ctx.mod = mod
        ctx.need_dx = x0.requires_grad
        ctx.n_params = len(params)
        return logits

    @staticmethod
    def backward(ctx, dlogit):
        mod = ctx.mod
        mod.ensure_grads()
        dx0 = mod._ws.backward(dlogit.float().contiguous(), [w.grad for w in mod.w], [b.grad for b in mod.b],
                               mod.w_out.view(-1), mod.w_out.grad.view(-1), mod.b_out.grad, ctx.need_dx)
        return (dx0 if ctx.need_dx else None, None) + (None,) * ctx.n_params


def fused_mlp(x: torch.Tensor, ws: Sequence[torch.Tensor], bs: Sequence[torch.Tensor],
              w_out: Optional[torch.Tensor], b_out: Optional[torch.Tensor], cache: List[torch.Tensor],
              k_split: int = 512) -> torch.Tensor:
    """x: [M, K0] (cast to bf16 and zero-padded to ws[0].shape[1])."""
    if x.dtype != torch.bfloat16:
        x = x.to(torch.bfloat16)
    if x.shape[1] != ws[0].shape[1]:
        x = torch.nn.functional.pad(x, (0, ws[0].shape[1] - x.shape[1]))
    params = list(ws) + list(bs) + ([w_out, b_out] if w_out is not None else [])
    return _MLPFn.apply(x.contiguous(), list(ws), list(bs), w_out, b_out, cache, k_split, *params)


class _MLP32Fn(torch.autograd.Function):
    """Exact-fp32 fc(relu) chain on library fp32 GEMMs (the reference fc
    precision, python/paddle/fluid/layers/nn.py:243 -> mul / matmul) for the
    lowered chains the fused fp32 tower does not take.  Same contract as
    _MLPFn: W [N, K] storage (K zero padded), gradients accumulated straight
    into ``p.grad`` (dense-arena views)."""

    @staticmethod
    def forward(ctx, x, ws, bs, w_out, b_out, *params):
        hs = [x]
        cur = x
        for w, b in zip(ws, bs):
            cur = torch.relu(torch.addmm(b.detach(), cur, w.detach().t()))
            hs.append(cur)
        ctx.ws, ctx.bs, ctx.w_out, ctx.b_out, ctx.hs = ws, bs, w_out, b_out, hs
        ctx.x_needs_grad = x.requires_grad
        ctx.n_params = len(params)
        if w_out is not None:
            return torch.addmm(b_out.detach(), cur, w_out.detach().t()).view(-1)
        return cur

    @staticmethod
    def backward(ctx, dout):
        hs = ctx.hs
        if ctx.w_out is not None:
            g = dout.float().reshape(-1, 1)
            _ensure_grad(ctx.w_out).add_(g.t() @ hs[-1])
            _ensure_grad(ctx.b_out).add_(g.sum(0))
            dh = g @ ctx.w_out.detach()
        else:
            dh = dout.float()
        for i in reversed(range(len(ctx.ws))):
            dh = dh * (hs[i + 1] > 0)
            _ensure_grad(ctx.ws[i]).add_(dh.t() @ hs[i])
            _ensure_grad(ctx.bs[i]).add_(dh.sum(0))
            if i > 0 or ctx.x_needs_grad:
                dh = dh @ ctx.ws[i].detach()
        ctx.hs = None
        dx = dh if ctx.x_needs_grad else None
        return (dx,) + (None,) * (4 + ctx.n_params)


def fused_mlp_fp32(x: torch.Tensor, ws: Sequence[torch.Tensor], bs: Sequence[torch.Tensor],
                   w_out: Optional[torch.Tensor], b_out: Optional[torch.Tensor]) -> torch.Tensor:
    """fp32 twin of fused_mlp: x [M, K0] zero-padded to ws[0].shape[1]."""
    x = x.float()
    if x.shape[1] != ws[0].shape[1]:
        x = torch.nn.functional.pad(x, (0, ws[0].shape[1] - x.shape[1]))
    params = list(ws) + list(bs) + ([w_out, b_out] if w_out is not None else [])
    return _MLP32Fn.apply(x.contiguous(), list(ws), list(bs), w_out, b_out, *params)


def tower_fp32_fits(widths: Sequence[int]) -> bool:
    """The exact-fp32 tower's LDS budget (FusedMLP.tower_fp32_ok) for the
    padded layer widths [in, hidden...]."""
    p16 = [(w + 15) // 16 * 16 for w in widths]
    return max(widths) <= 464 or (max(widths) <= 512 and all(p % 128 == 0 for p in p16))


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
        # split-K over the batch for the workspace dW GEMMs
        self.k_split_dw = int(os.environ.get("PBX_KSPLIT_DW", "1024"))
        self._ws = None
        self._tw = None
        # packed bf16 tower weights are valid (re-packed by FlatAdam's fused
        # kernel after every update when it owns this MLP; anything else that
        # writes the fp32 masters must call invalidate_pack())
        self._packed = False
        self.packed_by_optimizer = False

    # ---- fused tower path (csrc/hip/tower.hip)
    def tower_workspace(self, M: int, device: torch.device, fp32: bool = False, x3: bool = False):
        """Persistent buffers of the fused tower for batch M.  fp32=True is the
        exact-fp32 tower (csrc/hip/tower32.hip, the reference fc precision),
        else the bf16-operand tower (csrc/hip/tower.hip).  One workspace per
        (M, precision), kept for the module's lifetime: a HIP graph captured
        at one batch size keeps its workspace's addresses while steps of
        another size (a pass's last partial batch) use their own."""
        tws = self.__dict__.setdefault("_tws", {})
        key = (int(M), bool(fp32), bool(x3))
        tw = tws.get(key)
        if tw is None:
            dims = [self.in_dim] + list(self.hidden)
            # dW split over M (fp32: partial slabs summed in split order; bf16: fp32 atomics)
            if fp32:
                splits = int(os.environ.get("PBX_TOWER32_DW_SPLITS", "8"))
            else:
                splits = int(os.environ.get("PBX_TOWER_DW_SPLITS", "2"))
            if x3:
                # split-M partials summed in split order by the last split (bit-reproducible)
                splits = int(os.environ.get("PBX_TOWER_X3_DW_SPLITS", "2"))
            tw = tws[key] = _native.hip().TowerWorkspace(M, dims, device.index or 0, splits, bool(fp32), bool(x3))
        if self._tw is not tw:
            self._tw = tw
            self._packed = False
        return self._tw

    def tower_workspaces(self):
        """Every workspace of this MLP (the fused Adam re-packs all of them)."""
        return list(self.__dict__.get("_tws", {}).values())

    def tower_fp32_ok(self) -> bool:
        """The fp32 tower keeps two 32-row fp32 tiles in LDS, plus the
        remainder partial sums of its wave-stream schedule when a width is not
        a multiple of 128: widths <= 464, or <= 512 when all are multiples of
        128 (bindings_tower.cpp checks the exact budget)."""
        return tower_fp32_fits([self.in_dim] + list(self.hidden))

    def tower_x3_ok(self) -> bool:
        """The x3 tower (fp32 precision on bf16 MFMA, csrc/hip/tower_x3.hip)
        keeps hi + lo planes of two 32-row bf16 tiles in LDS: padded widths
        <= 592."""
        return max(pad32(d) for d in [self.in_dim] + list(self.hidden)) + 8 <= 600

    def ensure_packed(self):
        """Pack the current workspace's tower weights unless the optimizer
        keeps them packed.  With several batch-size workspaces the forward
        always packs its own: an optimizer launch captured before a
        workspace existed does not re-pack it."""
        if not self._packed or not self.packed_by_optimizer or len(self.__dict__.get("_tws", {})) > 1:
            self._tw.pack([w.detach() for w in self.w])
            self._packed = True

    def invalidate_pack(self):
        self._packed = False

    # ---- workspace path (csrc/hip/mlp.hip): persistent padded activations +
    # transposed copies so every GEMM streams both operands HBM -> LDS by DMA
    def workspace(self, M: int, device: torch.device):
        if self._ws is None or self._ws.M != M:
            dims = [self.in_dim] + list(self.hidden)
            self._ws = _native.hip().MlpWorkspace(M, dims, device.index or 0, self.k_split_dw)
        return self._ws

    def forward_ws(self, x0: torch.Tensor) -> torch.Tensor:
        """x0 = workspace.x(0) already filled (and x0^T = workspace.xt(0)) by
        the producer (the CTR head).  Returns [M] logits."""
        return _MLPWsFn.apply(x0, self, *self.parameters())

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

    def forward_fp32(self, x: torch.Tensor) -> torch.Tensor:
        """fp32 MLP on any device (library fp32 GEMMs on the GPU): the
        reference's fluid fc precision, kept for precision comparisons."""
        x = x.float()
        if x.shape[1] != self.in_dim:
            x = torch.nn.functional.pad(x, (0, self.in_dim - x.shape[1]))
        for w, b in zip(self.w, self.b):
            x = torch.relu(torch.addmm(b, x, w.t()))
        return torch.addmm(self.b_out, x, self.w_out.t()).view(-1)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if x.is_cuda:
            if x.dtype != torch.bfloat16:
                x = x.to(torch.bfloat16)
            if x.shape[1] != self.in_dim:
                x = torch.nn.functional.pad(x, (0, self.in_dim - x.shape[1]))
            return fused_mlp(x, list(self.w), list(self.b), self.w_out, self.b_out, self._bf16, self.k_split)
        x = x.float()
        if x.shape[1] != self.in_dim:
            x = torch.nn.functional.pad(x, (0, self.in_dim - x.shape[1]))
        for w, b in zip(self.w, self.b):
            x = torch.relu(x @ w.t() + b)
        return (x @ self.w_out.t() + self.b_out).view(-1)
