"""Dense CTR ops with autograd: data_norm, FM interaction, sigmoid+logloss,
streaming AUC.  GPU tensors run the hand-written gfx950 kernels
(csrc/hip/dense_ops.hip); CPU tensors run ``reference``.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from .. import _native
from ..parallel.comm import allreduce_sum, collective_active
from . import reference as ref


def _gpu(t: torch.Tensor) -> bool:
    return t.is_cuda


# ---------------------------------------------------------------- data_norm
class _DataNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bsize, bsum, bsq, scale_w, bias, eps, decay, sync_group, update, training):
        x = x.contiguous().float()
        if _gpu(x):
            y, means, scales = _native.hip().data_norm_fwd(x, bsize, bsum, bsq, scale_w, bias)
        else:
            y, means, scales = ref.data_norm_fwd(x, bsize, bsum, bsq, scale_w, bias)
        ctx.save_for_backward(x, means, scales, bsize, bsum, bsq, scale_w)
        ctx.eps, ctx.decay, ctx.group, ctx.update, ctx.training = eps, decay, sync_group, update, training
        ctx.has_sw = scale_w is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, means, scales, bsize, bsum, bsq, scale_w = ctx.saved_tensors
        dy = dy.contiguous().float()
        if _gpu(x):
            dx, stats = _native.hip().data_norm_bwd(x, dy, means, scales, ctx.eps, True, scale_w)
        else:
            dx, stats = ref.data_norm_bwd(x, dy, means, scales, ctx.eps, scale_w)
        if ctx.group is not None and collective_active(ctx.group):
            # one fused all-reduce of [3, C] (reference does 3 separate ones,
            # data_norm_op.cu:203-230); the group's IPC mesh when registered
            allreduce_sum(stats, ctx.group)
        if ctx.update and ctx.training:
            if _gpu(x):
                _native.hip().data_norm_update(bsize, bsum, bsq, stats, ctx.decay)
            else:
                ref.data_norm_update(bsize, bsum, bsq, stats, ctx.decay)
        dsw = dbias = None
        if ctx.has_sw:
            xn = (x - means) * scales
            dsw = (dy * xn).sum(0)
            dbias = dy.sum(0)
        return dx, None, None, None, dsw, dbias, None, None, None, None, None


class DataNorm(torch.nn.Module):
    """data_norm layer (py/fluid/layers/nn.py:3490-3676): running summary
    normalisation; summaries are updated by the backward with decay
    0.9999999 (not by the optimizer)."""

    def __init__(self, C: int, epsilon: float = 1e-5, summary_decay_rate: float = 0.9999999,
                 sync_stats: bool = False, enable_scale_and_shift: bool = False, batch_size_default: float = 1e4,
                 batch_sum_default: float = 0.0, batch_square_sum_default: float = 1e4, slot_dim: int = -1):
        super().__init__()
        self.C = C
        self.eps = epsilon
        self.decay = summary_decay_rate
        self.sync_stats = sync_stats
        self.slot_dim = slot_dim
        self.register_buffer("batch_size", torch.full((C,), float(batch_size_default)))
        self.register_buffer("batch_sum", torch.full((C,), float(batch_sum_default)))
        self.register_buffer("batch_square_sum", torch.full((C,), float(batch_square_sum_default)))
        if enable_scale_and_shift:
            self.scale_w = torch.nn.Parameter(torch.ones(C))
            self.bias = torch.nn.Parameter(torch.zeros(C))
        else:
            self.scale_w = None
            self.bias = None
        self.update_norm = True
        self.group = None
        # batch statistics [3, C] written by the fused tower backward; the
        # summary update is applied there, or by FlatAdam's fused kernel when
        # it owns this layer (fused_update = True)
        self.register_buffer("stats", torch.zeros(3 * C))
        self.fused_update = False

    def forward(self, x):
        return _DataNorm.apply(x, self.batch_size, self.batch_sum, self.batch_square_sum, self.scale_w, self.bias,
                               self.eps, self.decay, self.group if self.sync_stats else None, self.update_norm,
                               self.training)


# ---------------------------------------------------------------- fused CTR head
class _CtrHead(torch.autograd.Function):
    """y = data_norm(x) (bf16, padded to Cp) and lin = first-order + FM, one
    kernel each way on the GPU (csrc/hip/head_ops.hip)."""

    @staticmethod
    def forward(ctx, x, dn: Optional[DataNorm], S, Eo, ew_col, D, Cp, y_out=None, yT_out=None):
        x = x.contiguous().float()
        has_dn = dn is not None
        if _gpu(x):
            if has_dn:
                y, lin, means, scales = _native.hip().head_fwd(x, S, Eo, ew_col, D, Cp, dn.batch_size, dn.batch_sum,
                                                                dn.batch_square_sum, y_out, yT_out)
            else:
                y, lin, means, scales = _native.hip().head_fwd(x, S, Eo, ew_col, D, Cp, None, None, None, y_out,
                                                                yT_out)
        else:
            if has_dn:
                y, means, scales = ref.data_norm_fwd(x, dn.batch_size, dn.batch_sum, dn.batch_square_sum)
            else:
                y, means, scales = x, None, None
            if Cp > y.shape[1]:
                y = torch.nn.functional.pad(y, (0, Cp - y.shape[1]))
            lin = x[:, ew_col:S * Eo:Eo].sum(1) + ref.fm_fwd(x, S, D, ew_col + 1, Eo)
        ctx.save_for_backward(x)
        ctx.means, ctx.scales = means, scales
        ctx.dn, ctx.args = dn, (S, Eo, ew_col, D, Cp)
        return y, lin

    @staticmethod
    def backward(ctx, dy, dlin):
        (x,) = ctx.saved_tensors
        S, Eo, ew_col, D, Cp = ctx.args
        dn = ctx.dn
        if dlin is None:
            dlin = torch.zeros(x.shape[0], device=x.device)
        if _gpu(x):
            dyc = dy.contiguous() if dy is not None else None
            if dyc is not None and dyc.dtype != torch.bfloat16:
                dyc = dyc.to(torch.bfloat16)
            dx, stats = _native.hip().head_bwd(x, dyc, dlin.contiguous().float(), S, Eo, ew_col, D, Cp, ctx.means,
                                              ctx.scales, dn.eps if dn is not None else 0.0)
        else:
            with torch.enable_grad():
                xx = x.detach().requires_grad_(True)
                if dn is not None:
                    y = (xx - ctx.means) * ctx.scales
                else:
                    y = xx
                if Cp > y.shape[1]:
                    y = torch.nn.functional.pad(y, (0, Cp - y.shape[1]))
                lin = xx[:, ew_col:S * Eo:Eo].sum(1) + ref.fm_fwd(xx, S, D, ew_col + 1, Eo)
                outs, grads = [lin], [dlin]
                if dy is not None:
                    outs.append(y)
                    grads.append(dy.float())
                (dx,) = torch.autograd.grad(outs, xx, grads)
            stats = None
            if dn is not None:
                _, stats = ref.data_norm_bwd(x, x, ctx.means, ctx.scales, dn.eps)
        if dn is not None and dn.training and dn.update_norm:
            if dn.sync_stats and dn.group is not None and collective_active(dn.group):
                allreduce_sum(stats, dn.group)
            if _gpu(x):
                _native.hip().data_norm_update(dn.batch_size, dn.batch_sum, dn.batch_square_sum, stats, dn.decay)
            else:
                ref.data_norm_update(dn.batch_size, dn.batch_sum, dn.batch_square_sum, stats, dn.decay)
        return dx, None, None, None, None, None, None, None, None


def ctr_head(x: torch.Tensor, dn: Optional["DataNorm"], S: int, Eo: int, ew_col: int, D: int, Cp: int,
             y_out: Optional[torch.Tensor] = None, yT_out: Optional[torch.Tensor] = None):
    """(data_norm(x) as the MLP input [B, Cp] -- or written into the MLP
    workspace's X0 [B, ld] / X0^T buffers when given --, first-order + FM
    logit part [B])."""
    return _CtrHead.apply(x, dn, S, Eo, ew_col, D, Cp, y_out, yT_out)


# ---------------------------------------------------------------- FM
class _FM(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, S, D, col0, fstride):
        x = x.contiguous().float()
        if _gpu(x):
            out = _native.hip().fm_fwd(x, S, D, col0, fstride)
        else:
            out = ref.fm_fwd(x, S, D, col0, fstride)
        ctx.save_for_backward(x)
        ctx.args = (S, D, col0, fstride)
        return out

    @staticmethod
    def backward(ctx, dout):
        (x,) = ctx.saved_tensors
        S, D, col0, fstride = ctx.args
        dout = dout.contiguous().float()
        if _gpu(x):
            dx = torch.zeros_like(x)
            _native.hip().fm_bwd(x, dout, S, D, col0, fstride, dx, False)
        else:
            with torch.enable_grad():
                xx = x.detach().requires_grad_(True)
                y = ref.fm_fwd(xx, S, D, col0, fstride)
                (dx,) = torch.autograd.grad(y, xx, dout)
        return dx, None, None, None, None


def fm_interaction(x: torch.Tensor, S: int, D: int, col0: int, fstride: int) -> torch.Tensor:
    """DeepFM 2nd-order term 0.5*sum_d[(sum_s v)^2 - sum_s v^2] over S fields of
    dim D stored at x[:, col0 + s*fstride + d]."""
    return _FM.apply(x, S, D, col0, fstride)


# ---------------------------------------------------------------- loss
class _SigmoidLogLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logit, label):
        logit = logit.contiguous().float().view(-1)
        label = label.contiguous().float().view(-1)
        B = logit.numel()
        if _gpu(logit):
            pred, loss, dz = _native.hip().sigmoid_logloss(logit, label, 1.0 / B)
        else:
            pred, loss, dz = ref.sigmoid_logloss(logit, label, 1.0 / B)
        ctx.save_for_backward(dz)
        ctx.mark_non_differentiable(pred)
        return loss[0] / B, pred

    @staticmethod
    def backward(ctx, gl, gp):
        (dz,) = ctx.saved_tensors
        return dz * gl, None


def sigmoid_logloss(logit: torch.Tensor, label: torch.Tensor):
    """(mean log-loss, sigmoid prediction) with the gradient fused."""
    return _SigmoidLogLoss.apply(logit, label)


_LOSS_WS = {}


def _loss_ws(dev: torch.device) -> torch.Tensor:
    """Per-(device, stream) ticket + partials workspace of the loss kernel
    (zeroed once; the kernel re-arms it): launches on different streams never
    share a counter."""
    key = (dev.index, torch.cuda.current_stream(dev).cuda_stream)
    ws = _LOSS_WS.get(key)
    if ws is None:
        ws = _LOSS_WS[key] = torch.zeros(1 + 1024, dtype=torch.int32, device=dev)
    return ws


class _LogitLoss(torch.autograd.Function):
    """loss, pred = BCE(sigmoid(a + b), label): the sum of the two logit parts,
    the sigmoid, the mean log-loss and its gradient in one kernel; the
    backward is a single scale of the saved gradient, shared by both parts."""

    @staticmethod
    def forward(ctx, a, b, label):
        a = a.contiguous().float().view(-1)
        label = label.contiguous().float().view(-1)
        bb = b.contiguous().float().view(-1) if b is not None else None
        if _gpu(a):
            loss, pred, dz = _native.hip().logit_loss(a, bb, label, _loss_ws(a.device))
        else:
            z = a + bb if bb is not None else a
            pred, loss_sum, dz = ref.sigmoid_logloss(z, label, 1.0 / a.numel())
            loss = loss_sum / a.numel()
        ctx.save_for_backward(dz)
        ctx.has_b = b is not None
        ctx.mark_non_differentiable(pred)
        return loss.view(()), pred

    @staticmethod
    def backward(ctx, gl, gp):
        (dz,) = ctx.saved_tensors
        g = dz * gl
        return g, (g if ctx.has_b else None), None


def logit_logloss(a: torch.Tensor, b: Optional[torch.Tensor], label: torch.Tensor):
    """(mean log-loss, prediction) of logit = a + b, fused."""
    return _LogitLoss.apply(a, b, label)


# ---------------------------------------------------------------- AUC
def auc_accumulate(pred: torch.Tensor, label: torch.Tensor, table: torch.Tensor, stats: torch.Tensor,
                   mask: Optional[torch.Tensor] = None):
    pred = pred.detach().contiguous().float().view(-1)
    label = label.detach().contiguous().float().view(-1)
    if _gpu(pred):
        _native.hip().auc_accumulate(pred, label, mask, table, stats)
    else:
        ref.auc_accumulate(pred, label, table, stats, mask)
