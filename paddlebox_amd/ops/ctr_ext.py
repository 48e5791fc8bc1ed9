"""The PaddleBox CTR op family beyond the DeepFM hot path.

Semantics follow the reference kernels (cited per op); each op is an
autograd-aware function.  Where the reference gradient is not the true
derivative (CVM columns carrying show/click into the push, scaled_fc's bias
gradient) the reference behaviour is reproduced with a custom Function.
GPU tensors run the hand-written kernels in ``csrc/hip/ctr_ext.hip``
(batch_fc / scaled_fc / scaled_int8fc / rank_attention / cvm /
masked_data_norm / cross_norm_hadamard) and ``csrc/hip/seqpool_variants.hip``
(the fused_seqpool_cvm variant family, fused_seq_tensor); the torch
expressions here are the
CPU path and the fp32 reference the GPU tests compare against
(tests/test_gpu_ctr_ops.py).
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence

import torch
import torch.distributed as dist

from .. import _native
from ..parallel.comm import collective_active


def _seg_ids(offsets: torch.Tensor, L: int) -> torch.Tensor:
    """instance id of each of the L rows given [B+1] offsets."""
    return torch.searchsorted(offsets[1:].contiguous(), torch.arange(L, device=offsets.device), right=True)


# ================================================================== sequence_pool
def sequence_pool(x: torch.Tensor, offsets: torch.Tensor, B: int, pooltype: str = "SUM",
                  pad_value: float = 0.0) -> torch.Tensor:
    L = x.shape[0]
    seg = _seg_ids(offsets, L)
    x2 = x.reshape(L, -1)
    cnt = (offsets[1:] - offsets[:-1]).to(x.dtype).unsqueeze(1)
    out = torch.zeros(B, x2.shape[1], dtype=x.dtype, device=x.device).index_add(0, seg, x2)
    pt = pooltype.upper()
    if pt == "AVERAGE":
        out = out / cnt.clamp(min=1)
    elif pt == "SQRT":
        out = out / cnt.clamp(min=1).sqrt()
    elif pt == "MAX":
        out = torch.full((B, x2.shape[1]), float("-inf"), dtype=x.dtype, device=x.device)
        out = out.index_reduce(0, seg, x2, "amax")
    elif pt == "FIRST":
        out = x2[offsets[:-1].clamp(max=max(L - 1, 0))]
    elif pt == "LAST":
        out = x2[(offsets[1:] - 1).clamp(min=0)]
    empty = (cnt == 0)
    return torch.where(empty, torch.full_like(out, pad_value), out)


def auc_from_hist(pos: torch.Tensor, neg: torch.Tensor) -> torch.Tensor:
    """ROC AUC from per-threshold positive/negative counts (phi auc kernel)."""
    p = pos.double().flip(0)
    n = neg.double().flip(0)
    tp = torch.cumsum(p, 0)
    fp = torch.cumsum(n, 0)
    tp_prev = torch.cat([tp.new_zeros(1), tp[:-1]])
    fp_prev = torch.cat([fp.new_zeros(1), fp[:-1]])
    area = ((fp - fp_prev) * (tp + tp_prev) / 2).sum()
    denom = tp[-1] * fp[-1]
    return torch.where(denom > 0, area / denom.clamp(min=1e-300), torch.zeros_like(area))


# ================================================================== cvm
class _Cvm(torch.autograd.Function):
    """cvm op (operators/cvm_op.h:25-57): y = [log(show+1), log(clk+1)-log(show+1), rest]
    (use_cvm) or drop the two cvm columns; dx's cvm columns carry the CVM input."""

    @staticmethod
    def forward(ctx, x, cvm, use_cvm):
        ctx.use_cvm = use_cvm
        ctx.save_for_backward(cvm)
        ctx.width = x.shape[-1]
        if use_cvm:
            y = x.clone()
            y[..., 0] = torch.log(x[..., 0] + 1)
            y[..., 1] = torch.log(x[..., 1] + 1) - y[..., 0]
            return y
        return x[..., 2:].contiguous()

    @staticmethod
    def backward(ctx, dy):
        (cvm,) = ctx.saved_tensors
        n = dy.shape[0]
        dx = dy.new_empty(n, ctx.width)
        off = 0 if ctx.use_cvm else 2
        dx[:, off:] = dy
        dx[:, :2] = cvm.reshape(-1, 2)[:n] if cvm.shape[0] == n else cvm.reshape(-1, 2)[0]
        return dx, None, None


class _CvmHip(torch.autograd.Function):
    """GPU cvm: k_cvm_fwd / k_cvm_bwd (csrc/hip/ctr_ext.hip)."""

    @staticmethod
    def forward(ctx, x, cvm, use_cvm):
        ctx.use_cvm, ctx.width, ctx.lead = use_cvm, x.shape[-1], x.shape[:-1]
        ctx.save_for_backward(cvm)
        return _native.hip().cvm_fwd(x, use_cvm)

    @staticmethod
    def backward(ctx, dy):
        (cvm,) = ctx.saved_tensors
        dx = _native.hip().cvm_bwd(dy.float(), cvm.float(), ctx.width, ctx.use_cvm)
        return dx.reshape(*ctx.lead, ctx.width), None, None


def cvm(x: torch.Tensor, cvm_t: torch.Tensor, use_cvm: bool = True) -> torch.Tensor:
    if x.is_cuda:
        return _CvmHip.apply(x.float().contiguous(), cvm_t, use_cvm)
    return _Cvm.apply(x, cvm_t, use_cvm)


# ================================================================== seqpool-CVM family over records
def _quant(v: torch.Tensor, q: int) -> torch.Tensor:
    return torch.trunc(v * q + 0.5) / q if q > 0 else v


class _SeqpoolCvmVariant(torch.autograd.Function):
    """Generic fused_seqpool_cvm* over per-occurrence records.

    ``variant`` in {"std", "diff_thres", "conv", "pcoc", "tradew", "credit"};
    forward: filtered (+quantised) SUM pool (+pad) per (slot, instance) then the
    variant's CVM epilogue; backward: broadcast the pooled grad to every row of
    the sequence and overwrite the statistic columns with the CVM input, which
    is how show/click reach push_box_sparse (fused_seqpool_cvm_op.cu:813-1015
    and the per-variant grad kernels)."""

    @staticmethod
    def forward(ctx, cvm_in, variant, attrs, offsets_list, B, qvals, *xs):
        a = attrs
        outs, saved = [], []
        for x, off in zip(xs, offsets_list):
            L, E = x.shape
            seg = _seg_ids(off, L)
            show, clk = x[:, 0], x[:, 1] if E > 1 else x[:, 0]
            keep = torch.ones(L, dtype=torch.bool, device=x.device)
            need_f, embed_f = _filters(variant, a)
            if need_f:
                thr = a["threshold"]
                if variant == "diff_thres" and a.get("xbox_diff_thres_filter"):
                    thr = a["threshold_vec"][len(outs)]
                keep &= (show - clk) * a["show_coeff"] + clk * a["clk_coeff"] >= thr
            co = a.get("cvm_offset", 2)
            if embed_f:
                ets = a.get("embed_thres_size", 0)
                ets = ets if ets > 0 else E - co  # 0 = the whole embedding (op.cu:596-599)
                emb = x[:, co:co + ets]
                score = emb[:, 1:].pow(2).sum(1).sqrt() + emb[:, 0].abs()
                keep &= score >= a["embed_threshold"]
            q = a.get("quant_ratio", 0)
            mcol = a.get("max_cvm_offset", co) if variant == "pcoc" else co
            vals = x.clone()
            if q > 0:
                vals[:, mcol:] = _quant(vals[:, mcol:], q)
            if variant == "tradew":
                tn, tid = a["trade_num"], a["trade_id"]
                emb = vals[:, co + tn:]
                if tid >= 0:
                    emb = emb * vals[:, co + tid:co + tid + 1]
                vals = torch.cat([vals[:, :co], emb], 1)
            vals = vals * keep.unsqueeze(1).to(vals.dtype)
            pooled = torch.zeros(B, vals.shape[1], dtype=x.dtype, device=x.device).index_add(0, seg, vals)
            pooled = pooled + a.get("pad_value", 0.0)
            ecs = a.get("embedx_concate_size", 1)
            if ecs > 1:
                pooled = _concat_pool(vals, off, B, ecs, a.get("pad_value", 0.0))
            outs.append(_cvm_epilogue(variant, pooled, a, ecs))
            saved.append((L, E, seg))
        ctx.variant, ctx.attrs, ctx.B, ctx.saved = variant, a, B, saved
        ctx.offsets_list = offsets_list
        ctx.save_for_backward(cvm_in, qvals if qvals is not None else torch.zeros(0), *xs)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *douts):
        cvm_in, qvals, *xs = ctx.saved_tensors
        a, variant = ctx.attrs, ctx.variant
        co = a.get("cvm_offset", 2)
        grads = []
        for (L, E, seg), dout, x in zip(ctx.saved, douts, xs):
            dpool = _cvm_epilogue_grad(variant, dout, a, E, cvm_in, qvals, ctx.B)
            ecs = a.get("embedx_concate_size", 1)
            if ecs > 1:
                g = _concat_pool_grad(dpool, ctx.offsets_list[len(grads)], L, E, ecs)
            else:
                g = dpool[seg]
            if variant == "tradew":
                tn, tid = a["trade_num"], a["trade_id"]
                full = x.new_zeros(L, E)
                full[:, :co] = g[:, :co]
                emb_g = g[:, co:]
                if tid >= 0:
                    w = x[:, co + tid:co + tid + 1]
                    full[:, co + tn:] = emb_g * w
                    full[:, co + tid] = (emb_g * x[:, co + tn:]).sum(1)
                    full[:, :co] = 0.0
                else:
                    full[:, co + tn:] = emb_g
                g = full
            grads.append(g)
        return (None, None, None, None, None, None) + tuple(grads)


def _filters(variant, a):
    """(show/click filter, embedding-norm filter) as the reference applies
    them in the pooling kernels:
      * the embedding-norm filter only runs under need_filter
        (fused_seqpool_cvm_op.cu:580-581 nests it);
      * with embedx_concate_size > 1 a record is filtered only when
        embedx_concate_filter is set (op.cu:215, 352); the conv variant never
        filters in concat mode (fused_seqpool_cvm_with_conv_op.cu:345-383)."""
    need = bool(a.get("need_filter"))
    embed = need and bool(a.get("embed_threshold_filter")) if variant == "std" else False
    if a.get("embedx_concate_size", 1) > 1 and not (variant == "std" and a.get("embedx_concate_filter")):
        need = embed = False
    return need, embed


def _concat_pool(vals, off, B, ecs, pad):
    """embedx_concate: block k of an instance holds only its k-th row."""
    L, E = vals.shape
    out = torch.full((B, ecs, E), pad, dtype=vals.dtype, device=vals.device)
    starts = off[:-1]
    lens = off[1:] - off[:-1]
    for k in range(ecs):
        has = lens > k
        idx = (starts + k).clamp(max=max(L - 1, 0))
        out[:, k] += torch.where(has.unsqueeze(1), vals[idx], torch.zeros_like(vals[idx]))
    return out.reshape(B, ecs * E)


def _concat_pool_grad(dpool, off, L, E, ecs):
    """Reference grad: block k -> row k; the last block also feeds all
    remaining rows (FusedSeqpoolCVM*GradKernel*Concate)."""
    B = off.numel() - 1
    dp = dpool.reshape(B, ecs, E)
    seg = _seg_ids(off, L)
    pos = torch.arange(L, device=off.device) - off[seg]
    k = pos.clamp(max=ecs - 1)
    return dp[seg, k]


def _cvm_epilogue(variant, p, a, ecs=1):
    use_cvm = a.get("use_cvm", True)
    co = a.get("cvm_offset", 2)
    if ecs > 1:
        B = p.shape[0]
        E = p.shape[1] // ecs
        blocks = [_cvm_epilogue(variant, p[:, k * E:(k + 1) * E], a, 1) for k in range(ecs)]
        return torch.cat(blocks, 1) if blocks else p.new_zeros(B, 0)
    lg = lambda v: torch.log(v + 1)  # noqa: E731
    if variant in ("std", "diff_thres", "tradew"):
        if not use_cvm:
            return p[:, co + (a.get("embed_thres_size", 0) if variant == "std" else 0):]
        s = lg(p[:, 0])
        c = lg(p[:, 1]) - s
        if a.get("clk_filter"):
            return torch.cat([s[:, None], p[:, 2:]], 1)
        return torch.cat([s[:, None], c[:, None], p[:, 2:]], 1)
    if variant == "conv":
        if not use_cvm:
            return p[:, co:]
        s, c, v = lg(p[:, 0]), lg(p[:, 1]), lg(p[:, 2]) - lg(p[:, 1])
        if a.get("show_filter"):
            return torch.cat([c[:, None], v[:, None], p[:, 3:]], 1)
        return torch.cat([s[:, None], c[:, None], v[:, None], p[:, 3:]], 1)
    if variant == "credit":
        if not use_cvm:
            return p[:, co:]
        st = lg(p[:, :co])
        if a.get("show_filter"):
            return torch.cat([st[:, 1:], p[:, co:]], 1)
        return torch.cat([st, p[:, co:]], 1)
    if variant == "pcoc":
        mco = a.get("max_cvm_offset", co)
        if not use_cvm:
            return p[:, mco:]
        pk = co - 4
        diff = mco - 2 - 2 * pk
        s = lg(p[:, 0])
        cols = [s[:, None], (lg(p[:, 1]) - s)[:, None]]
        for j in range(pk):
            cols.append((lg(p[:, 4 + j]) - lg(p[:, 2]))[:, None])
        for j in range(pk):
            cols.append((lg(p[:, 4 + j]) - lg(p[:, 3]))[:, None])
        cols.append(p[:, 2 + 2 * pk + diff:])
        return torch.cat(cols, 1)
    raise ValueError(variant)


def _cvm_epilogue_grad(variant, dout, a, E, cvm_in, qvals, B):
    """[B, E_pool] gradient of the pooled value (statistic columns = CVM input)."""
    use_cvm = a.get("use_cvm", True)
    co = a.get("cvm_offset", 2)
    ecs = a.get("embedx_concate_size", 1)
    if variant == "tradew":
        E = E - a["trade_num"]
    if ecs > 1:
        Eo = dout.shape[1] // ecs
        blocks = [_cvm_epilogue_grad(variant, dout[:, k * Eo:(k + 1) * Eo], dict(a, embedx_concate_size=1), E,
                                     cvm_in, qvals, B) for k in range(ecs)]
        return torch.cat(blocks, 1)
    g = dout.new_zeros(B, E)
    cv = cvm_in.reshape(B, -1)
    if variant == "pcoc":
        mco = a.get("max_cvm_offset", co)
        pk = co - 4
        g[:, :4] = cv[:, :4]
        if pk > 0:
            q = qvals.reshape(B, pk) if qvals is not None and qvals.numel() == B * pk else dout.new_zeros(B, pk)
            g[:, 4:co] = q
        if use_cvm:
            diff = mco - 2 - 2 * pk
            g[:, mco:] = dout[:, mco - diff:]
        else:
            g[:, mco:] = dout
        return g
    ncv = min(co, cv.shape[1])
    skip = a.get("embed_thres_size", 0) if (variant == "std" and not use_cvm) else 0
    if skip == 0:  # with dropped columns the cvm grads are zero too (op.cu:958-969)
        g[:, :ncv] = cv[:, :ncv]
    if not use_cvm:
        g[:, co + skip:] = dout
        return g
    if variant in ("std", "diff_thres", "tradew"):
        if a.get("clk_filter"):
            g[:, 2:] = dout[:, 1:]
        else:
            g[:, 2:] = dout[:, 2:]
    elif variant in ("conv", "credit"):
        if a.get("show_filter"):
            g[:, co:] = dout[:, co - 1:]
        else:
            g[:, co:] = dout[:, co:]
    return g


_VARIANT = {
    "fused_seqpool_cvm": "std", "fused_seqpool_cvm_with_diff_thres": "diff_thres",
    "fused_seqpool_cvm_with_conv": "conv", "fused_seqpool_cvm_with_pcoc": "pcoc",
    "fused_seqpool_cvm_tradew": "tradew", "fused_seqpool_cvm_with_credit": "credit",
}


_F_COPY, _F_LOG, _F_LOGDIFF = 0, 1, 2
_G_ZERO, _G_CVM, _G_QVAL, _G_DOUT = 0, 1, 2, 3


def _spv_tables(variant: str, a: Dict, E: int, ncv: int, has_q: bool):
    """Column tables of one variant's CVM epilogue (forward: output column ->
    op on pooled columns) and its gradient (pooled column -> source), the
    same mapping _cvm_epilogue / _cvm_epilogue_grad spell out with slicing.
    Returns (ftab [(op, s1, s2)], btab [(op, idx)], Epool)."""
    use_cvm = a.get("use_cvm", True)
    co = a.get("cvm_offset", 2)
    Ep = E - a["trade_num"] if variant == "tradew" else E
    f: List = []
    g = [(_G_ZERO, 0)] * Ep

    def dout_from(pool0, out0):  # g[pool0 + i] = dout[out0 + i]
        for i in range(Ep - pool0):
            g[pool0 + i] = (_G_DOUT, out0 + i)

    if variant == "pcoc":
        mco = a.get("max_cvm_offset", co)
        pk = co - 4
        if use_cvm:
            f = [(_F_LOG, 0, 0), (_F_LOGDIFF, 1, 0)]
            f += [(_F_LOGDIFF, 4 + j, 2) for j in range(pk)] + [(_F_LOGDIFF, 4 + j, 3) for j in range(pk)]
        f += [(_F_COPY, c, 0) for c in range(mco, Ep)]
        for j in range(min(4, ncv)):
            g[j] = (_G_CVM, j)
        if pk > 0 and has_q:
            for j in range(pk):
                g[4 + j] = (_G_QVAL, j)
        dout_from(mco, mco - (mco - 2 - 2 * pk) if use_cvm else 0)
        return f, g, Ep
    skip = a.get("embed_thres_size", 0) if (variant == "std" and not use_cvm) else 0
    if skip == 0:
        for j in range(min(co, ncv)):
            g[j] = (_G_CVM, j)
    if not use_cvm:
        f = [(_F_COPY, c, 0) for c in range(co + skip, Ep)]
        dout_from(co + skip, 0)
        return f, g, Ep
    if variant in ("std", "diff_thres", "tradew"):
        f = [(_F_LOG, 0, 0)] + ([] if a.get("clk_filter") else [(_F_LOGDIFF, 1, 0)])
        f += [(_F_COPY, c, 0) for c in range(2, Ep)]
        dout_from(2, 1 if a.get("clk_filter") else 2)
    elif variant == "conv":
        f = ([] if a.get("show_filter") else [(_F_LOG, 0, 0)]) + [(_F_LOG, 1, 0), (_F_LOGDIFF, 2, 1)]
        f += [(_F_COPY, c, 0) for c in range(3, Ep)]
        dout_from(co, co - 1 if a.get("show_filter") else co)
    elif variant == "credit":
        f = [(_F_LOG, j, 0) for j in range(1 if a.get("show_filter") else 0, co)]
        f += [(_F_COPY, c, 0) for c in range(co, Ep)]
        dout_from(co, co - 1 if a.get("show_filter") else co)
    else:
        raise ValueError(variant)
    return f, g, Ep


def _enc_f(f):
    return [(op << 24) | (s1 << 12) | s2 for op, s1, s2 in f]


def _enc_g(g):
    return [(op << 24) | idx for op, idx in g]


class _SeqpoolCvmVariantHip(torch.autograd.Function):
    """GPU fused_seqpool_cvm variants: k_spv_fwd / k_spv_bwd
    (csrc/hip/seqpool_variants.hip) driven by _spv_tables."""

    @staticmethod
    def forward(ctx, cvm_in, variant, a, offsets_list, B, qvals, *xs):
        dev = xs[0].device
        E = xs[0].shape[1]
        S = len(xs)
        cv = cvm_in.float().reshape(B, -1).contiguous()
        has_q = variant == "pcoc" and qvals is not None and qvals.numel() == B * (a.get("cvm_offset", 2) - 4)
        f, g, Ep = _spv_tables(variant, a, E, cv.shape[1], has_q)
        co = a.get("cvm_offset", 2)
        ecs = a.get("embedx_concate_size", 1)
        ets = a.get("embed_thres_size", 0)
        need_f, embed_f = _filters(variant, a)
        ints = [int(need_f), int(embed_f),
                ets if ets > 0 else E - co, co, int(a.get("quant_ratio", 0)),
                a.get("max_cvm_offset", co) if variant == "pcoc" else co,
                int(variant == "tradew"), a.get("trade_num", 0) if variant == "tradew" else 0,
                a.get("trade_id", -1) if variant == "tradew" else -1, ecs, Ep, len(f)]
        fl = [a.get("show_coeff", 0.0), a.get("clk_coeff", 1.0), a.get("embed_threshold", 0.0),
              a.get("pad_value", 0.0)]
        if variant == "diff_thres" and a.get("xbox_diff_thres_filter"):
            thr = torch.tensor([float(t) for t in a["threshold_vec"][:S]], dtype=torch.float32)
        else:
            thr = torch.full((S,), float(a.get("threshold", 0.0)))
        lens = [x.shape[0] for x in xs]
        rb = torch.tensor([sum(lens[:i]) for i in range(S)], dtype=torch.int32)
        x = torch.cat([x.float() for x in xs]).contiguous()
        off = torch.stack([o.to(dev, torch.int32) for o in offsets_list]).contiguous()
        t = lambda v, dt=torch.int32: torch.tensor(v, dtype=dt).to(dev)  # noqa: E731
        ftab, btab = t(_enc_f(f)), t(_enc_g(g))
        rb, thr = rb.to(dev), thr.to(dev)
        h = _native.hip()
        out = h.spv_fwd(x, rb, off, thr, ftab, S, B, ints, fl)
        q = qvals.float().reshape(B, -1).contiguous() if has_q else None
        ctx.save_for_backward(x, rb, off, btab, cv, q if q is not None else torch.zeros(0))
        ctx.meta = (S, B, ints, fl, lens, has_q)
        return tuple(out.unbind(0))

    @staticmethod
    def backward(ctx, *douts):
        x, rb, off, btab, cv, q = ctx.saved_tensors
        S, B, ints, fl, lens, has_q = ctx.meta
        W = ints[9] * ints[11]
        d = torch.stack([dd.float() if dd is not None else x.new_zeros(B, W) for dd in douts]).contiguous()
        dx = _native.hip().spv_bwd(x, rb, off, btab, d, cv, q if has_q else None, S, B, ints, fl)
        return (None, None, None, None, None, None) + tuple(dx.split(lens))


def seqpool_cvm_variant(op_type: str, xs: Sequence[torch.Tensor], offsets: Sequence[torch.Tensor], B: int,
                        cvm_in: torch.Tensor, attrs: Dict, qvals: Optional[torch.Tensor] = None) -> List[torch.Tensor]:
    variant = _VARIANT[op_type]
    if xs and xs[0].is_cuda:
        return list(_SeqpoolCvmVariantHip.apply(cvm_in, variant, dict(attrs), list(offsets), B, qvals,
                                                *[x.float() for x in xs]))
    return list(_SeqpoolCvmVariant.apply(cvm_in, variant, dict(attrs), list(offsets), B, qvals,
                                         *[x.float() for x in xs]))


# ================================================================== masked data_norm
class _MaskedDataNorm(torch.autograd.Function):
    """masked_data_norm (operators/masked_data_norm_op.cu:39-130)."""

    @staticmethod
    def forward(ctx, x, mask, bsize, bsum, bsq, sw, bias, eps, decay, group, update, training):
        means = bsum / bsize
        scales = torch.sqrt(bsize / bsq)
        m = (mask > 0).unsqueeze(1)
        y = torch.where(m, (x - means) * scales, torch.zeros_like(x))
        if sw is not None:
            y = torch.where(m, y * sw + bias, y)
        ctx.save_for_backward(x, mask, means, scales, bsize, bsum, bsq, sw if sw is not None else torch.zeros(0))
        ctx.eps, ctx.decay, ctx.group, ctx.update, ctx.training = eps, decay, group, update, training
        ctx.has_sw = sw is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mask, means, scales, bsize, bsum, bsq, sw = ctx.saved_tensors
        m = (mask > 0).unsqueeze(1)
        g = dy * sw if ctx.has_sw else dy
        dx = torch.where(m, g * scales, torch.zeros_like(dy))
        n = m.sum()
        xm = x * m
        stats = torch.stack([
            (n > 0).to(x.dtype).expand(x.shape[1]),
            xm.sum(0) / n.clamp(min=1),
            (((x - means) ** 2) * m).sum(0) / n.clamp(min=1) + ctx.eps * (n > 0).to(x.dtype),
        ])
        _dn_update(stats, ctx.group, ctx.update, ctx.training, ctx.decay, bsize, bsum, bsq)
        dsw = dbias = None
        if ctx.has_sw:
            xn = torch.where(m, (x - means) * scales, torch.zeros_like(x))
            dsw = (dy * xn).sum(0)
            dbias = (dy * m).sum(0)
        return dx, None, None, None, None, dsw, dbias, None, None, None, None, None


def _dn_update(stats, group, update, training, decay, bsize, bsum, bsq):
    if group is not None and collective_active(group):
        dist.all_reduce(stats, group=group)
    if update and training:
        upd = stats[0] > 0
        with torch.no_grad():
            bsize.copy_(torch.where(upd, bsize * decay + stats[0], bsize))
            bsum.copy_(torch.where(upd, bsum * decay + stats[1], bsum))
            bsq.copy_(torch.where(upd, bsq * decay + stats[2], bsq))


class _MaskedDataNormHip(torch.autograd.Function):
    """GPU masked_data_norm: k_mdn_fwd normalises and emits per-block masked
    statistic partials in the same pass (reduced by k_mdn_stats), k_mdn_bwd
    produces dx and the scale/bias gradient partials; the summary update of
    the reference's backward (masked_data_norm_op.cu:200-290) uses the
    statistics computed in the forward."""

    @staticmethod
    def forward(ctx, x, mask, bsize, bsum, bsq, sw, bias, eps, decay, group, update, training):
        h = _native.hip()
        y, stats = h.masked_dn_fwd(x, mask, bsize, bsum, bsq, sw, bias, eps)
        ctx.save_for_backward(x, mask, bsize, bsum, bsq, sw if sw is not None else torch.zeros(0))
        ctx.stats, ctx.has_sw = stats, sw is not None
        ctx.args = (group, update, training, decay)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mask, bsize, bsum, bsq, sw = ctx.saved_tensors
        dx, dsw, dbias = _native.hip().masked_dn_bwd(x, dy.float().contiguous(), mask, bsize, bsum, bsq,
                                                     sw if ctx.has_sw else None)
        group, update, training, decay = ctx.args
        _dn_update(ctx.stats, group, update, training, decay, bsize, bsum, bsq)
        return dx, None, None, None, None, dsw, dbias, None, None, None, None, None


def masked_data_norm(x, mask, bsize, bsum, bsq, sw, bias, eps, decay, group, update, training):
    if x.is_cuda:
        return _MaskedDataNormHip.apply(x.float().contiguous(), mask.float().reshape(-1).contiguous(), bsize, bsum,
                                        bsq, sw, bias, eps, decay, group, update, training)
    return _MaskedDataNorm.apply(x, mask, bsize, bsum, bsq, sw, bias, eps, decay, group, update, training)


# ================================================================== cross_norm_hadamard
def _cross_raw(x: torch.Tensor, F: int, E: int) -> torch.Tensor:
    """[B, F*(3E+1)] un-normalised [a, b, a*b, <a,b>] blocks."""
    B = x.shape[0]
    xv = x.reshape(B, F, 2, E)
    a, b = xv[:, :, 0], xv[:, :, 1]
    ab = a * b
    return torch.cat([a, b, ab, ab.sum(-1, keepdim=True)], -1).reshape(B, F * (3 * E + 1))


class _CrossNormHadamard(torch.autograd.Function):
    """cross_norm_hadamard (operators/cross_norm_hadamard.cu.h:44-240).

    Forward matches the reference.  The input gradient is the exact
    derivative of the forward; the reference kernel
    (``nncross_normbackpropagate_multi``) reads b's direct term from a's
    column block, which this implementation does not reproduce (no reference
    unit test pins that path)."""

    @staticmethod
    def forward(ctx, x, summary, F, E, eps, decay, group, training):
        raw = _cross_raw(x, F, E)
        means = summary[1] / summary[0]
        scales = torch.sqrt(summary[0] / summary[2])
        ctx.save_for_backward(x, raw, means, scales, summary)
        ctx.F, ctx.E, ctx.eps, ctx.decay, ctx.group, ctx.training = F, E, eps, decay, group, training
        return (raw - means) * scales

    @staticmethod
    def backward(ctx, dy):
        x, raw, means, scales, summary = ctx.saved_tensors
        F, E = ctx.F, ctx.E
        B = x.shape[0]
        g = (dy * scales).reshape(B, F, 3 * E + 1)
        xv = x.reshape(B, F, 2, E)
        a, b = xv[:, :, 0], xv[:, :, 1]
        ga = g[..., :E] + g[..., 2 * E:3 * E] * b + g[..., 3 * E:] * b
        gb = g[..., E:2 * E] + g[..., 2 * E:3 * E] * a + g[..., 3 * E:] * a
        dx = torch.stack([ga, gb], 2).reshape(B, F * 2 * E)
        stats = torch.stack([torch.ones_like(means), raw.mean(0), ((raw - means) ** 2).mean(0) + ctx.eps])
        if ctx.group is not None and collective_active(ctx.group):
            dist.all_reduce(stats, group=ctx.group)
        if ctx.training:
            with torch.no_grad():
                summary.mul_(ctx.decay).add_(stats)
        return dx, None, None, None, None, None, None, None


class _CrossNormHadamardHip(torch.autograd.Function):
    """GPU cross_norm_hadamard: k_cnh_fwd builds [a, b, a*b, <a,b>] per field,
    normalises with the running summary and emits the batch-statistic
    partials in the same pass; k_cnh_bwd is the exact input gradient."""

    @staticmethod
    def forward(ctx, x, summary, F, E, eps, decay, group, training):
        y, stats = _native.hip().cnh_fwd(x, summary, F, E, eps)
        ctx.save_for_backward(x, summary)
        ctx.stats, ctx.args = stats, (F, E, decay, group, training)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, summary = ctx.saved_tensors
        F, E, decay, group, training = ctx.args
        dx = _native.hip().cnh_bwd(x, dy.float().contiguous(), summary, F, E)
        stats = ctx.stats
        if group is not None and collective_active(group):
            dist.all_reduce(stats, group=group)
        if training:
            with torch.no_grad():
                summary.mul_(decay).add_(stats.reshape(summary.shape))
        return dx, None, None, None, None, None, None, None


def cross_norm_hadamard(x, summary, F, E, eps, decay, group=None, training=True):
    if x.is_cuda and 2 * F * (3 * E + 1) * 4 <= 64 * 1024:
        return _CrossNormHadamardHip.apply(x.float().contiguous(), summary, F, E, eps, decay, group, training)
    return _CrossNormHadamard.apply(x, summary, F, E, eps, decay, group, training)


# ================================================================== rank_attention
def _rank_gather(x, rank_offset, W, max_rank):
    """Per instance i and peer k: (x[index_k] masked, W block (lower*R+faster_k))."""
    B, C = x.shape
    R = max_rank
    ro = rank_offset.long()
    lower = ro[:, 0] - 1
    P = W.shape[1]
    Wb = W.reshape(R * R, C, P)
    xs, ws, valid = [], [], []
    for k in range(R):
        faster = ro[:, 2 * k + 1] - 1
        raw = ro[:, 2 * k + 2]
        idx = raw.clamp(0, B - 1)
        ok = (lower >= 0) & (lower < R) & (faster >= 0) & (faster < R) & (raw >= 0) & (raw < B)
        blk = torch.where(ok, lower * R + faster, torch.zeros_like(lower))
        xs.append(x[idx] * ok.unsqueeze(1).to(x.dtype))
        ws.append(blk)
        valid.append(ok)
    return xs, ws, valid, Wb


def rank_attention(x: torch.Tensor, rank_offset: torch.Tensor, W: torch.Tensor, max_rank: int) -> torch.Tensor:
    """out[i] = sum_k [valid] x[index_k] @ W[(lower*R + faster_k)*C : +C]
    (rank_attention.cu.h:28-190 / numpy ref test_rank_attention_op.py:25-110)."""
    if x.is_cuda and 1 <= max_rank <= 8:
        return _RankAttentionHip.apply(x.float().contiguous(), rank_offset.to(torch.int32).contiguous(), W,
                                       max_rank)
    xs, blks, _, Wb = _rank_gather(x, rank_offset, W, max_rank)
    out = 0
    for xk, bk in zip(xs, blks):
        out = out + torch.bmm(xk.unsqueeze(1), Wb[bk]).squeeze(1)
    return out


class _RankAttentionHip(torch.autograd.Function):
    """GPU rank_attention, rank-bucketed (csrc/hip/ctr_ext.hip): k_ra_bucket
    counting-sorts the instances by their own rank; an instance of rank r uses
    only W_r = W[r*R*C:(r+1)*R*C], so each rank's tiles are dense GEMMs with
    the peer rows gathered on load -- k_ra_fwd (out = A W_r), k_ra_dexp
    (dout W_r^T scattered to the per-peer rows), k_ra_dx (the reference's
    gather-form merge, rank_attention.cu.h:120-190) and k_ra_dw (A^T dout per
    rank, split over instances)."""

    @staticmethod
    def forward(ctx, x, ro, W, R):
        h = _native.hip()
        out, bucket = h.rank_attention_fwd(x, ro, W.contiguous(), R)
        ctx.save_for_backward(x, ro, W, bucket)
        ctx.R = R
        return out

    @staticmethod
    def backward(ctx, dout):
        x, ro, W, bucket = ctx.saved_tensors
        h = _native.hip()
        dout = dout.contiguous()
        Wc = W.contiguous()
        # dW (per-rank A^T dout), then G + the gather merge, on the calling
        # stream (_ctr_side's default here: graphed R8 backward 41.3 us on one
        # stream vs 53.4 with dW on the side stream, R3 26.8 vs 37.2 --
        # profiles/r5_ctr_ops_side_ab_v2.txt)
        cur = torch.cuda.current_stream(dout.device)
        side = _ctr_side(dout.device, want=False)
        if side is cur:
            dx, dW = h.rank_attention_bwd(x, ro, Wc, dout, bucket, ctx.R, 0)
            return dx, None, dW, None
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            _, dW = h.rank_attention_bwd(x, ro, Wc, dout, bucket, ctx.R, 2)
        dx, _ = h.rank_attention_bwd(x, ro, Wc, dout, bucket, ctx.R, 1)
        cur.wait_stream(side)
        dW.record_stream(cur)  # allocated on the side stream, consumed here
        return dx, None, dW, None


# ================================================================== batch_fc
def _sg(A, B, C, M, N, K, batch, a_str, b_str, sC, ldc, bias=None, sBias=0, bias_scale=1.0):
    """C = A B (+ bias * bias_scale) through k_sgemm; strides are
    (batch, row, col) in elements, so permuted layouts need no copies."""
    _native.hip().sgemm(A, B, C, bias, M, N, K, batch, list(a_str), list(b_str), sC, ldc, sBias, bias_scale)
    return C


def _batch_fc_geom(mode, xs, ws):
    """Operand strides of the three batch_fc layouts as (batch, M, K, N, x
    strides, W strides, out strides (sC, ldc), bias stride, x shape)."""
    if mode == "default":  # x [P, N, in], W [P, in, out]
        P, N, I = xs
        O = ws[2]
        return P, N, I, O, (N * I, I, 1), (I * O, O, 1), (N * O, O), O, (P, N, O)
    if mode == "transpose":  # x [bc, N, in], W [in, bc*out]
        P, N, I = xs
        O = ws[1] // P
        return P, N, I, O, (N * I, I, 1), (O, P * O, 1), (N * O, O), O, (P, N, O)
    N, PI = xs  # batchcount: x [N, bc*in], W [in, bc*out]
    P = mode
    I, O = PI // P, ws[1] // P
    return P, N, I, O, (I, P * I, 1), (O, P * O, 1), (O, P * O), O, (N, P * O)


class _BatchFcHip(torch.autograd.Function):
    """GPU batch_fc (batch_fc_op.cu:195-567): every layout is one strided
    batched k_sgemm with the bias fused into the epilogue; backward is two
    more strided GEMMs (dx = dy W^T, dW = x^T dy) and a strided column sum."""

    @staticmethod
    def forward(ctx, x, W, b, mode):
        P, N, I, O, xst, wst, (sC, ldc), sb, oshape = _batch_fc_geom(mode, x.shape, W.shape)
        y = x.new_empty(oshape)
        # slots of at most 64 x 64 (CTR shapes): k_bfc_fwd keeps W_p in LDS and
        # streams x once; otherwise the strided batched k_mgemm
        st = [xst[0], xst[1], wst[0], wst[1], sC, ldc, sb]
        if not _native.hip().batch_fc_fwd(x, W, b, y, P, N, I, O, st):
            _sg(x, W, y, N, O, I, P, xst, wst, sC, ldc, b, sb)
        ctx.save_for_backward(x, W)
        ctx.geom, ctx.bshape = (P, N, I, O, xst, wst, sC, ldc, sb), b.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        x, W = ctx.saved_tensors
        P, N, I, O, xst, wst, sC, ldc, sb = ctx.geom
        dy = dy.float().contiguous()
        h = _native.hip()
        dx = torch.empty_like(x)
        # fused: dx, dW, db from one pass over x and dy (k_bfc_bwd + ordered reduce)
        dW = torch.empty_like(W)
        db = x.new_empty(ctx.bshape)
        if h.batch_fc_bwd(x, W, dy, dx, dW, db, P, N, I, O, [xst[0], xst[1], wst[0], wst[1], sC, ldc, sb]):
            return dx, dW, db, None
        # dx[p] (N x I) = dy[p] (N x O) . W[p]^T (O x I); dx shares x's strides
        _sg(dy, W, dx, N, I, O, P, (sC, ldc, 1), (wst[0], wst[2], wst[1]), xst[0], xst[1])
        # dW[p] (I x O) = x[p]^T (I x N) . dy[p] (N x O); dW shares W's strides
        _sg(x, dy, dW, I, O, N, P, (xst[0], xst[2], xst[1]), (sC, ldc, 1), wst[0], wst[1])
        h.colsum_strided(dy, P, N, O, sC, ldc, db, O, False)
        return dx, dW, db, None


def batch_fc(x: torch.Tensor, W: torch.Tensor, b: torch.Tensor, batchcount: int = 0,
             transpose_weight: bool = False) -> torch.Tensor:
    """batch_fc (operators/batch_fc_op.cu:195-330):
    * default: x [P, N, in], W [P, in, out], b [P, out] -> [P, N, out]
    * transpose_weight: x [bc, N, in], W [in, bc*out], b [1, bc*out] -> [bc, N, out]
    * batchcount>0: x [N, bc*in], W [in, bc*out], b [bc*out] -> [N, bc*out]
    """
    if x.is_cuda:
        mode = "transpose" if transpose_weight else (batchcount if batchcount > 0 else "default")
        return _BatchFcHip.apply(x.float().contiguous(), W.float().contiguous(), b.float().contiguous(), mode)
    if transpose_weight:
        bc = x.shape[0]
        od = W.shape[1] // bc
        Wb = W.reshape(W.shape[0], bc, od).permute(1, 0, 2)
        return torch.bmm(x, Wb) + b.reshape(bc, 1, od)
    if batchcount > 0:
        N = x.shape[0]
        inf = x.shape[1] // batchcount
        of = W.shape[1] // batchcount
        xb = x.reshape(N, batchcount, inf).permute(1, 0, 2)
        Wb = W.reshape(inf, batchcount, of).permute(1, 0, 2)
        y = torch.bmm(xb, Wb).permute(1, 0, 2).reshape(N, batchcount * of)
        return y + b.reshape(1, -1)
    return torch.baddbmm(b.unsqueeze(1), x, W)


# ================================================================== scaled fc family
def _ctr_side(device, want: bool = True):
    """Side stream of a CTR op backward: its weight-gradient GEMM runs there
    beside the input-gradient GEMM, or -- ``want`` False, or
    PBX_CTR_BWD_SIDE=0/1 forcing either way -- the calling stream.  Measured
    GPU time of the graphed backward, side vs one stream
    (profiles/r5_ctr_ops_side_ab.txt, r5_ctr_ops_side_ab_v2.txt after the
    rank_attention / split-K dW rework): scaled_fc 76.7 vs 62.2 us,
    scaled_int8fc 97.3 vs 82.3, rank_attention R8 53.4 vs 41.3, R3 37.2 vs
    26.8 -- both halves fill the GPU alone, so every op defaults to one stream."""
    from ..runtime.streams import side_stream

    force = os.environ.get("PBX_CTR_BWD_SIDE", "")
    if force in ("0", "1"):
        want = force == "1"
    return side_stream(device, "ctr_bwd") if want else torch.cuda.current_stream(device)


def _fc_backward_hip(x, W, dy):
    """dx = dy W^T, dW = x^T dy, db = colsum(dy) for x [N, K], W [K, O]."""
    N, K = x.shape
    O = W.shape[1]
    dy = dy.float().contiguous()
    dx = x.new_empty(N, K)
    _sg(dy, W, dx, N, K, O, 1, (0, O, 1), (0, 1, O), 0, K)
    dW = W.new_empty(K, O)
    _sg(x, dy, dW, K, O, N, 1, (0, 1, K), (0, O, 1), 0, O)
    db = W.new_empty(O)
    _native.hip().colsum_strided(dy, 1, N, O, 0, O, db, 0, False)
    return dx, dW, db


def scaled_fc_reference(x, W, b, in_scale, bias_scale):
    """The reference forward's arithmetic (scaled_fc_op.cu:144-227) in torch:
    fp16 operands, fp32-accumulated GEMM scaled by fp16(in_scale) and rounded
    to fp16, + fp16(fp16(bias) * fp16(bias_scale)) in fp16, then fp32 * 1/in_scale
    with inf -> NaN."""
    h = torch.float16
    acc = x.to(h).float() @ W.to(h).float()
    v = (float(torch.tensor(in_scale, dtype=h)) * acc).to(h)
    bb = (b.reshape(-1).to(h).float() * float(torch.tensor(bias_scale, dtype=h))).to(h)
    v = (v.float() + bb.float().reshape(1, -1)).to(h)
    y = v.float() * (1.0 / in_scale)
    return torch.where(torch.isinf(y), torch.full_like(y, float("nan")), y)


_MM16 = [None]  # torch.mm(fp16, fp16, out_dtype=float32) works on this build: None (untried) / True / False


def _mm16(a16, b16):
    """fp16 x fp16 -> fp32 (fp32 accumulate) on the library GEMM, or None
    when this torch build has no mixed-dtype mm (then k_hgemm runs)."""
    if _MM16[0] is False:
        return None
    try:
        r = torch.mm(a16, b16, out_dtype=torch.float32)
    except (RuntimeError, TypeError, NotImplementedError):
        _MM16[0] = False
        return None
    _MM16[0] = True
    return r.contiguous()


def _half_of(W: torch.Tensor, transposed: bool = False) -> torch.Tensor:
    """fp16 copy of a weight (transposed: of W^T, contiguous), cached on the
    tensor until it is modified in place (its version counter moves) -- one
    cast per optimizer step, not per forward."""
    key = (W._version, W.data_ptr(), tuple(W.shape))
    attr = "_pbx_half_t" if transposed else "_pbx_half"
    c = getattr(W, attr, None)
    if c is not None and c[0] == key:
        return c[1]
    W16 = (W.detach().t() if transposed else W.detach()).contiguous().half()
    try:
        setattr(W, attr, (key, W16))
    except (AttributeError, RuntimeError):
        pass
    return W16


def _sfc_dw_splits(N: int, K: int, O: int) -> int:
    """Workgroups per 80 x 80 dW tile of k_sfc_dw (split-K over the batch):
    about one workgroup per CU over the whole launch, at least 256 rows of
    the batch each; PBX_SFC_DW_SPLIT overrides."""
    env = os.environ.get("PBX_SFC_DW_SPLIT", "")
    if env:
        return max(1, int(env))
    tiles = ((K + 79) // 80) * ((O + 79) // 80)
    # ~200 workgroups (one per CU): N = 8192, 400 x 400 (25 tiles) -> 8 splits,
    # 25.5 us vs 28.5 at 16 and 34.6 at 20 (profiles/r6_ctr_bwd_kernels.txt)
    return max(1, min(200 // tiles, N // 256, 64))


class _ScaledFc(torch.autograd.Function):
    """scaled_fc (operators/scaled_fc_op.cu:144-330) with the reference's
    fp16 arithmetic on fp16 MFMA (csrc/hip/ctr_ext.hip k_hgemm):
      forward  y = fp32(fp16(fp16(in_scale) * x16 @ W16) + fp16(b16 * bs16)) / in_scale
      backward d16 = fp16(dy * grad_scale / in_scale);
               dx = fp32(fp16(fp16(in_scale) * d16 @ W16^T)) / grad_scale,
               dW = fp32(fp16(fp16(in_scale) * x16^T @ d16)) / grad_scale,
               db = colsum(dy) (fp32);  inf -> NaN on every cast back.
    CPU tensors run the same arithmetic in torch."""

    @staticmethod
    def forward(ctx, x, W, b, in_scale, bias_scale, grad_scale):
        ctx.bshape = b.shape
        ctx.sc = (in_scale, grad_scale)
        ctx.half_ops = False
        ctx.fused = False
        if x.is_cuda:
            N, K = x.shape
            O = W.shape[1]
            # one launch: the x cast, fp16 MFMA GEMM and fp16 epilogue fused (k_sfc)
            y = _native.hip().sfc(x, _half_of(W, True), b.reshape(-1), 1.0, in_scale, bias_scale, 1.0 / in_scale)
            if y is not None:
                ctx.save_for_backward(x, W)
                ctx.fused = True
                return y
            x16, W16 = x.half(), _half_of(W)
            acc = _mm16(x16, W16)
            if acc is not None:  # library fp16 GEMM (fp32 accumulate) + the fp16 epilogue
                _native.hip().h16_epi(acc, b.reshape(-1), in_scale, bias_scale, 1.0 / in_scale)
                ctx.save_for_backward(x16, W16)  # the backward's fp16 operands, cast once
                ctx.half_ops = True
                return acc
            ctx.save_for_backward(x, W)
            y = x.new_empty(N, O)
            _native.hip().hgemm(x, W, y, b.reshape(-1), N, O, K, [K, 1], [O, 1], O, 1.0, 1.0, in_scale, bias_scale,
                                1.0 / in_scale, 1)
            return y
        ctx.save_for_backward(x, W)
        return scaled_fc_reference(x, W, b, in_scale, bias_scale)

    @staticmethod
    def backward(ctx, dy):
        x, W = ctx.saved_tensors
        in_scale, gs = ctx.sc
        dy = dy.float().contiguous()
        N, K = x.shape
        O = W.shape[1]
        if ctx.fused:
            h = _native.hip()
            # dx = fp16(dy * gs / in_scale) @ W16^T in one launch (k_sfc, Bk = W16
            # [K, O]); dW = x16^T d16 in one split-K launch (k_hgemm: both casts
            # and the reference fp16 epilogue in the kernel, ~256 rows of N per
            # split) and db = colsum(dy) -- on _ctr_side's stream choice
            cur = torch.cuda.current_stream(dy.device)
            side = _ctr_side(dy.device, want=False)
            side.wait_stream(cur)
            dW = W.new_empty(K, O)
            db = dy.new_empty(O)
            if K % 4 == 0 and O % 8 == 0:  # k_sfc_dw (K, O % 4) and the dx k_sfc (O % 8)
                # dW and db in one launch (k_sfc_dw: split-K over N with a
                # fixed-order reduce), on _ctr_side's stream beside dx when
                # PBX_CTR_BWD_SIDE=1 (k_sfc_dw holds ~one workgroup per CU)
                with torch.cuda.stream(side):
                    ok = h.sfc_dw(x, dy, dW, db, 1.0, gs / in_scale, in_scale, 1.0 / gs, _sfc_dw_splits(N, K, O))
                if ok:
                    dx = h.sfc(dy, _half_of(W), None, gs / in_scale, in_scale, 1.0, 1.0 / gs)
                    cur.wait_stream(side)  # (everything side touched is ordered before cur's later work)
                    if dx is not None:
                        return dx, dW, db.reshape(ctx.bshape), None, None, None
            dx = h.sfc(dy, _half_of(W), None, gs / in_scale, in_scale, 1.0, 1.0 / gs)
            if dx is not None:
                with torch.cuda.stream(side):
                    # ~512 rows of N per split (scripts/micro/dw_gemm_sweep.py at
                    # N = 8192, 400 x 400: 4 splits 73 us, 8 44.7, 16 39.9, 32 42.7)
                    h.hgemm(x, dy, dW, None, K, O, N, [1, K], [O, 1], O, 1.0, gs / in_scale, in_scale, 1.0, 1.0 / gs,
                            max(1, min(64, N // 512)))
                    h.colsum_strided(dy, 1, N, O, 0, O, db, 0, False)
                cur.wait_stream(side)
                return dx, dW, db.reshape(ctx.bshape), None, None, None
            cur.wait_stream(side)
        if ctx.half_ops:  # x, W are the forward's fp16 casts
            h = _native.hip()
            d16 = (dy * (gs / in_scale)).half()
            dxa = _mm16(d16, W.t())
            dWa = _mm16(x.t(), d16) if dxa is not None else None
            if dWa is not None:
                h.h16_epi(dxa, None, in_scale, 1.0, 1.0 / gs)
                h.h16_epi(dWa, None, in_scale, 1.0, 1.0 / gs)
                db = dy.new_empty(O)
                h.colsum_strided(dy, 1, N, O, 0, O, db, 0, False)
                return dxa, dWa, db.reshape(ctx.bshape), None, None, None
            x, W = x.float(), W.float()  # fp16 values are exact in fp32: the kernel path below recasts
        if x.is_cuda:
            h = _native.hip()
            dx = x.new_empty(N, K)
            # dx [N, K] = d16 [N, O] @ W16^T: B[o][k] = W[k][o]
            h.hgemm(dy, W, dx, None, N, K, O, [O, 1], [1, O], K, gs / in_scale, 1.0, in_scale, 1.0, 1.0 / gs, 1)
            dW = W.new_empty(K, O)
            # dW [K, O] = x16^T [K, N] @ d16 [N, O]: A[k][n] = x[n][k]; split over N
            h.hgemm(x, dy, dW, None, K, O, N, [1, K], [O, 1], O, 1.0, gs / in_scale, in_scale, 1.0, 1.0 / gs,
                    max(1, min(16, N // 512)))
            db = W.new_empty(O)
            h.colsum_strided(dy, 1, N, O, 0, O, db, 0, False)
            return dx, dW, db.reshape(ctx.bshape), None, None, None
        hf = torch.float16
        a16 = float(torch.tensor(in_scale, dtype=hf))
        d16 = (dy * (gs / in_scale)).to(hf).float()

        def back(v):
            y = (a16 * v).to(hf).float() * (1.0 / gs)
            return torch.where(torch.isinf(y), torch.full_like(y, float("nan")), y)

        dx = back(d16 @ W.to(hf).float().t())
        dW = back(x.to(hf).float().t() @ d16)
        return dx, dW, dy.sum(0).reshape(ctx.bshape), None, None, None


def scaled_fc(x, W, b, in_scale, bias_scale, grad_scale=256.0):
    if x.is_cuda:
        x, W, b = x.float().contiguous(), W.float().contiguous(), b.float().contiguous()
    return _ScaledFc.apply(x, W, b, in_scale, bias_scale, grad_scale)


def int8_quantize(v: torch.Tensor, expand: float, clip: float, rng: float) -> torch.Tensor:
    """kernel_cast_and_padding (scaled_int8fc_op.cu:38-80): clip(v*expand, +-clip)
    quantised with interval 2*clip/range, trunc(v/interval + 0.5)."""
    e = v * expand
    e = torch.where(e >= 1e-6, torch.where(e - clip > 1e-6, torch.full_like(e, clip), e),
                    torch.where(e + clip < 1e-6, torch.full_like(e, -clip), e))
    interval = 2 * clip / rng
    return torch.trunc(e / interval + 0.5).clamp(-128, 127)


class _ScaledInt8Fc(torch.autograd.Function):
    """scaled_int8fc: int8 GEMM forward, fp32 straight-through backward
    (scaled_int8fc_op.cu:290-440).  Output scale reproduces the reference's
    cast_and_cut: acc * (2*input_clip/range) / (input_expand*weight_expand)."""

    @staticmethod
    def forward(ctx, x, W, b, a):
        rng = a["int8_range"]
        ctx.save_for_backward(x, W)
        ctx.bshape = b.shape
        if x.is_cuda:  # k_i8_quant x2 + k_i8_gemm (int8 MFMA, dequantising epilogue)
            return _native.hip().int8_fc(x, W, b.reshape(-1), a["input_expand_factor"], a["input_clip_factor"],
                                         a["weight_expand_factor"], a["weight_clip_factor"], rng)
        qx = int8_quantize(x, a["input_expand_factor"], a["input_clip_factor"], rng)
        qw = int8_quantize(W, a["weight_expand_factor"], a["weight_clip_factor"], rng)
        acc = qx.double() @ qw.double()
        interval = 2 * a["input_clip_factor"] / rng
        y = acc.float() / (a["input_expand_factor"] * a["weight_expand_factor"]) * interval
        return y + b.reshape(1, -1)

    @staticmethod
    def backward(ctx, dy):
        x, W = ctx.saved_tensors
        if x.is_cuda:
            # the reference straight-through backward is two fp32 GEMMs
            # (scaled_int8fc_op.cu:382-440), which its cuBLAS runs in TF32 in
            # training (gpu_context.cc:61-67, enable_cublas_tf32_op_math on).
            # Default here: exact fp32 library GEMMs (dW split-K batched with
            # a fixed-order sum).  PBX_INT8FC_BWD=bf16x3: both as three bf16
            # MFMA products of the operands' bf16 splits (~2^-16 relative per
            # product, tighter than TF32): dx in k_f3gemm_nt against W's split
            # (cached per optimizer step), dW + db in one k_sfc_dw launch --
            # measured slower than the library so far (dx 37 vs 36 us, dW 63
            # vs ~40 at 8192 x 512 x 512, profiles/r6_ctr_bwd_kernels.txt).
            dy = dy.float().contiguous()
            N, O = dy.shape
            K = x.shape[1]
            dW = torch.empty_like(W)
            db = dy.new_empty(O)
            h = _native.hip()
            if os.environ.get("PBX_INT8FC_BWD", "fp32") == "bf16x3":
                Wh, Wl = _bf16_split_of(W)
                dx = h.f3gemm_nt(dy, Wh, Wl)
                if dx is not None and h.sfc_dw(x, dy, dW, db, 1.0, 1.0, 1.0, 1.0, _sfc_dw_splits(N, K, O), mode=1):
                    return dx, dW, db.reshape(ctx.bshape), None
            cur = torch.cuda.current_stream(dy.device)
            side = _ctr_side(dy.device, want=False)
            side.wait_stream(cur)
            dx = torch.mm(dy, W.t())
            with torch.cuda.stream(side):
                _mm_tn_splitk(x, dy, dW)
                h.colsum_strided(dy, 1, N, O, 0, O, db, 0, False)
            cur.wait_stream(side)
        else:
            dx, dW, db = dy @ W.t(), x.t() @ dy, dy.sum(0)
        return dx, dW, db.reshape(ctx.bshape), None


def _bf16_split_of(W: torch.Tensor):
    """(hi, lo) bf16 split of an fp32 weight, W = hi + lo + O(2^-17 |W|)
    (round-to-nearest-even both times), cached on the tensor until it is
    modified in place -- one split per optimizer step."""
    key = (W._version, W.data_ptr(), tuple(W.shape))
    c = getattr(W, "_pbx_bf16_split", None)
    if c is not None and c[0] == key:
        return c[1]
    Wd = W.detach().contiguous()
    hi = Wd.to(torch.bfloat16)
    lo = (Wd - hi.float()).to(torch.bfloat16)
    try:
        setattr(W, "_pbx_bf16_split", (key, (hi, lo)))
    except (AttributeError, RuntimeError):
        pass
    return hi, lo


def _mm_tn_splitk(x: torch.Tensor, dy: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    """out = x^T dy for a long shared dimension N (a weight gradient over the
    batch): S library GEMMs over contiguous row blocks in one batched call,
    then their fixed-order sum -- deterministic, and at N = 8192, 512 x 512
    39.7 us vs 57.6 for the single library GEMM, whose tile choice leaves the
    long K serial (scripts/micro/dw_gemm_sweep.py; split 2 45.7, 4 41.1,
    16 41.2)."""
    N, K = x.shape
    S = 8
    while S > 1 and (N % S or N // S < 512):
        S //= 2
    if S == 1:
        return torch.mm(x.t(), dy, out=out)
    part = torch.bmm(x.reshape(S, N // S, K).transpose(1, 2), dy.reshape(S, N // S, dy.shape[1]))
    return torch.sum(part, 0, out=out)


def scaled_int8fc(x, W, b, attrs):
    if x.is_cuda:
        x, W, b = x.float().contiguous(), W.float().contiguous(), b.float().contiguous()
    return _ScaledInt8Fc.apply(x, W, b, dict(attrs))


# ================================================================== concat family
def partial_concat(xs: Sequence[torch.Tensor], start: int, length: int) -> torch.Tensor:
    """partial_concat (test_partial_concat_op.py np_partial_concat)."""
    size = xs[0].shape[1]
    if start < 0:
        start += size
    if length < 0:
        length = size - start
    return torch.cat([x[:, start:start + length] for x in xs], 1)


def partial_sum(xs: Sequence[torch.Tensor], start: int, length: int) -> torch.Tensor:
    size = xs[0].shape[1]
    if start < 0:
        start += size
    end = size if length < 0 else start + length
    out = xs[0][:, start:end]
    for x in xs[1:]:
        out = out + x[:, start:end]
    return out


def fused_concat(xs: Sequence[torch.Tensor], offset: int, length: int) -> torch.Tensor:
    """fused_concat (fused_concat_op.cu FusedColsConcatKernel): equal-width inputs,
    columns [offset, offset+length) of each, concatenated."""
    return torch.cat([x[:, offset:offset + length] for x in xs], 1)


def fused_seqpool_concat(groups: Sequence[Sequence[torch.Tensor]], col_ranges) -> List[torch.Tensor]:
    """fused_seqpool_concat (fused_concat_op.cu:34-115): output j = concat over
    groups i of groups[i][j][:, start_i:start_i+dim_i]."""
    n = len(groups[0])
    return [torch.cat([g[j][:, s:s + d] for g, (s, d) in zip(groups, col_ranges)], 1) for j in range(n)]


def shuffle_batch(x: torch.Tensor, gen: Optional[torch.Generator] = None) -> torch.Tensor:
    perm = torch.randperm(x.shape[0], generator=gen, device=gen.device if gen is not None else x.device) \
        if gen is not None else torch.randperm(x.shape[0], device=x.device)
    return x[perm.to(x.device)]


# ================================================================== fused_seq_tensor
def fused_seq_tensor(x: torch.Tensor, ad: torch.Tensor, batch_count: int, max_length: int, slot_num: int,
                     fea_emb_dim: int, ad_slot_num: int, ad_slot_offset: int):
    """DIN sequence tensors (fused_seq_tensor_op.cu): Input [ins, bc*slot*T*E],
    ADInput [ins, bc*ad_slot*E] -> DINOut [bc, ins*T, 4*ad_slot*E] =
    [seq, ad, seq-ad, seq*ad], MaskOut [bc, ins, T], SideInfoOut
    [bc, ins*T, side_slot*E], ADSlotSessionOut [bc, ins*T, ad_slot, E]."""
    ins = x.shape[0]
    bc, T, E, S, A = batch_count, max_length, fea_emb_dim, slot_num, ad_slot_num
    if x.is_cuda:  # k_fused_seq_tensor: all four outputs in one pass
        din, mask, side, sess = _native.hip().fused_seq_tensor(x.float(), ad.float(), bc, T, E, S, A, ad_slot_offset)
        sess = sess.reshape(bc, ins * T, A, E)
        if bc == 1:
            return (din.reshape(ins, T, 4 * A * E), mask.reshape(ins, T), side.reshape(ins, T, (S - A) * E),
                    sess.reshape(ins, T, A * E))
        return din, mask, side, sess
    xv = x.reshape(ins, bc, S, T, E).permute(1, 0, 3, 2, 4)  # [bc, ins, T, S, E]
    adv = ad.reshape(ins, bc, A, E).permute(1, 0, 2, 3).unsqueeze(2)  # [bc, ins, 1, A, E]
    seq = xv[:, :, :, ad_slot_offset:ad_slot_offset + A]  # [bc, ins, T, A, E]
    adb = adv.expand_as(seq)
    din = torch.cat([seq, adb, seq - adb, seq * adb], 3).reshape(bc, ins * T, 4 * A * E)
    side_off = A if ad_slot_offset == 0 else 0
    side = xv[:, :, :, side_off:side_off + (S - A)].reshape(bc, ins * T, (S - A) * E)
    mask = (xv.sum((3, 4)).abs() > 1e-8).to(x.dtype)  # [bc, ins, T]
    sess = seq.reshape(bc, ins * T, A, E)
    if bc == 1:
        din = din.reshape(ins, T, 4 * A * E)
        mask = mask.reshape(ins, T)
        side = side.reshape(ins, T, (S - A) * E)
        sess = sess.reshape(ins, T, A * E)
    return din, mask, side, sess
