"""Op kernels for the fluid executor.

A kernel is ``fn(ctx, op)``: it reads its inputs from ``ctx`` (torch tensors
or :class:`Ragged` LoD values) and writes its outputs back.  Autograd
provides every backward; ops whose backward is a side effect (the sparse
push, data_norm summary updates) use custom ``autograd.Function`` s from
``paddlebox_amd.ops``.  GPU tensors go to the hand-written gfx950 kernels
where one exists (pull/push, seqpool-CVM, data_norm, fused MLP, CTR-op
family); generic tensor algebra (concat, reshape, elementwise, reductions)
runs on PyTorch-ROCm.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Dict, List, Optional

import numpy as np
import torch
import torch.nn.functional as F

from ..ops import ctr as ctr_ops
from ..ops import ctr_ext
from ..ops import sparse as sparse_ops
from ..ps.sparse_engine import SeqpoolParams
from .framework import torch_dtype

KERNELS: Dict[str, Callable] = {}


def kernel(*names):
    def deco(fn):
        for n in names:
            KERNELS[n] = fn
        return fn

    return deco


@dataclass
class Ragged:
    """Level-1 LoD value: rows ``values[offsets[b]:offsets[b+1]]`` belong to
    instance b.  ``slot`` is the batch slot index for data variables."""

    values: torch.Tensor
    offsets: torch.Tensor  # int64 [B+1], offsets[0] == 0
    B: int
    slot: int = -1

    @property
    def shape(self):
        return self.values.shape


class LazyRagged(Ragged):
    """A batch slot as Ragged whose rebased offsets (``lod_row - base``) are
    only computed when an op reads them: the fused pull consumes the batch's
    flat keys and lod directly, so a captured step carries no per-slot
    offset kernels."""

    def __init__(self, values, lod_row, base: int, B: int, slot: int):
        self.values, self.B, self.slot = values, B, slot
        self._lod_row, self._base, self._offs = lod_row, base, None

    @property
    def offsets(self):
        if self._offs is None:
            self._offs = self._lod_row - self._base
        return self._offs

    @offsets.setter
    def offsets(self, v):
        self._offs = v


def _val(x):
    return x.values if isinstance(x, Ragged) else x


# ----------------------------------------------------------------- startup
@kernel("init_param")
def k_init_param(ctx, op):
    v = op.outputs["Out"][0]
    shape = [max(1, s) for s in v.shape]
    t = torch.empty(shape, dtype=torch_dtype(v.dtype))
    op.attrs["initializer"](t, ctx.generator)
    ctx.scope.set(v.name, t.to(ctx.device))


# ----------------------------------------------------------------- constants
def _batch(ctx) -> int:
    return ctx.B


@kernel("fill_constant")
def k_fill_constant(ctx, op):
    shape = [ctx.B if s < 0 else s for s in op.attrs["shape"]]
    ctx.set(op.outputs["Out"][0], torch.full(shape, op.attrs["value"], dtype=torch_dtype(op.attrs["dtype"]),
                                             device=ctx.device))


@kernel("fill_constant_batch_size_like")
def k_fill_bs_like(ctx, op):
    x = _val(ctx.get(op.inputs["Input"][0]))
    shape = list(op.attrs["shape"])
    shape[op.attrs["output_dim_idx"]] = x.shape[op.attrs["input_dim_idx"]]
    ctx.set(op.outputs["Out"][0], torch.full(shape, op.attrs["value"], dtype=torch_dtype(op.attrs["dtype"]),
                                             device=ctx.device))


@kernel("fill_zeros_like")
def k_zeros_like(ctx, op):
    ctx.set(op.outputs["Out"][0], torch.zeros_like(_val(ctx.get(op.inputs["X"][0]))))


@kernel("fill_ones_like")
def k_ones_like(ctx, op):
    ctx.set(op.outputs["Out"][0], torch.ones_like(_val(ctx.get(op.inputs["X"][0]))))


@kernel("assign")
def k_assign(ctx, op):
    ctx.set(op.outputs["Out"][0], ctx.get(op.inputs["X"][0]))


@kernel("cast")
def k_cast(ctx, op):
    x = ctx.get(op.inputs["X"][0])
    dt = torch_dtype(op.attrs["out_dtype"])
    if isinstance(x, Ragged):
        ctx.set(op.outputs["Out"][0], Ragged(x.values.to(dt), x.offsets, x.B, x.slot))
    else:
        ctx.set(op.outputs["Out"][0], x.to(dt))


# ----------------------------------------------------------------- elementwise
_UNARY = {
    "relu": torch.relu, "sigmoid": torch.sigmoid, "tanh": torch.tanh, "exp": torch.exp, "log": torch.log,
    "sqrt": torch.sqrt, "square": torch.square, "abs": torch.abs,
}


@kernel(*_UNARY)
def k_unary(ctx, op):
    x = ctx.get(op.inputs["X"][0])
    f = _UNARY[op.type]
    if isinstance(x, Ragged):
        ctx.set(op.outputs["Out"][0], Ragged(f(x.values.float()), x.offsets, x.B, x.slot))
    else:
        ctx.set(op.outputs["Out"][0], f(x.float() if x.dtype == torch.bfloat16 else x))


@kernel("softmax")
def k_softmax(ctx, op):
    ctx.set(op.outputs["Out"][0], torch.softmax(_val(ctx.get(op.inputs["X"][0])), op.attrs.get("axis", -1)))


@kernel("leaky_relu")
def k_leaky(ctx, op):
    ctx.set(op.outputs["Out"][0], F.leaky_relu(_val(ctx.get(op.inputs["X"][0])), op.attrs["alpha"]))


@kernel("clip")
def k_clip(ctx, op):
    ctx.set(op.outputs["Out"][0], torch.clamp(_val(ctx.get(op.inputs["X"][0])), op.attrs["min"], op.attrs["max"]))


@kernel("dropout")
def k_dropout(ctx, op):
    x = _val(ctx.get(op.inputs["X"][0]))
    p = op.attrs["dropout_prob"]
    test = op.attrs.get("is_test") or not ctx.training
    if op.attrs.get("dropout_implementation") == "upscale_in_train":
        y = x if test else F.dropout(x, p, True)
    else:  # downgrade_in_infer
        y = x * (1.0 - p) if test else x * (torch.rand_like(x) >= p).to(x.dtype)
    ctx.set(op.outputs["Out"][0], y)


@kernel("scale")
def k_scale(ctx, op):
    x = ctx.get(op.inputs["X"][0])
    s, b = op.attrs["scale"], op.attrs["bias"]
    f = (lambda t: t * s + b) if op.attrs.get("bias_after_scale", True) else (lambda t: (t + b) * s)
    if isinstance(x, Ragged):
        ctx.set(op.outputs["Out"][0], Ragged(f(x.values), x.offsets, x.B, x.slot))
    else:
        ctx.set(op.outputs["Out"][0], f(x))


def _bcast(x: torch.Tensor, y: torch.Tensor, axis: int) -> torch.Tensor:
    """Paddle elementwise broadcast: y's dims align with x's starting at axis."""
    if axis == -1 or y.dim() == x.dim():
        return y
    shape = [1] * x.dim()
    for i, s in enumerate(y.shape):
        shape[axis + i] = s
    return y.reshape(shape)


_BINARY = {
    "elementwise_add": torch.add, "elementwise_sub": torch.sub, "elementwise_mul": torch.mul,
    "elementwise_div": torch.div, "elementwise_max": torch.maximum, "elementwise_min": torch.minimum,
    "elementwise_pow": torch.pow,
}


@kernel(*_BINARY)
def k_binary(ctx, op):
    x = _val(ctx.get(op.inputs["X"][0])).float()
    y = _val(ctx.get(op.inputs["Y"][0])).float()
    ctx.set(op.outputs["Out"][0], _BINARY[op.type](x, _bcast(x, y, op.attrs.get("axis", -1))))


@kernel("sum")
def k_sum(ctx, op):
    xs = [_val(ctx.get(v)).float() for v in op.inputs["X"]]
    out = xs[0]
    for x in xs[1:]:
        out = out + x
    ctx.set(op.outputs["Out"][0], out)


# ----------------------------------------------------------------- linear algebra
@kernel("fc")
def k_fc(ctx, op):
    x = _val(ctx.get(op.inputs["Input"][0])).float()
    w = ctx.param(op.inputs["W"][0])
    nd = op.attrs.get("in_num_col_dims", 1)
    lead = x.shape[:nd]
    x2 = x.reshape(int(np.prod(lead)), -1)
    b = ctx.param(op.inputs["Bias"][0]) if op.inputs.get("Bias") else None
    y = torch.addmm(b, x2, w) if b is not None else x2 @ w
    act = op.attrs.get("activation_type", "")
    if act:
        y = _UNARY[act](y)
    ctx.set(op.outputs["Out"][0], y.reshape(*lead, w.shape[1]))


@kernel("matmul", "matmul_v2")
def k_matmul(ctx, op):
    x = _val(ctx.get(op.inputs["X"][0])).float()
    y = _val(ctx.get(op.inputs["Y"][0])).float()
    if op.attrs.get("transpose_X") or op.attrs.get("trans_x"):
        x = x.transpose(-1, -2)
    if op.attrs.get("transpose_Y") or op.attrs.get("trans_y"):
        y = y.transpose(-1, -2)
    out = torch.matmul(x, y)
    a = op.attrs.get("alpha", 1.0)
    ctx.set(op.outputs["Out"][0], out * a if a != 1.0 else out)


@kernel("mul")
def k_mul(ctx, op):
    x = _val(ctx.get(op.inputs["X"][0])).float()
    y = _val(ctx.get(op.inputs["Y"][0])).float()
    xn, yn = op.attrs["x_num_col_dims"], op.attrs["y_num_col_dims"]
    x2 = x.reshape(int(np.prod(x.shape[:xn])), -1)
    y2 = y.reshape(int(np.prod(y.shape[:yn])), -1)
    ctx.set(op.outputs["Out"][0], (x2 @ y2).reshape(*x.shape[:xn], *y.shape[yn:]))


@kernel("lookup_table", "lookup_table_v2")
def k_lookup_table(ctx, op):
    ids = ctx.get(op.inputs["Ids"][0])
    w = ctx.param(op.inputs["W"][0])
    idv = _val(ids).reshape(-1).long()
    out = F.embedding(idv, w, padding_idx=None)
    pad = op.attrs.get("padding_idx", -1)
    if pad >= 0:
        out = out * (idv != pad).unsqueeze(1).to(out.dtype)
    ctx.set(op.outputs["Out"][0], Ragged(out, ids.offsets, ids.B) if isinstance(ids, Ragged) else out)


# ----------------------------------------------------------------- shape ops
@kernel("concat")
def k_concat(ctx, op):
    xs = [_val(ctx.get(v)) for v in op.inputs["X"]]
    dt = torch.float32 if any(x.dtype.is_floating_point for x in xs) else xs[0].dtype
    ctx.set(op.outputs["Out"][0], torch.cat([x.to(dt) for x in xs], op.attrs.get("axis", 0)))


@kernel("split")
def k_split(ctx, op):
    x = _val(ctx.get(op.inputs["X"][0]))
    ax = op.attrs["axis"]
    if op.attrs.get("num"):
        parts = torch.chunk(x, op.attrs["num"], ax)
    else:
        secs = list(op.attrs["sections"])
        if -1 in secs:
            i = secs.index(-1)
            secs[i] = x.shape[ax] - (sum(secs) + 1)
        parts = torch.split(x, secs, ax)
    for v, p in zip(op.outputs["Out"], parts):
        ctx.set(v, p)


@kernel("slice")
def k_slice(ctx, op):
    x = _val(ctx.get(op.inputs["Input"][0]))
    idx = [slice(None)] * x.dim()
    for a, s, e in zip(op.attrs["axes"], op.attrs["starts"], op.attrs["ends"]):
        n = x.shape[a]
        e = min(e, n) if e >= 0 else n + e
        idx[a] = slice(s if s >= 0 else n + s, e)
    ctx.set(op.outputs["Out"][0], x[tuple(idx)])


@kernel("reshape2", "reshape")
def k_reshape(ctx, op):
    x = _val(ctx.get(op.inputs["X"][0]))
    shape = [x.shape[i] if s == 0 else s for i, s in enumerate(op.attrs["shape"])]
    ctx.set(op.outputs["Out"][0], x.reshape(shape))


@kernel("transpose2", "transpose")
def k_transpose(ctx, op):
    ctx.set(op.outputs["Out"][0], _val(ctx.get(op.inputs["X"][0])).permute(*op.attrs["axis"]))


@kernel("squeeze2", "squeeze")
def k_squeeze(ctx, op):
    x = _val(ctx.get(op.inputs["X"][0]))
    for a in sorted(op.attrs["axes"], reverse=True):
        x = x.squeeze(a)
    ctx.set(op.outputs["Out"][0], x)


@kernel("unsqueeze2", "unsqueeze")
def k_unsqueeze(ctx, op):
    x = _val(ctx.get(op.inputs["X"][0]))
    for a in sorted(op.attrs["axes"]):
        x = x.unsqueeze(a)
    ctx.set(op.outputs["Out"][0], x)


@kernel("stack")
def k_stack(ctx, op):
    ctx.set(op.outputs["Y"][0], torch.stack([_val(ctx.get(v)) for v in op.inputs["X"]], op.attrs["axis"]))


# ----------------------------------------------------------------- reductions / losses
def _reduce(fn, ctx, op):
    x = _val(ctx.get(op.inputs["X"][0])).float()
    d = op.attrs.get("dim")
    if d is None or d == [] or op.attrs.get("reduce_all"):
        y = fn(x)
        if op.attrs.get("keep_dim"):
            y = y.reshape([1] * x.dim())
    else:
        y = fn(x, dim=d if isinstance(d, int) else tuple(d), keepdim=bool(op.attrs.get("keep_dim")))
    ctx.set(op.outputs["Out"][0], y)


@kernel("reduce_sum")
def k_reduce_sum(ctx, op):
    _reduce(torch.sum, ctx, op)


@kernel("reduce_mean")
def k_reduce_mean(ctx, op):
    _reduce(torch.mean, ctx, op)


@kernel("reduce_max")
def k_reduce_max(ctx, op):
    _reduce(lambda x, **k: torch.amax(x, **k) if k else x.max(), ctx, op)


@kernel("mean")
def k_mean(ctx, op):
    ctx.set(op.outputs["Out"][0], _val(ctx.get(op.inputs["X"][0])).float().mean().reshape(1))


@kernel("log_loss")
def k_log_loss(ctx, op):
    p = _val(ctx.get(op.inputs["Predicted"][0])).float()
    y = _val(ctx.get(op.inputs["Labels"][0])).float().reshape(p.shape)
    eps = op.attrs["epsilon"]
    ctx.set(op.outputs["Loss"][0], -y * torch.log(p + eps) - (1 - y) * torch.log(1 - p + eps))


@kernel("sigmoid_cross_entropy_with_logits")
def k_sce(ctx, op):
    x = _val(ctx.get(op.inputs["X"][0])).float()
    y = _val(ctx.get(op.inputs["Label"][0])).float().reshape(x.shape)
    ign = op.attrs.get("ignore_index", -100)
    loss = F.binary_cross_entropy_with_logits(x, y, reduction="none")
    keep = (y != ign).to(loss.dtype)
    loss = loss * keep
    if op.attrs.get("normalize"):
        loss = loss / keep.sum().clamp(min=1)
    ctx.set(op.outputs["Out"][0], loss)


@kernel("cross_entropy", "cross_entropy2")
def k_cross_entropy(ctx, op):
    p = _val(ctx.get(op.inputs["X"][0])).float()
    lab = _val(ctx.get(op.inputs["Label"][0]))
    if op.attrs.get("soft_label"):
        y = -(lab.float() * torch.log(p)).sum(-1, keepdim=True)
    else:
        y = -torch.log(p.gather(-1, lab.long().reshape(-1, 1)))
    ctx.set(op.outputs["Y"][0], y)


@kernel("sequence_pool")
def k_sequence_pool(ctx, op):
    x = ctx.get(op.inputs["X"][0])
    ctx.set(op.outputs["Out"][0], ctr_ext.sequence_pool(x.values.float(), x.offsets, x.B, op.attrs["pooltype"],
                                                        op.attrs.get("pad_value", 0.0)))


@kernel("auc")
def k_auc(ctx, op):
    pred = _val(ctx.get(op.inputs["Predict"][0])).detach().float()
    lab = _val(ctx.get(op.inputs["Label"][0])).detach().reshape(-1)
    p1 = pred[:, -1] if pred.dim() == 2 else pred.reshape(-1)
    nt = op.attrs["num_thresholds"]
    pos = ctx.scope.get(op.inputs["StatPos"][0].name)
    neg = ctx.scope.get(op.inputs["StatNeg"][0].name)
    b = (p1 * nt).long().clamp(0, nt)
    lp = (lab > 0).double()
    bp = torch.zeros_like(pos).index_add_(0, b, lp)
    bn = torch.zeros_like(neg).index_add_(0, b, 1 - lp)
    pos += bp
    neg += bn
    ctx.set(op.outputs["AUC"][0], ctr_ext.auc_from_hist(pos, neg).reshape(1))
    ctx.set(op.outputs["BatchAUC"][0], ctr_ext.auc_from_hist(bp, bn).reshape(1))


# ----------------------------------------------------------------- PaddleBox sparse
def _sparse_inputs(ctx, ids_vars):
    """(keys, lod [S*(B+1)] absolute, B, S) for a list of slot variables.
    Zero-copy when they are exactly the batch's slots in order."""
    rs = [ctx.get(v) for v in ids_vars]
    b = ctx.batch
    S = len(rs)
    if b is not None and S == b.S and all(r.slot == i for i, r in enumerate(rs)):
        return b.keys, b.lod, b.B, S
    keys = torch.cat([r.values.reshape(-1) for r in rs])
    offs, base = [], 0
    for r in rs:
        offs.append(r.offsets + base)
        base += r.values.numel()
    return keys, torch.cat(offs), rs[0].B, S


@kernel("pull_box_sparse")
def k_pull_box_sparse(ctx, op):
    keys, lod, B, S = _sparse_inputs(ctx, op.inputs["Ids"])
    recs = sparse_ops.pull_box_sparse(ctx.engine, keys, lod, B, S)
    lod2 = lod.view(S, B + 1)
    for s, v in enumerate(op.outputs["Out"]):
        a = int(lod2[s, 0])
        e = int(lod2[s, B])
        ctx.set(v, Ragged(recs[a:e], lod2[s] - a, B, s))


def _pull_op_args(ctx, op):
    """(keys, lod, B, S, SeqpoolParams, dense or None) of a __pull_seqpool_cvm
    op over the batch bound to ctx."""
    keys, lod, B, S = _sparse_inputs(ctx, op.inputs["Ids"])
    a = op.attrs
    sp = SeqpoolParams(use_cvm=a["use_cvm"], cvm_offset=a["cvm_offset"], clk_filter=a["clk_filter"],
                       pad_value=a["pad_value"], need_filter=a["need_filter"], show_coeff=a["show_coeff"],
                       clk_coeff=a["clk_coeff"], threshold=a["threshold"], quant_ratio=a["quant_ratio"],
                       # the op nests the embedding-norm filter under need_filter (fused_seqpool_cvm_op.cu:580-581)
                       embed_threshold_filter=bool(a["need_filter"] and a["embed_threshold_filter"]),
                       embed_threshold=a["embed_threshold"],
                       embed_thres_size=a["embed_thres_size"])
    dense = None
    if op.inputs.get("Dense"):
        ds = [_val(ctx.get(v)).float().reshape(B, -1) for v in op.inputs["Dense"]]
        # one dense variable (a column slice of the batch's dense block) is
        # read in place by the seqpool launch: no concat copy
        dense = ds[0] if len(ds) == 1 else torch.cat(ds, 1)
    return keys, lod, B, S, sp, dense


def prefetch_pull_op(ctx, op, slot: int) -> bool:
    """Pool the batch bound to ctx for a __pull_seqpool_cvm op ahead of its
    step (the pipelined front: SparseEngine.prefetch_pull into pull slot
    ``slot``); that step's pull then launches nothing."""
    keys, lod, B, S, sp, dense = _pull_op_args(ctx, op)
    return sparse_ops.prefetch_seqpool_cvm_concat(ctx.engine, keys, lod, B, S, dense, sp, slot)


@kernel("__cvm_show_click")
def k_cvm_show_click(ctx, op):
    """[B, 2] (show = 1, click = label): a persistent buffer per batch size,
    its click column copied from the label (lowering._fuse_cvm)."""
    lab = _val(ctx.get(op.inputs["Label"][0]))
    B = int(lab.shape[0])
    key = ("cvm_show_click", id(op), B, lab.device)
    buf = ctx.cache.get(key)
    if buf is None:
        buf = ctx.cache[key] = torch.ones(B, 2, dtype=torch.float32, device=lab.device)
    buf[:, 1].copy_(lab.reshape(B, -1)[:, 0])
    ctx.set(op.outputs["Out"][0], buf)


@kernel("__pull_seqpool_cvm")
def k_pull_seqpool_cvm(ctx, op):
    """Lowered pull_box_sparse -> fused_seqpool_cvm (-> concat) chain."""
    keys, lod, B, S, sp, dense = _pull_op_args(ctx, op)
    cvm = _val(ctx.get(op.inputs["CVM"][0])).float().contiguous()
    out = sparse_ops.pull_seqpool_cvm_concat(ctx.engine, keys, lod, B, S, cvm, dense, sp)
    Eo = sp.out_width(ctx.engine.E)
    for s, v in enumerate(op.outputs["Out"]):
        ctx.set(v, out[:, s * Eo:(s + 1) * Eo])
    if op.outputs.get("Concat"):
        ctx.set(op.outputs["Concat"][0], out)


@kernel("fused_seqpool_cvm", "fused_seqpool_cvm_with_diff_thres", "fused_seqpool_cvm_with_conv",
        "fused_seqpool_cvm_with_pcoc", "fused_seqpool_cvm_tradew", "fused_seqpool_cvm_with_credit")
def k_fused_seqpool_cvm(ctx, op):
    """Unfused form over pulled records (Ragged [L_s, E] per slot)."""
    xs = [ctx.get(v) for v in op.inputs["X"]]
    cvm = _val(ctx.get(op.inputs["CVM"][0])).float()
    qv = ctx.batch.extra.get("q_values") if ctx.batch is not None else None
    outs = ctr_ext.seqpool_cvm_variant(op.type, [x.values for x in xs], [x.offsets for x in xs], xs[0].B, cvm,
                                       op.attrs, qv)
    for v, o in zip(op.outputs["Out"], outs):
        ctx.set(v, o)


@kernel("pull_box_extended_sparse")
def k_pull_box_extended_sparse(ctx, op):
    keys, lod, B, S = _sparse_inputs(ctx, op.inputs["Ids"])
    recs, ext = ctx.box.pull_extended(keys, lod, B, S, op.attrs["emb_size"], op.attrs["emb_extended_size"],
                                      op.attrs.get("mask"))
    lod2 = lod.view(S, B + 1)
    mask = op.attrs.get("mask") or [3] * S
    oi = ei = 0
    for s in range(S):
        a, e = int(lod2[s, 0]), int(lod2[s, B])
        if mask[s] & 1:
            ctx.set(op.outputs["Out"][oi], Ragged(recs[a:e], lod2[s] - a, B, s))
            oi += 1
        if mask[s] & 2:
            ctx.set(op.outputs["OutExtend"][ei], Ragged(ext[a:e], lod2[s] - a, B, s))
            ei += 1


@kernel("pull_cache_value")
def k_pull_cache_value(ctx, op):
    ids = ctx.get(op.inputs["Id"][0])
    out = ctx.box.replica_cache.pull(_val(ids).reshape(-1), op.attrs["size"])
    ctx.set(op.outputs["Out"][0], Ragged(out, ids.offsets, ids.B) if isinstance(ids, Ragged) else out)


@kernel("lookup_input")
def k_lookup_input(ctx, op):
    ids = ctx.get(op.inputs["Id"][0])
    out = ctx.box.input_table.lookup(_val(ids).reshape(-1), op.attrs["size"], ctx.device)
    ctx.set(op.outputs["Out"][0], Ragged(out, ids.offsets, ids.B) if isinstance(ids, Ragged) else out)


@kernel("store_q_value")
def k_store_q_value(ctx, op):
    """store_q_value (store_q_value_op.cc -> MiniBatchGpuPack::store_qvalue):
    input i holds one q value per instance and is written into extension
    float i of the batch's records, where the next batch over those records
    (next pass / epoch) finds it in its packed q tensor."""
    qs = [_val(ctx.get(v)).detach() for v in op.inputs["Ids"]]
    if ctx.batch is None:
        return
    src = getattr(ctx.batch, "src", None)
    if src is not None:
        native, begin, count, dim = src
        if len(qs) != dim:
            raise ValueError(f"store_q_value: {len(qs)} inputs for padbox_slotrecord_extend_dim={dim}")
        for i, q in enumerate(qs):
            native.store_ext(begin, count, dim, i, q.reshape(-1)[:count])
    ctx.batch.extra["q_values"] = torch.cat([q.reshape(q.shape[0], -1) for q in qs], 1)


@kernel("cvm")
def k_cvm(ctx, op):
    x = ctx.get(op.inputs["X"][0])
    cvm = _val(ctx.get(op.inputs["CVM"][0])).float()
    ctx.set(op.outputs["Y"][0], ctr_ext.cvm(_val(x).float(), cvm, op.attrs["use_cvm"]))


# ----------------------------------------------------------------- normalisation
@kernel("data_norm")
def k_data_norm(ctx, op):
    x = _val(ctx.get(op.inputs["X"][0])).float()
    a = op.attrs
    bsize, bsum, bsq = (ctx.scope.get(op.inputs[k][0].name) for k in ("BatchSize", "BatchSum", "BatchSquareSum"))
    sw = ctx.param(op.inputs["scale_w"][0]) if op.inputs.get("scale_w") else None
    bias = ctx.param(op.inputs["bias"][0]) if op.inputs.get("bias") else None
    training = ctx.training and not a.get("is_test")
    y = ctr_ops._DataNorm.apply(x, bsize, bsum, bsq, sw, bias, a["epsilon"], a["summary_decay_rate"],
                                _stats_group(ctx) if a.get("sync_stats") else None, a.get("update_norm", True), training)
    ctx.set(op.outputs["Y"][0], y)


def _stats_group(ctx):
    """The process group data_norm-family statistics are summed over when the
    op asks for sync_stats: the session's group, and for the default group
    (ctx.group None) the WORLD handle -- None would mean "no sync"."""
    if ctx.group is not None:
        return ctx.group
    import torch.distributed as dist

    return dist.group.WORLD if dist.is_available() and dist.is_initialized() else None


@kernel("masked_data_norm")
def k_masked_data_norm(ctx, op):
    x = _val(ctx.get(op.inputs["X"][0])).float()
    mask = _val(ctx.get(op.inputs["Mask"][0])).float().reshape(-1)
    a = op.attrs
    bsize, bsum, bsq = (ctx.scope.get(op.inputs[k][0].name) for k in ("BatchSize", "BatchSum", "BatchSquareSum"))
    sw = ctx.param(op.inputs["scale_w"][0]) if op.inputs.get("scale_w") else None
    bias = ctx.param(op.inputs["bias"][0]) if op.inputs.get("bias") else None
    training = ctx.training and not a.get("is_test")
    y = ctr_ext.masked_data_norm(x, mask, bsize, bsum, bsq, sw, bias, a["epsilon"], a["summary_decay_rate"],
                                 _stats_group(ctx) if a.get("sync_stats") else None, a.get("update_norm", True), training)
    ctx.set(op.outputs["Y"][0], y)


@kernel("cross_norm_hadamard")
def k_cross_norm_hadamard(ctx, op):
    x = _val(ctx.get(op.inputs["Input"][0])).float()
    summary = ctx.scope.get(op.inputs["SummaryInput"][0].name)
    a = op.attrs
    y = ctr_ext.cross_norm_hadamard(x, summary, a["fields_num"], a["embed_dim"], a["epsilon"],
                                    a["summary_decay_rate"], _stats_group(ctx) if a.get("sync_stats") else None,
                                    ctx.training)
    ctx.set(op.outputs["Out"][0], y)


# ----------------------------------------------------------------- CTR dense op family
@kernel("rank_attention", "rank_attention2")
def k_rank_attention(ctx, op):
    x = _val(ctx.get(op.inputs["X"][0])).float()
    ro = _val(ctx.get(op.inputs["RankOffset"][0]))
    w = ctx.param(op.inputs["RankParam"][0])
    ctx.set(op.outputs["Out"][0], ctr_ext.rank_attention(x, ro, w, op.attrs["MaxRank"]))


@kernel("batch_fc")
def k_batch_fc(ctx, op):
    x = _val(ctx.get(op.inputs["Input"][0])).float()
    w = ctx.param(op.inputs["W"][0])
    b = ctx.param(op.inputs["Bias"][0])
    ctx.set(op.outputs["Out"][0], ctr_ext.batch_fc(x, w, b, op.attrs["batchcount"], op.attrs["transpose_weight"]))


@kernel("scaled_fc")
def k_scaled_fc(ctx, op):
    x = _val(ctx.get(op.inputs["Input"][0])).float()
    a = op.attrs
    ctx.set(op.outputs["Out"][0], ctr_ext.scaled_fc(x, ctx.param(op.inputs["W"][0]), ctx.param(op.inputs["Bias"][0]),
                                                    a["input_scale_factor"], a["bias_scale_factor"],
                                                    a["grad_scale_factor"]))


@kernel("scaled_int8fc")
def k_scaled_int8fc(ctx, op):
    x = _val(ctx.get(op.inputs["Input"][0])).float()
    a = op.attrs
    ctx.set(op.outputs["Out"][0], ctr_ext.scaled_int8fc(x, ctx.param(op.inputs["W"][0]),
                                                        ctx.param(op.inputs["Bias"][0]), a))


@kernel("fused_concat")
def k_fused_concat(ctx, op):
    xs = [_val(ctx.get(v)) for v in op.inputs["X"]]
    ctx.set(op.outputs["Out"][0], ctr_ext.fused_concat(xs, op.attrs["offset"], op.attrs["length"]))


@kernel("fused_seqpool_concat")
def k_fused_seqpool_concat(ctx, op):
    groups = [[_val(ctx.get(v)) for v in op.inputs[f"X{i + 1}"]] for i in range(op.attrs["n_groups"])]
    outs = ctr_ext.fused_seqpool_concat(groups, op.attrs["col_ranges"])
    for v, o in zip(op.outputs["Out"], outs):
        ctx.set(v, o)


@kernel("partial_concat")
def k_partial_concat(ctx, op):
    xs = [_val(ctx.get(v)) for v in op.inputs["X"]]
    ctx.set(op.outputs["Out"][0], ctr_ext.partial_concat(xs, op.attrs["start_index"], op.attrs["length"]))


@kernel("partial_sum")
def k_partial_sum(ctx, op):
    xs = [_val(ctx.get(v)) for v in op.inputs["X"]]
    ctx.set(op.outputs["Out"][0], ctr_ext.partial_sum(xs, op.attrs["start_index"], op.attrs["length"]))


@kernel("shuffle_batch")
def k_shuffle_batch(ctx, op):
    x = _val(ctx.get(op.inputs["X"][0]))
    ctx.set(op.outputs["Out"][0], ctr_ext.shuffle_batch(x, ctx.generator_dev))


@kernel("fused_seq_tensor")
def k_fused_seq_tensor(ctx, op):
    x = _val(ctx.get(op.inputs["Input"][0])).float()
    ad = _val(ctx.get(op.inputs["ADInput"][0])).float()
    din, mask, side, sess = ctr_ext.fused_seq_tensor(x, ad, **{k: op.attrs[k] for k in (
        "batch_count", "max_length", "slot_num", "fea_emb_dim", "ad_slot_num", "ad_slot_offset")})
    ctx.set(op.outputs["DINOut"][0], din)
    ctx.set(op.outputs["MaskOut"][0], mask)
    ctx.set(op.outputs["SideInfoOut"][0], side)
    ctx.set(op.outputs["ADSlotSessionOut"][0], sess)


# ----------------------------------------------------------------- lowered dense chains
def _fc_fp32() -> bool:
    """FLAGS_padbox_fc_precision: fp32 (default, the reference fc precision,
    python/paddle/fluid/layers/nn.py:243), fp32x3 (fp32-class: bf16 hi + lo
    halves, three MFMA products, finer than the reference's default TF32
    math) or bf16 MFMA operands."""
    from ..utils import flags as _flags

    return _flags.get("padbox_fc_precision").lower() != "bf16"


def _fc_x3() -> bool:
    from ..utils import flags as _flags

    return _flags.get("padbox_fc_precision").lower() == "fp32x3"


def _tower_for(ctx, op, C: int):
    """CtrTower bound to the session's dense storage (fc weights already in
    the [out, in] padded layout the tower packs from) and data_norm summaries."""
    from ..ops.ctr import DataNorm
    from ..ops.mlp import FusedMLP
    from ..ops.tower import CtrTower

    key = ("tower", id(op))
    t = ctx.cache.get(key)
    if t is not None:
        return t
    ws = [ctx.storage(v) for v in op.inputs["W"]]
    bs = [ctx.storage(v) for v in op.inputs["B"]]
    mlp = FusedMLP.__new__(FusedMLP)
    torch.nn.Module.__init__(mlp)
    mlp.in_dim = ws[0].shape[1]
    mlp.hidden = [w.shape[0] for w in ws]
    mlp.w = torch.nn.ParameterList(ws)
    mlp.b = torch.nn.ParameterList(bs)
    mlp.w_out = ctx.storage(op.inputs["WOut"][0])
    mlp.b_out = ctx.storage(op.inputs["BOut"][0])
    mlp._bf16, mlp.k_split, mlp.k_split_dw = [], 512, 1024
    mlp._ws = mlp._tw = None
    mlp._packed = mlp.packed_by_optimizer = False
    a = op.attrs
    dn = DataNorm(C, epsilon=a.get("epsilon") or 1e-5, summary_decay_rate=a.get("summary_decay_rate") or 0.9999999,
                  sync_stats=bool(a.get("sync_stats")))
    for attr, k in (("batch_size", "BatchSize"), ("batch_sum", "BatchSum"), ("batch_square_sum", "BatchSquareSum")):
        setattr(dn, attr, ctx.scope.get(op.inputs[k][0].name))
    dn.stats = torch.zeros(3 * C, device=ctx.device)
    dn.update_norm = a.get("update_norm", True) is not False
    dn.group = _stats_group(ctx)
    # the reference fc precision by default (FLAGS_padbox_fc_precision):
    # the lowering only forms the tower when the fp32 tower takes its widths
    x3 = _fc_x3()
    t = CtrTower(mlp, dn, 0, 1, 0, 0, use_head_lin=False, fp32=_fc_fp32() and not x3)
    t.x3 = x3
    # Session.fuse_towers binds an AUC metric by these names
    t.io = (op.outputs["Pred"][0].name, {op.inputs["Label"][0].name, a.get("label_alias") or ""} - {""})
    if ctx.training and hasattr(ctx.s, "on_tower_grads"):
        import weakref

        sr, tr = weakref.ref(ctx.s), weakref.ref(t)  # no tower <-> hook reference cycle

        def hook():
            s_, t_ = sr(), tr()
            if s_ is not None and t_ is not None:
                s_.on_tower_grads(t_)
        t.on_dense_grads = hook
    ctx.cache[key] = t
    return t


@kernel("__ctr_tower")
def k_ctr_tower(ctx, op):
    x = _val(ctx.get(op.inputs["X"][0])).float().contiguous()
    label = _val(ctx.get(op.inputs["Label"][0])).float()
    if not (label.dim() == 2 and label.shape[1] == 1) and not label.dim() == 1:
        label = label.reshape(-1).contiguous()  # else a [B, 1] column view: the tower reads it strided
    t = _tower_for(ctx, op, x.shape[1])
    t.dn.train(ctx.training)
    loss, pred = t(x, label)
    if t.auc is not None and getattr(t, "auc_metric", None):
        ctx.fused_metrics.add(t.auc_metric)  # histogram added by the tower's loss tail
    ctx.set(op.outputs["Pred"][0], pred.view(-1, 1))
    ctx.set(op.outputs["Loss"][0], loss)


@kernel("__fused_mlp")
def k_fused_mlp(ctx, op):
    """Lowered fc(relu)^n [-> fc(size 1)] chain on the MFMA GEMM kernels."""
    from ..ops.mlp import fused_mlp, fused_mlp_fp32

    x = _val(ctx.get(op.inputs["X"][0]))
    ws = [ctx.storage(v) for v in op.inputs["W"]]
    bs = [ctx.storage(v) for v in op.inputs["B"]]
    wo = ctx.storage(op.inputs["WOut"][0]) if op.inputs.get("WOut") else None
    bo = ctx.storage(op.inputs["BOut"][0]) if op.inputs.get("BOut") else None
    if _fc_fp32():  # the reference fc precision: library fp32 GEMMs
        y = fused_mlp_fp32(x, ws, bs, wo, bo)
    else:
        cache = ctx.cache.setdefault(id(op), [])
        y = fused_mlp(x, ws, bs, wo, bo, cache)
    if wo is not None:
        y = y.view(-1, 1)
    else:
        y = y[:, : op.attrs["out_dim"]].float()
    ctx.set(op.outputs["Out"][0], y)
