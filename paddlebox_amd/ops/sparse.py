"""Autograd-aware sparse ops: fused pull+seqpool+CVM(+concat) and the plain
pull_box_sparse whose gradient is push_box_sparse.

Reference ops: ``pull_box_sparse``/``push_box_sparse``
(``paddle/fluid/operators/pull_box_sparse_op.{cc,h}``) and
``fused_seqpool_cvm`` (``operators/fused/fused_seqpool_cvm_op.*``).  As in the
reference, the backward of the embedding lookup *is* the sparse parameter
update: it runs the fused merge + Adagrad inside the engine and returns no
gradient for the ids.
"""
from __future__ import annotations

from typing import Optional

import torch

from ..ps.sparse_engine import SeqpoolParams, SparseEngine


_ANCHORS = {}


def _anchor(device) -> torch.Tensor:
    """A leaf that requires grad, fed to the sparse Functions so their output
    is part of the autograd graph even when no dense input requires grad
    (the sparse table update happens in their backward)."""
    d = torch.device(device)
    a = _ANCHORS.get(d)
    if a is None:
        a = torch.zeros((), device=d, requires_grad=True)
        _ANCHORS[d] = a
    return a


class _PullSeqpoolCvmConcat(torch.autograd.Function):
    @staticmethod
    def forward(ctx, anchor: torch.Tensor, dense: Optional[torch.Tensor], keys: torch.Tensor, lod: torch.Tensor,
                cvm: torch.Tensor, engine: SparseEngine, B: int, S: int, sp: SeqpoolParams, bs_scale: float):
        E = engine.E
        Eo = sp.out_width(E)
        Dd = 0 if dense is None else dense.shape[1]
        out = engine.prepared_output(keys)  # pooled ahead by prefetch_seqpool_cvm_concat
        if out is None or tuple(out.shape) != (B, S * Eo + Dd):
            out = torch.empty(B, S * Eo + Dd, dtype=torch.float32, device=keys.device)
        # the dense features are written by the same launch (no concat copy)
        st = engine.pull_seqpool_cvm(keys, lod, B, S, out, 0, sp, dense=dense if Dd else None, dense_col=S * Eo)
        ctx.engine, ctx.st, ctx.sp, ctx.bs_scale = engine, st, sp, bs_scale
        ctx.S, ctx.Eo, ctx.Dd = S, Eo, Dd
        ctx.save_for_backward(cvm)
        return out

    @staticmethod
    def backward(ctx, dout):
        (cvm,) = ctx.saved_tensors
        ctx.engine.push_seqpool_cvm(ctx.st, dout, cvm, 0, ctx.sp, ctx.bs_scale)
        ddense = dout[:, ctx.S * ctx.Eo:] if ctx.Dd else None
        return None, ddense, None, None, None, None, None, None, None, None


def pull_seqpool_cvm_concat(engine: SparseEngine, keys: torch.Tensor, lod: torch.Tensor, B: int, S: int,
                            cvm: torch.Tensor, dense: Optional[torch.Tensor] = None,
                            sp: Optional[SeqpoolParams] = None, bs_scale: Optional[float] = None) -> torch.Tensor:
    """[B, S*Eo (+Dd)]: pooled CVM'ed slot blocks followed by the dense features.

    The backward pushes per-key gradients (show/click from ``cvm``) into the
    sparse table and passes d(dense) through."""
    sp = sp or SeqpoolParams()
    bs = float(B if bs_scale is None else bs_scale)
    return _PullSeqpoolCvmConcat.apply(_anchor(keys.device), dense, keys, lod, cvm, engine, B, S, sp, bs)


def prefetch_seqpool_cvm_concat(engine: SparseEngine, keys: torch.Tensor, lod: torch.Tensor, B: int, S: int,
                                dense: Optional[torch.Tensor] = None, sp: Optional[SeqpoolParams] = None,
                                slot: int = 0) -> bool:
    """Pool a batch ahead of its step (SparseEngine.prefetch_pull): the
    step's pull_seqpool_cvm_concat on the same key buffer then launches
    nothing.  Returns False when the engine cannot prepare pulls."""
    return engine.prefetch_pull(keys, lod, B, S, sp or SeqpoolParams(), dense, slot)


def prefetch_pool_seqpool_cvm_concat(engine: SparseEngine, keys: torch.Tensor, lod: torch.Tensor, B: int, S: int,
                                     dense: Optional[torch.Tensor] = None, sp: Optional[SeqpoolParams] = None,
                                     slot: int = 0) -> bool:
    """The pooling half of prefetch_seqpool_cvm_concat, after an
    ``engine.prefetch_dedup(keys, slot)`` issued earlier (e.g. on a side
    stream beside the previous step's push)."""
    return engine.prefetch_pool(keys, lod, B, S, sp or SeqpoolParams(), dense, slot)


class _PullBoxSparse(torch.autograd.Function):
    @staticmethod
    def forward(ctx, anchor: torch.Tensor, keys: torch.Tensor, lod: torch.Tensor, engine: SparseEngine, B: int,
                S: int, bs_scale: float):
        recs, st = engine.pull_records(keys, lod, B, S)
        ctx.engine, ctx.st, ctx.bs_scale = engine, st, bs_scale
        return recs

    @staticmethod
    def backward(ctx, g):
        ctx.engine.push_records(ctx.st, g, 2, ctx.bs_scale)
        return None, None, None, None, None, None, None


def pull_box_sparse(engine: SparseEngine, keys: torch.Tensor, lod: torch.Tensor, B: int, S: int,
                    bs_scale: Optional[float] = None) -> torch.Tensor:
    """Per-occurrence pull records [L, 3+D] = [show, click, embed_w, embedx...]."""
    return _PullBoxSparse.apply(_anchor(keys.device), keys, lod, engine, B, S,
                                float(B if bs_scale is None else bs_scale))
