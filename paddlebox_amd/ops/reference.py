"""Plain-PyTorch fp32 reference implementations of every CTR kernel.

These are the numerics oracles for the HIP kernels (tests compare the two) and
the compute path when tensors live on the CPU (config 1: in-process CPU PS).
Semantics follow the reference PaddleBox kernels cited per function.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from ..ps.config import SparseSGDConfig, row_layout

_M64 = (1 << 64) - 1


def _s64(x: int) -> int:
    """uint64 constant -> int64 two's complement."""
    x &= _M64
    return x - (1 << 64) if x >= (1 << 63) else x


def _lsr(x: torch.Tensor, s: int) -> torch.Tensor:
    return (x >> s) & ((1 << (64 - s)) - 1)


_C1 = _s64(0xBF58476D1CE4E5B9)
_C2 = _s64(0x94D049BB133111EB)


def mix64(k: torch.Tensor) -> torch.Tensor:
    """splitmix64 finalizer on int64 tensors (bit-identical to pbx::mix64)."""
    z = k.to(torch.int64)
    z = (z ^ _lsr(z, 30)) * _C1
    z = (z ^ _lsr(z, 27)) * _C2
    return z ^ _lsr(z, 31)


def mix64_int(k: int) -> int:
    z = k & _M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


def _unxorshift(x: int, s: int) -> int:
    r = x
    for _ in range(64 // s + 1):
        r = x ^ (r >> s)
    return r


def unmix64_int(z: int) -> int:
    z &= _M64
    z = _unxorshift(z, 31)
    z = (z * 0x319642B2D24D8EC3) & _M64
    z = _unxorshift(z, 27)
    z = (z * 0x96DE1B173F119089) & _M64
    z = _unxorshift(z, 30)
    return z


def _unxorshift_t(x: torch.Tensor, s: int) -> torch.Tensor:
    r = x
    for _ in range(64 // s + 1):
        r = x ^ _lsr(r, s)
    return r


_I1 = _s64(0x96DE1B173F119089)
_I2 = _s64(0x319642B2D24D8EC3)


def unmix64(z: torch.Tensor) -> torch.Tensor:
    """Inverse of :func:`mix64` (recover feasigns from stored table keys)."""
    z = z.to(torch.int64)
    z = _unxorshift_t(z, 31)
    z = z * _I2
    z = _unxorshift_t(z, 27)
    z = z * _I1
    z = _unxorshift_t(z, 30)
    return z


def owner_of(h: torch.Tensor, n: int) -> torch.Tensor:
    """floor(uint64(h) * n / 2^64) (pbx::owner_of)."""
    if n == 1:
        return torch.zeros_like(h, dtype=torch.int64)
    hi = _lsr(h, 32)
    lo = h & 0xFFFFFFFF
    # (hi*2^32 + lo) * n >> 64 computed exactly with 2 32-bit halves
    t = lo * n
    t = hi * n + _lsr(t, 32)
    return _lsr(t, 32)


def dedup(keys: torch.Tensor, mixed: bool = False) -> Tuple[torch.Tensor, torch.Tensor]:
    """(uniq_h, uid) with uid[i] = index of keys[i] in uniq_h (BoxPS
    DedupKeysAndFillIdx semantics, box_wrapper_impl.h:128-136)."""
    h = keys if mixed else mix64(keys)
    uniq, inv = torch.unique(h, return_inverse=True)
    return uniq, inv.to(torch.int32)


def occurrence_map(lod: torch.Tensor, S: int, B: int) -> Tuple[torch.Tensor, torch.Tensor]:
    lod = lod.view(S, B + 1).to(torch.int64)
    L = int(lod[-1, -1].item()) if S > 0 else 0
    occ_slot = torch.empty(L, dtype=torch.int32)
    occ_ins = torch.empty(L, dtype=torch.int32)
    lens = (lod[:, 1:] - lod[:, :-1]).reshape(-1)
    ss = torch.arange(S).repeat_interleave(B)
    bb = torch.arange(B).repeat(S)
    occ_slot = torch.repeat_interleave(ss, lens).to(torch.int32)
    occ_ins = torch.repeat_interleave(bb, lens).to(torch.int32)
    return occ_slot, occ_ins


def seqpool_cvm(
    src: torch.Tensor,
    uid: torch.Tensor,
    lod: torch.Tensor,
    S: int,
    B: int,
    E: int,
    use_cvm: bool = True,
    cvm_offset: int = 2,
    clk_filter: bool = False,
    pad_value: float = 0.0,
    need_filter: bool = False,
    show_coeff: float = 0.2,
    clk_coeff: float = 1.0,
    threshold: float = 0.96,
    quant_ratio: int = 0,
    embed_threshold_filter: bool = False,
    embed_threshold: float = 0.0,
    embed_thres_size: int = 0,
    src_index: Optional[torch.Tensor] = None,
) -> torch.Tensor:
    """fused_seqpool_cvm forward (fused_seqpool_cvm_op.cu:34-527).

    src[u] is the pull record of unique u (first E columns used); occurrence k
    of slot s / instance b is lod[s*(B+1)+b] <= k < lod[s*(B+1)+b+1].
    Returns [B, S*Eo] (slot blocks concatenated).
    """
    dev = src.device
    lod = lod.view(S, B + 1).to(torch.int64)
    occ_slot, occ_ins = occurrence_map(lod.cpu(), S, B)
    occ_slot, occ_ins = occ_slot.to(dev), occ_ins.to(dev)
    uid = uid.to(torch.int64)
    L = occ_slot.numel()
    uid = uid[:L]
    idx = uid if src_index is None else torch.where(uid >= 0, src_index.to(torch.int64)[uid.clamp(min=0)], uid)
    valid = idx >= 0
    rows = torch.zeros(L, E, dtype=torch.float32, device=dev)
    rows[valid] = src[idx[valid], :E].float()
    keep = valid.clone()
    if need_filter or embed_threshold_filter:
        show, clk = rows[:, 0], rows[:, 1]
        keep &= (show - clk) * show_coeff + clk * clk_coeff >= threshold
        if embed_threshold_filter:
            # 0 means the whole embedding (fused_seqpool_cvm_op.cu:596-599)
            ets = embed_thres_size if embed_thres_size > 0 else E - cvm_offset
            e = rows[:, cvm_offset:]
            sc = torch.sqrt((e[:, 1:ets] ** 2).sum(1)) + e[:, 0].abs()
            keep &= sc >= embed_threshold
    if quant_ratio > 0:
        q = rows[:, cvm_offset:]
        rows = torch.cat([rows[:, :cvm_offset], (q * quant_ratio + 0.5).to(torch.int32).float() / quant_ratio], 1)
    rows = rows * keep.unsqueeze(1).float()
    seg = occ_ins.to(torch.int64) * S + occ_slot.to(torch.int64)
    pooled = torch.full((B * S, E), float(pad_value), dtype=torch.float32, device=dev)
    pooled.index_add_(0, seg, rows)
    pooled = pooled.view(B, S, E)
    if use_cvm:
        ls = torch.log(pooled[..., 0:1] + 1)
        if clk_filter:
            out = torch.cat([ls, pooled[..., 2:]], -1)
        else:
            out = torch.cat([ls, torch.log(pooled[..., 1:2] + 1) - ls, pooled[..., 2:]], -1)
    else:
        out = pooled[..., cvm_offset + embed_thres_size:]
    return out.reshape(B, -1)


def seqpool_cvm_out_width(E: int, use_cvm: bool, cvm_offset: int, clk_filter: bool, embed_thres_size: int = 0) -> int:
    """fused_seqpool_cvm output width (fused_seqpool_cvm_op.cc:85-96): without
    CVM the cvm columns and embed_thres_size more leading columns are dropped."""
    return (E - 1 if clk_filter else E) if use_cvm else E - cvm_offset - embed_thres_size


def push_merge(
    dout: torch.Tensor,
    cvm: torch.Tensor,
    uid: torch.Tensor,
    lod: torch.Tensor,
    S: int,
    B: int,
    U: int,
    dim: int,
    slot_ids: torch.Tensor,
    bs_scale: float,
    use_cvm: bool = True,
    clk_filter: bool = False,
    col_offset: int = 0,
    cvm_offset: int = 2,
    embed_thres_size: int = 0,
) -> torch.Tensor:
    """Per-unique push records [U, 4+dim] = [slot, show, click, embed_g, embedx_g]
    from the pooled-output gradient (fused_seqpool_cvm_op.cu:813-1015 +
    box_wrapper.cu:417-475): cvm columns take the CVM input, embed columns
    are scaled by -batch_size."""
    dev = dout.device
    E = 3 + dim
    occ_slot, occ_ins = occurrence_map(lod.cpu(), S, B)
    occ_slot, occ_ins = occ_slot.to(dev).long(), occ_ins.to(dev).long()
    L = occ_slot.numel()
    uid = uid[:L].to(torch.int64)
    ets = 0 if use_cvm else embed_thres_size
    Eo = seqpool_cvm_out_width(E, use_cvm, cvm_offset, clk_filter, ets)
    g = torch.zeros(L, 3 + dim, dtype=torch.float32, device=dev)
    if ets == 0:  # with dropped columns the cvm grads are zero too (op.cu:958-969)
        g[:, 0] = cvm[occ_ins, 0]
        g[:, 1] = cvm[occ_ins, 1]
    base = col_offset + occ_slot * Eo
    for c in range(cvm_offset + ets, E):
        oc = (c - 1 if clk_filter else c) if use_cvm else c - cvm_offset - ets
        g[:, 2 + c - cvm_offset] = dout[occ_ins, base + oc]
    valid = uid >= 0
    merged = torch.zeros(U, 3 + dim, dtype=torch.float32, device=dev)
    merged.index_add_(0, uid[valid], g[valid])
    merged[:, 2:] *= -bs_scale
    slot_col = torch.zeros(U, dtype=torch.float32, device=dev)
    slot_col[uid[valid]] = slot_ids.to(dev).float()[occ_slot[valid]]
    return torch.cat([slot_col.unsqueeze(1), merged], 1)


def adagrad_update(values: torch.Tensor, push: torch.Tensor, dim: int, cfg: SparseSGDConfig,
                   create_rand: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Sparse Adagrad + show/click/delta_score + embedx creation
    (heter_ps/optimizer.cuh.h:42-133).  values [U, stride] -> new values.
    create_rand [U, dim] supplies the U[0,1) draws for newly created embedx."""
    l = row_layout(dim)
    v = values.clone().float()
    slot, gs, gc = push[:, 0], push[:, 1], push[:, 2]
    v[:, l["slot"]] = slot
    v[:, 0] += gs
    v[:, 1] += gc
    v[:, l["delta_score"]] += cfg.nonclk_coeff * (gs - gc) + cfg.clk_coeff * gc
    v[:, l["unseen_days"]] = 0
    scale = torch.where(gs > 0, gs, torch.ones_like(gs))
    lr = torch.full_like(gs, cfg.learning_rate)
    mf_lr = torch.full_like(gs, cfg.mf_learning_rate)
    if cfg.use_feature_lr:
        m = slot != cfg.nodeid_slot
        lr = torch.where(m, torch.full_like(lr, cfg.feature_learning_rate), lr)
        mf_lr = torch.where(m, torch.full_like(lr, cfg.feature_learning_rate), mf_lr)
    g2 = v[:, l["embed_g2sum"]]
    ratio = lr * torch.sqrt(cfg.initial_g2sum / (cfg.initial_g2sum + g2))
    sg = push[:, 3] / scale
    v[:, 2] = (v[:, 2] + sg * ratio).clamp(cfg.min_bound, cfg.max_bound)
    v[:, l["embed_g2sum"]] = g2 + sg * sg
    created = v[:, l["mf_size"]] != 0
    show, click = v[:, 0], v[:, 1]
    create = (~created) & (cfg.nonclk_coeff * (show - click) + cfg.clk_coeff * click >= cfg.mf_create_thresholds)
    # update existing embedx
    g2x = v[:, l["embedx_g2sum"]]
    ratio_x = mf_lr * torch.sqrt(cfg.mf_initial_g2sum / (cfg.mf_initial_g2sum + g2x))
    sgx = push[:, 4:4 + dim] / scale.unsqueeze(1)
    newx = (v[:, 3:3 + dim] + sgx * ratio_x.unsqueeze(1)).clamp(cfg.mf_min_bound, cfg.mf_max_bound)
    v[:, 3:3 + dim] = torch.where(created.unsqueeze(1), newx, v[:, 3:3 + dim])
    v[:, l["embedx_g2sum"]] = torch.where(created, g2x + (sgx * sgx).sum(1) / dim, g2x)
    if create.any():
        r = create_rand if create_rand is not None else torch.rand(v.shape[0], dim, device=v.device)
        v[create, 3:3 + dim] = r[create] * cfg.mf_initial_range
        v[create, l["mf_size"]] = 1.0
    return v


def data_norm_fwd(x, bsize, bsum, bsq, scale_w=None, bias=None):
    """data_norm forward (data_norm_op.cu:38-60)."""
    means = bsum / bsize
    scales = torch.sqrt(bsize / bsq)
    y = (x - means) * scales
    if scale_w is not None:
        y = y * scale_w + bias
    return y, means, scales


def data_norm_bwd(x, dy, means, scales, eps, scale_w=None):
    """dx = dy*scale; per-batch summary stats (data_norm_op.cu:62-90)."""
    N = x.shape[0]
    sc = scales * (scale_w if scale_w is not None else 1.0)
    dx = dy * sc
    stats = torch.stack(
        [torch.ones_like(means), x.sum(0) / N, ((x - means) ** 2).sum(0) / N + eps]
    )
    return dx, stats


def data_norm_update(bsize, bsum, bsq, stats, decay):
    bsize.mul_(decay).add_(stats[0])
    bsum.mul_(decay).add_(stats[1])
    bsq.mul_(decay).add_(stats[2])


def fm_fwd(x: torch.Tensor, S: int, D: int, col0: int, fstride: int) -> torch.Tensor:
    B = x.shape[0]
    idx = col0 + torch.arange(S, device=x.device).unsqueeze(1) * fstride + torch.arange(D, device=x.device)
    v = x[:, idx.reshape(-1)].view(B, S, D)
    s1 = v.sum(1)
    s2 = (v * v).sum(1)
    return 0.5 * (s1 * s1 - s2).sum(1)


def sigmoid_logloss(logit: torch.Tensor, label: torch.Tensor, grad_scale: float):
    p = torch.sigmoid(logit)
    loss = torch.nn.functional.binary_cross_entropy_with_logits(logit, label, reduction="sum")
    dz = (p - label) * grad_scale
    return p, loss.reshape(1), dz


def auc_accumulate(pred, label, table, stats, mask=None):
    T = table.numel() // 2
    p = pred.double()
    lab = (label > 0.5).long()
    if mask is not None:
        keep = mask != 0
        p, lab = p[keep], lab[keep]
    pos = (p * T).long().clamp(0, T - 1)
    table.view(2, T).index_put_((lab, pos), torch.ones_like(p), accumulate=True)
    d = p - lab.double()
    stats += torch.stack([d.abs().sum(), (d * d).sum(), p.sum(), lab.double().sum(),
                          torch.tensor(float(p.numel()), dtype=torch.float64, device=p.device)])


def adam_flat(p, g, m, v, lr, b1, b2, eps, b1pow, b2pow, grad_scale=1.0, wd=0.0):
    """Paddle adam (phi adam_kernel): bias correction folded into lr."""
    gk = g * grad_scale + wd * p
    m.mul_(b1).add_((1 - b1) * gk)
    v.mul_(b2).add_((1 - b2) * gk * gk)
    lr_t = lr * (1 - b2pow) ** 0.5 / (1 - b1pow)
    p.sub_(lr_t * m / (v.sqrt() + eps * (1 - b2pow) ** 0.5))
