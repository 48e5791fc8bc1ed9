"""CPU semantics of the CTR op family (ops/ctr_ext.py): each op against a
direct evaluation of its definition, and autograd against finite
differences where the reference gradient is the true derivative.  The GPU
kernels are checked against these same torch paths in test_gpu_ctr_ops.py."""
import math

import torch

from paddlebox_amd.ops import ctr_ext as cx
from tests.ctr_data import page_view_ranks, rank_attention_loop


def test_rank_attention_forward_and_grad():
    g = torch.Generator().manual_seed(0)
    R, C, P = 3, 5, 4
    ro = page_view_ranks(12, R, g)
    B = ro.shape[0]
    x = torch.rand(B, C, generator=g, dtype=torch.float64)
    W = torch.rand(R * R * C, P, generator=g, dtype=torch.float64)
    torch.testing.assert_close(cx.rank_attention(x, ro, W, R), rank_attention_loop(x, ro, W, R))
    x.requires_grad_(True)
    W.requires_grad_(True)
    assert torch.autograd.gradcheck(lambda a, w: cx.rank_attention(a, ro, w, R), (x, W))


def test_batch_fc_layouts():
    g = torch.Generator().manual_seed(1)
    P, N, I, O = 3, 5, 4, 6
    x = torch.randn(P, N, I, generator=g, dtype=torch.float64)
    W = torch.randn(P, I, O, generator=g, dtype=torch.float64)
    b = torch.randn(P, O, generator=g, dtype=torch.float64)
    ref = torch.stack([x[p] @ W[p] + b[p] for p in range(P)])
    torch.testing.assert_close(cx.batch_fc(x, W, b), ref)
    # transpose_weight: W [in, bc*out]
    Wt = torch.randn(I, P * O, generator=g, dtype=torch.float64)
    bt = torch.randn(1, P * O, generator=g, dtype=torch.float64)
    ref = torch.stack([x[p] @ Wt[:, p * O:(p + 1) * O] + bt[0, p * O:(p + 1) * O] for p in range(P)])
    torch.testing.assert_close(cx.batch_fc(x, Wt, bt, transpose_weight=True), ref)
    # batchcount: x [N, bc*in]
    xb = torch.randn(N, P * I, generator=g, dtype=torch.float64)
    bb = torch.randn(P * O, generator=g, dtype=torch.float64)
    ref = torch.cat([xb[:, p * I:(p + 1) * I] @ Wt[:, p * O:(p + 1) * O] for p in range(P)], 1) + bb
    torch.testing.assert_close(cx.batch_fc(xb, Wt, bb, batchcount=P), ref)


def test_scaled_fc_and_int8fc():
    g = torch.Generator().manual_seed(2)
    x = torch.randn(7, 9, generator=g)
    W = torch.randn(9, 5, generator=g)
    b = torch.randn(1, 5, generator=g)
    y = cx.scaled_fc(x, W, b, 4.0, 2.0)
    # the reference's fp16 arithmetic (scaled_fc_op.cu): fp16-close to the fp32 product
    torch.testing.assert_close(y, x @ W + b * 0.5, rtol=4e-3, atol=1e-2)
    torch.testing.assert_close(y, cx.scaled_fc_reference(x, W, b, 4.0, 2.0), rtol=0, atol=0)
    # values past fp16 range come back NaN (inf -> NaN on the cast back)
    assert torch.isnan(cx.scaled_fc(x * 1e4, W, b, 4.0, 2.0)).any()
    xr = x.clone().requires_grad_()
    Wr = W.clone().requires_grad_()
    br = b.clone().requires_grad_()
    cx.scaled_fc(xr, Wr, br, 4.0, 2.0, grad_scale=256.0).sum().backward()
    d = torch.ones(7, 5)
    torch.testing.assert_close(xr.grad, d @ W.t(), rtol=4e-3, atol=1e-2)
    torch.testing.assert_close(Wr.grad, x.t() @ d, rtol=4e-3, atol=1e-2)
    torch.testing.assert_close(br.grad, d.sum(0, keepdim=True))
    a = dict(input_expand_factor=16.0, input_clip_factor=2.0, weight_expand_factor=32.0, weight_clip_factor=3.0,
             int8_range=127.0)
    y8 = cx.scaled_int8fc(x, W, b, a)
    qx = cx.int8_quantize(x, 16.0, 2.0, 127.0)
    qw = cx.int8_quantize(W, 32.0, 3.0, 127.0)
    exp = (qx.double() @ qw.double()).float() * (2 * 2.0 / 127.0) / (16.0 * 32.0) + b
    torch.testing.assert_close(y8, exp)
    # the quantiser clips to +-clip before rounding
    assert float(cx.int8_quantize(torch.tensor([10.0]), 1.0, 2.0, 127.0)) == 64.0  # trunc(2/(4/127)+.5)


def test_cvm_forward_and_backward():
    x = torch.tensor([[3.0, 1.0, 0.5, -1.0], [0.0, 0.0, 2.0, 4.0]], requires_grad=True)
    cvm = torch.tensor([[1.0, 0.0], [1.0, 1.0]])
    y = cx.cvm(x, cvm, True)
    torch.testing.assert_close(y[:, 0], torch.log(x[:, 0] + 1).detach())
    torch.testing.assert_close(y[:, 1], (torch.log(x[:, 1] + 1) - torch.log(x[:, 0] + 1)).detach())
    y.sum().backward()
    torch.testing.assert_close(x.grad[:, :2], cvm)
    torch.testing.assert_close(x.grad[:, 2:], torch.ones(2, 2))
    assert cx.cvm(x, cvm, False).shape == (2, 2)


def test_masked_data_norm_and_update():
    g = torch.Generator().manual_seed(3)
    N, C = 10, 4
    x = torch.randn(N, C, generator=g, dtype=torch.float64, requires_grad=True)
    mask = (torch.rand(N, generator=g) > 0.4).double()
    bsize = torch.full((C,), 5.0, dtype=torch.float64)
    bsum = torch.randn(C, generator=g, dtype=torch.float64)
    bsq = torch.full((C,), 7.0, dtype=torch.float64)
    sw = torch.rand(C, generator=g, dtype=torch.float64, requires_grad=True)
    bias = torch.randn(C, generator=g, dtype=torch.float64, requires_grad=True)
    s0 = (bsize.clone(), bsum.clone(), bsq.clone())
    y = cx.masked_data_norm(x, mask, bsize, bsum, bsq, sw, bias, 1e-4, 0.9, None, True, True)
    mean, scale = s0[1] / s0[0], torch.sqrt(s0[0] / s0[2])
    m = mask.bool().unsqueeze(1)
    exp = torch.where(m, (x - mean) * scale * sw + bias, torch.zeros_like(x))
    torch.testing.assert_close(y, exp)
    y.pow(2).sum().backward()
    n = mask.sum()
    xm = x.detach()[mask.bool()]
    torch.testing.assert_close(bsize, s0[0] * 0.9 + 1)
    torch.testing.assert_close(bsum, s0[1] * 0.9 + xm.sum(0) / n)
    torch.testing.assert_close(bsq, s0[2] * 0.9 + ((xm - mean) ** 2).sum(0) / n + 1e-4)
    # masked rows get no gradient; the rest is the true derivative
    assert float(x.grad[~mask.bool()].abs().sum()) == 0.0
    torch.testing.assert_close(x.grad, torch.where(m, 2 * exp * sw * scale, torch.zeros_like(x)))


def test_cross_norm_hadamard_grad_and_summary():
    g = torch.Generator().manual_seed(4)
    B, F, E = 6, 2, 3
    W = F * (3 * E + 1)
    x = torch.randn(B, F * 2 * E, generator=g, dtype=torch.float64, requires_grad=True)
    summary = torch.stack([torch.full((W,), 4.0), torch.randn(W, generator=g), torch.full((W,), 9.0)]).double()
    assert torch.autograd.gradcheck(
        lambda a: cx.cross_norm_hadamard(a, summary.clone(), F, E, 1e-4, 0.99, training=False), (x,))
    s_before = summary.clone()
    y = cx.cross_norm_hadamard(x, summary, F, E, 1e-4, 0.99)
    y.sum().backward()
    raw = cx._cross_raw(x.detach(), F, E)
    mean = s_before[1] / s_before[0]
    stats = torch.stack([torch.ones(W, dtype=torch.float64), raw.mean(0), ((raw - mean) ** 2).mean(0) + 1e-4])
    torch.testing.assert_close(summary, s_before * 0.99 + stats)
    assert math.isfinite(float(y.detach().sum()))


def _variant_cases():
    base = dict(use_cvm=True, cvm_offset=2)
    yield "std", dict(base)
    yield "std", dict(base, clk_filter=True)
    yield "std", dict(base, use_cvm=False, embed_thres_size=3)
    yield "diff_thres", dict(base, use_cvm=False)
    yield "tradew", dict(base, trade_num=2, trade_id=1)
    yield "conv", dict(base, cvm_offset=3)
    yield "conv", dict(base, cvm_offset=3, show_filter=True)
    yield "credit", dict(base, cvm_offset=4, show_filter=True)
    yield "credit", dict(base, cvm_offset=4)
    yield "pcoc", dict(base, cvm_offset=6, max_cvm_offset=8)
    yield "pcoc", dict(base, cvm_offset=6, max_cvm_offset=8, use_cvm=False)


def _apply_tables(f, g, p, dout, cv, qv):
    lg = lambda v: torch.log(v + 1)  # noqa: E731
    cols = []
    for op, s1, s2 in f:
        cols.append(p[:, s1] if op == cx._F_COPY else (lg(p[:, s1]) if op == cx._F_LOG else lg(p[:, s1]) - lg(p[:, s2])))
    grad = torch.stack([torch.zeros(p.shape[0]) if op == cx._G_ZERO else
                        (cv[:, i] if op == cx._G_CVM else (qv[:, i] if op == cx._G_QVAL else dout[:, i]))
                        for op, i in g], 1)
    return torch.stack(cols, 1), grad


def test_seqpool_variant_tables_match_epilogues():
    """The column tables the GPU kernels run reproduce the slicing-form
    epilogue and gradient of every variant."""
    g = torch.Generator().manual_seed(11)
    B, E = 5, 12
    for variant, a in _variant_cases():
        Ep = E - a.get("trade_num", 0) if variant == "tradew" else E
        p = torch.rand(B, Ep, generator=g) * 3
        cv = torch.rand(B, 4, generator=g)
        qv = torch.rand(B, 2, generator=g)
        f, gt, ep = cx._spv_tables(variant, a, E, cv.shape[1], variant == "pcoc")
        assert ep == Ep
        exp = cx._cvm_epilogue(variant, p, a)
        dout = torch.rand(B, exp.shape[1], generator=g)
        got, grad = _apply_tables(f, gt, p, dout, cv, qv)
        torch.testing.assert_close(got, exp, msg=f"{variant} {a}")
        eg = cx._cvm_epilogue_grad(variant, dout, a, E, cv, qv, B)
        torch.testing.assert_close(grad, eg, msg=f"{variant} {a} grad")
