"""GPU CTR op family (csrc/hip/ctr_ext.hip) against the fp32/fp64 torch paths
of ops/ctr_ext.py run on the CPU: forward values, every gradient and the
running-statistic updates."""
import pytest
import torch

from paddlebox_amd import _native
from paddlebox_amd.ops import ctr_ext as cx
from tests.ctr_data import page_view_ranks

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _pair(*ts):
    """(cpu fp64 leaf, gpu fp32 leaf) pairs of the same values."""
    out = []
    for t in ts:
        c = t.double().clone().requires_grad_(True)
        d = t.float().to(DEV).requires_grad_(True)
        out.append((c, d))
    return out


def _close(gpu, cpu, rtol=1e-4, atol=1e-4):
    torch.testing.assert_close(gpu.detach().cpu().double(), cpu.detach().double(), rtol=rtol, atol=atol)


def test_native_ctr_kernels_loaded():
    h = _native.hip()
    for name in ("sgemm", "int8_fc", "rank_attention_fwd", "cvm_fwd", "masked_dn_fwd", "cnh_fwd"):
        assert hasattr(h, name), name


@pytest.mark.parametrize("R", [1, 3, 8])
def test_rank_attention_gpu(R):
    g = torch.Generator().manual_seed(R)
    C, P = 37, 70
    ro = page_view_ranks(300, R, g)
    B = ro.shape[0]
    (xc, xg), (wc, wg) = _pair(torch.rand(B, C, generator=g), torch.rand(R * R * C, P, generator=g))
    yc = cx.rank_attention(xc, ro, wc, R)
    yg = cx.rank_attention(xg, ro.to(DEV), wg, R)
    _close(yg, yc)
    d = torch.randn(B, P, generator=g)
    yc.backward(d.double())
    yg.backward(d.to(DEV))
    _close(xg.grad, xc.grad)
    _close(wg.grad, wc.grad, rtol=1e-4, atol=1e-3)


def test_rank_attention_gpu_skewed_ranks():
    """Most instances have rank 1 (one bucket spans several dW segments and
    splits; B is not a tile multiple); page views larger than R give rank-less
    instances."""
    g = torch.Generator().manual_seed(11)
    R, C, P = 8, 64, 64
    ro = page_view_ranks(2400, R, g, p_single=0.85)
    B = ro.shape[0]
    (xc, xg), (wc, wg) = _pair(torch.rand(B, C, generator=g), torch.rand(R * R * C, P, generator=g))
    yc = cx.rank_attention(xc, ro, wc, R)
    yg = cx.rank_attention(xg, ro.to(DEV), wg, R)
    _close(yg, yc, atol=1e-3)
    d = torch.randn(B, P, generator=g)
    yc.backward(d.double())
    yg.backward(d.to(DEV))
    _close(xg.grad, xc.grad, atol=1e-3)
    _close(wg.grad, wc.grad, rtol=1e-4, atol=2e-3)


@pytest.mark.parametrize("R,C,P", [(3, 37, 70), (8, 64, 64)])
def test_rank_attention_gpu_inconsistent_ranks(R, C, P):
    """Random rank_offset rows (not page-view consistent): duplicate faster
    ranks among one instance's peers (k_ra_dw's multi-hit path), ranks and
    indices out of range.  out and dW against the fp64 torch path; dx against
    the reference's gather form (merge_input_gradient_kernel: dx[i] = sum over
    i's peers j of j's input-gradient row at slot rank_i - 1, zero for invalid
    pairs), which is what the GPU kernel implements."""
    g = torch.Generator().manual_seed(100 + R)
    B = 700
    ro = torch.empty(B, 2 * R + 1, dtype=torch.int32)
    ro[:, 0] = torch.randint(-1, R + 2, (B,), generator=g)
    ro[:, 1::2] = torch.randint(0, R + 2, (B, R), generator=g)  # faster rank + 1 (0 / > R: invalid)
    ro[:, 1::2][torch.rand(B, R, generator=g) < 0.5] = 1  # many duplicates of faster rank 1
    ro[:, 2::2] = torch.randint(-1, B + 1, (B, R), generator=g)
    (xc, xg), (wc, wg) = _pair(torch.rand(B, C, generator=g), torch.rand(R * R * C, P, generator=g))
    yc = cx.rank_attention(xc, ro, wc, R)
    yg = cx.rank_attention(xg, ro.to(DEV), wg, R)
    _close(yg, yc, atol=1e-3)
    d = torch.randn(B, P, generator=g, dtype=torch.float64)
    yc.backward(d)
    yg.backward(d.float().to(DEV))
    _close(wg.grad, wc.grad, rtol=1e-4, atol=2e-3)
    Wb = wc.detach().reshape(R * R, C, P)
    rol = ro.long()

    def dexp_row(j, k):
        q, f, idx = int(rol[j, 0]) - 1, int(rol[j, 2 * k + 1]) - 1, int(rol[j, 2 * k + 2])
        if not (0 <= q < R and 0 <= f < R and 0 <= idx < B):
            return torch.zeros(C, dtype=torch.float64)
        return Wb[q * R + f] @ d[j]

    dx_ref = torch.zeros(B, C, dtype=torch.float64)
    for i in range(B):
        r = int(rol[i, 0])
        if not 1 <= r <= R:
            continue
        for u in range(R):
            j = int(rol[i, 2 * u + 2])
            if 0 <= j < B:
                dx_ref[i] += dexp_row(j, r - 1)
    _close(xg.grad, dx_ref, atol=1e-3)


@pytest.mark.parametrize("dims", [(4, 150, 70, 90), (5, 1000, 64, 64), (3, 4133, 36, 20), (26, 8192, 64, 64)])
@pytest.mark.parametrize("mode", ["default", "transpose", "batchcount"])
def test_batch_fc_gpu(mode, dims):
    """(70, 90) runs the generic strided k_mgemm; the <= 64 x 64 slots run
    k_bfc_fwd / k_bfc_bwd (W_p in LDS, fused dx + dW + db with the ordered
    partial reduce), ragged row tiles and padded columns included."""
    g = torch.Generator().manual_seed(5)
    P, N, I, O = dims
    if mode == "default":
        shapes = [(P, N, I), (P, I, O), (P, O)]
        kw = {}
    elif mode == "transpose":
        shapes = [(P, N, I), (I, P * O), (1, P * O)]
        kw = dict(transpose_weight=True)
    else:
        shapes = [(N, P * I), (I, P * O), (P * O,)]
        kw = dict(batchcount=P)
    (xc, xg), (wc, wg), (bc, bg) = _pair(*[torch.randn(*s, generator=g) for s in shapes])
    yc = cx.batch_fc(xc, wc, bc, **kw)
    yg = cx.batch_fc(xg, wg, bg, **kw)
    _close(yg, yc)
    d = torch.randn(*yc.shape, generator=g)
    yc.backward(d.double())
    yg.backward(d.to(DEV))
    for a, b in ((xg, xc), (wg, wc), (bg, bc)):
        _close(a.grad, b.grad, atol=1e-3)


@pytest.mark.parametrize("shape", [(300, 130, 65), (1, 1, 1), (4096, 512, 256), (2053, 33, 97), (1000, 200, 130),
                                   (777, 400, 400), (65, 8, 8)])
def test_scaled_fc_gpu(shape):
    """fp16 MFMA (k_sfc when K % 8 == 0, else the library fp16 GEMM / k_hgemm)
    against the same fp16 rounding chain in torch: the
    products differ only in fp32 accumulation order, so results agree to one
    fp16 ulp; the fp32 bias gradient is exact up to summation order."""
    N, K, O = shape
    g = torch.Generator().manual_seed(6 + N)
    x, W, b = torch.randn(N, K, generator=g), torch.randn(K, O, generator=g) * 0.2, torch.randn(1, O, generator=g)
    xc, wc, bc = (t.clone().requires_grad_() for t in (x, W, b))
    xg, wg, bg = (t.to(DEV).requires_grad_() for t in (x, W, b))
    yc = cx.scaled_fc(xc, wc, bc, 8.0, 2.0)
    yg = cx.scaled_fc(xg, wg, bg, 8.0, 2.0)
    torch.testing.assert_close(yg.cpu(), yc, rtol=2e-3, atol=2e-3)
    # small upstream gradients: dout * grad_scale / in_scale summed over N stays
    # inside fp16 (past it both sides give NaN, the reference's inf -> NaN)
    d = torch.randn(N, O, generator=g) * 0.02
    yc.backward(d)
    yg.backward(d.to(DEV))
    for a, c in ((xg, xc), (wg, wc)):
        assert not torch.isnan(c.grad).any()
        scale = float(c.grad.abs().max()) + 1e-6
        torch.testing.assert_close(a.grad.cpu(), c.grad, rtol=2e-3, atol=2e-3 * scale)
    torch.testing.assert_close(bg.grad.cpu(), bc.grad, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("shape,splits", [((8192, 400, 400), 19), ((777, 132, 36), 3), ((777, 132, 36), 1),
                                          ((4096, 512, 256), 16), ((100, 8, 404), 1), ((3000, 84, 168), 7)])
def test_scaled_fc_dw_kernel(shape, splits):
    """k_sfc_dw (scaled_fc dW + db in one launch, split-K over the batch with
    a fixed-order slab reduce) against the fp16 rounding chain in torch (fp64
    accumulation): one fp16 ulp of the epilogue; db to fp32 summation order;
    two launches bit-identical (no atomics in the sums)."""
    from paddlebox_amd import _native

    N, K, O = shape
    g = torch.Generator().manual_seed(N + K + O)
    x = torch.randn(N, K, generator=g)
    d = torch.randn(N, O, generator=g) * 0.02
    in_scale, gs = 8.0, 256.0
    h = _native.hip()
    xg, dg = x.to(DEV), d.to(DEV)
    outs = []
    for _ in range(2):
        dW, db = torch.full((K, O), float("nan"), device=DEV), torch.full((O,), float("nan"), device=DEV)
        assert h.sfc_dw(xg, dg, dW, db, 1.0, gs / in_scale, in_scale, 1.0 / gs, splits)
        outs.append((dW.cpu(), db.cpu()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    hf = torch.float16
    acc = x.to(hf).double().t() @ (d * (gs / in_scale)).to(hf).double()
    ref = (float(torch.tensor(in_scale, dtype=hf)) * acc.float()).to(hf).float() * (1.0 / gs)
    scale = float(ref.abs().max()) + 1e-6
    torch.testing.assert_close(outs[0][0], ref, rtol=2e-3, atol=2e-3 * scale)
    torch.testing.assert_close(outs[0][1], d.double().sum(0).float(), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("shape", [(1, 1, 1), (257, 100, 65), (64, 32, 64)])
def test_scaled_int8fc_gpu_exact(shape):
    """int8 MFMA accumulation is exact: the GPU result equals the fp64 oracle
    up to the final fp32 scale/bias rounding."""
    N, K, O = shape
    g = torch.Generator().manual_seed(N + K)
    x, W, b = torch.randn(N, K, generator=g), torch.randn(K, O, generator=g) * 0.2, torch.randn(O, generator=g)
    a = dict(input_expand_factor=10.0, input_clip_factor=3.0, weight_expand_factor=40.0, weight_clip_factor=5.0,
             int8_range=127.0)
    yc = cx.scaled_int8fc(x, W, b, a)
    yg = cx.scaled_int8fc(x.to(DEV), W.to(DEV), b.to(DEV), a)
    torch.testing.assert_close(yg.cpu(), yc, rtol=1e-6, atol=1e-5)


@pytest.mark.parametrize("shape", [(4096, 96, 80), (1500, 64, 32), (300, 20, 10), (8192, 512, 512), (777, 136, 44)])
@pytest.mark.parametrize("mode", ["bf16x3", "fp32"])
def test_scaled_int8fc_gpu_backward(shape, mode, monkeypatch):
    """The straight-through backward: dx = dy W^T, dW = x^T dy, db = colsum(dy).
    fp32: library GEMMs (split-K batched + fixed-order sum for dW), fp32-close
    to the fp64 oracle (the default).  bf16x3: three bf16 MFMA products of the
    operands' bf16 splits -- every element within 2^-14 of the sum of |terms|
    (the GEMM error bound), and no worse than the TF32 arithmetic the
    reference's cuBLAS runs this GEMM in (10-bit mantissa operands, emulated
    here in fp64)."""
    monkeypatch.setenv("PBX_INT8FC_BWD", mode)
    N, K, O = shape
    g = torch.Generator().manual_seed(N)
    x, W, b = torch.randn(N, K, generator=g), torch.randn(K, O, generator=g) * 0.2, torch.randn(O, generator=g)
    a = dict(input_expand_factor=10.0, input_clip_factor=3.0, weight_expand_factor=40.0, weight_clip_factor=5.0,
             int8_range=127.0)
    (xc, xg), (wc, wg), (bc, bg) = _pair(x, W, b)
    d = torch.randn(N, O, generator=g)
    cx.scaled_int8fc(xc, wc, bc, a).backward(d.double())
    cx.scaled_int8fc(xg, wg, bg, a).backward(d.to(DEV))
    _close(bg.grad, bc.grad, rtol=1e-5, atol=1e-4)
    if mode == "fp32":
        _close(xg.grad, xc.grad, rtol=1e-5, atol=1e-4)
        _close(wg.grad, wc.grad, rtol=1e-5, atol=1e-3)
        return

    def tf32(t):  # round to a 10-bit mantissa (nearest): the TF32 operand format
        m, e = torch.frexp(t.double())
        return torch.ldexp(torch.round(m * 2048) / 2048, e)

    xd, wd, dd = x.double(), W.double(), d.double()
    for got, ref, bound, tf in ((xg.grad, xc.grad, dd.abs() @ wd.abs().t(), tf32(dd) @ tf32(wd).t()),
                                (wg.grad, wc.grad, xd.abs().t() @ dd.abs(), tf32(xd).t() @ tf32(dd))):
        err = (got.cpu().double() - ref.double()).abs()
        assert bool((err <= 2.0 ** -14 * bound + 1e-6).all()), float((err / (bound + 1e-30)).max())
        assert float(err.max()) <= float((tf - ref.double()).abs().max()), (float(err.max()),)


@pytest.mark.parametrize("use_cvm", [True, False])
def test_cvm_gpu(use_cvm):
    g = torch.Generator().manual_seed(7)
    x = torch.rand(500, 11, generator=g) * 5
    cv = torch.rand(500, 2, generator=g)
    (xc, xg), = _pair(x)
    yc = cx.cvm(xc, cv.double(), use_cvm)
    yg = cx.cvm(xg, cv.to(DEV), use_cvm)
    _close(yg, yc, rtol=1e-5, atol=1e-5)
    d = torch.randn(*yc.shape, generator=g)
    yc.backward(d.double())
    yg.backward(d.to(DEV))
    _close(xg.grad, xc.grad, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("with_sw", [True, False])
def test_masked_data_norm_gpu(with_sw):
    g = torch.Generator().manual_seed(8)
    N, C = 333, 70
    x = torch.randn(N, C, generator=g) * 2 + 1
    mask = (torch.rand(N, generator=g) > 0.3).float()
    stats = [torch.full((C,), 100.0), torch.randn(C, generator=g) * 10, torch.full((C,), 150.0)]
    (xc, xg), (swc, swg), (bc, bg) = _pair(x, torch.rand(C, generator=g) + 0.5, torch.randn(C, generator=g))
    sc = [s.double().clone() for s in stats]
    sg = [s.to(DEV).clone() for s in stats]
    yc = cx.masked_data_norm(xc, mask.double(), *sc, swc if with_sw else None, bc if with_sw else None, 1e-4, 0.99,
                             None, True, True)
    yg = cx.masked_data_norm(xg, mask.to(DEV), *sg, swg if with_sw else None, bg if with_sw else None, 1e-4, 0.99,
                             None, True, True)
    _close(yg, yc)
    d = torch.randn(N, C, generator=g)
    yc.backward(d.double())
    yg.backward(d.to(DEV))
    _close(xg.grad, xc.grad)
    if with_sw:
        _close(swg.grad, swc.grad, atol=1e-3)
        _close(bg.grad, bc.grad, atol=1e-3)
    for a, b in zip(sg, sc):
        _close(a, b, rtol=1e-5, atol=1e-4)


def test_cross_norm_hadamard_gpu():
    g = torch.Generator().manual_seed(9)
    B, F, E = 300, 5, 8
    W = F * (3 * E + 1)
    summary = torch.stack([torch.full((W,), 50.0), torch.randn(W, generator=g), torch.full((W,), 80.0)])
    sc, sg = summary.double().clone(), summary.to(DEV).clone()
    (xc, xg), = _pair(torch.randn(B, F * 2 * E, generator=g))
    yc = cx.cross_norm_hadamard(xc, sc, F, E, 1e-4, 0.999)
    yg = cx.cross_norm_hadamard(xg, sg, F, E, 1e-4, 0.999)
    _close(yg, yc)
    d = torch.randn(B, W, generator=g)
    yc.backward(d.double())
    yg.backward(d.to(DEV))
    _close(xg.grad, xc.grad)
    _close(sg, sc, rtol=1e-5, atol=1e-4)


def _records(g, B, S, E, max_len=4):
    xs, offs = [], []
    for _ in range(S):
        lens = torch.randint(0, max_len + 1, (B,), generator=g)
        off = torch.cat([torch.zeros(1, dtype=torch.long), lens.cumsum(0)])
        L = int(off[-1])
        x = torch.rand(L, E, generator=g) * 2
        x[:, 0] = torch.randint(0, 20, (L,), generator=g).float()  # show
        x[:, 1] = (x[:, 0] * torch.rand(L, generator=g)).floor()  # click <= show
        xs.append(x)
        offs.append(off)
    return xs, offs


_GPU_VARIANTS = [
    ("fused_seqpool_cvm", dict(use_cvm=True, cvm_offset=2, pad_value=0.5)),
    ("fused_seqpool_cvm", dict(use_cvm=True, cvm_offset=2, need_filter=True, show_coeff=0.2, clk_coeff=1.0,
                               threshold=1.5, quant_ratio=64, clk_filter=True)),
    ("fused_seqpool_cvm", dict(use_cvm=False, cvm_offset=2, need_filter=True, quant_ratio=128, threshold=0.5,
                               show_coeff=0.2, clk_coeff=1.0,
                               embed_threshold_filter=True, embed_threshold=1.2,
                               embed_thres_size=4)),
    ("fused_seqpool_cvm", dict(use_cvm=True, cvm_offset=2, embedx_concate_size=3, pad_value=0.1)),
    ("fused_seqpool_cvm_with_diff_thres", dict(use_cvm=True, cvm_offset=2, need_filter=True, show_coeff=0.2,
                                               clk_coeff=1.0, threshold=1.0, xbox_diff_thres_filter=True,
                                               threshold_vec=[0.5, 2.0, 4.0])),
    ("fused_seqpool_cvm_with_conv", dict(use_cvm=True, cvm_offset=3, show_filter=True)),
    ("fused_seqpool_cvm_with_conv", dict(use_cvm=True, cvm_offset=3)),
    ("fused_seqpool_cvm_with_pcoc", dict(use_cvm=True, cvm_offset=6, max_cvm_offset=8, quant_ratio=128)),
    ("fused_seqpool_cvm_tradew", dict(use_cvm=True, cvm_offset=2, trade_num=3, trade_id=1)),
    ("fused_seqpool_cvm_tradew", dict(use_cvm=False, cvm_offset=2, trade_num=3, trade_id=-1)),
    ("fused_seqpool_cvm_with_credit", dict(use_cvm=True, cvm_offset=4, show_filter=True)),
]


@pytest.mark.parametrize("case", range(len(_GPU_VARIANTS)))
def test_seqpool_cvm_variants_gpu(case):
    op, attrs = _GPU_VARIANTS[case]
    g = torch.Generator().manual_seed(100 + case)
    B, S, E = 97, 3, 18
    xs, offs = _records(g, B, S, E)
    co = attrs["cvm_offset"]
    cv = torch.rand(B, max(co, 4), generator=g)
    qv = torch.rand(B, co - 4, generator=g) if op.endswith("pcoc") else None
    pc = [x.double().requires_grad_(True) for x in xs]
    pg = [x.to(DEV).requires_grad_(True) for x in xs]
    oc = cx.seqpool_cvm_variant(op, pc, offs, B, cv.double(), attrs, qv.double() if qv is not None else None)
    og = cx.seqpool_cvm_variant(op, pg, [o.to(DEV) for o in offs], B, cv.to(DEV), attrs,
                                qv.to(DEV) if qv is not None else None)
    assert len(og) == S
    ds = []
    for a, b in zip(og, oc):
        _close(a, b, rtol=1e-5, atol=1e-5)
        ds.append(torch.randn(*b.shape, generator=g))
    torch.autograd.backward(oc, [d.double() for d in ds])
    torch.autograd.backward(og, [d.to(DEV) for d in ds])
    for a, b in zip(pg, pc):
        _close(a.grad, b.grad, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("bc,ad_off", [(1, 0), (3, 2)])
def test_fused_seq_tensor_gpu(bc, ad_off):
    g = torch.Generator().manual_seed(bc)
    ins, T, E, S, A = 37, 5, 8, 6, 2
    x = torch.randn(ins, bc * S * T * E, generator=g)
    x[:, : T * E] = 0.0  # some all-zero steps for the mask
    ad = torch.randn(ins, bc * A * E, generator=g)
    exp = cx.fused_seq_tensor(x, ad, bc, T, S, E, A, ad_off)
    got = cx.fused_seq_tensor(x.to(DEV), ad.to(DEV), bc, T, S, E, A, ad_off)
    for a, b in zip(got, exp):
        assert a.shape == b.shape
        torch.testing.assert_close(a.cpu(), b, rtol=1e-6, atol=1e-6)
