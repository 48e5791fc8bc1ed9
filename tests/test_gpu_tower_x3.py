"""fp32-precision fused tower on bf16 MFMA (csrc/hip/tower_x3.hip) vs fp64.

Every fp32 operand is carried as bf16 hi + lo halves and every product as
hi*hi + hi*lo + lo*hi.  The error of one dot product is then bounded by
~3 * 2^-16 of sum |a_k b_k| (the dropped lo*lo term and the split residues);
the tests assert 2^-13 of that sum per element -- TF32, which the reference's
fp32 fc uses by default (paddle/phi/backends/gpu/gpu_context.cc:65-67,580-588),
rounds each input to 2^-11 and so sits at ~2^-10.
"""
import copy

import pytest
import torch

from paddlebox_amd.ops.mlp import FusedMLP
from paddlebox_amd.ops.tower import CtrTower
from paddlebox_amd.parallel.dense import DenseArena, FlatAdam

from paddlebox_amd.ops.ctr import DataNorm

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
TOL = 2.0 ** -13


def _make(B, S, Eo, Dd, hidden, seed=0):
    torch.manual_seed(seed)
    g = torch.Generator().manual_seed(seed)
    C = S * Eo + Dd
    x = torch.randn(B, C, generator=g)
    x[:, 0:S * Eo:Eo] = torch.rand(B, S, generator=g) * 3
    label = (torch.rand(B, generator=g) < 0.3).float()
    dn = DataNorm(C)
    dn.batch_sum.normal_(0, 10, generator=g)
    mlp = FusedMLP(C, hidden, 1)
    with torch.no_grad():
        for b in mlp.b:
            b.normal_(0, 0.1, generator=g)
        mlp.b_out.fill_(0.05)
    return x, label, dn, mlp


def _fro(a, b):
    return float((a - b).norm() / (b.norm() + 1e-12))


def _unpack_mp2(t, M, N, Mp):
    """hi + lo m-packed halves [2][Mp/16][Np/32][64][8] -> fp32 [M, N]."""
    Np = (N + 31) // 32 * 32
    h = t.view(2, Mp // 16, Np // 32, 2, 32, 8).permute(0, 1, 3, 5, 2, 4).reshape(2, Mp, Np).float()
    return (h[0] + h[1])[:M, :N]


def _within(got, want, scale, what):
    err = (got.double() - want).abs()
    bound = TOL * scale + 1e-30
    bad = err > bound
    assert not bool(bad.any()), f"{what}: {int(bad.sum())} elements over 2^-13 sum|terms|, worst " \
                                f"{float((err / bound).max()):.3g}x"


@pytest.mark.parametrize("M,dims,splits", [(300, [304, 64, 48], 2), (8192, [304, 400, 400, 400], 1),
                                           (8192, [304, 400, 400, 400], 2), (8192, [304, 400, 400, 400], 4),
                                           (1000, [64, 136, 96], 4), (700, [128, 256, 512], 2)])
def test_x3_kernels_vs_fp64(M, dims, splits, monkeypatch):
    """k_tx3_fwd / bwd / dw against fp64 math on the kernels' own stored
    activations (hi + lo), element by element within 2^-13 of sum |terms|;
    the dW with 1, 2 and 4 split-M partials."""
    monkeypatch.setenv("PBX_TOWER_X3_DW_SPLITS", str(splits))
    torch.manual_seed(M)
    mlp = FusedMLP(dims[0], dims[1:], 1).to(DEV)
    with torch.no_grad():
        for b in mlp.b:
            b.normal_(0, 0.1)
        mlp.b_out.fill_(0.1)
    mlp.ensure_grads()
    dims = [mlp.in_dim] + list(mlp.hidden)
    ws = mlp.tower_workspace(M, torch.device(DEV), x3=True)
    assert ws.x3 and not ws.fp32 and ws.dw_splits in (splits, 2)
    mlp.ensure_packed()
    Mp = ws.Mp
    x = torch.randn(M, dims[0], device=DEV)
    ws.x0()[:, :dims[0]] = x
    lin = torch.randn(M, device=DEV)
    label = (torch.rand(M, device=DEV) < 0.4).float()
    loss, pred, dz = ws.forward(list(mlp.b), mlp.w_out.view(-1), mlp.b_out, lin, label)
    gl = torch.tensor([0.7], device=DEV)
    dx0 = ws.backward(gl, mlp.w_out.detach().view(-1), [w.grad for w in mlp.w], [b.grad for b in mlp.b],
                      mlp.w_out.grad.view(-1), mlp.b_out.grad, True)
    torch.cuda.synchronize()
    L = len(mlp.w)
    d64 = lambda t: t.detach().double()  # noqa: E731
    # the fwd m-packs X0's halves itself: they must reproduce X0 to 2^-16
    x0s = _unpack_mp2(ws.x0mp(), M, dims[0], Mp)
    assert float((x0s - x).abs().max()) <= 2.0 ** -16 * float(x.abs().max())
    hs = [x0s.double()] + [_unpack_mp2(ws.xmp(l), M, dims[l + 1], Mp).double() for l in range(L)]
    for l in range(L):
        w = d64(mlp.w[l])
        ref = torch.relu(hs[l] @ w.t() + d64(mlp.b[l]))
        scale = hs[l].abs() @ w.abs().t() + d64(mlp.b[l]).abs()
        # a pre-activation within the bound of 0 may land on either side of the ReLU
        _within(hs[l + 1], ref, scale, f"X{l + 1}")
    z = hs[L] @ d64(mlp.w_out).view(-1) + d64(mlp.b_out) + lin.double()
    pe = torch.sigmoid(z)
    torch.testing.assert_close(pred.double(), pe, rtol=1e-4, atol=1e-5)
    g = dz.double() * 0.7
    want = g[:, None] * d64(mlp.w_out).view(-1)[None, :] * (hs[L] > 0)
    want_scale = want.abs()
    for l in reversed(range(L)):
        dzu = _unpack_mp2(ws.dzmp(l), M, dims[l + 1], Mp).double()
        _within(dzu, want, want_scale, f"dZ{l + 1}")
        # from here on the reference runs on the kernel's stored halves
        gw = dzu.t() @ hs[l]
        _within(mlp.w[l].grad.double(), gw, dzu.abs().t() @ hs[l].abs(), f"dW{l}")
        gb = dzu.sum(0)
        torch.testing.assert_close(mlp.b[l].grad.double(), gb, rtol=1e-4, atol=1e-6 * float(dzu.abs().sum(0).max()))
        w = d64(mlp.w[l])
        dx, dx_scale = dzu @ w, dzu.abs() @ w.abs()
        if l > 0:
            want, want_scale = dx * (hs[l] > 0), dx_scale * (hs[l] > 0)
        else:
            _within(dx0[:, :dims[0]], dx, dx_scale, "dX0")
    g_wo = g @ hs[L]
    torch.testing.assert_close(mlp.w_out.grad.view(-1).double(), g_wo, rtol=1e-4,
                               atol=1e-6 * float((g.abs() @ hs[L].abs()).max()))


@pytest.mark.parametrize("B,hidden", [(300, (64, 48)), (2048, (400, 400, 400)), (8192, (400, 400, 400))])
def test_x3_tower_matches_fp32(B, hidden):
    """Whole fused tower (data_norm head + MLP + loss + AUC) at x3 vs the CPU
    fp32 path: same loss / predictions / grads to fp32-GEMM-level agreement."""
    S, Eo, Dd, D = 26, 11, 13, 8
    x, label, dn, mlp = _make(B, S, Eo, Dd, hidden)
    dn_c, mlp_c = copy.deepcopy(dn), copy.deepcopy(mlp)
    dn_g, mlp_g = copy.deepcopy(dn).to(DEV), copy.deepcopy(mlp).to(DEV)
    tc = CtrTower(mlp_c, dn_c, S, Eo, 2, D)
    tg = CtrTower(mlp_g, dn_g, S, Eo, 2, D)
    tg.x3 = True
    T = 1000
    tc.auc = (torch.zeros(2 * T, dtype=torch.float64), torch.zeros(5, dtype=torch.float64), None)
    tg.auc = (torch.zeros(2 * T, dtype=torch.float64, device=DEV), torch.zeros(5, dtype=torch.float64, device=DEV),
              None)
    xc = x.clone().requires_grad_(True)
    lc, pc = tc(xc, label)
    lc.backward()
    xg = x.to(DEV).requires_grad_(True)
    lg, pg = tg(xg, label.to(DEV))
    lg.backward()
    torch.cuda.synchronize()
    assert mlp_g._tw.x3
    assert abs(float(lg) - float(lc)) < 1e-5 * max(1.0, abs(float(lc)))
    assert float((pg.cpu() - pc.detach()).abs().max()) < 2e-5
    assert _fro(xg.grad.cpu(), xc.grad) < 2e-4
    # parameter grads sum B products per element over data_norm'ed inputs
    # with large column means (|grad| << sum |terms|), and a hidden layer's dZ
    # carries the error of the layer above it: relative agreement is bounded
    # by the cancellation, not by the GEMM (the per-element 2^-13 bounds on
    # the kernels' own operands are test_x3_kernels_vs_fp64).  2e-3 ~ 2^-9:
    # what the reference's TF32 fc reaches on such sums is ~8x coarser.
    for wc, wg in zip(list(mlp_c.w) + list(mlp_c.b) + [mlp_c.w_out, mlp_c.b_out],
                      list(mlp_g.w) + list(mlp_g.b) + [mlp_g.w_out, mlp_g.b_out]):
        assert _fro(wg.grad.cpu(), wc.grad) < 2e-3, wc.shape
    assert float(tg.auc[0].sum()) == float(tc.auc[0].sum()) == B


@pytest.mark.parametrize("B,hidden", [(700, (64, 48)), (8192, (400, 400, 400))])
def test_x3_deterministic(B, hidden):
    """One writer per dW element, ordered reductions: bitwise-equal reruns."""
    S, Eo, Dd, D = 26, 11, 13, 8
    x, label, dn, mlp = _make(B, S, Eo, Dd, hidden)
    outs = []
    for _ in range(3):
        d, m = copy.deepcopy(dn).to(DEV), copy.deepcopy(mlp).to(DEV)
        t = CtrTower(m, d, S, Eo, 2, D)
        t.x3 = True
        xg = x.to(DEV).requires_grad_(True)
        loss, pred = t(xg, label.to(DEV))
        loss.backward()
        torch.cuda.synchronize()
        outs.append([loss.detach().clone(), pred.clone(), xg.grad.clone()] + [p.grad.clone() for p in m.parameters()])
    assert m._tw.dw_splits > 1  # the split-M combine is exercised
    for run in outs[1:]:
        for a, b in zip(outs[0], run):
            assert torch.equal(a, b)


def test_x3_fused_adam_repack():
    """FlatAdam.fuse on the x3 tower re-packs hi AND lo halves: equal to an
    explicit pack of the updated masters."""
    S, Eo, Dd, D = 26, 11, 13, 8
    x, label, dn, mlp = _make(512, S, Eo, Dd, (96, 64))
    d, m = dn.to(DEV), mlp.to(DEV)
    t = CtrTower(m, d, S, Eo, 2, D)
    t.x3 = True
    arena = DenseArena(m.parameters(), torch.device(DEV))
    opt = FlatAdam(arena, lr=1e-2, clear_grad=True)
    opt.fuse(mlps=[m], data_norms=[d])
    for _ in range(3):
        loss, _ = t(x.to(DEV), label.to(DEV))
        loss.backward()
        opt.step()
    torch.cuda.synchronize()
    wp = [m._tw.wp(i).clone() for i in range(len(m.w))]
    wtp = [m._tw.wtp(i).clone() for i in range(len(m.w))]
    m._tw.pack([w.detach() for w in m.w])
    torch.cuda.synchronize()
    for i in range(len(m.w)):
        assert torch.equal(wp[i], m._tw.wp(i))
        assert torch.equal(wtp[i], m._tw.wtp(i))
        n = wp[i].numel() // 2
        assert bool(wp[i][n:].float().abs().max() > 0)  # the lo halves are live


def test_deepfm_x3_training_matches_fp32():
    """DeepFM trained at fp32x3 and at exact fp32 on the same stream: the
    held-out AUC agrees to 1e-3 and the final losses to 1e-3 relative."""
    from paddlebox_amd.data.synthetic import CriteoSynth
    from paddlebox_amd.models.deepfm import DeepFM
    from paddlebox_amd.ps.config import PSConfig
    from paddlebox_amd.ps.sparse_engine import SparseEngine

    dev = torch.device(DEV)
    B, steps = 2048, 100
    res = {}
    for prec in ("fp32", "fp32x3"):
        torch.manual_seed(7)
        synth = CriteoSynth(total_features=200_000, seed=3, device=DEV)
        eng = SparseEngine(PSConfig(embedx_dim=8), max_keys=B * 26, device=dev, capacity=400_000, auto_insert=True)
        model = DeepFM(eng, hidden=(400, 400, 400)).to(dev)
        model.set_precision(prec)
        assert model.tower.x3 == (prec == "fp32x3")
        arena = DenseArena(model.parameters(), dev)
        opt = FlatAdam(arena, lr=1e-3, clear_grad=True)
        opt.fuse(mlps=[model.mlp], data_norms=[model.dn])
        preds, labels, losses = [], [], []
        for i in range(2 * steps):
            b = synth.batch(B)
            loss, pred = model(b)
            if i >= 2 * steps - 20:
                preds.append(pred.detach().float().cpu())
                labels.append(b.label.cpu())
                losses.append(float(loss))
            loss.backward()
            opt.step()
        p, y = torch.cat(preds), torch.cat(labels)
        order = torch.argsort(p)
        ranks = torch.empty_like(p)
        ranks[order] = torch.arange(1, p.numel() + 1, dtype=p.dtype)
        npos = float(y.sum())
        nneg = p.numel() - npos
        res[prec] = ((float(ranks[y > 0.5].sum()) - npos * (npos + 1) / 2) / (npos * nneg), sum(losses) / len(losses))
    assert res["fp32"][0] > 0.6, res
    assert abs(res["fp32"][0] - res["fp32x3"][0]) < 1e-3, res
    assert abs(res["fp32"][1] - res["fp32x3"][1]) < 1e-3 * res["fp32"][1], res


@pytest.mark.parametrize("B,use_dn", [(700, True), (8192, True), (513, False)])
def test_x3_fused_head_backward_equals_head_kernel(B, use_dn, monkeypatch):
    """The DeepFM head backward fused into k_tx3_bwd's dX0 epilogue
    (PBX_X3_FUSED_HEAD=1, opt-in) gives the
    gradient of the separate k_head_bwd launch (same fp32 ops; the compilers'
    multiply-add contraction may differ by an ulp); every parameter gradient
    is bitwise unchanged."""
    S, Eo, Dd, D = 26, 11, 13, 8
    x, label, dn, mlp = _make(B, S, Eo, Dd, (400, 400, 400))
    grads = {}
    for fused in ("1", "0"):
        monkeypatch.setenv("PBX_X3_FUSED_HEAD", fused)
        d, m = (copy.deepcopy(dn).to(DEV) if use_dn else None), copy.deepcopy(mlp).to(DEV)
        t = CtrTower(m, d, S, Eo, 2, D)
        t.x3 = True
        xg = x.to(DEV).requires_grad_(True)
        loss, _ = t(xg, label.to(DEV))
        loss.backward()
        torch.cuda.synchronize()
        grads[fused] = [xg.grad.clone()] + [p.grad.clone() for p in m.parameters()]
    ref = grads["0"][0]
    torch.testing.assert_close(grads["1"][0], ref, rtol=1e-6, atol=1e-6 * float(ref.abs().max()))
    for a, b in zip(grads["1"][1:], grads["0"][1:]):
        assert torch.equal(a, b)
