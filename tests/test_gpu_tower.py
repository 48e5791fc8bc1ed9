"""Fused dense tower (csrc/hip/tower.hip) vs the fp32 PyTorch path.

The GPU path runs head -> k_tower_fwd -> k_tower_bwd -> k_tower_dw ->
k_head_bwd with bf16 MFMA inputs; the oracle is the CPU fp32 composition
(ctr_head + FusedMLP fp32 + logit_logloss) on copies of the same parameters.
"""
import copy

import pytest
import torch

from paddlebox_amd.ops.ctr import DataNorm
from paddlebox_amd.ops.mlp import FusedMLP
from paddlebox_amd.ops.tower import CtrTower
from paddlebox_amd.parallel.dense import DenseArena, FlatAdam

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _make(B, S, Eo, Dd, hidden, seed=0):
    torch.manual_seed(seed)  # FusedMLP init draws from the global generator
    g = torch.Generator().manual_seed(seed)
    C = S * Eo + Dd
    x = torch.randn(B, C, generator=g)
    x[:, 0:S * Eo:Eo] = torch.rand(B, S, generator=g) * 3  # show-like columns
    label = (torch.rand(B, generator=g) < 0.3).float()
    dn = DataNorm(C)
    dn.batch_sum.normal_(0, 10, generator=g)
    mlp = FusedMLP(C, hidden, 1)
    with torch.no_grad():
        for b in mlp.b:
            b.normal_(0, 0.1, generator=g)
        mlp.b_out.fill_(0.05)
    return x, label, dn, mlp


def _rel(a, b):
    return float((a - b).abs().max() / (b.abs().max() + 1e-6))


def _fro(a, b):
    return float((a - b).norm() / (b.norm() + 1e-12))


def _bf(t):
    return t.to(torch.bfloat16).float()


def _unpack_mp(t, M, N):
    """m-packed [Mp/16][Np/32][64][8] -> [M, N] (see csrc/hip/kernels.h)."""
    Np = (N + 31) // 32 * 32
    Mp = t.numel() // Np
    z = t.view(Mp // 16, Np // 32, 2, 32, 8).permute(0, 2, 4, 1, 3).reshape(Mp, Np)
    return z[:M, :N].float()


@pytest.mark.parametrize("B,hidden", [(300, (64, 48)), (2048, (400, 400, 400)), (8192, (400, 400, 400))])
def test_tower_matches_fp32(B, hidden):
    S, Eo, Dd, D = 26, 11, 13, 8
    x, label, dn, mlp = _make(B, S, Eo, Dd, hidden)
    dn_c, mlp_c = copy.deepcopy(dn), copy.deepcopy(mlp)
    dn_g, mlp_g = copy.deepcopy(dn).to(DEV), copy.deepcopy(mlp).to(DEV)
    tc = CtrTower(mlp_c, dn_c, S, Eo, 2, D)
    tg = CtrTower(mlp_g, dn_g, S, Eo, 2, D)
    T = 1000
    auc_c = (torch.zeros(2 * T, dtype=torch.float64), torch.zeros(5, dtype=torch.float64), None)
    auc_g = (torch.zeros(2 * T, dtype=torch.float64, device=DEV), torch.zeros(5, dtype=torch.float64, device=DEV),
             None)
    tc.auc, tg.auc = auc_c, auc_g

    xc = x.clone().requires_grad_(True)
    lc, pc = tc(xc, label)
    lc.backward()
    xg = x.to(DEV).requires_grad_(True)
    lg, pg = tg(xg, label.to(DEV))
    lg.backward()
    torch.cuda.synchronize()

    # end to end vs pure fp32: bf16 MFMA inputs, so Frobenius-relative bounds
    assert abs(float(lg) - float(lc)) < 2e-3 * max(1.0, abs(float(lc)))
    assert _rel(pg.cpu(), pc.detach()) < 2e-2
    assert _fro(xg.grad.cpu(), xc.grad) < 3e-2
    for wc, wg in zip(list(mlp_c.w) + list(mlp_c.b) + [mlp_c.w_out, mlp_c.b_out],
                      list(mlp_g.w) + list(mlp_g.b) + [mlp_g.w_out, mlp_g.b_out]):
        assert _fro(wg.grad.cpu(), wc.grad) < 8e-2, wc.shape
    # data_norm summaries updated from the fused batch statistics
    for name in ("batch_size", "batch_sum", "batch_square_sum"):
        assert _rel(getattr(dn_g, name).cpu(), getattr(dn_c, name)) < 1e-4, name
    # fused AUC histogram: counts agree up to bucket-boundary rounding
    assert float(auc_g[0].sum()) == float(auc_c[0].sum()) == B
    assert abs(float(auc_g[1][4]) - float(auc_c[1][4])) == 0
    assert abs(float(auc_g[1][2]) - float(auc_c[1][2])) < 1e-2 * B


def test_tower_extra_logit_and_no_dn():
    """External logit term (DCN-style) gets d loss / d logit; no data_norm."""
    S, Eo, Dd = 4, 11, 3
    x, label, _, mlp = _make(200, S, Eo, Dd, (32,))
    mlp_c, mlp_g = copy.deepcopy(mlp), copy.deepcopy(mlp).to(DEV)
    tc = CtrTower(mlp_c, None, S, Eo, 2, 0, use_head_lin=False)
    tg = CtrTower(mlp_g, None, S, Eo, 2, 0, use_head_lin=False)
    e = torch.randn(200)
    ec, eg = e.clone().requires_grad_(True), e.to(DEV).requires_grad_(True)
    xc, xg = x.clone().requires_grad_(True), x.to(DEV).requires_grad_(True)
    lc, _ = tc(xc, label, ec)
    (2.0 * lc).backward()
    lg, _ = tg(xg, label.to(DEV), eg)
    (2.0 * lg).backward()
    assert abs(float(lg) - float(lc)) < 2e-3
    assert _rel(eg.grad.cpu(), ec.grad) < 1e-2
    assert _fro(xg.grad.cpu(), xc.grad) < 3e-2


@pytest.mark.parametrize("M,dims", [(300, [304, 64, 48]), (8192, [304, 400, 400, 400]), (1000, [64, 130, 96])])
def test_tower_kernels_exact(M, dims):
    """k_tower_fwd/bwd/dw vs an fp32 reference that rounds to bf16 exactly
    where the kernels store bf16 (input, activations, dZ), using the kernels'
    own stored activations so ReLU masks agree."""
    from paddlebox_amd import _native

    torch.manual_seed(M)
    mlp = FusedMLP(dims[0], dims[1:], 1).to(DEV)
    with torch.no_grad():
        for b in mlp.b:
            b.normal_(0, 0.1)
        mlp.b_out.fill_(0.1)
    mlp.ensure_grads()
    dims = [mlp.in_dim] + list(mlp.hidden)  # widths as padded to multiples of 8
    ws = mlp.tower_workspace(M, torch.device(DEV))
    mlp.ensure_packed()
    x = _bf(torch.randn(M, dims[0], device=DEV))
    ws.x0()[:, :dims[0]] = x
    ws.x0mp().view(-1)[:] = 0
    Mp, K0p = ws.Mp, (dims[0] + 31) // 32 * 32
    xp = torch.zeros(Mp, K0p, device=DEV)
    xp[:M, :dims[0]] = x
    ws.x0mp().copy_(xp.view(Mp // 16, 2, 8, K0p // 32, 32).permute(0, 3, 1, 4, 2).reshape(-1).to(torch.bfloat16))
    lin = torch.randn(M, device=DEV)
    label = (torch.rand(M, device=DEV) < 0.4).float()
    loss, pred, dz = ws.forward(list(mlp.b), mlp.w_out.view(-1), mlp.b_out, lin, label)
    gl = torch.tensor([0.7], device=DEV)
    dx0 = ws.backward(gl, mlp.w_out.detach().view(-1), [w.grad for w in mlp.w], [b.grad for b in mlp.b],
                      mlp.w_out.grad.view(-1), mlp.b_out.grad, True)
    torch.cuda.synchronize()
    L = len(mlp.w)
    hs = [x] + [_unpack_mp(ws.xmp(l), M, dims[l + 1]) for l in range(L)]
    assert _fro(_unpack_mp(ws.x0mp(), M, dims[0]), x) == 0
    for l in range(L):  # each layer from the stored previous activations
        ref = _bf(torch.relu(hs[l] @ _bf(mlp.w[l].detach()).t() + mlp.b[l].detach()))
        torch.testing.assert_close(hs[l + 1], ref, rtol=2e-2, atol=2e-2)
    z = hs[L] @ mlp.w_out.detach().view(-1) + mlp.b_out.detach() + lin
    pe = torch.sigmoid(z)
    torch.testing.assert_close(pred, pe, rtol=1e-3, atol=1e-4)
    le = torch.nn.functional.binary_cross_entropy_with_logits(z, label)
    assert float(loss) == pytest.approx(float(le), rel=1e-3)
    torch.testing.assert_close(dz, (pe - label) / M, rtol=1e-3, atol=1e-6)
    g = dz * 0.7
    wo = mlp.w_out.detach().view(-1)
    dxl = g[:, None] * wo[None, :]
    dzs = [None] * L
    dzu = dxl * (hs[L] > 0)
    gw, gb = [None] * L, [None] * L
    for l in reversed(range(L)):
        dzb = _bf(dzu)
        dzs[l] = dzb
        gb[l] = dzu.sum(0)
        gw[l] = dzb.t() @ hs[l]
        dx = dzb @ _bf(mlp.w[l].detach())
        if l > 0:
            dzu = dx * (hs[l] > 0)
    for l in range(L):
        torch.testing.assert_close(_unpack_mp(ws.dzmp(l), M, dims[l + 1]), dzs[l], rtol=2e-2,
                                   atol=2e-2 * float(dzs[l].abs().max()))
        torch.testing.assert_close(mlp.w[l].grad, gw[l], rtol=2e-2, atol=1e-2 * float(gw[l].abs().max()))
        torch.testing.assert_close(mlp.b[l].grad, gb[l], rtol=2e-2, atol=1e-2 * float(gb[l].abs().max()))
    g_wo = g @ hs[L]
    torch.testing.assert_close(mlp.w_out.grad.view(-1), g_wo, rtol=2e-2, atol=1e-2 * float(g_wo.abs().max()))
    assert float(mlp.b_out.grad) == pytest.approx(float(g.sum()), rel=1e-3, abs=1e-6)
    torch.testing.assert_close(dx0[:, :dims[0]].float(), dx, rtol=2e-2, atol=1e-2 * float(dx.abs().max()))
    assert _native.hip() is not None


def test_fused_adam_pack_and_dn_update():
    """FlatAdam.fuse: one kernel = Adam + bf16 re-pack + data_norm update,
    equal to plain Adam + explicit pack + data_norm_update."""
    from paddlebox_amd import _native

    S, Eo, Dd, D = 26, 11, 13, 8
    B = 512
    x, label, dn, mlp = _make(B, S, Eo, Dd, (96, 64))
    runs = []
    for fused in (False, True):
        d, m = copy.deepcopy(dn).to(DEV), copy.deepcopy(mlp).to(DEV)
        t = CtrTower(m, d, S, Eo, 2, D)
        arena = DenseArena(m.parameters(), torch.device(DEV))
        opt = FlatAdam(arena, lr=1e-2, clear_grad=True)
        if fused:
            opt.fuse(mlps=[m], data_norms=[d])
        for _ in range(3):
            loss, _ = t(x.to(DEV), label.to(DEV))
            loss.backward()
            opt.step()
        torch.cuda.synchronize()
        runs.append((arena.flat.clone(), d.batch_size.clone(), d.batch_sum.clone(), d.batch_square_sum.clone(),
                     [m._tw.wp(i).clone() for i in range(len(m.w))], m, opt))
    a, b = runs
    assert torch.allclose(a[0], b[0], rtol=1e-5, atol=1e-6)
    for i in (1, 2, 3):
        assert torch.allclose(a[i], b[i], rtol=1e-6)
    assert torch.equal(a[6].pows, b[6].pows)
    # the fused re-pack equals an explicit pack of the updated masters
    m = b[5]
    m._tw.pack([w.detach() for w in m.w])
    torch.cuda.synchronize()
    for i in range(len(m.w)):
        assert torch.equal(b[4][i], m._tw.wp(i))
    assert _native.hip() is not None


def test_tower_deterministic():
    """Two identical steps give bitwise-identical loss, grads and dx (the
    split-2 dW atomics add two partials onto zero; reductions are ordered)."""
    S, Eo, Dd, D = 26, 11, 13, 8
    x, label, dn, mlp = _make(300, S, Eo, Dd, (64, 48))
    outs = []
    for _ in range(2):
        d, m = copy.deepcopy(dn).to(DEV), copy.deepcopy(mlp).to(DEV)
        t = CtrTower(m, d, S, Eo, 2, D)
        xg = x.to(DEV).requires_grad_(True)
        loss, pred = t(xg, label.to(DEV))
        loss.backward()
        torch.cuda.synchronize()
        outs.append([loss.detach().clone(), pred.clone(), xg.grad.clone(), m._tw.x0().clone(), m._tw.x0mp().clone()]
                    + [m._tw.xmp(i).clone() for i in range(2)] + [m._tw.dzmp(i).clone() for i in range(2)]
                    + [m._tw.dx0().clone()] + [p.grad.clone() for p in m.parameters()])
    names = ["loss", "pred", "dx", "x0", "x0mp", "xmp0", "xmp1", "dzmp0", "dzmp1", "dx0"] + [
        f"g{i}" for i in range(len(outs[0]) - 10)]
    bad = [n for n, a, b in zip(names, outs[0], outs[1]) if not torch.equal(a, b)]
    assert not bad, bad
