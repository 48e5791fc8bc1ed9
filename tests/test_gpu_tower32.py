"""Exact-fp32 fused tower (csrc/hip/tower32.hip) vs the fp32 PyTorch path.

The reference's dense `fc` runs fp32 GEMMs (paddle/phi/kernels/gpu/matmul_kernel.cu);
tower32 keeps every operand in fp32 (v_mfma_f32_16x16x4_f32), so the bounds
here are fp32-summation-order tight, not bf16 ones.
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


def _unpack_mp32(t, M, N):
    """MP32 [Mp/16][Np/16][64][4] -> [M, N] (see csrc/hip/kernels.h)."""
    Np = (N + 15) // 16 * 16
    Mp = t.numel() // Np
    z = t.view(Mp // 16, Np // 16, 4, 16, 4).permute(0, 2, 4, 1, 3).reshape(Mp, Np)
    return z[:M, :N]


@pytest.mark.parametrize("B,hidden", [(300, (64, 48)), (1000, (130, 96)), (2048, (400, 400, 400)),
                                      (8192, (400, 400, 400))])
def test_tower32_matches_fp32(B, hidden):
    S, Eo, Dd, D = 26, 11, 13, 8
    x, label, dn, mlp = _make(B, S, Eo, Dd, hidden)
    dn_c, mlp_c = copy.deepcopy(dn), copy.deepcopy(mlp)
    dn_g, mlp_g = copy.deepcopy(dn).to(DEV), copy.deepcopy(mlp).to(DEV)
    tc = CtrTower(mlp_c, dn_c, S, Eo, 2, D)
    tg = CtrTower(mlp_g, dn_g, S, Eo, 2, D, fp32=True)
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
    assert mlp_g._tw.fp32
    assert abs(float(lg) - float(lc)) < 1e-5 * max(1.0, abs(float(lc)))
    assert float((pg.cpu() - pc.detach()).abs().max()) < 1e-5
    assert _fro(xg.grad.cpu(), xc.grad) < 1e-4
    for wc, wg in zip(list(mlp_c.w) + list(mlp_c.b) + [mlp_c.w_out, mlp_c.b_out],
                      list(mlp_g.w) + list(mlp_g.b) + [mlp_g.w_out, mlp_g.b_out]):
        assert _fro(wg.grad.cpu(), wc.grad) < 1e-4, wc.shape
    for name in ("batch_size", "batch_sum", "batch_square_sum"):
        a, b = getattr(dn_g, name).cpu(), getattr(dn_c, name)
        assert float((a - b).abs().max() / (b.abs().max() + 1e-6)) < 1e-5, name
    assert float(tg.auc[0].sum()) == float(tc.auc[0].sum()) == B


@pytest.mark.parametrize("M,dims", [(300, [304, 64, 48]), (8192, [304, 400, 400, 400]), (1000, [64, 136, 96]),
                                    (700, [128, 256, 512])])
def test_tower32_kernels_exact(M, dims):
    """k_t32_fwd/bwd/dw against fp64 math on the kernels' own stored
    activations (ReLU masks agree), checking every MP32 buffer."""
    torch.manual_seed(M)
    mlp = FusedMLP(dims[0], dims[1:], 1).to(DEV)
    with torch.no_grad():
        for b in mlp.b:
            b.normal_(0, 0.1)
        mlp.b_out.fill_(0.1)
    mlp.ensure_grads()
    dims = [mlp.in_dim] + list(mlp.hidden)
    ws = mlp.tower_workspace(M, torch.device(DEV), fp32=True)
    mlp.ensure_packed()
    K0p = ws.K0p
    x = torch.randn(M, dims[0], device=DEV)
    ws.x0()[:, :dims[0]] = x
    Mp = ws.Mp
    xp = torch.zeros(Mp, K0p, device=DEV)
    xp[:M, :dims[0]] = x
    ws.x0mp().copy_(xp.view(Mp // 16, 4, 4, K0p // 16, 16).permute(0, 3, 1, 4, 2).reshape(-1))
    assert torch.equal(_unpack_mp32(ws.x0mp(), M, dims[0]), x)
    lin = torch.randn(M, device=DEV)
    label = (torch.rand(M, device=DEV) < 0.4).float()
    loss, pred, dz = ws.forward(list(mlp.b), mlp.w_out.view(-1), mlp.b_out, lin, label)
    gl = torch.tensor([0.7], device=DEV)
    dx0 = ws.backward(gl, mlp.w_out.detach().view(-1), [w.grad for w in mlp.w], [b.grad for b in mlp.b],
                      mlp.w_out.grad.view(-1), mlp.b_out.grad, True)
    torch.cuda.synchronize()
    L = len(mlp.w)
    d64 = lambda t: t.detach().double()  # noqa: E731
    hs = [x.double()] + [_unpack_mp32(ws.xmp(l), M, dims[l + 1]).double() for l in range(L)]
    for l in range(L):
        ref = torch.relu(hs[l] @ d64(mlp.w[l]).t() + d64(mlp.b[l]))
        torch.testing.assert_close(hs[l + 1], ref, rtol=1e-5, atol=1e-5)
    z = hs[L] @ d64(mlp.w_out).view(-1) + d64(mlp.b_out) + lin.double()
    pe = torch.sigmoid(z)
    torch.testing.assert_close(pred.double(), pe, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(dz.double(), (pe - label.double()) / M, rtol=1e-4, atol=1e-8)
    g = dz.double() * 0.7
    dzu = g[:, None] * d64(mlp.w_out).view(-1)[None, :] * (hs[L] > 0)
    for l in reversed(range(L)):
        torch.testing.assert_close(_unpack_mp32(ws.dzmp(l), M, dims[l + 1]).double(), dzu, rtol=1e-4,
                                   atol=1e-5 * float(dzu.abs().max()))
        gw, gb = dzu.t() @ hs[l], dzu.sum(0)
        torch.testing.assert_close(mlp.w[l].grad.double(), gw, rtol=1e-4, atol=1e-5 * float(gw.abs().max()))
        torch.testing.assert_close(mlp.b[l].grad.double(), gb, rtol=1e-4, atol=1e-5 * float(gb.abs().max()))
        dx = dzu @ d64(mlp.w[l])
        if l > 0:
            dzu = dx * (hs[l] > 0)
    g_wo = g @ hs[L]
    torch.testing.assert_close(mlp.w_out.grad.view(-1).double(), g_wo, rtol=1e-4, atol=1e-5 * float(g_wo.abs().max()))
    torch.testing.assert_close(dx0[:, :dims[0]].double(), dx, rtol=1e-4, atol=1e-5 * float(dx.abs().max()))


def test_tower32_fused_adam_repack():
    """FlatAdam.fuse on the fp32 tower: the fused re-pack writes the fp32
    packed copies, equal to an explicit pack of the updated masters; the
    update equals the unfused Adam."""
    S, Eo, Dd, D = 26, 11, 13, 8
    x, label, dn, mlp = _make(512, S, Eo, Dd, (96, 64))
    runs = []
    for fused in (False, True):
        d, m = copy.deepcopy(dn).to(DEV), copy.deepcopy(mlp).to(DEV)
        t = CtrTower(m, d, S, Eo, 2, D, fp32=True)
        arena = DenseArena(m.parameters(), torch.device(DEV))
        opt = FlatAdam(arena, lr=1e-2, clear_grad=True)
        if fused:
            opt.fuse(mlps=[m], data_norms=[d])
        for _ in range(3):
            loss, _ = t(x.to(DEV), label.to(DEV))
            loss.backward()
            opt.step()
        torch.cuda.synchronize()
        runs.append((arena.flat.clone(), [m._tw.wp(i).clone() for i in range(len(m.w))],
                     [m._tw.wtp(i).clone() for i in range(len(m.w))], m))
    a, b = runs
    # the fused Adam kernel and the unfused torch update round differently
    # (Adam's m / sqrt(v) amplifies it for near-zero grads): the update is
    # compared at that tolerance, the re-pack exactly below
    assert torch.allclose(a[0], b[0], rtol=1e-5, atol=1e-5)
    m = b[3]
    m._tw.pack([w.detach() for w in m.w])
    torch.cuda.synchronize()
    for i in range(len(m.w)):
        assert torch.equal(b[1][i], m._tw.wp(i))
        assert torch.equal(b[2][i], m._tw.wtp(i))


@pytest.mark.parametrize("B,hidden", [(700, (64, 48)), (8192, (400, 400, 400))])
def test_tower32_deterministic(B, hidden):
    """Bit-reproducible: the dW split-M partials are summed in split order by
    the tile's last arriving split (no fp32 atomics), every other reduction
    is ordered too -- two runs give bitwise-equal grads."""
    S, Eo, Dd, D = 26, 11, 13, 8
    x, label, dn, mlp = _make(B, S, Eo, Dd, hidden)
    outs = []
    for _ in range(3):
        d, m = copy.deepcopy(dn).to(DEV), copy.deepcopy(mlp).to(DEV)
        t = CtrTower(m, d, S, Eo, 2, D, fp32=True)
        xg = x.to(DEV).requires_grad_(True)
        loss, pred = t(xg, label.to(DEV))
        loss.backward()
        torch.cuda.synchronize()
        outs.append([loss.detach().clone(), pred.clone(), xg.grad.clone()] + [p.grad.clone() for p in m.parameters()])
    assert m._tw.dw_splits > 1  # the split-M combine is exercised
    for run in outs[1:]:
        for a, b in zip(outs[0], run):
            assert torch.equal(a, b)


def test_deepfm_fp32_vs_bf16_training_auc():
    """Two passes of DeepFM training on the same synthetic stream with the
    fp32 tower and with the bf16 tower: the held-out AUC differs by < 0.002
    (the bf16 tower's precision costs no model quality at this scale)."""
    from paddlebox_amd.data.synthetic import CriteoSynth
    from paddlebox_amd.models.deepfm import DeepFM
    from paddlebox_amd.ps.config import PSConfig
    from paddlebox_amd.ps.sparse_engine import SparseEngine

    dev = torch.device(DEV)
    B, steps = 2048, 150
    aucs = {}
    for prec in ("fp32", "bf16"):
        torch.manual_seed(7)
        synth = CriteoSynth(total_features=200_000, seed=3, device=DEV)
        eng = SparseEngine(PSConfig(embedx_dim=8), max_keys=B * 26, device=dev, capacity=400_000, auto_insert=True)
        model = DeepFM(eng, hidden=(400, 400, 400)).to(dev)
        model.set_precision(prec)
        arena = DenseArena(model.parameters(), dev)
        opt = FlatAdam(arena, lr=1e-3, clear_grad=True)
        opt.fuse(mlps=[model.mlp], data_norms=[model.dn])
        preds, labels = [], []
        for i in range(2 * steps):
            b = synth.batch(B)
            loss, pred = model(b)
            if i >= 2 * steps - 20:  # held-out: evaluated before training on them
                preds.append(pred.detach().float().cpu())
                labels.append(b.label.cpu())
            loss.backward()
            opt.step()
        p, y = torch.cat(preds), torch.cat(labels)
        order = torch.argsort(p)
        ranks = torch.empty_like(p)
        ranks[order] = torch.arange(1, p.numel() + 1, dtype=p.dtype)
        npos = float(y.sum())
        nneg = p.numel() - npos
        aucs[prec] = (float(ranks[y > 0.5].sum()) - npos * (npos + 1) / 2) / (npos * nneg)
    assert aucs["fp32"] > 0.6, aucs
    assert abs(aucs["fp32"] - aucs["bf16"]) < 0.002, aucs


@pytest.mark.parametrize("T", [4, 1000])
def test_tower_auc_histogram_exact(T):
    """The fused loss tail's AUC histogram (wave-merged adds) equals a
    bincount of the stored predictions; T = 4 puts most rows of every wave on
    one bucket (the converged-model case the per-wave merge is for)."""
    B = 8192
    S, Eo, Dd, D = 26, 11, 13, 8
    x, label, dn, mlp = _make(B, S, Eo, Dd, (400, 400, 400))
    tg = CtrTower(copy.deepcopy(mlp).to(DEV), copy.deepcopy(dn).to(DEV), S, Eo, 2, D, fp32=True)
    tg.auc = (torch.zeros(2 * T, dtype=torch.float64, device=DEV), torch.zeros(5, dtype=torch.float64, device=DEV),
              None)
    _, pg = tg(x.to(DEV), label.to(DEV))
    torch.cuda.synchronize()
    p = pg.detach().float().cpu().view(-1)
    pos = (p * T).to(torch.int64).clamp(0, T - 1)
    lab = (label.view(-1) > 0.5).to(torch.int64)
    want = torch.bincount(lab * T + pos, minlength=2 * T).double()
    assert torch.equal(tg.auc[0].cpu(), want)
