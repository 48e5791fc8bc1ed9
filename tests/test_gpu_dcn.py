"""DCN-V2 cross stack on the MFMA GEMM (gemm.hip EPI_CROSS_* epilogues +
cross.hip) against an fp64 torch oracle of the same recurrence on the same
bf16 inputs."""
import pytest
import torch

from paddlebox_amd.models.dcn_v2 import CrossNetV2, cross_logit

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


def _p64(n):
    return (n + 63) // 64 * 64


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("M,C,L", [(1000, 304, 3), (4096, 64, 1), (333, 136, 2)])
def test_cross_stack_matches_fp64(M, C, L, fused, monkeypatch):
    """C = the padded MLP input width D; x0 / x0^T laid out as the MLP
    workspace's X_0 [M, pad64(D)] / X_0^T [pad64(D+1), pad64(M)] (ones row).
    fused: the one-launch forward (tower.hip k_cross_fwd) vs the per-layer
    GEMMs (PBX_CROSS_FUSED=0)."""
    monkeypatch.setenv("PBX_CROSS_FUSED", "1" if fused else "0")
    ld = _p64(C)
    torch.manual_seed(M + C)
    dev = torch.device("cuda:0")
    net = CrossNetV2(C, L).to(dev)
    with torch.no_grad():
        for w, b in zip(net.w, net.b):
            w.copy_(torch.randn(C, C, device=dev) * (0.5 / C ** 0.5))
            b.copy_(torch.randn(C, device=dev) * 0.1)
    w_c = torch.nn.Parameter(torch.randn(C, device=dev) * 0.3)
    y = torch.zeros(M, ld, dtype=torch.bfloat16, device=dev)
    y[:, :C] = (torch.randn(M, C, device=dev) * 0.7).to(torch.bfloat16)
    yt = torch.zeros(_p64(C + 1), _p64(M), dtype=torch.bfloat16, device=dev)
    yt[:C, :M] = y[:, :C].t()
    yt[C, :M] = 1.0
    r = torch.randn(M, device=dev)
    # HIP path (grads accumulate into .grad; start from zero)
    for p in list(net.parameters()) + [w_c]:
        p.grad = torch.zeros_like(p)
    yh = y.clone().requires_grad_(True)
    s = cross_logit(yh, net, w_c, yt)
    assert net._xw.fused_forward == fused
    (s * r).sum().backward()
    # fp64 oracle
    x0 = y[:, :C].double().requires_grad_(True)
    ws = [w.detach().double().requires_grad_(True) for w in net.w]
    bs = [b.detach().double().requires_grad_(True) for b in net.b]
    wc = w_c.detach().double().requires_grad_(True)
    x = x0
    for w, b in zip(ws, bs):
        x = x0 * (x @ w.t() + b) + x
    sr = x @ wc
    (sr * r.double()).sum().backward()
    # bf16 GEMM operands (x_l, W) with fp32 accumulation and fp32 state
    assert _rel(s, sr) < 2e-2
    assert _rel(w_c.grad, wc.grad) < 2e-2
    for l in range(L):
        assert _rel(net.w[l].grad, ws[l].grad) < 3e-2, l
        assert _rel(net.b[l].grad, bs[l].grad) < 3e-2, l
    assert _rel(yh.grad[:, :C].float(), x0.grad) < 3e-2
    assert bool((yh.grad[:, C:] == 0).all())


def test_dcn_tower_path_matches_workspace_path():
    """DCN-V2 with the cross stack inside the fused tower (head + MLP + loss +
    cross on the normalised input) vs the same parameters through the MLP
    workspace + standalone cross: same loss and gradients up to the bf16
    operands of both (the tower's cross is 64-padded wider; the extra
    features are zero padding)."""
    from paddlebox_amd.data.synthetic import CriteoSynth
    from paddlebox_amd.models.dcn_v2 import DCNv2
    from paddlebox_amd.parallel.dense import join_grad_producers
    from paddlebox_amd.ps.config import PSConfig
    from paddlebox_amd.ps.sparse_engine import SparseEngine

    dev = torch.device("cuda:0")
    torch.manual_seed(3)
    synth = CriteoSynth(total_features=20000, alpha=1.2, seed=5, device="cuda:0")
    B = 1024
    b = synth.batch(B)
    eng = SparseEngine(PSConfig(embedx_dim=8), max_keys=B * 26, device=dev, auto_insert=True, capacity=100000)
    mt = DCNv2(eng, hidden=(64, 32), cross_layers=2).to(dev)
    mw = DCNv2(eng, hidden=(64, 32), cross_layers=2, fused_tower=False).to(dev)
    assert mt.use_tower and not mw.use_tower
    D = mw.cross.dim
    with torch.no_grad():
        mt.w_c.normal_(0, 0.3)
        mt.w_c[mt.C:] = 0
        mw.w_c.copy_(mt.w_c[:D])
        for wt, ww, bt, bw in zip(mt.cross.w, mw.cross.w, mt.cross.b, mw.cross.b):
            ww.copy_(wt[:D, :D])
            bw.copy_(bt[:D])
        for pt, pw in zip(mt.mlp.parameters(), mw.mlp.parameters()):
            pw.copy_(pt)
    mt.mlp.invalidate_pack()
    for m in (mt, mw):
        m.dn.training = False  # keep the data_norm summaries fixed
    with torch.no_grad():
        mt(b)  # auto-insert the batch's keys
    join_grad_producers()
    eng.test_mode = True  # pulls only: both models see the same embeddings, no push
    res = {}
    for tag, m in (("tower", mt), ("ws", mw)):
        for p in m.parameters():
            p.grad = torch.zeros_like(p)
        loss, pred = m(b)
        loss.backward()
        join_grad_producers()
        torch.cuda.synchronize()
        res[tag] = (float(loss), m)
    assert abs(res["tower"][0] - res["ws"][0]) < 2e-3
    for gt, gw in [(mt.w_c.grad[:D], mw.w_c.grad)] + \
            [(a.grad[:D, :D], c.grad) for a, c in zip(mt.cross.w, mw.cross.w)] + \
            [(a.grad[:D], c.grad) for a, c in zip(mt.cross.b, mw.cross.b)] + \
            [(a.grad, c.grad) for a, c in zip(mt.mlp.parameters(), mw.mlp.parameters())]:
        if gw.abs().max() > 0:
            assert _rel(gt, gw) < 5e-2
