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


@pytest.mark.parametrize("M,C,L", [(1000, 304, 3), (4096, 64, 1), (333, 136, 2)])
def test_cross_stack_matches_fp64(M, C, L):
    """C = the padded MLP input width D; x0 / x0^T laid out as the MLP
    workspace's X_0 [M, pad64(D)] / X_0^T [pad64(D+1), pad64(M)] (ones row)."""
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
