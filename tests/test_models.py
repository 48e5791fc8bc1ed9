"""Model families beyond DeepFM on the same sparse stack: Wide&Deep and
DCN-V2 (BASELINE configs 4/5).  CPU training runs here, GPU runs marked."""
import math

import numpy as np
import pytest
import torch

from paddlebox_amd.data.synthetic import CriteoSynth
from paddlebox_amd.models.dcn_v2 import CrossNetV2, DCNv2
from paddlebox_amd.models.wide_deep import WideDeep
from paddlebox_amd.parallel.dense import DenseArena, FlatAdam
from paddlebox_amd.ps.config import PSConfig
from paddlebox_amd.ps.sparse_engine import SparseEngine


def _train(cls, dev, steps, B, hidden, **kw):
    torch.manual_seed(0)
    synth = CriteoSynth(total_features=50000, alpha=1.2, seed=0, device=dev)
    extra = {"capacity": 300000} if dev != "cpu" else {}
    eng = SparseEngine(PSConfig(embedx_dim=8), max_keys=B * 26, device=torch.device(dev), auto_insert=True, **extra)
    model = cls(eng, hidden=hidden, **kw).to(dev)
    arena = DenseArena(model.parameters(), torch.device(dev))
    opt = FlatAdam(arena, lr=5e-3)
    losses = []
    for _ in range(steps):
        b = synth.batch(B)
        arena.zero_grad()
        loss, pred = model(b)
        loss.backward()
        opt.step()
        losses.append(float(loss.detach()))
    return model, eng, losses


@pytest.mark.parametrize("cls,kw", [(WideDeep, {}), (DCNv2, {"cross_layers": 2})])
def test_model_trains_on_cpu(cls, kw):
    model, eng, losses = _train(cls, "cpu", 50, 256, (32, 16), **kw)
    assert all(math.isfinite(x) for x in losses)
    assert np.mean(losses[-10:]) < np.mean(losses[:10])
    h, v = eng.table.export(True)
    assert float(v[:, 0].sum()) == pytest.approx(50 * 256 * 26)  # push reached every occurrence


def test_dcn_cross_matches_explicit_recurrence():
    torch.manual_seed(1)
    net = CrossNetV2(12, 3)
    x0 = torch.randn(5, 12, requires_grad=True)
    out = net(x0)
    out.sum().backward()
    x0r = x0.detach().clone().requires_grad_(True)
    x = x0r
    for w, b in zip(net.w, net.b):
        x = x0r * (x @ w.detach().t() + b.detach()) + x
    x.sum().backward()
    torch.testing.assert_close(out, x)
    torch.testing.assert_close(x0.grad, x0r.grad)


@pytest.mark.gpu
@pytest.mark.parametrize("cls,kw", [(WideDeep, {}), (DCNv2, {"cross_layers": 2})])
def test_model_trains_on_gpu(cls, kw):
    model, eng, losses = _train(cls, "cuda:0", 60, 1024, (64, 32), **kw)
    assert all(math.isfinite(x) for x in losses)
    assert np.mean(losses[-10:]) < np.mean(losses[:10])
