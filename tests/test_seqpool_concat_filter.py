"""embedx_concate_filter / need_filter / embed_threshold_filter matrix of
fused_seqpool_cvm against a numpy transcription of the reference kernels
(tests/seqpool_concat_oracle.py; fused_seqpool_cvm_op.cu:180-227,317-365).
CPU: the torch path; GPU: k_spv_fwd (csrc/hip/seqpool_variants.hip)."""
import itertools

import numpy as np
import pytest
import torch

from paddlebox_amd.ops import ctr_ext as cx

from .seqpool_concat_oracle import ref_fused_seqpool_cvm

MATRIX = list(itertools.product([False, True], [1, 3], [False, True], [False, True]))


def _records(seed, B=41, S=2, E=10):
    g = torch.Generator().manual_seed(seed)
    xs, offs = [], []
    for _ in range(S):
        lens = torch.randint(0, 6, (B,), generator=g)
        off = torch.zeros(B + 1, dtype=torch.int64)
        off[1:] = torch.cumsum(lens, 0)
        L = int(off[-1])
        x = torch.rand(L, E, generator=g, dtype=torch.float64) * 2 - 0.5
        x[:, 0] = torch.randint(0, 12, (L,), generator=g).double()  # show
        x[:, 1] = (x[:, 0] * torch.rand(L, generator=g, dtype=torch.float64)).floor()  # click <= show
        xs.append(x)
        offs.append(off)
    return xs, offs


def _attrs(need, ecs, cflag, embf):
    return dict(use_cvm=True, cvm_offset=2, pad_value=0.25, need_filter=need, show_coeff=0.2, clk_coeff=1.0,
                threshold=1.3, quant_ratio=128 if need else 0, embed_threshold_filter=embf, embed_threshold=1.1,
                embed_thres_size=5, embedx_concate_size=ecs, embedx_concate_filter=cflag)


def _oracle(xs, offs, B, a):
    kw = {k: v for k, v in a.items() if k != "use_cvm"}
    return ref_fused_seqpool_cvm([x.numpy() for x in xs], [o.numpy() for o in offs], B, **kw)


@pytest.mark.parametrize("need,ecs,cflag,embf", MATRIX)
def test_concat_filter_matrix_cpu(need, ecs, cflag, embf):
    B = 41
    xs, offs = _records(7 + ecs, B)
    a = _attrs(need, ecs, cflag, embf)
    exp = _oracle(xs, offs, B, a)
    got = cx.seqpool_cvm_variant("fused_seqpool_cvm", xs, offs, B, torch.rand(B, 2, dtype=torch.float64), a)
    for g, e in zip(got, exp):
        np.testing.assert_allclose(g.detach().double().numpy(), e, rtol=1e-5, atol=1e-5)


def test_concat_filter_changes_result():
    """The flag matters: with need_filter and concat, filtering on and off differ."""
    B = 41
    xs, offs = _records(11, B)
    on = _oracle(xs, offs, B, _attrs(True, 3, True, False))
    off = _oracle(xs, offs, B, _attrs(True, 3, False, False))
    assert any(not np.allclose(a, b) for a, b in zip(on, off))


@pytest.mark.gpu
@pytest.mark.parametrize("need,ecs,cflag,embf", MATRIX)
def test_concat_filter_matrix_gpu(need, ecs, cflag, embf):
    B = 41
    xs, offs = _records(7 + ecs, B)
    a = _attrs(need, ecs, cflag, embf)
    exp = _oracle(xs, offs, B, a)
    dev = torch.device("cuda:0")
    got = cx.seqpool_cvm_variant("fused_seqpool_cvm", [x.float().to(dev) for x in xs], [o.to(dev) for o in offs],
                                 B, torch.rand(B, 2).to(dev), a)
    for g, e in zip(got, exp):
        np.testing.assert_allclose(g.detach().double().cpu().numpy(), e, rtol=2e-5, atol=2e-5)
