"""CPU tests of the fp32 reference ops (the oracles) against naive loops and
autograd."""
import math

import numpy as np
import pytest
import torch

from paddlebox_amd.data.synthetic import ragged_batch
from paddlebox_amd.ops import reference as ref
from paddlebox_amd.ps.config import SparseSGDConfig, row_layout


def test_mix64_roundtrip_and_owner():
    k = torch.randint(-(2**62), 2**62, (1000,), dtype=torch.int64)
    h = ref.mix64(k)
    assert torch.equal(ref.unmix64(h), k)
    for a, b in zip(k[:20].tolist(), h[:20].tolist()):
        assert (b & ((1 << 64) - 1)) == ref.mix64_int(a)
        assert ref.unmix64_int(ref.mix64_int(a)) == a & ((1 << 64) - 1)
    for n in (1, 2, 3, 7, 8):
        o = ref.owner_of(h, n)
        exp = [((x & ((1 << 64) - 1)) * n) >> 64 for x in h.tolist()]
        assert o.tolist() == exp
        assert o.min() >= 0 and o.max() < n


def test_owner_monotone_in_unsigned_h():
    h = ref.mix64(torch.arange(1, 5000, dtype=torch.int64))
    u = [(x & ((1 << 64) - 1)) for x in h.tolist()]
    o = ref.owner_of(h, 8).tolist()
    pairs = sorted(zip(u, o))
    assert all(pairs[i][1] <= pairs[i + 1][1] for i in range(len(pairs) - 1))


def _naive_seqpool(src, uid, lod, S, B, E, use_cvm, cvm_offset=2, pad=0.0):
    lod = lod.view(S, B + 1)
    Eo = E if use_cvm else E - cvm_offset
    out = torch.zeros(B, S * Eo)
    for s in range(S):
        for b in range(B):
            acc = [pad] * E
            for k in range(int(lod[s, b]), int(lod[s, b + 1])):
                row = src[int(uid[k])]
                for c in range(E):
                    acc[c] += float(row[c])
            if use_cvm:
                vals = [math.log(acc[0] + 1), math.log(acc[1] + 1) - math.log(acc[0] + 1)] + acc[2:]
            else:
                vals = acc[cvm_offset:]
            out[b, s * Eo:(s + 1) * Eo] = torch.tensor(vals)
    return out


@pytest.mark.parametrize("use_cvm", [True, False])
def test_seqpool_cvm_vs_naive(use_cvm):
    b = ragged_batch(8, 3, 3, 10, seed=1)
    uniq, uid = ref.dedup(b.keys)
    src = torch.rand(uniq.numel(), 11) * 3
    got = ref.seqpool_cvm(src, uid, b.lod, b.S, b.B, 11, use_cvm=use_cvm, pad_value=0.25)
    exp = _naive_seqpool(src, uid, b.lod, b.S, b.B, 11, use_cvm, pad=0.25)
    torch.testing.assert_close(got, exp, rtol=1e-5, atol=1e-5)


def test_push_merge_vs_naive():
    b = ragged_batch(6, 3, 4, 8, seed=2)
    uniq, uid = ref.dedup(b.keys)
    U = uniq.numel()
    dout = torch.randn(b.B, b.S * 11)
    slot_ids = torch.tensor([10.0, 20.0, 30.0])
    push = ref.push_merge(dout, b.cvm, uid, b.lod, b.S, b.B, U, 8, slot_ids, float(b.B))
    lod = b.lod.view(b.S, b.B + 1)
    exp = torch.zeros(U, 12)
    for s in range(b.S):
        for i in range(b.B):
            for k in range(int(lod[s, i]), int(lod[s, i + 1])):
                u = int(uid[k])
                exp[u, 0] = slot_ids[s]
                exp[u, 1] += b.cvm[i, 0]
                exp[u, 2] += b.cvm[i, 1]
                exp[u, 3:] += -b.B * dout[i, s * 11 + 2:s * 11 + 11]
    torch.testing.assert_close(push, exp, rtol=1e-5, atol=1e-4)


def test_adagrad_update_semantics():
    cfg = SparseSGDConfig(mf_create_thresholds=5.0)
    l = row_layout(8)
    v = torch.zeros(3, l["stride"])
    v[1, l["mf_size"]] = 1
    v[1, 3:11] = 0.5
    push = torch.zeros(3, 12)
    push[:, 0] = 7
    push[:, 1] = torch.tensor([2.0, 4.0, 10.0])  # show
    push[:, 2] = torch.tensor([1.0, 0.0, 5.0])  # click
    push[:, 3] = torch.tensor([0.2, -0.4, 1.0])
    push[:, 4:] = 0.1
    r = torch.rand(3, 8)
    nv = ref.adagrad_update(v, push, 8, cfg, r)
    assert nv[:, l["slot"]].tolist() == [7, 7, 7]
    torch.testing.assert_close(nv[:, 0], push[:, 1])
    # embed_w: ratio = lr*sqrt(g0/(g0+0)) = lr ; w = g/show*lr
    torch.testing.assert_close(nv[:, 2], push[:, 3] / push[:, 1] * 0.05)
    # row1 existing embedx updated, row2 created (score 0.1*5+5=5.5 >= 5), row0 not (0.1*1+1=1.1)
    assert nv[0, l["mf_size"]] == 0 and nv[2, l["mf_size"]] == 1
    torch.testing.assert_close(nv[2, 3:11], r[2] * cfg.mf_initial_range)
    torch.testing.assert_close(nv[1, 3:11], torch.full((8,), 0.5) + 0.1 / 4 * 0.05)
    assert float(nv[0, l["delta_score"]]) == pytest.approx(0.1 * 1 + 1 * 1)


def test_data_norm_and_fm_grads():
    x = torch.randn(50, 9)
    bs, bsum, bsq = torch.full((9,), 1e4), torch.randn(9), torch.full((9,), 1e4)
    y, m, s = ref.data_norm_fwd(x, bs, bsum, bsq)
    torch.testing.assert_close(y, (x - bsum / bs) * torch.sqrt(bs / bsq))
    dx, st = ref.data_norm_bwd(x, torch.ones_like(x), m, s, 1e-5)
    torch.testing.assert_close(st[1], x.mean(0))
    xx = torch.randn(4, 26 * 11 + 13, requires_grad=True)
    f = ref.fm_fwd(xx, 26, 8, 3, 11)
    v = xx[:, [3 + s * 11 + d for s in range(26) for d in range(8)]].view(4, 26, 8)
    exp = 0.5 * ((v.sum(1) ** 2) - (v ** 2).sum(1)).sum(1)
    torch.testing.assert_close(f, exp)


def test_sigmoid_logloss_and_auc_tables():
    z = torch.randn(200)
    y = (torch.rand(200) < 0.4).float()
    p, l, dz = ref.sigmoid_logloss(z, y, 1 / 200)
    zz = z.clone().requires_grad_(True)
    loss = torch.nn.functional.binary_cross_entropy_with_logits(zz, y, reduction="mean")
    (g,) = torch.autograd.grad(loss, zz)
    torch.testing.assert_close(dz, g)
    tab = torch.zeros(2 * 100, dtype=torch.float64)
    st = torch.zeros(5, dtype=torch.float64)
    ref.auc_accumulate(p, y, tab, st)
    assert tab.sum().item() == 200 and st[4].item() == 200


def test_adam_flat_matches_closed_form():
    p = torch.ones(10)
    g = torch.full((10,), 0.5)
    m, v = torch.zeros(10), torch.zeros(10)
    ref.adam_flat(p, g, m, v, 0.1, 0.9, 0.999, 1e-8, 0.9, 0.999)
    # first step: m=0.05, v=0.00025; lr_t=0.1*sqrt(.001)/.1 ; step = lr_t*m/(sqrt(v)+eps*sqrt(.001)) ~ 0.1
    torch.testing.assert_close(p, torch.full((10,), 0.9), rtol=1e-4, atol=1e-4)
