"""Numerics of the hand-written gfx950 kernels vs plain-PyTorch fp32 references.

All tests need an MI355X (marker ``gpu``); they fail loudly if the HIP
extension is missing (no eager fallback on GPU tensors).
"""
import math

import pytest
import torch

from paddlebox_amd import _native
from paddlebox_amd.data.synthetic import CriteoSynth, ragged_batch
from paddlebox_amd.ops import reference as ref
from paddlebox_amd.ps.config import PSConfig, SparseSGDConfig, row_layout
from paddlebox_amd.ps.sparse_engine import SeqpoolParams, SparseEngine

pytestmark = pytest.mark.gpu
DEV = "cuda"


def hip():
    return _native.hip()


def test_mix64_matches_reference():
    keys = torch.randint(0, 2**62, (1000,), dtype=torch.int64)
    for k in keys[:10].tolist():
        assert hip().mix64(k) == ref.mix64_int(k)
        assert hip().unmix64(hip().mix64(k)) == k
    t = ref.mix64(keys)
    assert [ (x & ((1 << 64) - 1)) for x in t[:10].tolist()] == [ref.mix64_int(k) for k in keys[:10].tolist()]


@pytest.mark.parametrize("hash_mode", [True, False])
def test_dedup_matches_unique(hash_mode):
    torch.manual_seed(0)
    n = 50000
    ws = hip().DedupWorkspace(n, 0, hash_mode)
    # a first, different batch: the hash table must be cleaned between runs
    ws.run(torch.randint(0, 10**9, (n // 2,), dtype=torch.int64, device=DEV), False)
    keys = torch.randint(0, 3000, (n,), dtype=torch.int64, device=DEV)
    keys[:2000] = 7  # one Zipf-hot key
    keys[-100:] = -1  # padding
    ws.run(keys, False)
    U = int(ws.u_count[0])
    nvalid = int(ws.u_count[1])
    h = ref.mix64(keys[:-100])
    uq = torch.unique(h)
    assert U == uq.numel()
    assert nvalid == n - 100
    got = ws.uniq_h[:U]
    # sorted as uint64: compare as sets
    assert torch.equal(torch.sort(got).values, torch.sort(uq).values)
    uid = ws.uid[: n - 100].long()
    assert torch.equal(got[uid], h)
    assert bool((ws.uid[n - 100:] == -1).all())
    seg = ws.seg[: U + 1].long()
    perm = ws.perm[:nvalid].long()
    counts = torch.bincount(uid, minlength=U)
    if hash_mode:
        # runs are contiguous but in no particular order: [seg[u], seg[u] + cnt[u])
        assert torch.equal(ws.cnt[:U].long(), counts)
        ends = seg[:U] + counts
        order = torch.argsort(seg[:U])
        assert int(seg[order[0]]) == 0 and torch.equal(seg[order[1:]], ends[order[:-1]])
        assert int(ends[order[-1]]) == nvalid
    else:
        ends = seg[1:U + 1]
    # every segment holds exactly the occurrences of one key
    for u in [0, 1, U // 2, U - 1]:
        occ = perm[seg[u]:ends[u]]
        assert occ.numel() == int(counts[u])
        assert bool((h[occ] == got[u]).all())
    assert torch.equal(torch.sort(perm).values, torch.arange(nvalid, device=perm.device))


def test_table_insert_probe_high_load():
    t = hip().GpuTable(8, 200_000, 1024, 0)
    cap = t.capacity
    n = int(cap * 0.9)
    keys = torch.unique(ref.mix64(torch.randint(0, 2**60, (n,), dtype=torch.int64, device=DEV)))
    fails = t.insert(keys, None, SparseSGDConfig().to_native(hip()), 7, True)
    assert fails == 0
    assert t.size() == keys.numel()
    rows = t.probe(keys, None)
    assert bool((rows >= 0).all())
    assert torch.unique(rows).numel() == keys.numel()
    other = ref.mix64(torch.randint(2**61, 2**62, (1000,), dtype=torch.int64, device=DEV))
    assert bool((t.probe(other, None) == -1).all())
    # embedx initialised and flagged created
    l = row_layout(8)
    v = t.values[rows[:100]]
    assert bool((v[:, l["mf_size"]] == 1).all())
    assert float(v[:, 3:11].abs().max()) <= 1e-4 + 1e-9
    # re-inserting existing keys is a no-op
    t.insert(keys[:1000], None, SparseSGDConfig().to_native(hip()), 8, False)
    assert t.size() == keys.numel()
    k, vals = t.export_all(True)
    assert k.numel() == keys.numel()
    assert torch.equal(torch.sort(k).values, torch.sort(keys).values)


def _engine(dim=8, max_keys=100000, cap=1 << 18, device=DEV):
    cfg = PSConfig(embedx_dim=dim)
    cfg.sgd.mf_create_thresholds = 2.0
    return SparseEngine(cfg, max_keys=max_keys, device=torch.device(device), capacity=cap)


@pytest.mark.parametrize("ragged", [False, True])
@pytest.mark.parametrize("use_cvm", [True, False])
def test_seqpool_cvm_matches_reference(ragged, use_cvm):
    torch.manual_seed(1)
    if ragged:
        b = ragged_batch(64, 5, 4, 50, seed=3, device=DEV)
    else:
        b = CriteoSynth(total_features=100000, seed=2, device=DEV).batch(128)
    eng = _engine()
    eng.register_keys(b.keys, init_embedx=True)
    sp = SeqpoolParams(use_cvm=use_cvm)
    # give rows non-trivial show/click/embed values
    vals = eng.table.values
    vals[:, :3] = torch.rand_like(vals[:, :3]) * 5
    Eo = sp.out_width(eng.E)
    out = torch.zeros(b.B, b.S * Eo, device=DEV)
    st = eng.pull_seqpool_cvm(b.keys, b.lod, b.B, b.S, out, 0, sp)
    # reference from the table rows
    uniq, uid = ref.dedup(b.keys)
    rows = eng.table.probe(uniq)
    src = vals[rows]
    exp = ref.seqpool_cvm(src, uid, b.lod, b.S, b.B, eng.E, use_cvm=use_cvm)
    torch.testing.assert_close(out, exp, rtol=1e-5, atol=1e-5)


def test_seqpool_filter_quant():
    b = ragged_batch(32, 4, 5, 40, seed=5, device=DEV)
    eng = _engine()
    eng.register_keys(b.keys, init_embedx=True)
    vals = eng.table.values
    vals[:, :2] = torch.rand_like(vals[:, :2]) * 3
    vals[:, 2:11] = torch.randn_like(vals[:, 2:11])
    sp = SeqpoolParams(need_filter=True, quant_ratio=128, threshold=0.5, pad_value=0.1)
    out = torch.zeros(b.B, b.S * 11, device=DEV)
    eng.pull_seqpool_cvm(b.keys, b.lod, b.B, b.S, out, 0, sp)
    uniq, uid = ref.dedup(b.keys)
    src = vals[eng.table.probe(uniq)]
    exp = ref.seqpool_cvm(src, uid, b.lod, b.S, b.B, 11, need_filter=True, quant_ratio=128, threshold=0.5,
                          pad_value=0.1)
    torch.testing.assert_close(out, exp, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("push_finish", ["0", "1"])
@pytest.mark.parametrize("ragged", [False, True])
def test_push_adagrad_matches_reference(ragged, push_finish, monkeypatch):
    """Fused merge + Adagrad vs the reference, in both straddling-run forms:
    per-unique arrival counters (one launch, default) and k_push_finish."""
    monkeypatch.setenv("PBX_PUSH_FINISH", push_finish)
    torch.manual_seed(4)
    if ragged:
        b = ragged_batch(64, 6, 6, 30, seed=9, device=DEV)
    else:
        b = CriteoSynth(total_features=20000, alpha=1.3, seed=5, device=DEV).batch(512)
    eng = _engine()
    eng.register_keys(b.keys, init_embedx=False)
    vals = eng.table.values
    vals[:, 2] = torch.randn_like(vals[:, 2]) * 0.1
    # half the rows already have embedx created
    l = row_layout(8)
    created = torch.rand(vals.shape[0], device=DEV) < 0.5
    vals[created, l["mf_size"]] = 1
    vals[created, 3:11] = torch.randn_like(vals[created, 3:11]) * 0.01
    sp = SeqpoolParams()
    uniq, uid = ref.dedup(b.keys)
    rows = eng.table.probe(uniq)
    before = vals[rows].clone()
    out = torch.zeros(b.B, b.S * 11, device=DEV)
    st = eng.pull_seqpool_cvm(b.keys, b.lod, b.B, b.S, out, 0, sp)
    dout = torch.randn_like(out) * 0.01
    eng.push_seqpool_cvm(st, dout, b.cvm, 0, sp, float(b.B))
    after = vals[rows]
    push = ref.push_merge(dout, b.cvm, uid, b.lod, b.S, b.B, uniq.numel(), 8, eng._slot_ids(b.S), float(b.B))
    exp = ref.adagrad_update(before, push, 8, eng.cfg.sgd)
    # newly created embedx are random: compare them by range only
    newly = (before[:, l["mf_size"]] == 0) & (exp[:, l["mf_size"]] == 1)
    cols = [c for c in range(exp.shape[1]) if not (3 <= c < 11)]
    torch.testing.assert_close(after[:, cols], exp[:, cols], rtol=2e-4, atol=2e-5)
    keep = ~newly
    torch.testing.assert_close(after[keep, 3:11], exp[keep, 3:11], rtol=2e-4, atol=2e-5)
    if bool(newly.any()):
        x = after[newly, 3:11]
        assert float(x.min()) >= 0 and float(x.max()) <= eng.cfg.sgd.mf_initial_range


def test_pull_box_sparse_records_and_push():
    b = ragged_batch(16, 3, 3, 20, seed=11, device=DEV)
    eng = _engine()
    eng.register_keys(b.keys, init_embedx=True)
    eng.table.values[:, :3] = torch.rand_like(eng.table.values[:, :3])
    recs, st = eng.pull_records(b.keys, b.lod, b.B, b.S)
    uniq, uid = ref.dedup(b.keys)
    exp = eng.table.values[eng.table.probe(uniq)][uid.long(), :11]
    torch.testing.assert_close(recs, exp)
    g = torch.randn_like(recs) * 0.01
    before = eng.table.values.clone()
    eng.push_records(st, g, 2, float(b.B))
    assert not torch.equal(before, eng.table.values)


def test_data_norm_fm_loss_auc_adam():
    torch.manual_seed(0)
    N, C = 300, 77
    x = torch.randn(N, C, device=DEV)
    bs = torch.full((C,), 1e4, device=DEV)
    bsum = torch.randn(C, device=DEV)
    bsq = torch.full((C,), 1e4, device=DEV) + torch.rand(C, device=DEV)
    y, m, s = hip().data_norm_fwd(x, bs, bsum, bsq, None, None)
    ye, me, se = ref.data_norm_fwd(x, bs, bsum, bsq)
    torch.testing.assert_close(y, ye)
    dy = torch.randn_like(x)
    dx, st = hip().data_norm_bwd(x, dy, m, s, 1e-5, True, None)
    dxe, ste = ref.data_norm_bwd(x, dy, me, se, 1e-5)
    torch.testing.assert_close(dx, dxe)
    torch.testing.assert_close(st, ste, rtol=1e-4, atol=1e-5)
    # FM
    B, S, D, Eo = 64, 26, 8, 11
    xx = torch.randn(B, S * Eo + 13, device=DEV)
    f = hip().fm_fwd(xx, S, D, 3, Eo)
    torch.testing.assert_close(f, ref.fm_fwd(xx, S, D, 3, Eo), rtol=1e-4, atol=1e-4)
    go = torch.randn(B, device=DEV)
    dxx = torch.zeros_like(xx)
    hip().fm_bwd(xx, go, S, D, 3, Eo, dxx, False)
    xr = xx.clone().requires_grad_(True)
    (gr,) = torch.autograd.grad(ref.fm_fwd(xr, S, D, 3, Eo), xr, go)
    torch.testing.assert_close(dxx, gr, rtol=1e-4, atol=1e-4)
    # loss
    z = torch.randn(1000, device=DEV)
    lab = (torch.rand(1000, device=DEV) < 0.3).float()
    p, l, dz = hip().sigmoid_logloss(z, lab, 1e-3)
    pe, le, dze = ref.sigmoid_logloss(z, lab, 1e-3)
    torch.testing.assert_close(p, pe)
    torch.testing.assert_close(l, le, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(dz, dze)
    # auc
    T = 1000
    tab = torch.zeros(2 * T, dtype=torch.float64, device=DEV)
    stt = torch.zeros(5, dtype=torch.float64, device=DEV)
    hip().auc_accumulate(p, lab, None, tab, stt)
    tab2 = torch.zeros_like(tab)
    st2 = torch.zeros_like(stt)
    ref.auc_accumulate(p, lab, tab2, st2)
    torch.testing.assert_close(tab, tab2)
    torch.testing.assert_close(stt, st2)
    # adam
    n = 1003
    pp = torch.randn(n, device=DEV)
    gg = torch.randn(n, device=DEV)
    m1 = torch.zeros(n, device=DEV)
    v1 = torch.zeros(n, device=DEV)
    p2, m2, v2 = pp.clone(), m1.clone(), v1.clone()
    pows = torch.ones(2, device=DEV)
    hip().adam_flat(pp, gg, m1, v1, pows, 1e-3, 0.9, 0.999, 1e-8, 0.5, 0.0)
    torch.testing.assert_close(pows, torch.tensor([0.9, 0.999], device=DEV))
    ref.adam_flat(p2, gg, m2, v2, 1e-3, 0.9, 0.999, 1e-8, 0.9, 0.999, 0.5, 0.0)
    torch.testing.assert_close(pp, p2)


def test_deepfm_trains_on_gpu():
    from paddlebox_amd.models.deepfm import DeepFM
    from paddlebox_amd.parallel.dense import DenseArena, FlatAdam

    synth = CriteoSynth(total_features=200000, alpha=1.1, seed=0, device=DEV)
    eng = SparseEngine(PSConfig(embedx_dim=8), max_keys=1024 * 26, device=torch.device(DEV), capacity=300000,
                       auto_insert=True)
    model = DeepFM(eng, hidden=(64, 32)).to(DEV)
    arena = DenseArena(model.parameters(), torch.device(DEV))
    opt = FlatAdam(arena, lr=3e-3)
    losses = []
    for i in range(60):
        b = synth.batch(1024)
        arena.zero_grad()
        loss, pred = model(b)
        loss.backward()
        opt.step()
        losses.append(float(loss))
    assert math.isfinite(losses[-1])
    assert sum(losses[-10:]) / 10 < sum(losses[:10]) / 10


def _bf(x):
    return x.to(torch.bfloat16)


@pytest.mark.parametrize("M,N,K", [(300, 400, 304), (8192, 400, 400), (64, 64, 64), (130, 72, 24)])
def test_mfma_linear_fwd_bwd(M, N, K):
    torch.manual_seed(M + N + K)
    x = _bf(torch.randn(M, K, device=DEV))
    w = _bf(torch.randn(N, K, device=DEV) * 0.1)
    b = torch.randn(N, device=DEV)
    y = hip().linear_fwd(x, w, b, True)
    ye = torch.relu(x.float() @ w.float().t() + b)
    torch.testing.assert_close(y.float(), ye, rtol=2e-2, atol=2e-2)
    y2 = hip().linear_fwd(x, w, b, False)
    torch.testing.assert_close(y2.float(), x.float() @ w.float().t() + b, rtol=2e-2, atol=2e-2)
    dy = _bf(torch.randn(M, N, device=DEV))
    dW = torch.zeros(N, K, device=DEV)
    db = torch.zeros(N, device=DEV)
    dx = hip().linear_bwd(dy, y, x, w, dW, db, True, 128)
    dz = dy.float() * (y.float() > 0)
    torch.testing.assert_close(dx.float(), dz @ w.float(), rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(dW, dz.t() @ x.float(), rtol=1e-2, atol=5e-2)
    torch.testing.assert_close(db, dz.sum(0), rtol=1e-2, atol=5e-2)


def test_gemv_out():
    h = _bf(torch.rand(777, 400, device=DEV))
    w = torch.randn(400, device=DEV)
    b = torch.randn(1, device=DEV)
    out = hip().gemv_out(h, w, b)
    torch.testing.assert_close(out, h.float() @ w + b, rtol=1e-4, atol=1e-3)
    dout = torch.randn(777, device=DEV)
    dw = torch.zeros(400, device=DEV)
    db = torch.zeros(1, device=DEV)
    dh = hip().gemv_out_bwd(h, w, dout, dw, db)
    torch.testing.assert_close(dh.float(), dout[:, None] * w[None, :], rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(dw, dout @ h.float(), rtol=1e-3, atol=1e-2)
    torch.testing.assert_close(db, dout.sum().view(1), rtol=1e-4, atol=1e-3)


def test_ctr_head_gpu_matches_cpu():
    from paddlebox_amd.ops.ctr import DataNorm, ctr_head

    torch.manual_seed(0)
    B, S, Eo, D = 100, 26, 11, 8
    C = S * Eo + 13
    Cp = (C + 7) // 8 * 8
    x = torch.randn(B, C)
    dn_c = DataNorm(C)
    dn_c.batch_sum.normal_()
    dn_g = DataNorm(C).to(DEV)
    dn_g.load_state_dict(dn_c.state_dict())
    xc = x.clone().requires_grad_(True)
    xg = x.to(DEV).requires_grad_(True)
    yc, lc = ctr_head(xc, dn_c, S, Eo, 2, D, Cp)
    yg, lg = ctr_head(xg, dn_g, S, Eo, 2, D, Cp)
    torch.testing.assert_close(yg.float().cpu(), yc, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(lg.cpu(), lc, rtol=1e-4, atol=1e-3)
    dy = torch.randn(B, Cp).to(torch.bfloat16).float()
    dl = torch.randn(B)
    ((yc * dy).sum() + (lc * dl).sum()).backward()  # one backward -> one summary update
    ((yg.float() * dy.to(DEV)).sum() + (lg * dl.to(DEV)).sum()).backward()
    torch.testing.assert_close(xg.grad.cpu(), xc.grad, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(dn_g.batch_sum.cpu(), dn_c.batch_sum, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(dn_g.batch_square_sum.cpu(), dn_c.batch_square_sum, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("M,dims", [(8192, [280, 400, 400, 400]), (300, [24, 72, 8]), (1000, [64, 128, 64])])
def test_mlp_workspace_matches_fp32(M, dims):
    """Workspace MLP (DMA-staged NT GEMMs, transposed activations, fused
    masks, split-K atomics) vs an fp32 reference on the same bf16 inputs."""
    from paddlebox_amd.ops.mlp import FusedMLP

    torch.manual_seed(M)
    mlp = FusedMLP(dims[0], dims[1:], 1).to(DEV)
    mlp.ensure_grads()
    for p in mlp.parameters():
        p.grad.zero_()
    ws = mlp.workspace(M, torch.device(DEV))
    x = _bf(torch.randn(M, dims[0], device=DEV))
    ws.x(0)[:, :dims[0]] = x
    ws.xt(0)[:dims[0], :M] = x.t()
    x0 = ws.x(0).detach().requires_grad_(True)
    logits = mlp.forward_ws(x0)
    # reference with bf16-rounded weights and activations
    h = x.float()
    hs = [h]
    for w, b in zip(mlp.w, mlp.b):
        h = torch.relu(h @ _bf(w).float().t() + b).to(torch.bfloat16).float()
        hs.append(h)
    ref_logit = h @ mlp.w_out.view(-1) + mlp.b_out
    torch.testing.assert_close(logits, ref_logit, rtol=3e-2, atol=3e-2)
    dl = torch.randn(M, device=DEV)
    logits.backward(dl)
    # reference backward on the activations the kernels stored (so ReLU masks
    # agree exactly), gradients rounded to bf16 where the kernels store them
    torch.testing.assert_close(ws.x(len(dims) - 1)[:, :dims[-1]].float(), hs[-1], rtol=3e-2, atol=3e-2)
    hs = [ws.x(i)[:, :dims[i]].float() for i in range(len(dims))]
    wo = mlp.w_out.detach().view(-1)
    dz = (dl[:, None] * wo[None, :] * (hs[-1] > 0)).to(torch.bfloat16).float()
    gw, gb = [None] * len(hs[:-1]), [None] * len(hs[:-1])
    g_wo = dl @ hs[-1]
    dx = None
    for l in reversed(range(len(mlp.w))):
        gw[l] = dz.t() @ hs[l]
        gb[l] = dz.sum(0)
        dx = dz @ _bf(mlp.w[l].detach()).float()
        if l > 0:
            dz = (dx * (hs[l] > 0)).to(torch.bfloat16).float()
    for w, g in zip(mlp.w, gw):
        torch.testing.assert_close(w.grad, g, rtol=2e-2, atol=1e-2 * float(g.abs().max()))
    for b, g in zip(mlp.b, gb):
        torch.testing.assert_close(b.grad, g, rtol=2e-2, atol=1e-2 * float(g.abs().max()))
    torch.testing.assert_close(mlp.w_out.grad.view(-1), g_wo, rtol=2e-2, atol=1e-2 * float(g_wo.abs().max()))
    torch.testing.assert_close(x0.grad[:, :dims[0]].float(), dx, rtol=2e-2, atol=1e-2 * float(dx.abs().max()))


@pytest.mark.parametrize("B", [1, 300, 8192, 300001])
def test_logit_loss_multiblock(B):
    torch.manual_seed(B)
    a = torch.randn(B, device=DEV) * 3
    b = torch.randn(B, device=DEV)
    y = (torch.rand(B, device=DEV) < 0.3).float()
    ws = torch.zeros(1025, dtype=torch.int32, device=DEV)
    for _ in range(2):  # second launch checks the ticket re-arms
        loss, pred, dz = hip().logit_loss(a, b, y, ws)
    assert int(ws[0]) == 0
    z = (a + b).double()
    pe = torch.sigmoid(z)
    le = torch.nn.functional.binary_cross_entropy_with_logits(z, y.double())
    torch.testing.assert_close(pred.double(), pe, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(dz.double(), (pe - y.double()) / B, rtol=1e-5, atol=1e-9)
    assert float(loss) == pytest.approx(float(le), rel=1e-5)


def test_two_outstanding_pulls_push_their_own_state():
    """Two pulls before either push (two pull ops in one program): each push
    must use its own pull's dedup/occurrence buffers (pull ring).  Expected:
    the same table as pull2 -> push2 -> pull1 -> push1 on a fresh engine (push
    results depend on the gradients and key structure, not on pulled values)."""
    b1 = ragged_batch(48, 5, 4, 40, seed=21, device=DEV)
    b2 = ragged_batch(48, 5, 4, 40, seed=22, device=DEV)
    g = torch.Generator(device=DEV).manual_seed(7)
    d1 = torch.randn(b1.B, b1.S * 11, device=DEV, generator=g) * 0.01
    d2 = torch.randn(b2.B, b2.S * 11, device=DEV, generator=g) * 0.01
    sp = SeqpoolParams()
    tables = []
    for mode in ("interleaved", "one_at_a_time"):
        eng = _engine()
        eng.register_keys(torch.cat([b1.keys, b2.keys]), init_embedx=True)
        l = row_layout(8)
        vals = eng.table.values
        vals[:, l["mf_size"]] = 1  # embedx already created: updates are deterministic
        o1 = torch.zeros(b1.B, b1.S * 11, device=DEV)
        o2 = torch.zeros(b2.B, b2.S * 11, device=DEV)
        if mode == "interleaved":
            s1 = eng.pull_seqpool_cvm(b1.keys, b1.lod, b1.B, b1.S, o1, 0, sp)
            s2 = eng.pull_seqpool_cvm(b2.keys, b2.lod, b2.B, b2.S, o2, 0, sp)
            eng.push_seqpool_cvm(s2, d2, b2.cvm, 0, sp, float(b2.B))
            eng.push_seqpool_cvm(s1, d1, b1.cvm, 0, sp, float(b1.B))
        else:
            s2 = eng.pull_seqpool_cvm(b2.keys, b2.lod, b2.B, b2.S, o2, 0, sp)
            eng.push_seqpool_cvm(s2, d2, b2.cvm, 0, sp, float(b2.B))
            s1 = eng.pull_seqpool_cvm(b1.keys, b1.lod, b1.B, b1.S, o1, 0, sp)
            eng.push_seqpool_cvm(s1, d1, b1.cvm, 0, sp, float(b1.B))
        uq = torch.unique(torch.cat([b1.keys, b2.keys]))
        uq = uq[uq != -1]
        tables.append(eng.table.read(ref.mix64(uq)))
    torch.testing.assert_close(tables[0], tables[1], rtol=1e-5, atol=1e-6)


def test_stale_pull_state_raises():
    b = ragged_batch(16, 3, 3, 20, seed=11, device=DEV)
    cfg = PSConfig(embedx_dim=8)
    eng = SparseEngine(cfg, max_keys=100000, device=torch.device(DEV), capacity=1 << 16, pull_ring=1)
    eng.register_keys(b.keys)
    sp = SeqpoolParams()
    out = torch.zeros(b.B, b.S * 11, device=DEV)
    s1 = eng.pull_seqpool_cvm(b.keys, b.lod, b.B, b.S, out, 0, sp)
    eng.pull_seqpool_cvm(b.keys, b.lod, b.B, b.S, out, 0, sp)
    with pytest.raises(RuntimeError, match="stale pull state"):
        eng.push_seqpool_cvm(s1, torch.zeros_like(out), b.cvm, 0, sp, float(b.B))


@pytest.mark.parametrize("ets", [0, 3])
def test_seqpool_embed_threshold_no_cvm(ets):
    """embed_threshold_filter with embed_thres_size 0 (= whole embedding) and
    use_cvm=False dropping cvm_offset + embed_thres_size columns, fwd + push."""
    b = ragged_batch(32, 4, 5, 40, seed=5, device=DEV)
    eng = _engine()
    eng.register_keys(b.keys, init_embedx=True)
    vals = eng.table.values
    torch.manual_seed(8)
    vals[:, :2] = torch.rand_like(vals[:, :2]) * 3
    vals[:, 2:11] = torch.randn_like(vals[:, 2:11]) * 0.5
    sp = SeqpoolParams(use_cvm=False, embed_threshold_filter=True, embed_threshold=1.0, embed_thres_size=ets,
                       threshold=0.0)
    Eo = sp.out_width(11)
    assert Eo == 11 - 2 - ets
    out = torch.zeros(b.B, b.S * Eo, device=DEV)
    st = eng.pull_seqpool_cvm(b.keys, b.lod, b.B, b.S, out, 0, sp)
    uniq, uid = ref.dedup(b.keys)
    rows = eng.table.probe(uniq)
    src = vals[rows].clone()
    exp = ref.seqpool_cvm(src, uid, b.lod, b.S, b.B, 11, use_cvm=False, embed_threshold_filter=True,
                          embed_threshold=1.0, embed_thres_size=ets, threshold=0.0)
    torch.testing.assert_close(out, exp, rtol=1e-5, atol=1e-5)
    dout = torch.randn_like(out) * 0.01
    before = vals[rows].clone()
    eng.push_seqpool_cvm(st, dout, b.cvm, 0, sp, float(b.B))
    push = ref.push_merge(dout, b.cvm, uid, b.lod, b.S, b.B, uniq.numel(), 8, eng._slot_ids(b.S), float(b.B),
                          use_cvm=False, embed_thres_size=ets)
    exp_rows = ref.adagrad_update(before, push, 8, eng.cfg.sgd)
    after = vals[rows]
    torch.testing.assert_close(after[:, :3], exp_rows[:, :3], rtol=2e-4, atol=2e-5)


def test_shrink_reaches_stash_rows():
    """Keys that overflowed the buckets into the stash are decayed / aged /
    deleted by shrink like bucket rows (the stash is compacted)."""
    from paddlebox_amd.ps.config import ShrinkConfig
    from paddlebox_amd.ps.gpu_table import GpuSparseTable

    t = GpuSparseTable(8, 64, DEV, stash_cap=1024, load_factor=1.0)
    h = ref.mix64(torch.arange(1, 301, dtype=torch.int64, device=DEV))
    t.insert_mixed(h, SparseSGDConfig())
    assert bool((t.probe(h) >= 0).all()) and int(t.t.stash_n()) > 0
    n0 = t.size()
    # keep everything once: rows age by a day, nothing deleted, all still found
    assert t.shrink(ShrinkConfig(delete_threshold=-1.0, delete_after_unseen_days=5.0)) == 0
    assert bool((t.probe(h) >= 0).all()) and t.size() == n0
    # rows unseen for more than 1 day go, stash included
    deleted = t.shrink(ShrinkConfig(delete_threshold=-1.0, delete_after_unseen_days=1.5))
    assert deleted == 300
    assert bool((t.probe(h) < 0).all())
    assert int(t.t.stash_n()) == 0


def test_split_pull_matches_inline_dedup():
    """Split pull (fused probe in the seqpool, table dedup on a side stream
    joined by the push) == the inline table dedup, over batches of different
    sizes in -1 padded key buffers (the rows buffer must read -1 outside the
    lod on every pull)."""
    synth = CriteoSynth(total_features=30000, alpha=1.2, seed=11, device=DEV)
    batches = [synth.batch(n) for n in (512, 128, 384, 256)]
    engs = []
    for split in (True, False):
        torch.manual_seed(0)
        e = _engine()
        e.split_pull = split
        for b in batches:
            e.register_keys(b.keys, init_embedx=True)
        engs.append(e)
    allk = torch.cat([b.keys.reshape(-1) for b in batches])
    h = torch.unique(ref.mix64(allk[allk != -1]))
    engs[1].table.assign(h, engs[0].table.read(h))
    sp = SeqpoolParams()
    for it in range(6):
        b = batches[it % len(batches)]
        pad = torch.full((97,), -1, dtype=torch.int64, device=DEV)
        keys = torch.cat([b.keys.reshape(-1), pad])
        outs = []
        for e in engs:
            out = torch.zeros(b.B, b.S * 11, device=DEV)
            st = e.pull_seqpool_cvm(keys, b.lod, b.B, b.S, out, 0, sp)
            dout = torch.sin(out * 7.0 + it) * 0.01
            e.push_seqpool_cvm(st, dout, b.cvm, 0, sp, float(b.B))
            outs.append(out)
        torch.cuda.synchronize()
        torch.testing.assert_close(outs[0], outs[1], rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(engs[0].table.read(h), engs[1].table.read(h), rtol=1e-5, atol=1e-6)
    rows = engs[0]._slots[0].ws.table_rows_occ()
    assert bool((rows == -1).all()), "rows buffer not handed back all -1"


def test_big_table_falls_back_to_hash_dedup(monkeypatch):
    """Single-GPU tables past the table dedup's int32 row space take the hash
    dedup (VERDICT r3 #6a); forced here by lowering the limit: the engine
    selects the fallback and trains exactly like the table dedup."""
    import paddlebox_amd.ps.sparse_engine as se

    synth = CriteoSynth(total_features=30000, alpha=1.2, seed=12, device=DEV)
    batches = [synth.batch(n) for n in (512, 256)]
    engs = []
    for limit in (se.TABLE_DEDUP_MAX_ROWS, 1000):
        monkeypatch.setattr(se, "TABLE_DEDUP_MAX_ROWS", limit)
        torch.manual_seed(0)
        e = _engine()
        for b in batches:
            e.register_keys(b.keys, init_embedx=True)
        engs.append(e)
    assert engs[0].table_dedup and not engs[1].table_dedup
    allk = torch.cat([b.keys.reshape(-1) for b in batches])
    h = torch.unique(ref.mix64(allk[allk != -1]))
    engs[1].table.assign(h, engs[0].table.read(h))
    sp = SeqpoolParams()
    for it in range(4):
        b = batches[it % len(batches)]
        outs = []
        for e in engs:
            out = torch.zeros(b.B, b.S * 11, device=DEV)
            st = e.pull_seqpool_cvm(b.keys.reshape(-1), b.lod, b.B, b.S, out, 0, sp)
            dout = torch.sin(out * 5.0 + it) * 0.01
            e.push_seqpool_cvm(st, dout, b.cvm, 0, sp, float(b.B))
            outs.append(out)
        torch.cuda.synchronize()
        torch.testing.assert_close(outs[0], outs[1], rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(engs[0].table.read(h), engs[1].table.read(h), rtol=1e-5, atol=1e-6)
