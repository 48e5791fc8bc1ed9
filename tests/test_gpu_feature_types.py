"""GPU PS feature types (csrc/hip/feature_ops.hip): int16 embedx with
pull_embedx_scale, the expand block of pull_box_extended_sparse and the
SparseAdam rule, each against the torch oracle in ps/feature_types.py, plus
the engine end to end (codec path == the fused fp32 path for kind 0)."""
import pytest
import torch

from paddlebox_amd.ops import reference as ref
from paddlebox_amd.ps.config import PSConfig, SparseSGDConfig
from paddlebox_amd.ps.feature_types import KIND_ADAM, KIND_FP32, KIND_INT16, FeatureCodec
from paddlebox_amd.ps.gpu_table import GpuSparseTable

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
QS = 2.0 ** -12


def _sgd():
    c = SparseSGDConfig()
    c.mf_create_thresholds = 0.0
    return c


def _random_canon(codec: FeatureCodec, n: int, g: torch.Generator) -> torch.Tensor:
    c = codec.canon
    v = torch.zeros(n, codec.canon_width)
    v[:, 0] = torch.randint(1, 50, (n,), generator=g).float()
    v[:, 1] = (v[:, 0] * torch.rand(n, generator=g)).floor()
    v[:, 2] = torch.randn(n, generator=g) * 0.1
    v[:, 3:3 + codec.DX] = torch.randn(n, codec.DX, generator=g) * 0.05
    v[:, c["embed_g2sum"]] = torch.rand(n, generator=g)
    v[:, c["embedx_g2sum"]] = torch.rand(n, generator=g)
    v[:, c["delta_score"]] = torch.rand(n, generator=g)
    v[:, c["slot"]] = 3.0
    v[:, c["mf_size"]] = 1.0
    base = c["stride"]
    if codec.De:
        v[:, base + codec.eg2 - codec.raw["mf_size"] - 1] = torch.rand(n, generator=g)
    if codec.kind == KIND_ADAM:
        a = base + codec.adam - codec.raw["mf_size"] - 1
        DX = codec.DX
        v[:, a] = torch.randn(n, generator=g) * 0.01
        v[:, a + 1] = torch.rand(n, generator=g) * 0.01
        v[:, a + 2] = 0.9 ** torch.randint(1, 5, (n,), generator=g).float()
        v[:, a + 3] = 0.999 ** torch.randint(1, 5, (n,), generator=g).float()
        v[:, a + 4:a + 4 + DX] = torch.randn(n, DX, generator=g) * 0.01
        v[:, a + 4 + DX:a + 4 + 2 * DX] = torch.rand(n, DX, generator=g) * 0.01
        v[:, a + 4 + 2 * DX] = 0.9 ** 3
        v[:, a + 5 + 2 * DX] = 0.999 ** 3
    if codec.kind == KIND_INT16:  # start on the int16 grid
        v[:, 3:3 + codec.DX] = codec.quantize(v[:, 3:3 + codec.DX]) * codec.qscale
    return v


@pytest.mark.parametrize("kind", [KIND_FP32, KIND_INT16, KIND_ADAM])
@pytest.mark.parametrize("De", [0, 5])
def test_codec_update_matches_oracle(kind, De):
    g = torch.Generator().manual_seed(kind * 10 + De)
    codec = FeatureCodec(kind, 8, De, QS)
    t = GpuSparseTable(8, 5000, DEV, codec=codec)
    n = 777
    h = torch.unique(ref.mix64(torch.randint(0, 1 << 40, (n,), generator=g))).to(DEV)
    n = h.numel()
    cfg = _sgd()
    t.insert_mixed(h, cfg, init_embedx=True)
    canon = _random_canon(codec, n, g)
    t.assign(h, canon.to(DEV))
    got0 = t.read(h).cpu()
    torch.testing.assert_close(got0, canon, rtol=0, atol=0)  # exact round trip (values start on the grid)
    # pull records
    rows = t.probe(h)
    out = torch.zeros(n, 3 + codec.DX + 3, device=DEV)
    t.t.codec_pull(codec.native(), rows, None, None, n, out)
    torch.testing.assert_close(out[:, :3 + codec.DX].cpu(), canon[:, :3 + codec.DX], rtol=0, atol=0)
    # update
    push = torch.zeros(n, 4 + codec.DX + 2)
    push[:, 0] = 3.0
    push[:, 1] = torch.randint(0, 4, (n,), generator=g).float()
    push[:, 2] = (push[:, 1] * torch.rand(n, generator=g)).floor()
    push[:, 3:4 + codec.DX] = torch.randn(n, 1 + codec.DX, generator=g) * 0.3
    t.t.codec_update(codec.native(), rows, push.to(DEV), None, cfg.to_native(t._mod), 7)
    got = t.read(h).cpu()
    exp = codec.update_ref(canon, push, cfg)
    atol = QS * 1.01 if kind == KIND_INT16 else 1e-6
    torch.testing.assert_close(got, exp, rtol=1e-5, atol=atol)
    if kind == KIND_INT16:
        q = got[:, 3:3 + codec.DX] / QS
        assert torch.equal(q, q.round())


def test_int16_table_memory_and_creation():
    codec = FeatureCodec(KIND_INT16, 8, 0, QS)
    assert codec.raw_stride < FeatureCodec(KIND_FP32, 8).raw_stride  # 64 B vs 80 B rows
    t = GpuSparseTable(8, 1000, DEV, codec=codec)
    h = ref.mix64(torch.arange(100)).to(DEV)
    cfg = _sgd()
    cfg.mf_initial_range = 0.01
    t.insert_mixed(h, cfg, init_embedx=True)
    v = t.read(h).cpu()
    x = v[:, 3:11]
    assert bool((v[:, codec.canon["mf_size"]] == 1).all())
    assert float(x.abs().max()) <= 0.01 + QS and float(x.abs().sum()) > 0
    assert torch.equal(x / QS, (x / QS).round())


def _engine(cfg, B=64, S=4):
    from paddlebox_amd.ps.sparse_engine import SparseEngine

    return SparseEngine(cfg, max_keys=B * S * 4, device=DEV, capacity=50000,
                        slot_ids=[float(s + 1) for s in range(S)])


def _batches(n, B=64, S=4):
    from paddlebox_amd.data.synthetic import ragged_batch

    return [ragged_batch(B, S, 3, 300, seed=500 + i) for i in range(n)]


def _train(eng, batches):
    from paddlebox_amd.models.deepfm import DeepFM

    torch.manual_seed(0)
    model = DeepFM(eng, num_slots=4, dense_dim=13, hidden=(32, 32), use_data_norm=False).to(DEV)
    opt = torch.optim.SGD(model.parameters(), lr=0.01)
    losses = []
    for b in batches:
        b = b.to(DEV)
        eng.register_keys(b.keys, init_embedx=True)
        opt.zero_grad()
        loss, _ = model(b)
        loss.backward()
        opt.step()
        losses.append(float(loss.detach()))
    return losses


def test_engine_codec_fp32_equals_fused_path():
    """force_codec routes the default fp32 Adagrad rows through the codec
    kernels (decode -> seqpool, push_merge -> codec_update): same training."""
    batches = _batches(4)
    cfg = PSConfig(embedx_dim=8)
    cfg.sgd.mf_create_thresholds = 0.0
    e1 = _engine(cfg)
    l1 = _train(e1, batches)
    cfg2 = PSConfig(embedx_dim=8, force_codec=True)
    cfg2.sgd.mf_create_thresholds = 0.0
    e2 = _engine(cfg2)
    assert e2.codec is not None
    l2 = _train(e2, batches)
    assert l1 == pytest.approx(l2, rel=1e-4, abs=1e-5)
    h1, v1 = e1.table.export(True)
    o1 = torch.argsort(h1)
    h2, v2 = e2.table.export(True)
    o2 = torch.argsort(h2)
    assert torch.equal(h1[o1], h2[o2])
    torch.testing.assert_close(v2[o2][:, :v1.shape[1]], v1[o1], rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("ftype,opt", [(1, "adagrad"), (0, "adam")])
def test_engine_trains_with_feature_type(ftype, opt):
    cfg = PSConfig(embedx_dim=8, feature_type=ftype, pull_embedx_scale=QS, sparse_optimizer=opt)
    cfg.sgd.mf_create_thresholds = 0.0
    cfg.sgd.mf_initial_range = 0.01
    eng = _engine(cfg)
    assert eng.codec is not None and eng.codec.kind == (KIND_INT16 if ftype == 1 else KIND_ADAM)
    losses = _train(eng, _batches(6))
    assert all(torch.isfinite(torch.tensor(losses)))
    _, v = eng.table.export(True)
    x = v[:, 3:11].cpu()
    if ftype == 1:
        assert torch.equal(x / QS, (x / QS).round())
    assert float(x.abs().sum()) > 0


def test_extended_pull_push_codec():
    """pull_box_extended_sparse with the expand block in the same rows: the
    pull returns [embedx part | expand part] and the push applies both."""
    from paddlebox_amd.ps.extras import pull_extended_codec

    De, B, S = 4, 32, 2
    cfg = PSConfig(embedx_dim=8, expand_embed_dim=De)
    cfg.sgd.mf_create_thresholds = 0.0
    eng = _engine(cfg, B, S)
    g = torch.Generator().manual_seed(3)
    keys = torch.randperm(10000, generator=g)[: B * S].to(torch.int64)  # all distinct
    lod = torch.cat([torch.arange(B + 1), torch.arange(B, 2 * B + 1)]).to(torch.int64)
    keys, lod = keys.to(DEV), lod.to(DEV)
    eng.register_keys(keys, init_embedx=True)
    hk = ref.mix64(keys)
    before = eng.table.read(hk).cpu()
    out, ex = pull_extended_codec(eng, keys, lod, B, S, 11, De)
    torch.testing.assert_close(out.cpu(), before[:, :11], rtol=0, atol=0)
    torch.testing.assert_close(ex.cpu(), before[:, 11:11 + De], rtol=0, atol=0)
    go = torch.randn(B * S, 11, generator=g)
    ge = torch.randn(B * S, De, generator=g)
    torch.autograd.backward([out, ex], [go.to(DEV), ge.to(DEV)])
    push = torch.zeros(B * S, 4 + 8 + De)
    push[:, 0] = torch.tensor([1.0] * B + [2.0] * B)
    push[:, 1:3] = go[:, :2]
    push[:, 3:12] = go[:, 2:11] * (-float(B))
    push[:, 12:] = ge * (-float(B))
    exp = eng.codec.update_ref(before, push, cfg.sgd)
    torch.testing.assert_close(eng.table.read(hk).cpu(), exp, rtol=1e-5, atol=1e-6)


def test_variable_feature_pull_push():
    """Variable feature type (codec kind 3, reference PullCopyVariable /
    PushMergeCopyVariable): features of the expand slot are created with De
    columns, the others with D; each slot reads / writes only its own output
    and the update touches only the feature's live columns."""
    from paddlebox_amd.ps.extras import pull_extended_var
    from paddlebox_amd.ps.feature_types import KIND_VAR

    D, De, B, S = 8, 16, 32, 2
    cfg = PSConfig(embedx_dim=D, expand_embed_dim=De, feature_type=2)
    cfg.sgd.mf_create_thresholds = 0.0
    cfg.sgd.mf_initial_range = 0.01
    eng = _engine(cfg, B, S)
    c = eng.codec
    assert c.kind == KIND_VAR and c.DX == De
    g = torch.Generator().manual_seed(5)
    keys = torch.randperm(10000, generator=g)[: B * S].to(torch.int64) + 1  # all distinct
    lod = torch.cat([torch.arange(B + 1), torch.arange(B, 2 * B + 1)]).to(torch.int64)
    keys, lod = keys.to(DEV), lod.to(DEV)
    mask = [1, 2]  # slot 0 -> embedx output, slot 1 -> expand output
    eng.register_keys(keys, init_embedx=False)
    hk = ref.mix64(keys)
    size_col = c.canon["stride"] + (c.xsz - c.raw["mf_size"] - 1)
    # pass 1: nothing created yet -> zero embeddings; the push creates them
    out, ex = pull_extended_var(eng, keys, lod, B, S, 3 + D, 3 + De, mask)
    assert out.shape == (B * S, 3 + D) and ex.shape == (B * S, 3 + De)
    assert float(out[B:].abs().sum()) == 0 and float(ex[:B].abs().sum()) == 0
    assert float(out[:B, 3:].abs().sum()) == 0 and float(ex[B:, 3:].abs().sum()) == 0
    g1, g2 = torch.randn(out.shape, generator=g), torch.randn(ex.shape, generator=g)
    g1[:, :2] = g1[:, :2].abs() + 1  # show / click (cvm inputs) > 0: score passes the create threshold
    g2[:, :2] = g2[:, :2].abs() + 1
    torch.autograd.backward([out, ex], [g1.to(DEV), g2.to(DEV)])
    before = eng.table.read(hk).cpu()
    sizes = before[:, size_col]
    assert torch.equal(sizes[:B], torch.full((B,), float(D)))
    assert torch.equal(sizes[B:], torch.full((B,), float(De)))
    assert float(before[:B, 3 + D:3 + De].abs().sum()) == 0  # past the size: untouched zeros
    assert float(before[B:, 3:3 + De].abs().sum()) > 0
    # pass 2: pull values masked by size, push against the oracle
    out, ex = pull_extended_var(eng, keys, lod, B, S, 3 + D, 3 + De, mask)
    torch.testing.assert_close(out[:B].cpu(), before[:B, :3 + D], rtol=0, atol=0)
    torch.testing.assert_close(ex[B:].cpu(), before[B:, :3 + De], rtol=0, atol=0)
    go = torch.randn(B * S, 3 + D, generator=g)
    ge = torch.randn(B * S, 3 + De, generator=g)
    torch.autograd.backward([out, ex], [go.to(DEV), ge.to(DEV)])
    push = torch.zeros(B * S, 4 + De)
    push[:, 0] = torch.tensor([1.0] * B + [2.0] * B)
    push[:B, 1:3] = go[:B, :2]
    push[:B, 3:4 + D] = go[:B, 2:3 + D] * (-float(B))
    push[B:, 1:3] = ge[B:, :2]
    push[B:, 3:4 + De] = ge[B:, 2:3 + De] * (-float(B))
    exp = c.update_ref(before, push, cfg.sgd)
    after = eng.table.read(hk).cpu()
    torch.testing.assert_close(after, exp, rtol=1e-5, atol=1e-6)
