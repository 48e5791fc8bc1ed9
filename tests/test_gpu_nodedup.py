"""FLAGS_enable_pullpush_dedup_keys=false: the single-shard GPU step without a
key dedup (per-occurrence probe, seqpool from the rows, leader-elected push
merge + Adagrad; sparse_engine._pull_nodedup, sparse_ops.hip k_push_occ_*).
Checked against the fp32 torch oracle of ops/reference.py and against the
dedup engine over several training steps (reference: box_wrapper.cu:1049-1060)."""
import pytest
import torch

from paddlebox_amd.data.synthetic import CriteoSynth, ragged_batch
from paddlebox_amd.ops import reference as ref
from paddlebox_amd.ps.config import PSConfig
from paddlebox_amd.ps.sparse_engine import SeqpoolParams, SparseEngine
from paddlebox_amd.ps.config import row_layout

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _engine(dedup, dim=8, thr=2.0):
    cfg = PSConfig(embedx_dim=dim)
    cfg.sgd.mf_create_thresholds = thr
    return SparseEngine(cfg, max_keys=100000, device=torch.device(DEV), capacity=1 << 18, dedup=dedup)


def test_flag_selects_nodedup():
    from paddlebox_amd.utils import flags

    old = flags.get("enable_pullpush_dedup_keys")
    try:
        flags.set_flags({"enable_pullpush_dedup_keys": "false"})
        assert SparseEngine(PSConfig(embedx_dim=8), max_keys=1000, device=torch.device(DEV), capacity=4096).dedup is False
    finally:
        flags.set_flags({"enable_pullpush_dedup_keys": old})
    assert _engine(True).dedup is True


@pytest.mark.parametrize("ragged", [False, True])
def test_nodedup_pull_push_matches_reference(ragged):
    torch.manual_seed(4)
    if ragged:
        b = ragged_batch(64, 6, 6, 30, seed=9, device=DEV)
    else:
        b = CriteoSynth(total_features=20000, alpha=1.3, seed=5, device=DEV).batch(512)
    eng = _engine(False)
    assert not eng.dedup
    eng.register_keys(b.keys, init_embedx=False)
    vals = eng.table.values
    vals[:, :3] = torch.rand_like(vals[:, :3]) * 3
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
    assert st.extra.get("nodedup")
    exp_out = ref.seqpool_cvm(before, uid, b.lod, b.S, b.B, eng.E)
    torch.testing.assert_close(out, exp_out, rtol=1e-5, atol=1e-5)
    dout = torch.randn_like(out) * 0.01
    eng.push_seqpool_cvm(st, dout, b.cvm, 0, sp, float(b.B))
    after = vals[rows]
    push = ref.push_merge(dout, b.cvm, uid, b.lod, b.S, b.B, uniq.numel(), 8, eng._slot_ids(b.S), float(b.B))
    exp = ref.adagrad_update(before, push, 8, eng.cfg.sgd)
    newly = (before[:, l["mf_size"]] == 0) & (exp[:, l["mf_size"]] == 1)
    cols = [c for c in range(exp.shape[1]) if not (3 <= c < 11)]
    torch.testing.assert_close(after[:, cols], exp[:, cols], rtol=2e-4, atol=2e-5)
    torch.testing.assert_close(after[~newly, 3:11], exp[~newly, 3:11], rtol=2e-4, atol=2e-5)
    assert float(eng.push_acc_occ.abs().sum()) == 0.0


@pytest.mark.parametrize("dim", [8, 16])
def test_nodedup_trains_like_dedup(dim):
    """Several steps on power-law batches: same pooled outputs and table."""
    synth = CriteoSynth(total_features=50000, alpha=1.2, seed=7, device=DEV)
    batches = [synth.batch(256) for _ in range(4)]
    engs = [_engine(True, dim, 0.0), _engine(False, dim, 0.0)]
    E = 3 + dim
    for e in engs:
        for bt in batches:
            e.register_keys(bt.keys, init_embedx=True)
    outs = {0: [], 1: []}
    torch.manual_seed(0)
    douts = [torch.randn(256, synth.S * E, device=DEV) * 0.01 for _ in batches]
    sp = SeqpoolParams()
    for i, e in enumerate(engs):
        for bt, d in zip(batches, douts):
            out = torch.zeros(bt.B, bt.S * E, device=DEV)
            st = e.pull_seqpool_cvm(bt.keys, bt.lod, bt.B, bt.S, out, 0, sp)
            e.push_seqpool_cvm(st, d, bt.cvm, 0, sp, float(bt.B))
            outs[i].append(out)
    for a, b in zip(outs[0], outs[1]):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)
    k0, v0 = engs[0].table.export(True)
    k1, v1 = engs[1].table.export(True)
    o0, o1 = torch.argsort(k0), torch.argsort(k1)
    assert torch.equal(k0[o0], k1[o1])
    torch.testing.assert_close(v0[o0], v1[o1], rtol=1e-4, atol=1e-5)
