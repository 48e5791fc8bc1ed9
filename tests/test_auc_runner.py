"""AucRunner (slot importance by feature replacement, native columnar
replacement in csrc/host/auc_runner.cc): replacing an informative slot costs
AUC, replacing a noise slot does not; replace/restore is exact."""
import types

import numpy as np
import torch
from sklearn.metrics import roc_auc_score

from paddlebox_amd.data.dataset import PadBoxSlotDataset, SlotVar
from paddlebox_amd.ps.auc_runner import AucRunner
from paddlebox_amd.ps.config import PSConfig
from paddlebox_amd.ps.sparse_engine import SparseEngine

N = 3000
SLOTS = ["inf", "noise", "weak"]


def _lines(n, seed=0):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        y = int(rng.random() < 0.5)
        inf = [1000 + 2 * int(rng.integers(0, 20)) + (y if rng.random() < 0.9 else 1 - y)]  # parity ~ label
        noise = rng.integers(5000, 5200, size=int(rng.integers(1, 3))).tolist()
        weak = [9000 + (y if rng.random() < 0.6 else 1 - y)]
        toks = ["1", str(y)]
        for v in (inf, noise, weak):
            toks += [str(len(v))] + [str(x) for x in v]
        toks += ["2", f"{rng.random():.3f}", f"{rng.random():.3f}"]
        out.append(" ".join(toks))
    return out


def _dataset():
    ds = PadBoxSlotDataset(rank=0, world=1)
    ds.set_use_var([SlotVar("label", "int64", (1,), 0)] + [SlotVar(s) for s in SLOTS] +
                   [SlotVar("dense", "float32", (2,), 0)])
    ds.set_batch_size(500)
    ds.set_label_var("label")
    ds.add_lines(_lines(N))
    return ds


def _batch(ds, b0, cnt):
    b = ds.build_batch(b0, cnt)
    return types.SimpleNamespace(keys=b.keys, lod=b.lod, dense=b.dense_var("dense").contiguous(), label=b.label,
                                 cvm=b.cvm, B=b.B, S=b.S)


def _snapshot(ds):
    return [ds.build_batch(b0, c).keys.clone() for b0, c in ds.prepare_train(shuffle=False)]


def test_replace_and_restore_are_exact():
    ds = _dataset()
    before = _snapshot(ds)
    r = AucRunner([["noise"], ["inf", "weak"]], thread_num=3, pool_size=64, seed=1)
    cand = r.prepare(ds)
    assert r.pool_entries() == 3 * 64 and cand.numel() > 0
    n = r.shuffle(ds, ["inf", "weak"])
    assert n > 0
    after = _snapshot(ds)
    changed = sum(int((a != b).sum()) for a, b in zip(before, after) if a.shape == b.shape)
    assert changed > 0 or any(a.shape != b.shape for a, b in zip(before, after))
    # replaced values come from the candidate pool
    allk = torch.cat(after)
    assert bool(torch.isin(allk[(allk >= 1000) & (allk < 1100)], cand).all())
    r.shuffle(ds, [])
    for a, b in zip(before, _snapshot(ds)):
        assert torch.equal(a, b)


def test_slot_importance_informative_vs_noise():
    torch.manual_seed(0)
    ds = _dataset()
    cfg = PSConfig(embedx_dim=4)
    cfg.sgd.mf_create_thresholds = 0.0
    eng = SparseEngine(cfg, max_keys=20000, device=torch.device("cpu"), capacity=100000, auto_insert=True)
    from paddlebox_amd.models.deepfm import DeepFM

    model = DeepFM(eng, num_slots=3, dense_dim=2, hidden=(16,), use_data_norm=False)
    opt = torch.optim.Adam(model.parameters(), lr=0.02)
    plan = ds.prepare_train(shuffle=False)
    for _ in range(4):
        for b0, c in plan:
            b = _batch(ds, b0, c)
            opt.zero_grad()
            loss, _ = model(b)
            loss.backward()
            opt.step()

    def evaluate():
        eng.test_mode = True
        preds, labels = [], []
        with torch.no_grad():
            for b0, c in plan:
                b = _batch(ds, b0, c)
                _, p = model(b)
                preds.append(p.detach().view(-1))
                labels.append(b.label.view(-1))
        eng.test_mode = False
        return roc_auc_score(torch.cat(labels).numpy(), torch.cat(preds).numpy())

    r = AucRunner([["inf"], ["noise"], ["weak"]], thread_num=2, pool_size=500, seed=3)
    eng.register_keys(r.prepare(ds))  # AddReplaceFeasign: candidates are in the table
    res = r.slot_importance(ds, evaluate)
    assert res["base"] > 0.9
    assert res["inf"] < res["base"] - 0.2  # informative slot: large AUC drop
    assert abs(res["noise"] - res["base"]) < 0.02  # noise slot: no drop
    assert res["inf"] < res["weak"] < res["base"]
    assert abs(evaluate() - res["base"]) < 1e-9  # restored


def test_boxwrapper_auc_runner_mode():
    """initialize_auc_runner + feed pass (candidates registered with the PS)
    + BoxHelper.slots_shuffle (phase flip, replace, restore)."""
    from paddlebox_amd.ps.box_wrapper import BoxWrapper

    box = BoxWrapper(4, device="cpu")
    try:
        box.initialize_gpu_and_load_model(slot_vector=[1, 2, 3], max_keys=50000)
        box.initialize_auc_runner([["inf"], ["noise"]], thread_num=2, pool_size=100)
        assert box.auc_runner_mode() == 1
        ds = _dataset()
        ds.box = box
        before = _snapshot(ds)
        box.feed_pass(ds)
        cand = box.auc_runner._n.candidate_keys()
        from paddlebox_amd.ops import reference as ref

        rows = box.engine.table.probe(ref.mix64(cand))
        assert bool((rows >= 0).all())  # AddReplaceFeasign
        p0 = box.phase
        ds.slots_shuffle(["inf"])
        assert box.phase != p0
        assert any(not torch.equal(a, b) for a, b in zip(before, _snapshot(ds)))
        ds.slots_shuffle([])
        for a, b in zip(before, _snapshot(ds)):
            assert torch.equal(a, b)
    finally:
        BoxWrapper._instance = None
