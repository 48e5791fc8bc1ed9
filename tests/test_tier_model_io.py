"""Tiered model IO over host + SSD: SaveBase / SaveDelta /
load / ShrinkTable see every feature, including the rows the host-tier cap
spilled to the SSD log, and agree with an all-in-memory oracle trained on
the same batches (reference: box_wrapper.cc:1286-1318, box_wrapper.h:638,
ctr_accessor.cc:63-170)."""
import os

import numpy as np
import torch

from paddlebox_amd.data.synthetic import ragged_batch
from paddlebox_amd.ops import reference as ref
from paddlebox_amd.ps import checkpoint as ck
from paddlebox_amd.ps.box_wrapper import BoxWrapper
from paddlebox_amd.ps.sparse_engine import SeqpoolParams

S = 3


def _batches():
    out = []
    for p in range(4):
        b = ragged_batch(64, S, 3, 300, seed=40 + p)
        k = b.keys.clone()
        # pass p shares keys with the pass before it; key 0 is never fed
        k[k != -1] = k[k != -1] % 300 + 150 * p + 1
        b.keys = k
        out.append(b)
    return out


def _box(mode, tmp_path=None, cap=0):
    box = BoxWrapper(8, device="cpu")
    box.cfg.sgd.mf_create_thresholds = 0.0
    box.cfg.sgd.mf_initial_range = 0.0  # placement-independent rows
    box.cfg.tier.spill_unseen_days = 1e9  # only the host cap spills
    box.cfg.tier.ssd_spill_threshold = cap
    box.cfg.save.base_threshold = 0.5
    box.cfg.save.delta_threshold = 0.3
    box.initialize_gpu_and_load_model(slot_vector=list(range(1, S + 1)), max_keys=50000, mode=mode,
                                      ssd_path=str(tmp_path / "ssd") if mode == "tiered" else None)
    return box


def _run_pass(box, b, p):
    eng = box.engine
    sp = SeqpoolParams()
    box.feed_pass(b.keys)
    box.begin_pass()
    out = torch.zeros(b.B, b.S * 11)
    st = eng.pull_seqpool_cvm(b.keys, b.lod, b.B, b.S, out, 0, sp)
    g = torch.Generator().manual_seed(1000 + p)
    eng.push_seqpool_cvm(st, torch.randn(out.shape, generator=g) * 0.05, b.cvm, 0, sp, float(b.B))
    box.end_pass()


def _rows(table):
    h, v = table.export(True)
    o = torch.argsort(h)
    return h[o], v[o]


def _part(path):
    k = np.load(os.path.join(path, "part-00000.keys.npy"), allow_pickle=False)
    v = np.load(os.path.join(path, "part-00000.vals.npy"), allow_pickle=False)
    o = np.argsort(k)
    return k[o], v[o]


def _xbox(path):
    k, v = ck.load_xbox_text(os.path.join(path, "part-00000.txt"), 8)
    o = np.argsort(k)
    return k[o], v[o]


def _same_rows(a, b, slot_col):
    keep = [c for c in range(a.shape[1]) if c != slot_col]
    np.testing.assert_allclose(a[:, keep], b[:, keep], rtol=1e-6, atol=1e-7)


def test_tiered_save_delta_load_shrink_cover_ssd(tmp_path):
    batches = _batches()
    try:
        ob = _box("hbm")
        for p, b in enumerate(batches):
            _run_pass(ob, b, p)
    finally:
        BoxWrapper._instance = None
    n_all = ob.engine.table.size()
    tb = _box("tiered", tmp_path, cap=int(n_all * 0.5))
    try:
        for p, b in enumerate(batches):
            _run_pass(tb, b, p)
        view = tb._authoritative()
        n_ssd = len(tb.ssd)
        assert n_ssd >= 0.3 * n_all, (n_ssd, n_all)  # a third of the table is cold, on SSD
        assert view.size() == n_all
        # no key in both tiers
        assert bool((tb.host.probe(tb.ssd.keys()) < 0).all())
        slot = tb.host.layout["slot"]
        oh, ov = _rows(ob.engine.table)
        th, tv = _rows(view)
        assert torch.equal(oh, th)
        _same_rows(tv.numpy(), ov.numpy(), slot)

        # SaveBase: batch model + xbox base, every tier
        tb.save_base(str(tmp_path / "t_batch"), str(tmp_path / "t_xbox"))
        ob.save_base(str(tmp_path / "o_batch"), str(tmp_path / "o_xbox"))
        assert ck.last_save_stats.get("ssd_rows", 0) > 0
        tk, tvv = _part(str(tmp_path / "t_batch"))
        okk, ovv = _part(str(tmp_path / "o_batch"))
        assert tk.shape[0] == n_all  # the repro: every row, not just the host tier's
        assert np.array_equal(tk, okk)
        _same_rows(tvv, ovv, slot)
        xk, xv = _xbox(str(tmp_path / "t_xbox"))
        yk, yv = _xbox(str(tmp_path / "o_xbox"))
        assert 0 < xk.shape[0] < n_all and np.array_equal(xk, yk)
        _same_rows(xv, yv, slot)
        # the base save reset delta_score everywhere it saved (both tiers)
        th, tv = _rows(view)
        oh, ov = _rows(ob.engine.table)
        _same_rows(tv.numpy(), ov.numpy(), slot)

        # one more pass, then SaveDelta: the delta row sets agree
        extra = ragged_batch(64, S, 3, 300, seed=99)
        extra.keys[extra.keys != -1] = extra.keys[extra.keys != -1] % 300 + 1  # pass-0 keys: back from SSD
        _run_pass(tb, extra, 9)
        _run_pass(ob, extra, 9)
        tb.save_delta(str(tmp_path / "t_delta"))
        ob.save_delta(str(tmp_path / "o_delta"))
        dk, dv = _xbox(str(tmp_path / "t_delta"))
        ek, ev = _xbox(str(tmp_path / "o_delta"))
        assert dk.shape[0] > 0 and np.array_equal(dk, ek)
        _same_rows(dv, ev, slot)

        # the tiered batch model loads back into an all-in-memory table whole
        tb.save_base(str(tmp_path / "t_batch2"), str(tmp_path / "t_xbox2"))
        ob.save_base(str(tmp_path / "o_batch2"), str(tmp_path / "o_xbox2"))
        BoxWrapper._instance = None
        lb = _box("hbm")
        assert lb.load_model(str(tmp_path / "t_batch2")) == view.size()
        lh, lv = _rows(lb.engine.table)
        okk, ovv = _part(str(tmp_path / "o_batch2"))  # rows as saved (before the xbox delta reset)
        assert np.array_equal(ref.unmix64(lh).numpy().view(np.uint64), okk[np.argsort(ref.mix64(
            torch.from_numpy(okk.view(np.int64))).numpy())])
        o = np.argsort(ref.mix64(torch.from_numpy(okk.view(np.int64))).numpy())
        _same_rows(lv.numpy(), ovv[o], slot)

        # ShrinkTable: decay + age + delete over host AND SSD rows
        tb.cfg.shrink.delete_threshold = 0.4
        ob.cfg.shrink.delete_threshold = 0.4
        assert len(tb.ssd) > 0
        g1 = tb.shrink_table()
        g2 = ob.shrink_table()
        assert g1 == g2 > 0
        th, tv = _rows(tb._authoritative())
        oh, ov = _rows(ob.engine.table)
        assert torch.equal(th, oh)
        _same_rows(tv.numpy(), ov.numpy(), slot)
        # the SSD log is replayed to the same (aged, pruned) state
        n_ssd = len(tb.ssd)
        del view
        tb._tier_view = None
        from paddlebox_amd.ps.tiered import SsdTier

        path, stride = tb.ssd.path, tb.ssd.stride
        tb.ssd = None
        re = SsdTier(path, stride)
        assert len(re) == n_ssd
        f, rv = re.get(re.keys())
        assert bool(f.all())
        oi = torch.searchsorted(oh, re.keys())
        _same_rows(rv.numpy(), ov[oi].numpy(), slot)
    finally:
        BoxWrapper._instance = None


def test_ssd_shrink_and_rewrite_rule(tmp_path):
    """SsdLog::shrink applies the accessor rule to every live record in place
    (superseded records and tombstones untouched), survives a reopen."""
    from paddlebox_amd.ps.config import ShrinkConfig, row_layout
    from paddlebox_amd.ps.tiered import SsdTier

    l = row_layout(8)
    st = l["stride"]
    s = SsdTier(str(tmp_path / "ssd"), st, segment_bytes=1 << 15)
    g = torch.Generator().manual_seed(3)
    h = torch.unique(ref.mix64(torch.randint(1, 1 << 40, (3000,), generator=g)))
    v = torch.zeros(h.numel(), st)
    v[:, 0] = torch.rand(h.numel(), generator=g) * 5
    v[:, 1] = v[:, 0] * torch.rand(h.numel(), generator=g) * 0.5
    v[:, l["unseen_days"]] = torch.randint(0, 40, (h.numel(),), generator=g).float()
    s.put(h, v)
    s.put(h[:500], v[:500])  # superseded copies in older segments
    s.delete(h[-100:])
    live = torch.ones(h.numel(), dtype=torch.bool)
    live[-100:] = False
    cfg = ShrinkConfig(show_click_decay_rate=0.9, delete_threshold=0.8, delete_after_unseen_days=30.0)
    exp = v.clone()
    exp[:, 0] *= 0.9
    exp[:, 1] *= 0.9
    exp[:, l["unseen_days"]] += 1
    score = (exp[:, 0] - exp[:, 1]) * cfg.nonclk_coeff + exp[:, 1] * cfg.clk_coeff
    keep = live & (score >= cfg.delete_threshold) & (exp[:, l["unseen_days"]] <= cfg.delete_after_unseen_days)
    gone = s._native.shrink(0.9, l["unseen_days"], cfg.nonclk_coeff, cfg.clk_coeff, 0.8, 30.0)
    assert gone == int((live & ~keep).sum()) > 0
    assert len(s) == int(keep.sum())
    f, got = s.get(h)
    assert torch.equal(f, keep)
    torch.testing.assert_close(got[keep], exp[keep])
    s.compact(0.9)
    del s
    s2 = SsdTier(str(tmp_path / "ssd"), st, segment_bytes=1 << 15)
    f, got = s2.get(h)
    assert torch.equal(f, keep)
    torch.testing.assert_close(got[keep], exp[keep])


def test_host_insert_stamps_current_epoch():
    """rows inserted outside a write-back carry the newest pass
    stamp, so spill_oldest does not take them first."""
    from paddlebox_amd.ps.tiered import HostTable

    t = HostTable(8, threads=2, chunk_rows=1024)
    a = ref.mix64(torch.arange(1, 101))
    r, _ = t._native.insert(a)
    t._native.stamp(r, 5)
    b = ref.mix64(torch.arange(1000, 1050))
    t._native.insert(b)  # e.g. a model load: no stamp() follows
    assert bool((t._native.epochs(t.probe(b)) == 5).all())
    t.erase(a[:10])
    c = ref.mix64(torch.arange(5000, 5010))  # recycled rows
    rc, fresh = t._native.insert_fresh(torch.cat([c, a[10:12]]))
    assert fresh.tolist() == [True] * 10 + [False] * 2
    assert bool((t._native.epochs(rc[:10]) == 5).all())


def test_load_ssd2mem_streams_within_host_cap(tmp_path):
    """LoadSSD2Mem moves SSD rows into the host tier in
    bounded chunks and never past the host-tier row cap; the rows it moves
    keep their values and leave the SSD (one tier per key)."""
    box = _box("tiered", tmp_path, cap=120)
    try:
        for p, b in enumerate(_batches()):
            _run_pass(box, b, p)
        total = box.host.size() + len(box.ssd)
        assert len(box.ssd) > 100
        before_h, before_v = _rows(box._authoritative())
        box.SSD2MEM_CHUNK_ROWS = 7  # many chunks
        box.cfg.tier.ssd_spill_threshold = box.host.size() + 50
        moved = box.load_ssd2mem()
        assert moved == 50 and box.host.size() == box.cfg.tier.ssd_spill_threshold
        assert box.host.size() + len(box.ssd) == total
        assert box.load_ssd2mem() == 0  # host tier at its cap
        box.cfg.tier.ssd_spill_threshold = 0  # no cap: everything
        rest = len(box.ssd)
        assert box.load_ssd2mem() == rest
        assert len(box.ssd) == 0 and box.host.size() == total
        after_h, after_v = _rows(box._authoritative())
        assert torch.equal(before_h, after_h)
        torch.testing.assert_close(after_v, before_v)
    finally:
        BoxWrapper._instance = None
