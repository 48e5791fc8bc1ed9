"""Native host tier (sharded open addressing over a NUMA-first-touched row
arena) and log-structured SSD tier (csrc/host/tier_store.cc)."""
import numpy as np
import torch

from paddlebox_amd.ops import reference as ref
from paddlebox_amd.ps.tiered import HostTable, SsdTier

STRIDE = 20


def _keys(n, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.unique(ref.mix64(torch.randint(0, 1 << 40, (n,), generator=g)))


def test_host_tier_roundtrip_growth_erase():
    t = HostTable(8, threads=4, chunk_rows=1024)
    h = _keys(20000, 0)  # forces shard growth and several arena chunks
    rows, fresh = t._native.insert(h)
    assert fresh == h.numel() and t.size() == h.numel()
    v = torch.randn(h.numel(), STRIDE)
    t.assign(h, v)
    assert torch.equal(t.read(h), v)
    # duplicates / re-insert are no-ops
    _, fresh2 = t._native.insert(torch.cat([h[:100], h[:100]]))
    assert fresh2 == 0
    gone = t.erase(h[::2])
    assert gone == h[::2].numel() and t.size() == h.numel() - gone
    assert bool((t.probe(h[::2]) == -1).all())
    assert torch.equal(t.read(h[1::2]), v[1::2])
    # freed rows are reused, re-inserted keys start zeroed
    t._native.insert(h[::2])
    assert float(t.read(h[::2]).abs().sum()) == 0.0
    k, vals = t.export(True)
    assert k.numel() == h.numel()
    cold_k, _ = t._native.select_ge(t.layout["slot"], 0.5)
    assert cold_k.numel() == int((torch.cat([torch.zeros(h[::2].numel()), v[1::2, t.layout["slot"]]]) >= 0.5).sum())


def test_ssd_log_put_get_erase_compact_and_replay(tmp_path):
    d = str(tmp_path / "ssd")
    s = SsdTier(d, STRIDE, segment_bytes=1 << 16)  # small segments: many files
    h = _keys(5000, 1)
    v = torch.randn(h.numel(), STRIDE)
    s.put(h, v)
    assert len(s) == h.numel() and s._native.segments() > 3
    f, got = s.get(h)
    assert bool(f.all()) and torch.equal(got, v)
    # overwrite half, delete a quarter
    v2 = v.clone()
    v2[: h.numel() // 2] += 1
    s.put(h[: h.numel() // 2], v2[: h.numel() // 2])
    s.delete(h[-h.numel() // 4:])
    live = h.numel() - h.numel() // 4
    assert len(s) == live
    f, got = s.get(h)
    assert int(f.sum()) == live
    assert torch.equal(got[f], v2[f])
    moved = s.compact(0.9)
    assert moved > 0
    f2, got2 = s.get(h)
    assert torch.equal(f2, f) and torch.equal(got2[f2], v2[f2])
    # a new process rebuilds the same index by replaying the segment log
    del s
    s2 = SsdTier(d, STRIDE, segment_bytes=1 << 16)
    assert len(s2) == live
    f3, got3 = s2.get(h)
    assert torch.equal(f3, f) and torch.equal(got3[f3], v2[f3])
    assert set(np.asarray(s2.keys()).tolist()) == set(np.asarray(h[f]).tolist())


def test_ssd_compaction_keeps_tombstones_that_shadow_survivors(tmp_path):
    """a tombstone living in a compacted (victim) segment must not
    vanish while an older surviving segment still holds the key's previous
    put -- otherwise a reopen replays the old record and the key comes back."""
    d = str(tmp_path / "ssd")
    stride = 4
    per_seg = (4096 // (12 + 4 * stride)) * 2  # records per 2-page segment
    s = SsdTier(d, stride, segment_bytes=2 * 4096)
    k_old = torch.arange(1, per_seg + 1, dtype=torch.int64)  # fills segment 0
    s.put(k_old, torch.ones(per_seg, stride))
    victim_keys = torch.arange(10_000, 10_000 + per_seg // 2, dtype=torch.int64)
    s.put(victim_keys, torch.full((victim_keys.numel(), stride), 2.0))  # segment 1
    gone = k_old[5:6]
    s.delete(gone)  # tombstone in segment 1; segment 0 still holds the old put
    s.put(victim_keys, torch.full((victim_keys.numel(), stride), 3.0))  # segment 1 -> mostly dead
    assert s._native.segments() >= 3
    moved = s.compact(0.5)  # segment 1 is a victim, segment 0 (live ~100%) survives
    assert moved > 0
    f, _ = s.get(gone)
    assert not bool(f.any())
    del s
    s2 = SsdTier(d, stride, segment_bytes=2 * 4096)
    f, _ = s2.get(gone)
    assert not bool(f.any()), "deleted key resurrected by replay after compaction"
    f, v = s2.get(victim_keys)
    assert bool(f.all()) and bool((v == 3.0).all())
    f, _ = s2.get(k_old[6:])
    assert bool(f.all())


def test_host_tier_native_shrink_matches_rule():
    from paddlebox_amd.ps.config import ShrinkConfig

    t = HostTable(8, threads=4, chunk_rows=1024)
    h = _keys(5000, 3)
    t._native.insert(h)
    g = torch.Generator().manual_seed(9)
    v = torch.zeros(h.numel(), t.stride)
    v[:, 0] = torch.rand(h.numel(), generator=g) * 5
    v[:, 1] = v[:, 0] * torch.rand(h.numel(), generator=g) * 0.5
    l = t.layout
    v[:, l["unseen_days"]] = torch.randint(0, 40, (h.numel(),), generator=g).float()
    t.assign(h, v)
    cfg = ShrinkConfig(show_click_decay_rate=0.9, delete_threshold=0.8, delete_after_unseen_days=30.0)
    exp = v.clone()
    exp[:, 0] *= 0.9
    exp[:, 1] *= 0.9
    exp[:, l["unseen_days"]] += 1
    score = (exp[:, 0] - exp[:, 1]) * cfg.nonclk_coeff + exp[:, 1] * cfg.clk_coeff
    keep = (score >= cfg.delete_threshold) & (exp[:, l["unseen_days"]] <= cfg.delete_after_unseen_days)
    gone = t.shrink(cfg)
    assert gone == int((~keep).sum()) > 0
    assert t.size() == int(keep.sum())
    assert bool((t.probe(h[~keep]) == -1).all())
    torch.testing.assert_close(t.read(h[keep]), exp[keep])


def test_host_tier_spill_oldest_passes_first():
    """spill_oldest moves whole older passes first, then part of the boundary
    pass, and returns exactly the removed rows with their values."""
    t = HostTable(8, threads=4, chunk_rows=1024)
    passes = [_keys(3000, 10 + p) for p in range(3)]
    vals = {}
    for p, h in enumerate(passes, start=1):
        rows, _ = t._native.insert(h)
        v = torch.randn(h.numel(), STRIDE)
        t._native.scatter(rows, v)
        t._native.stamp(rows, p)
        for k, row in zip(h.tolist(), v):
            vals[k] = row
    union = torch.unique(torch.cat(passes))
    total = t.size()
    assert total == union.numel()
    ep = t._native.epochs(t.probe(union))
    n1 = int((ep == 1).sum())
    keep = total - n1 - 500  # all of pass 1's surviving rows + 500 of pass 2's
    k, v = t._native.spill_oldest(keep)
    assert k.numel() == n1 + 500 and t.size() == keep
    kep = dict(zip(union.tolist(), ep.tolist()))
    spilled_ep = torch.tensor([kep[x] for x in k.tolist()])
    assert int((spilled_ep == 1).sum()) == n1 and int((spilled_ep == 2).sum()) == 500
    for i, x in enumerate(k.tolist()):
        assert torch.equal(v[i], vals[x])
    assert bool((t.probe(k) == -1).all())
    # under the cap: nothing moves
    k2, _ = t._native.spill_oldest(keep)
    assert k2.numel() == 0
    # clear releases the arena: re-inserted keys start from zero rows
    t.clear()
    t._native.insert(passes[0])
    assert float(t.read(passes[0]).abs().sum()) == 0.0


def test_ssd_log_bulk_sharded_index_duplicates_and_partial_pages(tmp_path):
    """Bulk paths of the 64-shard SSD index (> 64K keys: per-thread bucketing,
    shard-parallel set / erase): a key repeated inside one put keeps its LAST
    record, erase of present + absent keys, and puts that end inside a page
    (its unused slots must read as empty on replay now that a new segment's
    mirror is no longer cleared up front) continue in the same page."""
    d = str(tmp_path / "ssd")
    s = SsdTier(d, STRIDE, segment_bytes=1 << 20)
    h = _keys(150_000, 7)
    n = h.numel()
    v = torch.randn(n, STRIDE)
    # one batch holding every key twice: the second copy (v + 1) wins
    s.put(torch.cat([h, h]), torch.cat([v, v + 1]))
    assert len(s) == n
    f, got = s.get(h)
    assert bool(f.all()) and torch.equal(got, v + 1)
    # odd-sized puts: each ends inside a page, the next continues it
    for a, b in ((0, 1001), (1001, 70_003), (70_003, n)):
        s.put(h[a:b], v[a:b] * 2)
    absent = _keys(80_000, 8)
    absent = absent[~torch.isin(absent, h)]
    gone = s._native.erase(torch.cat([h[: n // 3], absent]))
    assert gone == n // 3
    live = n - n // 3
    assert len(s) == live
    f, got = s.get(h)
    assert int(f.sum()) == live and not bool(f[: n // 3].any())
    assert torch.equal(got[f], v[f] * 2)
    del s
    s2 = SsdTier(d, STRIDE, segment_bytes=1 << 20)  # replay: same index, no phantom records
    assert len(s2) == live
    f2, got2 = s2.get(h)
    assert torch.equal(f2, f) and torch.equal(got2[f2], v[f2] * 2)
