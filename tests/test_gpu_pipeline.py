"""Pipelined front (bench.py --pipeline): each captured step pools the NEXT
batch (table dedup + fused seqpool/CVM) right after its own sparse push, so
the next step starts at the data_norm head.  Training must be unchanged: the
pooled values are read after the push they depend on.  Oracle: the same
batches through the plain graphed step (no pipelining), from identical
initial states -- dense parameters, losses and table rows agree exactly.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _setup(seed_batches=7, ring=3, n_batches=8):
    from paddlebox_amd.data.synthetic import CriteoSynth
    from paddlebox_amd.ops import reference as ref
    from paddlebox_amd.ps.config import PSConfig
    from paddlebox_amd.ps.sparse_engine import SparseEngine
    from paddlebox_amd.runtime.graph_step import pack_batch

    synth = CriteoSynth(total_features=200_000, alpha=1.1, seed=seed_batches, device="cpu")
    bs = [synth.batch(512) for _ in range(n_batches)]
    S = bs[0].S
    eng = SparseEngine(PSConfig(embedx_dim=8), max_keys=512 * S, device=DEV, capacity=300_000,
                       slot_ids=[float(s + 1) for s in range(S)], pull_ring=ring)
    allk = torch.cat([b.keys for b in bs])
    eng.insert_local_mixed(torch.unique(ref.mix64(allk[allk != -1])).to(DEV), init_embedx=True)
    hbs = [pack_batch(b, pin=True) for b in bs]
    return eng, hbs, S


def _train(pipeline: bool, precision: str, K: int = 1, n_batches: int = 8):
    eng, hbs, S = _setup(ring=3 * K, n_batches=n_batches)
    flat, losses = _run(eng, hbs, S, pipeline, precision, K)
    hk, v = eng.table.export(True)
    o = torch.argsort(hk)
    return flat, losses, hk[o].cpu(), v[o].cpu()


def _run(eng, hbs, S, pipeline: bool, precision: str, K: int = 1, model: str = "deepfm"):
    """One training program over the engine: warm batch 0 eagerly, then the
    rest of the batches through the graphed step (K steps per graph)."""
    from paddlebox_amd.runtime.ctr_step import CtrTrainStep
    from paddlebox_amd.runtime.graph_step import GraphedTrainStep

    eng.clear_prefetch(reset_rows=True)
    torch.manual_seed(0)
    step = CtrTrainStep(eng, model, precision, num_slots=S, hidden=(64, 64, 64))
    pipe = (lambda b, j: step.prefetch(b, j), step.set_next, eng.clear_prefetch) if pipeline else None
    losses = []
    g = GraphedTrainStep(step.train_step, hbs[0], DEV, warmup=0, warm_batches=[hbs[0]],
                         on_warm=lambda out: losses.append(float(out)), n_buffers=3 if pipeline else 2,
                         pipeline=pipe, steps_per_graph=K, join_each_step=not step.adam_overlap)
    if K == 1:
        ahead = 2 if pipeline else 1
        for a in range(1, 1 + ahead):
            g.load(a % g.n, hbs[a])
        for i in range(1, len(hbs)):
            if i + ahead < len(hbs):
                g.load((i + ahead) % g.n, hbs[i + ahead])
            out = g.run(i % g.n)
            torch.cuda.synchronize()
            losses.append(float(out))
    else:  # batches 1.. in groups of K (the graph returns its last step's loss)
        groups = [hbs[1 + q * K:1 + (q + 1) * K] for q in range((len(hbs) - 1) // K)]
        ahead = 2 if pipeline else 1
        for a in range(min(ahead, len(groups))):
            g.load(a % g.n, groups[a])
        for q in range(len(groups)):
            if q + ahead < len(groups):
                g.load((q + ahead) % g.n, groups[q + ahead])
            out = g.run(q % g.n)
            torch.cuda.synchronize()
            losses.append(float(out))
    flat = step.arena.flat.cpu()
    del g, step
    return flat, losses


@pytest.mark.parametrize("precision,K,split,overlap,fs", [("fp32", 3, "0", "0", "0"), ("fp32", 4, "0", "0", "0"),
                                                          ("fp32", 1, "0", "0", "0"), ("bf16", 1, "0", "0", "0"),
                                                          ("fp32", 2, "0", "0", "0"), ("fp32", 1, "2", "0", "0"),
                                                          ("fp32", 2, "1", "0", "0"), ("fp32", 2, "0", "1", "0"),
                                                          ("bf16", 2, "0", "1", "0"), ("fp32", 2, "3", "0", "0"),
                                                          ("fp32", 1, "0", "0", "1"), ("fp32", 2, "0", "0", "1"),
                                                          ("fp32", 2, "2", "0", "1")])
def test_pipelined_front_matches_plain_graphed_step(precision, K, split, overlap, fs, monkeypatch):
    # split: the next batch's key dedup on its own stream (PBX_SPLIT_PREFETCH,
    # forked at the dX chain (1) or after the head backward (2)); overlap:
    # Adam on the dW side stream, the next head not waiting for it
    # (PBX_ADAM_OVERLAP, the step's side work joined by the next step)
    nb = 1 + 3 * K if K > 2 else 8  # K = 3, 4 (bench's default): three graphs of K steps
    f0, l0, k0, v0 = _train(False, precision, K, nb)
    monkeypatch.setenv("PBX_SPLIT_PREFETCH", split)
    monkeypatch.setenv("PBX_ADAM_OVERLAP", overlap)
    monkeypatch.setenv("PBX_FUSED_SCATTER", fs)  # the dedup scatter inside the prefetched pooling launch
    f1, l1, k1, v1 = _train(True, precision, K, nb)
    # the dense update is bit-reproducible (fixed-order dW split reduce,
    # test_gpu_tower32.py::test_tower32_deterministic); the sparse push is
    # not: a key's occurrences are summed in fp32 in the order the dedup's
    # atomics placed them (rank within the key, run placement) and the pieces
    # of a run that straddles waves meet in fp32 atomics, so two runs differ
    # at fp32 rounding level (seen: 4e-7 abs / 1.7e-6 rel in 1 of 190k table
    # values), which Adam's m / sqrt(v) can lift a little in the dense params
    rt, at = (1e-5, 1e-6) if precision == "fp32" else (1e-4, 1e-5)
    assert l1 == pytest.approx(l0, rel=rt, abs=at)
    torch.testing.assert_close(f1, f0, rtol=rt, atol=at)
    assert torch.equal(k1, k0)
    torch.testing.assert_close(v1, v0, rtol=rt, atol=at)


def test_pipelined_program_then_plain_multistep_on_same_engine():
    """bench.py runs a pipelined K = 4 fp32 program and then
    other programs (bf16 K = 2, plain) over the SAME engine.  No pull-ring
    reset between them: the second program must train exactly like a fresh
    plain sequence (fp32 K = 1 then bf16 K = 1) from the same initial state."""
    eng, hbs, S = _setup(ring=12, n_batches=13)
    _, la = _run(eng, hbs, S, True, "fp32", 4)
    fb, lb = _run(eng, hbs, S, False, "bf16", 2)
    ha, va = eng.table.export(True)
    del eng
    ref_eng, hbs2, _ = _setup(ring=12, n_batches=13)
    _, lc = _run(ref_eng, hbs2, S, False, "fp32", 1)
    fd, ld = _run(ref_eng, hbs2, S, False, "bf16", 1)
    hr, vr = ref_eng.table.export(True)
    assert la == pytest.approx(lc[:1] + lc[4::4], rel=1e-5, abs=1e-6)
    assert lb == pytest.approx(ld[:1] + ld[2::2], rel=2e-3, abs=1e-4)
    torch.testing.assert_close(fb, fd, rtol=2e-3, atol=1e-4)
    oa, orr = torch.argsort(ha), torch.argsort(hr)
    assert torch.equal(ha[oa], hr[orr])
    torch.testing.assert_close(va[oa], vr[orr], rtol=2e-3, atol=1e-4)


@pytest.mark.parametrize("K,overlap", [(1, "0"), (4, "0"), (4, "1")])
def test_dedup_finish_on_side_stream_matches_plain(K, overlap, monkeypatch):
    """PBX_TD_FINISH_SIDE=1: the prefetched dedup's run starts + scatter run
    on a side stream beside the pooling (joined with the step's side work);
    with and without Adam on the dW stream (PBX_ADAM_OVERLAP)."""
    nb = 1 + 3 * K if K > 2 else 8
    f0, l0, k0, v0 = _train(False, "fp32", K, nb)
    monkeypatch.setenv("PBX_TD_FINISH_SIDE", "1")
    monkeypatch.setenv("PBX_ADAM_OVERLAP", overlap)
    f1, l1, k1, v1 = _train(True, "fp32", K, nb)
    # tolerance: the sparse push's fp32 summation order (see above)
    assert l1 == pytest.approx(l0, rel=1e-5, abs=1e-6)
    torch.testing.assert_close(f1, f0, rtol=1e-5, atol=1e-6)
    assert torch.equal(k1, k0)
    torch.testing.assert_close(v1, v0, rtol=1e-5, atol=1e-6)


def test_dcn_v2_adam_overlap_matches_plain(monkeypatch):
    """with PBX_ADAM_OVERLAP=1 the DCN-V2 cross forward must see
    the updated cross weights (the overlapped Adam is joined before it)."""
    eng, hbs, S = _setup(ring=4, n_batches=9)
    f0, l0 = _run(eng, hbs, S, False, "bf16", 2, model="dcn_v2")
    k0, v0 = eng.table.export(True)
    eng2, hbs2, _ = _setup(ring=4, n_batches=9)
    monkeypatch.setenv("PBX_ADAM_OVERLAP", "1")
    f1, l1 = _run(eng2, hbs2, S, False, "bf16", 2, model="dcn_v2")
    k1, v1 = eng2.table.export(True)
    assert l1 == pytest.approx(l0, rel=1e-4, abs=1e-5)
    torch.testing.assert_close(f1, f0, rtol=1e-4, atol=1e-5)
    o0, o1 = torch.argsort(k0), torch.argsort(k1)
    torch.testing.assert_close(v1[o1], v0[o0], rtol=1e-4, atol=1e-5)
