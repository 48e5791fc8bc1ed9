"""The W-rank graph-captured DeepFM step equals one rank on the union batch
(SURVEY §7.4 M4 exit test).

W processes share the test box's one GPU (same-GPU rehearsal: gloo control
plane, every in-step collective on the IPC meshes -- the same kernels that run
over xGMI on a node).  Each rank trains its slice of every union batch through
``runtime.ctr_step.CtrTrainStep`` -- bench.py's step: sharded sparse pull /
push over the IPC exchange (owner-side merged Adagrad), the exact-fp32 tower,
the IPC dense gradient all-reduce launched from the tower's dense-grads hook,
data_norm batch statistics summed in the tail of the same all-reduce, fused
Adam -- the first step eagerly, the rest as replays of the captured graphs.

The oracle is one unsharded rank training the union batches eagerly.  Dense
parameters, data_norm summaries and every table row must agree to fp32
rounding.  One reference semantic is modelled explicitly: with sync_stats the
reference all-reduces each GPU's normalised batch statistics (1, sum/N,
sqsum/N + eps) (data_norm_op.cu:38-104), i.e. W times the union batch's
normalised statistics, so the oracle scales its statistics by W before the
summary update.  Reference step: boxps_worker.cc:1191-1258.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

HIDDEN = (400, 400, 400)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _data(W, B, steps):
    from paddlebox_amd.data.synthetic import CriteoSynth
    from tests.test_sharded_loopback import concat_batches

    synth = CriteoSynth(total_features=300_000, alpha=1.1, seed=5, device="cpu")
    per_rank = [[synth.batch(B) for _ in range(W)] for _ in range(steps)]
    union = [concat_batches(bs) for bs in per_rank]
    return per_rank, union


def _cfg():
    from paddlebox_amd.ps.config import PSConfig

    return PSConfig(embedx_dim=8)


def _union_keys(union):
    from paddlebox_amd.ops import reference as ref

    allk = torch.cat([u.keys for u in union])
    return torch.unique(ref.mix64(allk[allk != -1]))


def _worker(rank, W, port, B, steps, q, mode="plain"):
    try:
        if mode in ("overlap_dw", "both", "both_split3", "both_adam"):
            os.environ["PBX_OVERLAP_DW_IPC"] = "1"
        # the overlapped multi-rank Adam (default) only in its own mode: the
        # others keep covering the in-order update
        os.environ["PBX_ADAM_OVERLAP_MULTI"] = "1" if mode == "both_adam" else "0"
        # the multi-rank defaults: the next batch's dedup at the step start
        # (split 3) in the both_split3 / both_adam modes, off in the others
        os.environ["PBX_SPLIT_PREFETCH"] = "3" if mode in ("both_split3", "both_adam") else "0"
        import torch.distributed as dist

        from paddlebox_amd.ops import reference as ref
        from paddlebox_amd.parallel.comm import TorchDistComm
        from paddlebox_amd.ps.sparse_engine import SparseEngine
        from paddlebox_amd.runtime.ctr_step import CtrTrainStep
        from paddlebox_amd.runtime.graph_step import GraphedTrainStep, pack_batch

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        os.environ.setdefault("PBX_IPC_MAX_BLOCKS", str(max(8, 256 // W)))
        dist.init_process_group("gloo", rank=rank, world_size=W)
        torch.cuda.set_device(0)
        dev = torch.device("cuda:0")
        per_rank, union = _data(W, B, steps)
        S = union[0].S
        eng = SparseEngine(_cfg(), max_keys=B * S, device=dev, capacity=400_000, comm=TorchDistComm(),
                           exchange="ipc", exchange_capacity=B * S, slot_ids=[float(s + 1) for s in range(S)],
                           pull_ring=3)
        assert eng.exchange_mode == "ipc", eng.exchange_mode
        h = _union_keys(union)
        eng.insert_local_mixed(h[ref.owner_of(h, W) == rank].to(dev), init_embedx=True)
        torch.manual_seed(0)
        step = CtrTrainStep(eng, "deepfm", "fp32", num_slots=S, hidden=HIDDEN, multi=True, same_gpu=True)
        assert step.fused and step.ipc is not None
        hbs = [pack_batch(per_rank[i][rank], pin=True) for i in range(steps)]
        losses = []
        # step 0 eagerly through the graph's buffers, then the captured replays
        pipe = None
        if mode in ("pipeline", "both", "both_split3", "both_adam"):
            # sharded pipelined front: each step pulls the next batch (dedup,
            # both exchanges, owner gather, pooling) right after its own push
            assert eng.can_prefetch_pull()
            pipe = (lambda b, j: step.prefetch(b, j), step.set_next, eng.clear_prefetch)
        g = GraphedTrainStep(step.train_step, hbs[0], dev, warmup=0, warm_batches=[hbs[0]],
                             on_warm=lambda out: losses.append(float(out)), n_buffers=3 if pipe else 2,
                             pipeline=pipe, join_each_step=not step.adam_overlap_multi)
        assert step.adam_overlap_multi == (mode == "both_adam")
        ahead = 2 if pipe else 1
        for a in range(1, min(1 + ahead, steps)):
            g.load(a % g.n, hbs[a])
        for i in range(1, steps):
            if i + ahead < steps:
                g.load((i + ahead) % g.n, hbs[i + ahead])
            out = g.run(i % g.n)
            torch.cuda.synchronize()
            losses.append(float(out))  # the graphs' loss outputs share the tower's workspace scalar

        dn = step.model.dn
        res = dict(flat=step.arena.flat.cpu(), dn=torch.stack([dn.batch_size, dn.batch_sum, dn.batch_square_sum]).cpu(),
                   keys=None, vals=None, losses=losses, ovf=eng.check_overflow())
        hk, v = eng.table.export(True)
        res["keys"], res["vals"] = hk.cpu(), v.cpu()
        eng.check_exchange()
        step.ipc.check()
        dist.barrier()
        # numpy, not torch: a torch tensor crosses the queue as a shared fd that dies with the worker
        q.put((rank, {k: (v.numpy() if torch.is_tensor(v) else v) for k, v in res.items()}))
        step.close()
        for m in eng.xmesh:
            m.close()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback

        q.put((rank, repr(e) + traceback.format_exc()))


def _oracle(W, B, steps):
    from paddlebox_amd.parallel.dense import join_grad_producers
    from paddlebox_amd.ps.sparse_engine import SparseEngine
    from paddlebox_amd.runtime.ctr_step import CtrTrainStep

    dev = torch.device("cuda:0")
    _, union = _data(W, B, steps)
    S = union[0].S
    eng = SparseEngine(_cfg(), max_keys=W * B * S, device=dev, capacity=400_000,
                       slot_ids=[float(s + 1) for s in range(S)])
    eng.insert_local_mixed(_union_keys(union).to(dev), init_embedx=True)
    torch.manual_seed(0)
    # the plain eager step: the loop below runs Adam itself, after scaling the
    # statistics (no optimizer inside the backward)
    prev = os.environ.get("PBX_ADAM_OVERLAP")
    os.environ["PBX_ADAM_OVERLAP"] = "0"
    try:
        step = CtrTrainStep(eng, "deepfm", "fp32", num_slots=S, hidden=HIDDEN, multi=False)
    finally:
        if prev is None:
            os.environ.pop("PBX_ADAM_OVERLAP", None)
        else:
            os.environ["PBX_ADAM_OVERLAP"] = prev
    assert not step.adam_overlap
    model = step.model
    losses = []
    for u in union:
        b = u.to(dev)
        loss, _ = model(b)
        loss.backward(step.one)
        join_grad_producers()
        model.dn.stats.mul_(W)  # W ranks' normalised statistics, summed (module docstring)
        step.opt.step(1.0)
        losses.append(float(loss.detach()))
    torch.cuda.synchronize()
    dn = model.dn
    return dict(flat=step.arena.flat.cpu(), dn=torch.stack([dn.batch_size, dn.batch_sum, dn.batch_square_sum]).cpu(),
                eng=eng, losses=losses)


@pytest.mark.parametrize("W,mode", [(2, "plain"), (4, "plain"), (2, "overlap_dw"), (2, "pipeline"),
                                    (4, "pipeline"), (2, "both"), (2, "both_split3"), (4, "both_split3"),
                                    (2, "both_adam"), (4, "both_adam")])
def test_nrank_graphed_deepfm_step_matches_union_oracle(W, mode):
    """mode: plain graphed step; overlap_dw = the dW GEMM and its IPC dense
    all-reduce on the side stream (PBX_OVERLAP_DW_IPC); pipeline = the sharded
    pipelined front (SparseEngine prefetch_pull with the exchanges inside)."""
    from paddlebox_amd.ops import reference as ref

    B, steps = 256, 4 if mode in ("pipeline", "both", "both_split3", "both_adam") else 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, W, port, B, steps, q, mode)) for r in range(W)]
    for p in ps:
        p.start()
    res = {}
    try:
        for _ in range(W):
            r, out = q.get(timeout=300)
            res[r] = out
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in range(W):
        assert not isinstance(res[r], str), res[r]
        res[r] = {k: (torch.from_numpy(v) if isinstance(v, np.ndarray) else v) for k, v in res[r].items()}
        assert res[r]["ovf"] is False
    orc = _oracle(W, B, steps)
    # every replica holds the same dense parameters (one-shot all-reduce: same
    # summation order on every rank), equal to the union oracle
    for r in range(1, W):
        torch.testing.assert_close(res[r]["flat"], res[0]["flat"], rtol=0, atol=0)
    torch.testing.assert_close(res[0]["flat"], orc["flat"], rtol=2e-4, atol=2e-6)
    torch.testing.assert_close(res[0]["dn"], orc["dn"], rtol=2e-5, atol=1e-4)
    # the per-rank losses average to the union loss
    for i in range(steps):
        mean = sum(res[r]["losses"][i] for r in range(W)) / W
        assert mean == pytest.approx(orc["losses"][i], rel=2e-5, abs=2e-6)
    # table: every key lives at its owner, rows equal the oracle's
    allh = torch.cat([res[r]["keys"] for r in range(W)])
    allv = torch.cat([res[r]["vals"] for r in range(W)])
    assert allh.numel() == torch.unique(allh).numel() == orc["eng"].table.size()
    for r in range(W):
        assert bool((ref.owner_of(res[r]["keys"], W) == r).all())
    exp = orc["eng"].table.read(allh.to("cuda:0")).cpu()
    torch.testing.assert_close(allv[:, :14], exp[:, :14], rtol=2e-4, atol=2e-6)
