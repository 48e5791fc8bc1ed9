"""The user-facing fluid path on W ranks: the canonical
PaddleBox program (pull_box_sparse -> fused_seqpool_cvm -> data_norm
(sync_stats) -> fc x3 -> log-loss, BoxPSOptimizer(Adam)) trained by
``exe.train_from_dataset`` in W processes on the test box's one GPU, with the
step captured in HIP graphs.  Dense sync is either the GradAllReduce
transpiler's program ops (coalesce_tensor -> c_allreduce_sum -> scale) or the
executor's built-in grad all-reduce, launched from the fused tower's
dense-grads hook; both, and the data_norm statistics, run on the session's
self-tested IPC mesh, the sparse exchange on the engine's.

Oracle: one rank training the union of the rank files (each union batch = the
W rank batches of that step, concatenated).  With sync_stats the reference
sums each GPU's normalised statistics (data_norm_op.cu:38-104), W times the
union batch's, so the oracle scales its statistics by W before the summary
update.  Reference: boxps_worker.cc:1216-1236, c_allreduce_x_op.cc:45-190.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

B, NB = 64, 4  # rank batch, batches per rank file


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _build(fluid):
    from tests.test_fluid import DENSE, S

    main, startup = fluid.Program(), fluid.Program()
    main.random_seed = startup.random_seed = 11
    with fluid.program_guard(main, startup), fluid.unique_name.guard():
        label = fluid.layers.data("label", shape=[1], dtype="int64")
        slots = [fluid.layers.data(f"slot{i}", shape=[1], dtype="int64", lod_level=1) for i in range(S)]
        dense = fluid.layers.data("dense", shape=[DENSE], dtype="float32")
        show = fluid.layers.fill_constant_batch_size_like(label, shape=[-1, 1], dtype="float32", value=1.0)
        click = fluid.layers.cast(label, "float32")
        cvm = fluid.layers.concat([show, click], axis=1)
        embs = fluid.layers._pull_box_sparse(slots, size=11)
        pooled = fluid.contrib.layers.fused_seqpool_cvm(embs, "sum", cvm)
        x = fluid.layers.concat(pooled + [dense], axis=1)
        x = fluid.layers.data_norm(x, name="dn", sync_stats=True)
        h = x
        for i, n in enumerate((64, 32, 16)):
            h = fluid.layers.fc(h, n, act="relu", name=f"fc{i}")
        logit = fluid.layers.fc(h, 1, name="out")
        loss = fluid.layers.reduce_mean(fluid.layers.sigmoid_cross_entropy_with_logits(logit, click))
        fluid.optimizer.BoxPSOptimizer(fluid.optimizer.Adam(learning_rate=0.01)).minimize(loss)
    return main, startup, slots, label, dense, loss


def _write_files(d, W):
    """W rank files of NB*B records and the union file whose batch i (W*B
    records) is the W rank batches i in rank order."""
    from tests.test_fluid import _lines

    ranks = [_lines(NB * B, seed=40 + r) for r in range(W)]
    paths = []
    for r, ls in enumerate(ranks):
        p = os.path.join(d, f"rank-{r}.txt")
        with open(p, "w") as f:
            f.write("\n".join(ls) + "\n")
        paths.append(p)
    union = []
    for i in range(NB):
        for r in range(W):
            union += ranks[r][i * B:(i + 1) * B]
    up = os.path.join(d, "union.txt")
    with open(up, "w") as f:
        f.write("\n".join(union) + "\n")
    return paths, up


def _train(fluid, files, batch, rank, W, transpile):
    from paddlebox_amd.ps.box_wrapper import BoxWrapper
    from tests.test_fluid import S

    BoxWrapper._instance = None
    box = fluid.core.BoxWrapper(8, device="cuda:0", new=True)
    box.cfg.sgd.mf_create_thresholds = 0.0
    box.initialize_gpu_and_load_model(slot_vector=list(range(S)), max_keys=60000)
    scope = fluid.Scope()
    main, startup, slots, label, dense, loss = _build(fluid)
    main._pipeline_opt = dict(main._pipeline_opt or {}, use_graph=os.environ.get("PBX_TEST_FLUID_GRAPH", "1") == "1")
    if transpile:
        eps = [f"127.0.0.1:{6170 + r}" for r in range(W)]
        fluid.transpiler.GradAllReduce().transpile(startup, main, rank, eps, eps[rank])
    exe = fluid.Executor(fluid.CUDAPlace(0))
    exe.run(startup, scope=scope)
    ds = fluid.DatasetFactory().create_dataset("PadBoxSlotDataset")
    ds.set_use_var([label] + slots + [dense])
    ds.set_batch_size(batch)
    ds.set_thread(1)
    ds.set_filelist(files)
    ds.disable_shuffle()
    boxps = fluid.core.BoxPS(ds)
    boxps.read_ins_into_memory()
    boxps.begin_pass()
    stats = exe.train_from_dataset(main, ds, scope=scope, fetch_list=[loss], print_period=1000)
    boxps.end_pass()
    torch.cuda.synchronize()
    names = sorted(p.name for p in main.all_parameters())
    out = {n: np.array(scope.find_var(n).get_tensor()).copy() for n in names}
    for n in ("batch_size", "batch_sum", "batch_square_sum"):
        out["dn." + n] = np.array(scope.find_var(f"dn.{n}").get_tensor()).copy()
    h, v = box.engine.table.export(True)
    sess = exe.sessions_for(main)[0]
    info = dict(ipc=sess.ipc is not None, replays=stats.get("graph_replays", 0) if isinstance(stats, dict) else 0)
    BoxWrapper._instance = None
    # numpy, not torch: a torch tensor crosses the result queue as a shared fd
    # that dies with the worker process
    return out, h.cpu().numpy(), v.cpu().numpy(), info


def _worker(rank, W, port, d, transpile, q):
    import faulthandler
    import sys

    faulthandler.dump_traceback_later(90, exit=False, file=sys.stderr)  # a stuck rank shows where
    try:
        import torch.distributed as dist

        import paddlebox_amd.fluid as fluid

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        os.environ.setdefault("PBX_IPC_MAX_BLOCKS", str(max(8, 256 // W)))
        dist.init_process_group("gloo", rank=rank, world_size=W)
        torch.cuda.set_device(0)
        paths, _ = _write_files(d, W) if rank == 0 else (None, None)
        dist.barrier()
        # every rank gets the whole filelist and reads its rank stride of it
        # (data_set.cc:1963-1975): rank r trains rank-r.txt
        paths = [os.path.join(d, f"rank-{r}.txt") for r in range(W)]
        out = _train(fluid, paths, B, rank, W, transpile)
        dist.barrier()
        q.put((rank, out))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback

        q.put((rank, repr(e) + traceback.format_exc()))


@pytest.mark.parametrize("transpile,graph", [(True, True), (False, True), (False, False)])
def test_fluid_two_ranks_match_union_oracle(tmp_path, monkeypatch, transpile, graph):
    """graph=False: the eager loop (a device batch read on the compute stream
    after its H2D copy on a side stream once returned its memory to the copy
    stream's pool early: corrupted batches / a stalled rank, round 5)."""
    from paddlebox_amd import _native
    from paddlebox_amd.ops import reference as ref

    import paddlebox_amd.fluid as fluid

    W = 2
    d = str(tmp_path)
    monkeypatch.setenv("PBX_TEST_FLUID_GRAPH", "1" if graph else "0")  # inherited by the spawned ranks
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, W, port, d, transpile, q)) for r in range(W)]
    for p in ps:
        p.start()
    res = {}
    try:
        for _ in range(W):
            r, out = q.get(timeout=400)
            res[r] = out
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    errs = {r: res[r] for r in range(W) if isinstance(res.get(r), str)}
    assert not errs, "\n".join(f"rank {r}: {e}" for r, e in errs.items())
    for r in range(W):
        assert res[r][3]["ipc"], "the session did not set up its IPC mesh"
    # oracle: one rank, the union file, W*B batches, statistics x W
    h = _native.hip()
    orig = h.data_norm_update
    monkeypatch.setattr(h, "data_norm_update", lambda bs, bsum, bsq, st, dec: orig(bs, bsum, bsq, st * W, dec))
    # ... which the oracle must call: keep its summary update out of the
    # fused Adam launch (where the statistics are not scaled)
    from paddlebox_amd.parallel.dense import FlatAdam

    fuse = FlatAdam.fuse
    monkeypatch.setattr(FlatAdam, "fuse", lambda self, mlps=(), data_norms=(), **kw: fuse(self, mlps=mlps, **kw))
    _, union = _write_files(d, W)
    o_dense, o_h, o_v, _ = _train(fluid, [union], W * B, 0, 1, False)
    o_h, o_v = torch.from_numpy(o_h), torch.from_numpy(o_v)
    for r in range(W):
        res[r] = (res[r][0], torch.from_numpy(res[r][1]), torch.from_numpy(res[r][2]), res[r][3])
    for n, a in o_dense.items():
        for r in range(W):
            np.testing.assert_allclose(res[r][0][n], a, rtol=2e-4, atol=2e-5, err_msg=f"rank {r} {n}")
    allh = torch.cat([res[r][1] for r in range(W)])
    allv = torch.cat([res[r][2] for r in range(W)])
    assert allh.numel() == torch.unique(allh).numel() == o_h.numel()
    for r in range(W):
        assert bool((ref.owner_of(res[r][1], W) == r).all())
    oi = torch.argsort(o_h)
    ai = torch.argsort(allh)
    assert torch.equal(o_h[oi], allh[ai])
    torch.testing.assert_close(allv[ai][:, :14], o_v[oi][:, :14], rtol=2e-4, atol=2e-5)
