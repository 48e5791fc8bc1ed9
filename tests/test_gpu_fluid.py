"""The fluid / BoxPS user path on the GPU: the canonical PaddleBox program
(pull_box_sparse -> fused_seqpool_cvm -> concat ->
data_norm -> fc x3 -> sigmoid log-loss, BoxPSOptimizer(Adam)) trained with
``exe.train_from_dataset`` on cuda:0, eagerly and with the step captured in
HIP graphs; both must train and agree with each other."""
import numpy as np
import pytest
import torch

import paddlebox_amd.fluid as fluid
from paddlebox_amd.ps.box_wrapper import BoxWrapper
from paddlebox_amd.utils.flags import set_flags
from tests.test_fluid import DENSE, S, _build, _files

pytestmark = pytest.mark.gpu


def _box():
    b = fluid.core.BoxWrapper(8, device="cuda:0", new=True)
    b.cfg.sgd.mf_create_thresholds = 0.0
    b.initialize_gpu_and_load_model(slot_vector=list(range(S)), max_keys=200000)
    return b


def _run(tmp_path, graph: bool, passes: int = 3, device_pass: bool = True, transpile: bool = False,
         steps_per_graph: int = 0, pipelined: bool = True, n_per_file: int = 320):
    tmp_path.mkdir(parents=True, exist_ok=True)
    set_flags({"FLAGS_padbox_device_pass": device_pass, "FLAGS_padbox_train_steps_per_graph": steps_per_graph,
               "FLAGS_padbox_pipelined_front": pipelined})
    box = _box()
    try:
        scope = fluid.Scope()
        main, startup, slots, label, dense, pred, loss = _build()
        main._pipeline_opt = dict(main._pipeline_opt or {}, use_graph=graph)
        if transpile:  # gradient sync carried by the program (coalesce_tensor -> c_allreduce_sum -> scale)
            fluid.transpiler.GradAllReduce().transpile(startup, main, 0, ["127.0.0.1:6170"], "127.0.0.1:6170")
        exe = fluid.Executor(fluid.CUDAPlace(0))
        exe.run(startup, scope=scope)
        ds = fluid.DatasetFactory().create_dataset("PadBoxSlotDataset")
        ds.set_use_var([label] + slots + [dense])
        ds.set_batch_size(64)
        ds.set_filelist(_files(tmp_path, 2, n_per_file))
        ds.disable_shuffle()
        box.init_metric("AucCalculator", "auc", label.name, pred.name, bucket_size=1000)
        boxps = fluid.core.BoxPS(ds)
        boxps.read_ins_into_memory()
        w0 = np.array(scope.find_var("fc0.w_0").get_tensor()).copy()
        all_stats = []
        for _ in range(passes):
            boxps.begin_pass()
            all_stats.append(exe.train_from_dataset(main, ds, scope=scope, fetch_list=[loss], print_period=1000))
            boxps.end_pass()
        w1 = np.array(scope.find_var("fc0.w_0").get_tensor()).copy()
        msg = box.get_metric_msg("auc")
        h, v = box.engine.table.export(True)
        o = torch.argsort(h)
        dn = {n: np.array(scope.find_var(f"dn.{n}").get_tensor()).copy()
              for n in ("batch_size", "batch_sum", "batch_square_sum")}
        return dict(stats=all_stats, w0=w0, w1=w1, auc=msg[0], n=msg[7], table=v[o].cpu(), dn=dn)
    finally:
        set_flags({"FLAGS_padbox_device_pass": True, "FLAGS_padbox_train_steps_per_graph": 0,
                   "FLAGS_padbox_pipelined_front": True})
        BoxWrapper._instance = None


def test_train_from_dataset_gpu_eager_and_graph(tmp_path):
    eager = _run(tmp_path / "e", graph=False)
    st = eager["stats"][0]
    assert st["batches"] == 10 and st["instances"] == 640
    assert not np.allclose(eager["w0"], eager["w1"])
    assert eager["n"] == 3 * 640 and eager["auc"] > 0.55
    # graphed step fed by the device-resident pass (batches assembled on the
    # GPU) and by the native host assembler thread (pinned ring + H2D)
    for tag, dpass in (("g", True), ("h", False)):
        graphed = _run(tmp_path / tag, graph=True, device_pass=dpass)
        gst = graphed["stats"][-1]
        assert gst["batches"] == 10 and gst.get("graph_replays", 0) > 0
        assert bool(gst.get("device_pass", False)) == dpass
        # same data, same order, same init: the captured step trains the same
        # model (lazily created embedx rows draw from their key, not from the
        # push counter a capture would freeze -- that made graph replays and
        # eager steps diverge by ~1e-4 before round 5)
        np.testing.assert_allclose(graphed["w1"], eager["w1"], rtol=0, atol=1e-4)
        keep = [c for c in range(eager["table"].shape[1]) if c != 14]  # "slot" field: last occurrence, racy
        torch.testing.assert_close(graphed["table"][:, keep], eager["table"][:, keep], rtol=1e-4, atol=1e-5)
        assert abs(graphed["auc"] - eager["auc"]) < 0.01


def test_graphed_loop_is_bench_step(tmp_path):
    """the graphed train_from_dataset loop runs bench.py's
    step -- K = 4 steps per graph with the pipelined front (the next batch
    pooled right after the sparse push) and the AUC accumulated inside the
    graph -- and trains exactly like the plain one-step graphed loop."""
    plain = _run(tmp_path / "p", graph=True, steps_per_graph=1, pipelined=False)
    fast = _run(tmp_path / "f", graph=True)
    st = fast["stats"][-1]
    assert st["steps_per_graph"] == 4 and st["pipelined_front"] and st["graph_replays"] == 8
    assert plain["stats"][-1]["steps_per_graph"] == 1 and not plain["stats"][-1]["pipelined_front"]
    assert fast["n"] == plain["n"] == 3 * 640  # every batch's AUC counted (inside the graphs)
    assert abs(fast["auc"] - plain["auc"]) < 1e-6
    # up to the float atomics of the dW split / sparse push
    np.testing.assert_allclose(fast["w1"], plain["w1"], rtol=0, atol=1e-4)
    keep = [c for c in range(plain["table"].shape[1]) if c != 14]  # "slot" field: last occurrence, racy
    torch.testing.assert_close(fast["table"][:, keep], plain["table"][:, keep], rtol=1e-4, atol=1e-5)
    for k in fast["dn"]:
        np.testing.assert_allclose(fast["dn"][k], plain["dn"][k], rtol=1e-4, atol=1e-4)


def test_graphed_loop_mixed_batch_sizes_keeps_order(tmp_path):
    """a pass whose plan mixes batch sizes (1204 records in 19
    batches: 7 of 64, then 12 of 63) trains in plan order under K = 4 steps
    per graph with the pipelined front -- the batches short of a whole graph
    and the filled sets of one size run before the first batch of the next
    size -- so it matches the eager loop."""
    eager = _run(tmp_path / "e", graph=False, n_per_file=602)
    fast = _run(tmp_path / "f", graph=True, n_per_file=602)
    st = fast["stats"][-1]
    assert st["batches"] == 19 and st["steps_per_graph"] == 4 and st.get("graph_replays", 0) > 0
    assert fast["n"] == eager["n"] == 3 * 1204
    np.testing.assert_allclose(fast["w1"], eager["w1"], rtol=0, atol=1e-4)
    keep = [c for c in range(eager["table"].shape[1]) if c != 14]
    torch.testing.assert_close(fast["table"][:, keep], eager["table"][:, keep], rtol=1e-4, atol=1e-5)


def test_fc_precision_fp32_matches_cpu_oracle(tmp_path):
    """at the default FLAGS_padbox_fc_precision=fp32 the
    lowered GPU program (fused pull + exact-fp32 tower) predicts what the
    op-by-op program computes in float64 on the CPU from the same weights."""
    from paddlebox_amd.fluid.executor import ExecContext, Session
    from tests.test_fluid import _lines

    box = _box()
    try:
        main, startup, slots, label, dense, pred, loss = _build()
        ds = fluid.DatasetFactory().create_dataset("PadBoxSlotDataset")
        ds.set_use_var([label] + slots + [dense])
        ds.set_batch_size(128)
        ds.add_lines(_lines(128, seed=5))
        box.feed_pass(ds)
        scope = fluid.Scope()
        exe = fluid.Executor(fluid.CUDAPlace(0))
        exe.run(startup, scope=scope)
        batch = ds.build_batch(0, 128).to(torch.device("cuda:0"))
        s = Session(main, scope, torch.device("cuda:0"))
        assert "__ctr_tower" in [op.type for op in s.lowered.steps]
        s.training = False
        ctx = ExecContext(s, batch, training=False)
        s.feed_batch(ctx, batch)
        s.forward(ctx)
        gp = ctx.get(pred).detach().double().view(-1).cpu()
        t = next(v for k, v in s.cache.items() if isinstance(k, tuple) and k[0] == "tower")
        assert t.fp32
        # float64 oracle from the same pooled input, weights and summaries
        x = ctx.get(next(op for op in s.lowered.steps if op.type == "__ctr_tower").inputs["X"][0])
        from paddlebox_amd.fluid.kernels import Ragged

        x = (x.values if isinstance(x, Ragged) else x).detach().double().cpu()
        dn = t.dn
        mean = (dn.batch_sum / dn.batch_size).double().cpu()
        scale = torch.sqrt(dn.batch_size / dn.batch_square_sum).double().cpu()
        h = (x - mean) * scale
        h = torch.nn.functional.pad(h, (0, t.mlp.in_dim - h.shape[1]))
        for w, b in zip(t.mlp.w, t.mlp.b):
            h = torch.relu(h @ w.detach().double().cpu().t() + b.detach().double().cpu())
        z = h @ t.mlp.w_out.detach().double().cpu().t() + t.mlp.b_out.detach().double().cpu()
        torch.testing.assert_close(gp, torch.sigmoid(z.view(-1)), rtol=0, atol=2e-6)
    finally:
        BoxWrapper._instance = None


def test_tower_lowering_matches_unfused_program(tmp_path):
    """On the GPU the canonical program lowers to __pull_seqpool_cvm +
    __ctr_tower; its predictions and loss match the op-by-op program (fp32
    data_norm, fc, sigmoid, log-loss) -- both at the reference fc precision
    (fp32, default), and within bf16 tolerance at FLAGS_padbox_fc_precision=bf16."""
    from paddlebox_amd.fluid.executor import ExecContext, Session
    from tests.test_fluid import _lines

    box = _box()
    try:
        main, startup, slots, label, dense, pred, loss = _build()
        ds = fluid.DatasetFactory().create_dataset("PadBoxSlotDataset")
        ds.set_use_var([label] + slots + [dense])
        ds.set_batch_size(128)
        ds.add_lines(_lines(128, seed=3))
        box.feed_pass(ds)
        batch = ds.build_batch(0, 128).to(torch.device("cuda:0"))
        outs = {}
        for fuse in (True, False):
            scope = fluid.Scope()
            exe = fluid.Executor(fluid.CUDAPlace(0))
            exe.run(startup, scope=scope)
            s = Session(main, scope, torch.device("cuda:0"), fuse=fuse)
            if fuse:
                assert "__ctr_tower" in [op.type for op in s.lowered.steps]
            s.training = False
            ctx = ExecContext(s, batch, training=False)
            s.feed_batch(ctx, batch)
            s.forward(ctx)
            outs[fuse] = (ctx.get(pred).detach().float().view(-1).cpu(), float(ctx.get(loss)))
        torch.testing.assert_close(outs[True][0], outs[False][0], rtol=0, atol=2e-5)
        assert abs(outs[True][1] - outs[False][1]) < 2e-5
        # fp32x3: the x3 tower (bf16 hi + lo halves, three products per step)
        set_flags({"FLAGS_padbox_fc_precision": "fp32x3"})
        scope = fluid.Scope()
        exe = fluid.Executor(fluid.CUDAPlace(0))
        exe.run(startup, scope=scope)
        s = Session(main, scope, torch.device("cuda:0"), fuse=True)
        s.training = False
        ctx = ExecContext(s, batch, training=False)
        s.feed_batch(ctx, batch)
        s.forward(ctx)
        t = next(v for k, v in s.cache.items() if isinstance(k, tuple) and k[0] == "tower")
        assert t.x3 and not t.fp32
        torch.testing.assert_close(ctx.get(pred).detach().float().view(-1).cpu(), outs[False][0], rtol=0, atol=1e-4)
        set_flags({"FLAGS_padbox_fc_precision": "bf16"})
        scope = fluid.Scope()
        exe = fluid.Executor(fluid.CUDAPlace(0))
        exe.run(startup, scope=scope)
        s = Session(main, scope, torch.device("cuda:0"), fuse=True)
        s.training = False
        ctx = ExecContext(s, batch, training=False)
        s.feed_batch(ctx, batch)
        s.forward(ctx)
        torch.testing.assert_close(ctx.get(pred).detach().float().view(-1).cpu(), outs[False][0], rtol=0, atol=2e-2)
    finally:
        set_flags({"FLAGS_padbox_fc_precision": "fp32"})
        BoxWrapper._instance = None


def test_profile_mode_on_gpu(tmp_path):
    """train_from_dataset(debug=True): eager steps with every lowered op and
    its grad op timed by HIP events."""
    tmp_path.mkdir(parents=True, exist_ok=True)
    box = _box()
    try:
        scope = fluid.Scope()
        main, startup, slots, label, dense, pred, loss = _build()
        exe = fluid.Executor(fluid.CUDAPlace(0))
        exe.run(startup, scope=scope)
        ds = fluid.DatasetFactory().create_dataset("PadBoxSlotDataset")
        ds.set_use_var([label] + slots + [dense])
        ds.set_batch_size(64)
        ds.set_filelist(_files(tmp_path, 1, 320))
        ds.disable_shuffle()
        boxps = fluid.core.BoxPS(ds)
        boxps.read_ins_into_memory()
        boxps.begin_pass()
        st = exe.train_from_dataset(main, ds, scope=scope, debug=True, print_period=1000)
        boxps.end_pass()
        prof = st["op_profile"]
        assert st["batches"] == 5 and st.get("graph_replays", 0) == 0
        assert prof["dense sync + optimizer"]["calls"] == 5
        assert any(k.endswith("_grad") for k in prof)
        assert all(r["ms"] >= 0 for r in prof.values())
    finally:
        BoxWrapper._instance = None


def test_transpiled_program_captured_on_gpu(tmp_path):
    """A GradAllReduce-transpiled program: the inserted sync ops run after
    backward inside the captured step and train the same model."""
    plain = _run(tmp_path / "p", graph=True, passes=1)
    tr = _run(tmp_path / "t", graph=True, passes=1, transpile=True)
    assert tr["stats"][-1].get("graph_replays", 0) > 0
    np.testing.assert_allclose(tr["w1"], plain["w1"], rtol=0, atol=1e-4)


def test_checkpoint_resume_on_gpu(tmp_path):
    """Save after pass 1 (BoxPS batch model + persistables + Adam state),
    restore into a fresh wrapper / scope and train pass 2 with the captured
    step: equals uninterrupted training up to float atomics."""
    from tests.test_fluid import _resume_run

    files = _files(tmp_path, 2, 320)
    ck = tmp_path / "ck"
    ref_dense, ref_h, _ = _resume_run(tmp_path, files, 1, 1, ckpt=ck, device="cuda:0")
    res_dense, res_h, _ = _resume_run(tmp_path, files, 0, 1, restore=ck, device="cuda:0")
    assert torch.equal(res_h, ref_h)
    for n in ref_dense:
        np.testing.assert_allclose(res_dense[n], ref_dense[n], rtol=0, atol=1e-4, err_msg=n)
