"""HIP-graph captured training step == eager step (same state evolution), and
the sparse table / data_norm are updated through the model's backward."""
import pytest
import torch

from paddlebox_amd.data.synthetic import CriteoSynth
from paddlebox_amd.models.deepfm import DeepFM
from paddlebox_amd.parallel.dense import DenseArena, FlatAdam
from paddlebox_amd.ps.config import PSConfig
from paddlebox_amd.ps.sparse_engine import SparseEngine
from paddlebox_amd.runtime.graph_step import GraphedTrainStep

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _setup(seed=0):
    torch.manual_seed(seed)
    synth = CriteoSynth(total_features=50000, alpha=1.1, seed=3, device="cuda:0")
    eng = SparseEngine(PSConfig(embedx_dim=8), max_keys=256 * 26, device=DEV, capacity=60000)
    for chunk in synth.all_keys_chunks(1 << 20):
        from paddlebox_amd.ops import reference as ref

        eng.insert_local_mixed(ref.mix64(chunk), init_embedx=True)
    model = DeepFM(eng, hidden=(32, 16)).to(DEV)
    arena = DenseArena(model.parameters(), DEV)
    opt = FlatAdam(arena, lr=1e-3)
    batches = [synth.batch(256) for _ in range(6)]
    return eng, model, arena, opt, batches


def _step_fn(model, arena, opt):
    def step(b):
        arena.zero_grad()
        loss, _ = model(b)
        loss.backward()
        opt.step()
        return loss.detach()

    return step


def test_sparse_and_data_norm_updated_through_backward():
    eng, model, arena, opt, batches = _setup()
    h0, v0 = eng.table.export(True)
    step = _step_fn(model, arena, opt)
    step(batches[0])
    torch.cuda.synchronize()
    v1 = eng.table.read(h0)
    assert float(v1[:, 0].sum() - v0[:, 0].sum()) == pytest.approx(256 * 26)
    assert float(model.dn.batch_size[0]) != 1e4


@pytest.mark.parametrize("use_ws", [False, True])
def test_graph_replay_matches_eager(use_ws):
    # eager reference, run to completion first (interleaving eager steps of a
    # second model with graph replays is covered by test_two_models_eager)
    eng_e, model_e, arena_e, opt_e, batches = _setup()
    model_e.use_workspace = use_ws
    step_e = _step_fn(model_e, arena_e, opt_e)
    for _ in range(3):
        step_e(batches[0])
    for i in range(1, 6):
        step_e(batches[i])
    torch.cuda.synchronize()
    flat_e = arena_e.flat.clone()
    h, ve = eng_e.table.export(True)
    # graphed run from identical initial state
    eng_g, model_g, arena_g, opt_g, _ = _setup()
    model_g.use_workspace = use_ws
    step_g = _step_fn(model_g, arena_g, opt_g)
    g = GraphedTrainStep(step_g, batches[0], DEV, warmup=3)
    for i in range(1, 6):
        g.load(i % 2, batches[i])
        g.run(i % 2)
    torch.cuda.synchronize()
    torch.testing.assert_close(arena_g.flat, flat_e, rtol=1e-3, atol=1e-4)
    vg = eng_g.table.read(h)
    torch.testing.assert_close(vg[:, :13], ve[:, :13], rtol=1e-3, atol=1e-4)


def test_mlp_workspace_graph_replay():
    """The MLP workspace path captured in a HIP graph replays like eager."""
    from paddlebox_amd.ops.mlp import FusedMLP

    torch.manual_seed(0)
    M, dims = 256, [304, 32, 16]
    mlp = FusedMLP(dims[0], dims[1:], 1).to(DEV)
    mlp.ensure_grads()
    ws = mlp.workspace(M, DEV)
    x = torch.randn(M, dims[0], device=DEV).to(torch.bfloat16)
    ws.x(0)[:, :dims[0]] = x
    ws.xt(0)[:dims[0], :M] = x.t()
    dl = torch.randn(M, device=DEV)

    def step():
        for p in mlp.parameters():
            p.grad.zero_()
        lg = mlp.forward_ws(ws.x(0).requires_grad_(False))
        out = ws.backward(dl, [w.grad for w in mlp.w], [b.grad for b in mlp.b], mlp.w_out.view(-1),
                          mlp.w_out.grad.view(-1), mlp.b_out.grad, True)
        return lg

    step()
    ref = [p.grad.clone() for p in mlp.parameters()]
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    g.replay()
    torch.cuda.synchronize()
    for p, r in zip(mlp.parameters(), ref):
        torch.testing.assert_close(p.grad, r, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("pipelined", [True, False])
def test_prefetched_pull_graph_matches_eager(pipelined):
    """Pipelined pull (graph j dedups + probes buffer j+1 on a side stream):
    same training as eager steps, both with the load-ahead order (the
    prefetch is used) and with load-then-run (each buffer is re-prepared)."""
    eng_e, model_e, arena_e, opt_e, batches = _setup()
    step_e = _step_fn(model_e, arena_e, opt_e)
    for i in [0, 0, 0] + list(range(6)):  # 3 warm-up steps on the example batch
        step_e(batches[i])
    torch.cuda.synchronize()
    flat_e = arena_e.flat.clone()
    h, ve = eng_e.table.export(True)
    eng_g, model_g, arena_g, opt_g, _ = _setup()
    step_g = _step_fn(model_g, arena_g, opt_g)
    g = GraphedTrainStep(step_g, batches[0], DEV, warmup=3, prefetch=(eng_g, lambda b: b.keys))
    if pipelined:
        g.load(0, batches[0])
        for i in range(6):
            if i + 1 < 6:
                g.load((i + 1) % 2, batches[i + 1])
            g.run(i % 2)
    else:
        for i in range(6):
            g.load(i % 2, batches[i])
            g.run(i % 2)
    torch.cuda.synchronize()
    torch.testing.assert_close(arena_g.flat, flat_e, rtol=1e-3, atol=1e-4)
    vg = eng_g.table.read(h)
    torch.testing.assert_close(vg[:, :13], ve[:, :13], rtol=1e-3, atol=1e-4)


def test_multistep_graph_matches_eager():
    """steps_per_graph = 2: each replay trains two batches (two buffer sets
    of two), identical to eager training on the same sequence."""
    eng_e, model_e, arena_e, opt_e, batches = _setup()
    step_e = _step_fn(model_e, arena_e, opt_e)
    for _ in range(3):
        step_e(batches[0])
    seq = [batches[i % 6] for i in range(1, 9)]
    for b in seq:
        step_e(b)
    torch.cuda.synchronize()
    flat_e = arena_e.flat.clone()
    h, ve = eng_e.table.export(True)
    eng_g, model_g, arena_g, opt_g, _ = _setup()
    step_g = _step_fn(model_g, arena_g, opt_g)
    g = GraphedTrainStep(step_g, batches[0], DEV, warmup=3, steps_per_graph=2)
    assert g.n == 2 and len(g.bufs) == 4
    for j in range(4):
        g.load(j % 2, seq[2 * j:2 * j + 2])
        g.run(j % 2)
    torch.cuda.synchronize()
    torch.testing.assert_close(arena_g.flat, flat_e, rtol=1e-3, atol=1e-4)
    vg = eng_g.table.read(h)
    torch.testing.assert_close(vg[:, :13], ve[:, :13], rtol=1e-3, atol=1e-4)
