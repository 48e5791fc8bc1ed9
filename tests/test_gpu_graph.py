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


def test_graph_replay_matches_eager():
    # eager reference
    eng_e, model_e, arena_e, opt_e, batches = _setup()
    step_e = _step_fn(model_e, arena_e, opt_e)
    # graphed run from identical initial state
    eng_g, model_g, arena_g, opt_g, _ = _setup()
    step_g = _step_fn(model_g, arena_g, opt_g)
    # GraphedTrainStep warms up 3 eager steps on batch 0: mirror that
    for _ in range(3):
        step_e(batches[0])
    g = GraphedTrainStep(step_g, batches[0], DEV, warmup=3)
    for i in range(1, 6):
        step_e(batches[i])
        g.load(i % 2, batches[i])
        g.run(i % 2)
    torch.cuda.synchronize()
    torch.testing.assert_close(arena_g.flat, arena_e.flat, rtol=1e-3, atol=1e-4)
    h, ve = eng_e.table.export(True)
    vg = eng_g.table.read(h)
    torch.testing.assert_close(vg[:, :13], ve[:, :13], rtol=1e-3, atol=1e-4)
