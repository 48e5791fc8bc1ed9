#!/usr/bin/env python3
"""Debug: eager model + graphed model interleaved (tests/test_gpu_graph.py)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddlebox_amd.data.synthetic import CriteoSynth  # noqa: E402
from paddlebox_amd.models.deepfm import DeepFM  # noqa: E402
from paddlebox_amd.ops import reference as ref  # noqa: E402
from paddlebox_amd.parallel.dense import DenseArena, FlatAdam  # noqa: E402
from paddlebox_amd.ps.config import PSConfig  # noqa: E402
from paddlebox_amd.ps.sparse_engine import SparseEngine  # noqa: E402
from paddlebox_amd.runtime.graph_step import GraphedTrainStep  # noqa: E402

DEV = torch.device("cuda:0")
mode = sys.argv[1]


def setup(use_ws=True):
    torch.manual_seed(0)
    synth = CriteoSynth(total_features=50000, alpha=1.1, seed=3, device="cuda:0")
    eng = SparseEngine(PSConfig(embedx_dim=8), max_keys=256 * 26, device=DEV, capacity=60000)
    for chunk in synth.all_keys_chunks(1 << 20):
        eng.insert_local_mixed(ref.mix64(chunk), init_embedx=True)
    model = DeepFM(eng, hidden=(32, 16)).to(DEV)
    model.use_workspace = use_ws
    model.head_into_workspace = os.environ.get("E_HEAD", "direct") == "direct"
    arena = DenseArena(model.parameters(), DEV)
    opt = FlatAdam(arena, lr=1e-3)
    batches = [synth.batch(256) for _ in range(6)]

    def step(b):
        arena.zero_grad()
        loss, _ = model(b)
        loss.backward()
        opt.step()
        return loss.detach()

    return step, batches


e_ws = os.environ.get("E_WS", "1") == "1"
g_ws = os.environ.get("G_WS", "1") == "1"
step_e, batches = setup(e_ws)
if mode == "eager2":
    step_f, _ = setup()
    for i in range(6):
        print("e", i, float(step_e(batches[i])), flush=True)
        torch.cuda.synchronize()
        print("f", i, float(step_f(batches[i])), flush=True)
        torch.cuda.synchronize()
else:
    step_g, _ = setup(g_ws)
    for _ in range(3):
        step_e(batches[0])
    torch.cuda.synchronize()
    print("warm e ok", flush=True)
    g = GraphedTrainStep(step_g, batches[0], DEV, warmup=3)
    print("captured", flush=True)
    for i in range(1, 6):
        print("e", i, float(step_e(batches[i])), flush=True)
        torch.cuda.synchronize()
        g.load(i % 2, batches[i])
        out = g.run(i % 2)
        torch.cuda.synchronize()
        print("g", i, float(out), flush=True)
print("OK", flush=True)
