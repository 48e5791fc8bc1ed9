#!/usr/bin/env python3
"""Debug: DeepFM workspace path under GraphedTrainStep with knobs.
usage: debug_graph_ws.py <head_direct 0|1> <n_buffers>"""
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
head_direct = bool(int(sys.argv[1]))
nbuf = int(sys.argv[2])
torch.manual_seed(0)
synth = CriteoSynth(total_features=50000, alpha=1.1, seed=3, device="cuda:0")
eng = SparseEngine(PSConfig(embedx_dim=8), max_keys=256 * 26, device=DEV, capacity=60000)
for chunk in synth.all_keys_chunks(1 << 20):
    eng.insert_local_mixed(ref.mix64(chunk), init_embedx=True)
model = DeepFM(eng, hidden=(32, 16)).to(DEV)
model.head_into_workspace = head_direct
arena = DenseArena(model.parameters(), DEV)
opt = FlatAdam(arena, lr=1e-3)
batches = [synth.batch(256) for _ in range(6)]


def step(b):
    arena.zero_grad()
    loss, _ = model(b)
    loss.backward()
    opt.step()
    return loss.detach()


g = GraphedTrainStep(step, batches[0], DEV, n_buffers=nbuf, warmup=3)
for i in range(1, 6):
    g.load(i % nbuf, batches[i])
    out = g.run(i % nbuf)
    torch.cuda.synchronize()
    print("step", i, float(out), flush=True)
print("OK", flush=True)
