"""Diagnostic: max difference between the fused and unfused Adam runs of
tests/test_gpu_tower32.py::test_tower32_fused_adam_repack, over repeats."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_gpu_tower32 import DEV, _make  # noqa: E402

from paddlebox_amd.ops.tower import CtrTower  # noqa: E402
from paddlebox_amd.parallel.dense import DenseArena, FlatAdam  # noqa: E402

S, Eo, Dd, D = 26, 11, 13, 8
x, label, dn, mlp = _make(512, S, Eo, Dd, (96, 64))
for rep in range(3):
    runs = []
    for fused in (False, True, False):
        d, m = copy.deepcopy(dn).to(DEV), copy.deepcopy(mlp).to(DEV)
        t = CtrTower(m, d, S, Eo, 2, D, fp32=True)
        arena = DenseArena(m.parameters(), torch.device(DEV))
        opt = FlatAdam(arena, lr=1e-2, clear_grad=True)
        if fused:
            opt.fuse(mlps=[m], data_norms=[d])
        for _ in range(3):
            loss, _ = t(x.to(DEV), label.to(DEV))
            loss.backward()
            opt.step()
        torch.cuda.synchronize()
        runs.append(arena.flat.clone())
    d_fu = (runs[0] - runs[1]).abs()
    d_uu = (runs[0] - runs[2]).abs()
    print(f"rep {rep}: unfused-vs-fused max {float(d_fu.max()):.3e} at {int(d_fu.argmax())} (n>1e-6: {int((d_fu > 1e-6).sum())}); "
          f"unfused-vs-unfused max {float(d_uu.max()):.3e}", flush=True)
