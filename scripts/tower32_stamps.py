#!/usr/bin/env python3
"""Timing experiment: per-wave s_memtime stamps of the fp32 tower forward
(stamp 0 start, 2l+1 layer l units done, 2l+2 after the layer barrier, 7 before the loss reduction)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddlebox_amd.ops.mlp import FusedMLP  # noqa: E402

dev = torch.device("cuda:0")
M, dims = 8192, [304, 400, 400, 400]
mlp = FusedMLP(dims[0], dims[1:], 1).to(dev)
ws = mlp.tower_workspace(M, dev, fp32=True)
mlp.ensure_packed()
ws.x0()[:, :dims[0]] = torch.randn(M, dims[0], device=dev)
lin = torch.randn(M, device=dev)
label = (torch.rand(M, device=dev) < 0.3).float()
nwg = ws.Mp // 32
st = torch.zeros(nwg * 8 * 8, dtype=torch.int64, device=dev)
for i in range(5):
    if i == 4:
        ws.set_stamps(st)
    ws.forward(list(mlp.b), mlp.w_out.view(-1), mlp.b_out, lin, label)
torch.cuda.synchronize()
s = st.view(nwg, 8, 8).double().cpu()
t0 = s[:, :, 0].min()
s = s - t0
print("kernel span (ticks)", float(s[:, :, 7].max()))
for l in range(3):
    units = s[:, :, 1 + 2 * l] - (s[:, :, 0] if l == 0 else s[:, :, 2 * l])
    bar = s[:, :, 2 + 2 * l] - s[:, :, 1 + 2 * l]
    print(f"layer {l}: units ticks mean {float(units.mean()):.0f} min {float(units.min()):.0f} max {float(units.max()):.0f}; "
          f"barrier wait mean {float(bar.mean()):.0f} max {float(bar.max()):.0f}")
    for w in range(8):
        print(f"   wave {w}: units mean {float(units[:, w].mean()):.0f}")
print("start skew", float(s[:, :, 0].max()), "staging", float((s[:, :, 1] * 0).mean()))
print("end of layers", float(s[:, :, 6].mean()), "loss part", float((s[:, :, 7] - s[:, :, 6]).mean()))
