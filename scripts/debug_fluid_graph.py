"""Compare the eager and graph-captured fluid trainer on the GPU."""
import pathlib
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from tests.test_gpu_fluid import _run  # noqa: E402

base = pathlib.Path("/tmp/pbx_dbg")
e = _run(base / "e", graph=False, passes=1)
g = _run(base / "g", graph=True, passes=1)
for k in ("stats",):
    print("eager", e[k], flush=True)
    print("graph", g[k], flush=True)
print("nan eager", np.isnan(e["w1"]).sum(), "nan graph", np.isnan(g["w1"]).sum())
print("w diff", np.nanmax(np.abs(e["w1"] - g["w1"])))
print("table nan eager", torch.isnan(e["table"]).sum().item(), "graph", torch.isnan(g["table"]).sum().item())
print("auc", e["auc"], g["auc"])
print("nan rows graph", np.where(np.isnan(g["w1"]).any(1))[0], "w shape", g["w1"].shape)
for n in g["dn"]:
    print(n, "nan eager", np.isnan(e["dn"][n]).sum(), "graph", np.isnan(g["dn"][n]).sum(),
          "maxdiff", np.nanmax(np.abs(e["dn"][n] - g["dn"][n])), "cols", np.where(np.isnan(g["dn"][n]))[0])
import os
os.environ["PBX_GRAPH_DEBUG_EAGER"] = "1"
g2 = _run(base / "g2", graph=True, passes=1)
print("eager-through-buffers: nan", np.isnan(g2["w1"]).sum(), "w diff vs eager", np.nanmax(np.abs(e["w1"] - g2["w1"])))
