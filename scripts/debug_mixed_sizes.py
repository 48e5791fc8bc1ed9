"""Mixed batch sizes in one pass (1204 records: 7 x 64 then 12 x 63): which
configuration of the graphed device-pass loop departs from the eager loop.
usage (GPU box): python scripts/debug_mixed_sizes.py"""
import os
import sys
import tempfile
from pathlib import Path

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_gpu_fluid import _run  # noqa: E402

tmp = Path(tempfile.mkdtemp())
n = int(os.environ.get("N_PER_FILE", "602"))
passes = int(os.environ.get("PASSES", "1"))
eager = _run(tmp / "e", graph=False, n_per_file=n, passes=passes)
print("eager batches", eager["stats"][-1]["batches"], flush=True)
for K, pipe in ((1, False), (4, False), (1, True), (4, True)):
    r = _run(tmp / f"g{K}{int(pipe)}", graph=True, n_per_file=n, steps_per_graph=K, pipelined=pipe, passes=passes)
    st = r["stats"][-1]
    d = float(np.abs(r["w1"] - eager["w1"]).max())
    dt = float((r["table"] - eager["table"]).abs().max())
    print(f"K={K} pipe={pipe}: replays={st.get('graph_replays')} w1 maxdiff={d:.3e} table maxdiff={dt:.3e}",
          flush=True)
