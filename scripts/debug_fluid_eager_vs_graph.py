#!/usr/bin/env python3
"""One rank, the multirank test's union data: the graphed device-pass loop
(K steps per graph) against the same batches trained eagerly (a K larger than
the pass, so nothing is captured): per-parameter max |difference| and the
table rows.

    python scripts/debug_fluid_eager_vs_graph.py [--k 1]
"""
import argparse
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=1)
    ap.add_argument("--pipe", default="false")
    a = ap.parse_args()
    import paddlebox_amd.fluid as fluid
    from paddlebox_amd.utils import flags
    from tests.test_gpu_fluid_multirank import B, _train, _write_files

    d = tempfile.mkdtemp()
    _, union = _write_files(d, 2)
    flags.set_flags({"padbox_pipelined_front": a.pipe, "padbox_train_steps_per_graph": str(a.k)})
    g_dense, g_h, g_v, gi = _train(fluid, [union], 2 * B, 0, 1, False)
    flags.set_flags({"padbox_train_steps_per_graph": "64"})
    e_dense, e_h, e_v, ei = _train(fluid, [union], 2 * B, 0, 1, False)
    print(f"graphed {gi}  eager {ei}", flush=True)
    for n in g_dense:
        print(f"{n:24s} |graph - eager| {float(np.abs(g_dense[n] - e_dense[n]).max()):.3e}", flush=True)
    og, oe = np.argsort(g_h), np.argsort(e_h)
    assert np.array_equal(g_h[og], e_h[oe])
    dv = np.abs(g_v[og] - e_v[oe])
    print(f"table rows: max |diff| {float(dv.max()):.3e} per column {np.round(dv.max(0), 8).tolist()}", flush=True)


if __name__ == "__main__":
    main()
