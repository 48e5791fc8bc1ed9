#!/usr/bin/env python3
"""Run the 2-rank fluid training of tests/test_gpu_fluid_multirank.py once and
print each rank's outcome as it arrives (for diagnosing the multi-rank fluid
path outside pytest: output streams, a stuck rank is killed after --timeout).

    PBX_TEST_FLUID_GRAPH=0 python scripts/debug_fluid_mr.py
"""
import argparse
import os
import sys
import tempfile

import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tests.test_gpu_fluid_multirank import B as B_  # noqa: E402
from tests.test_gpu_fluid_multirank import _free_port, _worker  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--timeout", type=float, default=120)
    ap.add_argument("--transpile", action="store_true")
    ap.add_argument("--oracle", action="store_true", help="also train the 1-rank union oracle and diff the params")
    a = ap.parse_args()
    W = 2
    d = tempfile.mkdtemp()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, W, port, d, a.transpile, q)) for r in range(W)]
    for p in ps:
        p.start()
    bad = False
    res = {}
    try:
        for _ in range(W):
            r, out = q.get(timeout=a.timeout)
            res[r] = out
            if isinstance(out, str):
                bad = True
                print(f"[rank {r}] ERROR\n{out}", flush=True)
            else:
                print(f"[rank {r}] ok: {out[3]}", flush=True)
    except Exception as e:  # queue timeout
        bad = True
        print(f"[parent] {e!r}", flush=True)
    finally:
        for p in ps:
            p.join(timeout=10)
            if p.is_alive():
                p.kill()
    if not bad and a.oracle:
        compare(res, d, W)
    sys.exit(1 if bad else 0)


def compare(res, d, W):
    """Per-parameter max |difference|: rank vs rank and rank 0 vs the union oracle."""
    import numpy as np

    from paddlebox_amd import _native
    from paddlebox_amd.parallel.dense import FlatAdam
    from tests.test_gpu_fluid_multirank import _train, _write_files

    import paddlebox_amd.fluid as fluid

    h = _native.hip()
    orig = h.data_norm_update
    h.data_norm_update = lambda bs, bsum, bsq, st, dec: orig(bs, bsum, bsq, st * W, dec)
    fuse = FlatAdam.fuse
    FlatAdam.fuse = lambda self, mlps=(), data_norms=(), **kw: fuse(self, mlps=mlps, **kw)
    _, union = _write_files(d, W)
    o_dense, _, _, info = _train(fluid, [union], W * B_, 0, 1, False)
    print(f"[oracle] {info}", flush=True)
    for n, ov in o_dense.items():
        r0, r1 = res[0][0][n], res[1][0][n]
        print(f"{n:28s} r0-r1 {float(np.abs(r0 - r1).max()):.3e}  r0-oracle {float(np.abs(r0 - ov).max()):.3e}"
              f"  |oracle| {float(np.abs(ov).max()):.3e}", flush=True)


if __name__ == "__main__":
    main()
