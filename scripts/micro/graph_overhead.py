#!/usr/bin/env python3
"""Per-kernel cost of dependent tiny kernels: eager vs HIP graph (one stream),
and with the repo's own 1-block fill kernel.  Prints us per kernel."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from paddlebox_amd import _native  # noqa: E402

h = _native.hip()
dev = torch.device("cuda:0")
t = torch.zeros(256, device=dev)
big = torch.zeros(1 << 20, device=dev)
N = 200


def run_eager(fn, reps=5):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best / N * 1e6


def chain_small():
    for i in range(N):
        t.add_(1.0)


def chain_big():
    for i in range(N):
        big.add_(1.0)


for name, fn in (("tiny add_ (1 WG)", chain_small), ("1M add_ (4K WG)", chain_big)):
    e = run_eager(fn)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        fn()
    gr = run_eager(g.replay)
    print(f"{name:20s}: eager {e:6.2f} us/kernel, graph replay {gr:6.2f} us/kernel", flush=True)
