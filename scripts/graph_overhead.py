#!/usr/bin/env python3
"""Measure HIP-graph replay cost vs node count on the GPU box.

For N tiny dependent kernels captured in one graph, reports per replay:
host enqueue time (replay call only), GPU wall per replay (events, back to
back), first-window vs steady-state, and the same N kernels launched eagerly.
Also times hipGraphUpload (if reachable through ctypes) on the first replay.
"""
import ctypes
import time

import torch


def build(n, x):
    for _ in range(n):
        x.add_(1.0)


def main():
    dev = torch.device("cuda:0")
    x = torch.zeros(64, device=dev)
    try:
        hip = ctypes.CDLL("libamdhip64.so")
    except OSError:
        hip = None
    for n in (1, 8, 16, 32, 64, 128):
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            build(n, x)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            build(n, x)
        torch.cuda.synchronize()
        uploaded = False
        if hip is not None and hasattr(g, "raw_cuda_graph_exec"):
            try:
                ex = g.raw_cuda_graph_exec()
                rc = hip.hipGraphUpload(ctypes.c_void_p(ex), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
                torch.cuda.synchronize()
                uploaded = rc == 0
            except Exception:
                uploaded = False
        res = []
        for w in range(6):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(20):
                g.replay()
            th = time.perf_counter() - t0
            torch.cuda.synchronize()
            tw = time.perf_counter() - t0
            res.append((th / 20 * 1e6, tw / 20 * 1e6))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            build(n, x)
        te = time.perf_counter() - t0
        torch.cuda.synchronize()
        tew = time.perf_counter() - t0
        print(f"N={n:4d} upload={uploaded} graph host/wall us per replay by 20-window: "
              + " ".join(f"{a:.0f}/{b:.0f}" for a, b in res)
              + f" | eager host/wall {te / 20 * 1e6:.0f}/{tew / 20 * 1e6:.0f}", flush=True)


if __name__ == "__main__":
    main()
