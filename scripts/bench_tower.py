#!/usr/bin/env python3
"""Microbenchmark of the fused dense tower kernels (csrc/hip/tower.hip).

    python scripts/bench_tower.py [--M 8192] [--dims 304,400,400,400] [--iters 50]

Times forward (k_tower_fwd), backward (k_tower_bwd + k_tower_dw) and the
fused Adam with re-pack, each as back-to-back launches bracketed by events.
Run under rocprofv3 --kernel-trace --stats for per-kernel numbers.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from paddlebox_amd.ops.mlp import FusedMLP  # noqa: E402
from paddlebox_amd.parallel.dense import DenseArena, FlatAdam  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=8192)
    ap.add_argument("--dims", type=str, default="304,400,400,400")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--fp32", action="store_true", help="exact-fp32 tower (tower32.hip)")
    ap.add_argument("--x3", action="store_true", help="fp32 precision on bf16 MFMA (tower_x3.hip)")
    args = ap.parse_args()
    dims = [int(d) for d in args.dims.split(",")]
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    mlp = FusedMLP(dims[0], dims[1:], 1).to(dev)
    arena = DenseArena(mlp.parameters(), dev)
    opt = FlatAdam(arena, lr=1e-3, clear_grad=True).fuse(mlps=[mlp])
    ws = mlp.tower_workspace(args.M, dev, fp32=args.fp32, x3=args.x3)
    mlp.ensure_packed()
    ws.x0()[:, :dims[0]] = torch.randn(args.M, dims[0], device=dev).to(ws.x0().dtype)
    lin = torch.randn(args.M, device=dev)
    label = (torch.rand(args.M, device=dev) < 0.3).float()
    gl = torch.ones(1, device=dev)

    def fwd():
        ws.forward(list(mlp.b), mlp.w_out.view(-1), mlp.b_out, lin, label)

    def bwd(parts=3):
        ws.backward(gl, mlp.w_out.detach().view(-1), [w.grad for w in mlp.w], [b.grad for b in mlp.b],
                    mlp.w_out.grad.view(-1), mlp.b_out.grad, True, parts=parts)

    def step():
        opt.step()

    flops = 2 * args.M * sum(a * b for a, b in zip(dims[:-1], dims[1:]))
    mlp.ensure_grads()
    for name, fn, fl in (("forward", fwd, flops), ("backward", bwd, 2 * flops), ("dX chain", lambda: bwd(1), flops),
                         ("dW", lambda: bwd(2), flops), ("adam+pack", step, 0)):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / args.iters * 1e3
        tf = f"  {fl / us / 1e6:.0f} TFLOP/s" if fl else ""
        print(f"[tower] {name:10s} {us:8.1f} us/launch-set{tf}", flush=True)


if __name__ == "__main__":
    main()
