#!/usr/bin/env python3
"""Microbenchmark: DeepFM MLP (M=8192, 280-400-400-400-1) forward+backward,
workspace engine (csrc/hip/mlp.hip) vs the register-staged GEMM path
(csrc/hip/gemm.hip) vs torch fp32->bf16 autocast reference."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddlebox_amd.ops.mlp import FusedMLP  # noqa: E402

dev = torch.device("cuda")


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e6


def main():
    out = []
    for M, dims in [(8192, [280, 400, 400, 400]), (16384, [280, 400, 400, 400]), (8192, [512, 1024, 1024, 512])]:
        mlp = FusedMLP(dims[0], dims[1:], 1).to(dev)
        mlp.ensure_grads()
        x = torch.randn(M, dims[0], device=dev).to(torch.bfloat16)
        ws = mlp.workspace(M, dev)
        ws.x(0)[:, :dims[0]] = x
        ws.xt(0)[:dims[0], :M] = x.t()
        x0 = ws.x(0)
        dl = torch.randn(M, device=dev)

        def ws_step():
            lg = mlp.forward_ws(x0.requires_grad_(True))
            lg.backward(dl)

        def old_step():
            xx = x.detach().requires_grad_(True)
            lg = mlp(xx)
            lg.backward(dl)

        def ws_fwd():
            with torch.no_grad():
                ws.forward(list(mlp.w), list(mlp.b), mlp.w_out.view(-1), mlp.b_out)

        r = {"M": M, "dims": dims}
        for _ in range(2):  # interleaved rounds
            r["ws_fwd_us"] = timeit(ws_fwd)
            r["ws_step_us"] = timeit(ws_step)
            r["old_step_us"] = timeit(old_step)
        flops = 0
        for a, b in zip(dims[:-1], dims[1:]):
            flops += 2 * M * a * b * 3
        r["ws_tflops"] = flops / r["ws_step_us"] / 1e6
        out.append(r)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
