#!/usr/bin/env python3
"""Microbenchmark: hand-written MFMA MLP GEMMs vs torch (hipBLASLt) for the
DeepFM shapes.  Interleaved rounds in one process (guide §5.4 rule 24)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddlebox_amd import _native  # noqa: E402

h = _native.hip()
dev = "cuda"


def timeit(fn, iters=50):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e6


def main():
    res = []
    for (M, N, K) in [(8192, 400, 304), (8192, 400, 400), (16384, 400, 400), (8192, 1024, 1024)]:
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
        b = torch.randn(N, device=dev)
        dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
        dW = torch.zeros(N, K, device=dev)
        db = torch.zeros(N, device=dev)
        y = h.linear_fwd(x, w, b, True)
        err = (y.float() - torch.relu(x.float() @ w.float().t() + b)).abs().max().item()
        rounds = {"fwd_pbx": [], "fwd_torch": [], "bwd_pbx": [], "bwd_torch": []}
        xt = x.clone().requires_grad_(True)
        wt = w.clone().requires_grad_(True)
        for _ in range(5):
            rounds["fwd_pbx"].append(timeit(lambda: h.linear_fwd(x, w, b, True)))
            rounds["fwd_torch"].append(timeit(lambda: torch.relu(torch.addmm(b.to(torch.bfloat16), x, w.t()))))
            rounds["bwd_pbx"].append(timeit(lambda: h.linear_bwd(dy, y, x, w, dW, db, True, 512)))

            def tb():
                dz = dy * (y > 0)
                _ = dz @ w
                _ = dz.t() @ x
                _ = dz.sum(0)

            rounds["bwd_torch"].append(timeit(tb))
        flop = 2 * M * N * K
        r = {"M": M, "N": N, "K": K, "max_err": err}
        for k, v in rounds.items():
            us = sorted(v)[len(v) // 2]
            r[k + "_us"] = round(us, 2)
            r[k + "_tflops"] = round((flop * (1 if "fwd" in k else 2)) / us / 1e6, 1)
        res.append(r)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
