#!/usr/bin/env python3
"""Timing experiment: the weight-gradient GEMMs of the CTR op backwards
(C = A^T B over a long K = the batch) under different schedules, graph-replay
GPU time.  scaled_fc dW (fp16 k_hgemm, split-K sweep) at N=8192, 400x400;
scaled_int8fc dW (fp32) at N=8192, 512x512: library mm in both operand
orders, library batched split-K + sum, k_mgemm split-K.  One JSON line each."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from paddlebox_amd import _native  # noqa: E402
from paddlebox_amd.ops import ctr_ext as cx  # noqa: E402

DEV = torch.device("cuda:0")


def graph_us(fn, reps=20, iters=10):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / (reps * iters)


def main():
    h = _native.hip()
    torch.manual_seed(0)
    N, K, O = 8192, 400, 400
    x = torch.randn(N, K, device=DEV)
    dy = torch.randn(N, O, device=DEV)
    dW = torch.empty(K, O, device=DEV)
    ref = None
    for ks in (4, 8, 16, 32, 64):
        f = lambda ks=ks: h.hgemm(x, dy, dW, None, K, O, N, [1, K], [O, 1], O, 1.0, 0.25, 8.0, 1.0, 0.5, ks)
        us = graph_us(f)
        f()
        torch.cuda.synchronize()
        if ref is None:
            ref = dW.clone()
        err = float((dW - ref).abs().max())
        print(json.dumps({"gemm": "scaled_fc_dW_hgemm", "ksplit": ks, "us": round(us, 2), "maxdiff_vs_ks4": err}),
              flush=True)

    # library alternative: fp16 casts, S row-block fp16 GEMMs with fp32
    # outputs (fp32 accumulate), fixed-order sum, the fp16 epilogue
    ref16 = dW.clone()
    h.hgemm(x, dy, ref16, None, K, O, N, [1, K], [O, 1], O, 1.0, 0.25, 8.0, 1.0, 0.5, 16)
    for S in (4, 8, 16):
        part = torch.empty(S, K, O, device=DEV)

        def f(S=S, part=part):
            x16 = x.half()
            d16 = (dy * 0.25).half()
            torch.bmm(x16.view(S, N // S, K).transpose(1, 2), d16.view(S, N // S, O), out_dtype=torch.float32,
                      out=part)
            torch.sum(part, 0, out=dW)
            h.h16_epi(dW, None, 8.0, 1.0, 0.5)
        try:
            us = graph_us(f)
        except Exception as e:  # noqa: BLE001
            print(json.dumps({"gemm": "scaled_fc_dW_lib16", "S": S, "error": str(e)[:200]}), flush=True)
            break
        f()
        torch.cuda.synchronize()
        err = float(((dW - ref16).abs() / (ref16.abs() + 1e-3)).max())
        print(json.dumps({"gemm": "scaled_fc_dW_lib16", "S": S, "us": round(us, 2), "max_rel_vs_hgemm": err}),
              flush=True)

    N, K, O = 8192, 512, 512
    x = torch.randn(N, K, device=DEV)
    dy = torch.randn(N, O, device=DEV)
    dW = torch.empty(K, O, device=DEV)
    ref = x.t().double() @ dy.double()

    def rec(name, fn, out):
        us = graph_us(fn)
        fn()
        torch.cuda.synchronize()
        err = float((out().double() - ref).abs().max() / ref.abs().max())
        print(json.dumps({"gemm": "int8fc_dW_fp32", "schedule": name, "us": round(us, 2), "rel_err": err}), flush=True)

    rec("mm(x^T, dy)", lambda: torch.mm(x.t(), dy, out=dW), lambda: dW)
    dWt = torch.empty(O, K, device=DEV)
    rec("mm(dy^T, x)^T", lambda: torch.mm(dy.t(), x, out=dWt), lambda: dWt.t())
    for S in (2, 4, 8, 16):
        part = torch.empty(S, K, O, device=DEV)

        def f(S=S, part=part):
            torch.bmm(x.view(S, N // S, K).transpose(1, 2), dy.view(S, N // S, O), out=part)
            torch.sum(part, 0, out=dW)
        rec(f"bmm split {S} + sum", f, lambda: dW)
    rec("k_mgemm split-K", lambda: cx._sg(x, dy, dW, K, O, N, 1, (0, 1, K), (0, O, 1), 0, O), lambda: dW)


if __name__ == "__main__":
    main()
