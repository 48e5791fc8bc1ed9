"""Microbenchmarks of the CTR GEMM ops at CTR shapes:
batch_fc (slot-batched fp32 MFMA GEMM), scaled_fc (fp16 MFMA, the reference's
fp16 rounding chain), rank_attention (grouped
MFMA GEMMs with gather-on-load) and scaled_int8fc (int8 MFMA, LDS-staged),
forward and forward+backward, timed with HIP events over many iterations.
A torch.matmul (hipBLASLt) fp32 GEMM of the same FLOP shape is printed next
to each as a library reference point.  One JSON line per op on stdout.

  python scripts/micro/bench_ctr_ops.py [--iters 50]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from paddlebox_amd.ops import ctr_ext as cx  # noqa: E402
from tests.ctr_data import page_view_ranks  # noqa: E402

DEV = torch.device("cuda:0")


def timed(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3  # us


def graphed(fn, iters):
    """GPU time of fn without the host launch/autograd overhead: fn captured
    once into a HIP graph (warmed on a side stream first), the replay timed.
    None when fn cannot be captured (a host sync inside)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(g):
            fn()
    except RuntimeError:
        return None
    return timed(g.replay, iters)


def report(name, shape, flops_fwd, f_fwd, f_train, ref_fn, iters, bwd_args=None, fwd_of=None):
    """bwd_args = (inputs, d): the backward alone, timed as
    torch.autograd.grad over a retained graph (no .grad accumulation kernels,
    no forward) -- the number the VERDICT targets."""
    us_f = timed(f_fwd, iters)
    if bwd_args is not None:  # a training step starts from zero_grad(set_to_none=True): no .grad accumulation adds
        f_train0 = f_train

        def f_train():
            for t in bwd_args[0]:
                t.grad = None
            f_train0()
    us_t = timed(f_train, iters)
    us_r = timed(ref_fn, iters)
    rec = {"op": name, "shape": shape, "fwd_us": round(us_f, 1), "fwd_bwd_us": round(us_t, 1),
           "fwd_tflops": round(flops_fwd / us_f / 1e6, 2), "fwd_bwd_tflops": round(3 * flops_fwd / us_t / 1e6, 2),
           "torch_fp32_matmul_same_flops_us": round(us_r, 1)}
    if bwd_args is not None:
        ins, d = bwd_args
        fwd_of = fwd_of or (lambda *a: f_fwd())
        y = f_fwd()
        us_b = timed(lambda: torch.autograd.grad(y, ins, d, retain_graph=True), iters)
        rec["bwd_us"] = round(us_b, 1)
        rec["bwd_tflops"] = round(2 * flops_fwd / us_b / 1e6, 2)
        # forward and forward+backward replayed from HIP graphs: GPU time
        # alone (the eager numbers above include the autograd engine's host
        # time, which dominates at these ~50 us shapes).  The forward is
        # captured with its backward: autograd runs a backward op on the
        # stream its forward ran on, so both must be on the capture stream.
        # fresh leaves: the eager runs above left AccumulateGrad nodes bound
        # to the default stream on the originals
        fresh = [t.detach().clone().requires_grad_() for t in ins]
        print(f"# {name}: capturing", file=sys.stderr, flush=True)
        gf = graphed(lambda: fwd_of(*fresh), iters)
        gt = graphed(lambda: torch.autograd.grad(fwd_of(*fresh), fresh, d), iters)
        rec["fwd_graph_us"] = None if gf is None else round(gf, 1)
        rec["fwd_bwd_graph_us"] = None if gt is None else round(gt, 1)
        rec["bwd_graph_us"] = None if gf is None or gt is None else round(gt - gf, 1)
    print(json.dumps(rec), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    it = a.iters
    g = torch.Generator().manual_seed(0)

    # batch_fc: one fc per slot group (P groups, N instances, I -> O)
    P, N, I, O = 26, 8192, 64, 64
    x = torch.randn(P, N, I, generator=g).to(DEV).requires_grad_()
    W = (torch.randn(P, I, O, generator=g) * 0.1).to(DEV).requires_grad_()
    bb = torch.randn(P, O, generator=g).to(DEV).requires_grad_()
    d = torch.randn(P, N, O, device=DEV)
    xr, wr = x.detach(), W.detach()
    report("batch_fc", [P, N, I, O], 2.0 * P * N * I * O, lambda: cx.batch_fc(x, W, bb),
           lambda: cx.batch_fc(x, W, bb).backward(d), lambda: torch.bmm(xr, wr), it, ([x, W, bb], d),
           fwd_of=lambda x, W, bb: cx.batch_fc(x, W, bb))

    # scaled_fc: [N, K] x [K, O]
    N, K, O = 8192, 400, 400
    x = torch.randn(N, K, generator=g).to(DEV).requires_grad_()
    W = (torch.randn(K, O, generator=g) * 0.05).to(DEV).requires_grad_()
    bb = torch.randn(1, O, generator=g).to(DEV).requires_grad_()
    d = torch.randn(N, O, device=DEV)
    xr, wr = x.detach(), W.detach()
    report("scaled_fc", [N, K, O], 2.0 * N * K * O, lambda: cx.scaled_fc(x, W, bb, 8.0, 2.0),
           lambda: cx.scaled_fc(x, W, bb, 8.0, 2.0).backward(d), lambda: xr @ wr, it, ([x, W, bb], d),
           fwd_of=lambda x, W, bb: cx.scaled_fc(x, W, bb, 8.0, 2.0))

    # rank_attention: B instances, R ranks, x width C, output P
    for R in (3, 8):
        ro = page_view_ranks(8192 // R, R, g).to(DEV)
        B = ro.shape[0]
        C, Pp = 64, 64
        x = torch.rand(B, C, generator=g).to(DEV).requires_grad_()
        W = (torch.rand(R * R * C, Pp, generator=g) * 0.1).to(DEV).requires_grad_()
        d = torch.randn(B, Pp, device=DEV)
        xr = torch.randn(B, R * C, device=DEV)
        wr = torch.randn(R * C, Pp, device=DEV)
        report(f"rank_attention_R{R}", [B, R, C, Pp], 2.0 * B * R * C * Pp, lambda: cx.rank_attention(x, ro, W, R),
               lambda: cx.rank_attention(x, ro, W, R).backward(d), lambda: xr @ wr, it, ([x, W], d),
               fwd_of=lambda x, W, ro=ro, R=R: cx.rank_attention(x, ro, W, R))

    # scaled_int8fc: int8 MFMA forward, fp32 straight-through backward
    # (scaled_int8fc_op.cu:290-440 registers both)
    N, K, O = 8192, 512, 512
    x = torch.randn(N, K, device=DEV).requires_grad_()
    W = (torch.randn(K, O, device=DEV) * 0.2).requires_grad_()
    bb = torch.randn(O, device=DEV).requires_grad_()
    d = torch.randn(N, O, device=DEV)
    xr, wr = x.detach(), W.detach()
    at = dict(input_expand_factor=10.0, input_clip_factor=3.0, weight_expand_factor=40.0, weight_clip_factor=5.0,
              int8_range=127.0)
    report("scaled_int8fc", [N, K, O], 2.0 * N * K * O, lambda: cx.scaled_int8fc(x, W, bb, at),
           lambda: cx.scaled_int8fc(x, W, bb, at).backward(d), lambda: xr @ wr, it, ([x, W, bb], d),
           fwd_of=lambda x, W, bb: cx.scaled_int8fc(x, W, bb, at))


if __name__ == "__main__":
    main()
