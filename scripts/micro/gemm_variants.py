"""Library-GEMM layouts for the CTR backwards' weight gradients (graph-replay
GPU time, us): dW = x^T dy with x [N, K], dy [N, O] computed as a transposed
-A GEMM, on a materialised x^T, or as (dy^T x)^T.

    python scripts/micro/gemm_variants.py
"""
import json

import torch


def gpu_us(fn, iters=50):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) / iters * 1e3, 1)


def main():
    dev = torch.device("cuda:0")
    out = {}
    for (N, K, O, dt) in ((8192, 512, 512, torch.float32), (8192, 400, 400, torch.float16)):
        x = torch.randn(N, K, device=dev).to(dt)
        dy = torch.randn(N, O, device=dev).to(dt)
        W = torch.randn(K, O, device=dev).to(dt)
        tag = f"{N}x{K}x{O}_{str(dt)[6:]}"
        kw = {"out_dtype": torch.float32} if dt == torch.float16 else {}
        out[tag + "_xT_dy"] = gpu_us(lambda: torch.mm(x.t(), dy, **kw))
        out[tag + "_contig_xT_dy"] = gpu_us(lambda: torch.mm(x.t().contiguous(), dy, **kw))
        out[tag + "_dyT_x_T"] = gpu_us(lambda: torch.mm(dy.t(), x, **kw).t().contiguous())
        out[tag + "_dx_dy_WT"] = gpu_us(lambda: torch.mm(dy, W.t(), **kw))
        out[tag + "_transpose_only"] = gpu_us(lambda: x.t().contiguous())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
