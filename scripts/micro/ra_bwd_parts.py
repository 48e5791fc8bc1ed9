#!/usr/bin/env python3
"""Timing experiment: rank_attention backward parts on their own (graph
replays): part 1 (dexp + gather merge) and part 2 (dW), at the microbench
shapes (R = 3 / 8, C = P = 64).  Knobs read by the launcher: PBX_RA_DEBUG,
PBX_RA_DW_SPLITS.  One JSON line per (R, part)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from paddlebox_amd import _native  # noqa: E402
from tests.ctr_data import page_view_ranks  # noqa: E402

DEV = torch.device("cuda:0")


def main():
    h = _native.hip()
    g = torch.Generator().manual_seed(0)
    iters = int(os.environ.get("ITERS", "50"))
    for R in (3, 8):
        ro = page_view_ranks(8192 // R, R, g).to(DEV).to(torch.int32).contiguous()
        B, C, P = ro.shape[0], 64, 64
        x = torch.rand(B, C, generator=g).to(DEV)
        W = (torch.rand(R * R * C, P, generator=g) * 0.1).to(DEV)
        d = torch.randn(B, P, device=DEV)
        _, bucket = h.rank_attention_fwd(x, ro, W, R)
        for part in (1, 2):
            for _ in range(5):
                h.rank_attention_bwd(x, ro, W, d, bucket, R, part)
            # graph replay: GPU time without the eager launch / allocation cost
            gr = torch.cuda.CUDAGraph()
            st = torch.cuda.Stream()
            st.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(st):
                with torch.cuda.graph(gr, stream=st):
                    for _ in range(20):
                        h.rank_attention_bwd(x, ro, W, d, bucket, R, part)
            torch.cuda.current_stream().wait_stream(st)
            gr.replay()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(iters // 20 + 1):
                gr.replay()
            e1.record()
            torch.cuda.synchronize()
            iters_done = 20 * (iters // 20 + 1)
            print(json.dumps({"R": R, "B": B, "part": part, "us": round(e0.elapsed_time(e1) * 1e3 / iters_done, 2),
                              "debug": os.environ.get("PBX_RA_DEBUG", "0"),
                              "splits": os.environ.get("PBX_RA_DW_SPLITS") or "auto"}), flush=True)


if __name__ == "__main__":
    main()
