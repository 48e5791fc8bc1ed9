"""Per-launch times of the scaled_fc / scaled_int8fc backward pieces at the
microbench shapes (HIP events, many iterations): which launch the backward
spends its time in.

  python scripts/micro/scaled_fc_parts.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from paddlebox_amd import _native  # noqa: E402
from paddlebox_amd.ops import ctr_ext as cx  # noqa: E402

DEV = torch.device("cuda:0")


def timed(fn, iters=100):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) / iters * 1e3, 1)


def main():
    h = _native.hip()
    out = {}
    N, K, O = 8192, 400, 400
    g = torch.Generator().manual_seed(0)
    x = torch.randn(N, K, generator=g).to(DEV)
    W = (torch.randn(K, O, generator=g) * 0.05).to(DEV)
    dy = torch.randn(N, O, device=DEV)
    in_scale, gs = 8.0, 256.0
    W16 = cx._half_of(W)
    out["sfc_dx"] = timed(lambda: h.sfc(dy, W16, None, gs / in_scale, in_scale, 1.0, 1.0 / gs))
    out["d16_cast"] = timed(lambda: (dy * (gs / in_scale)).half())
    out["x_half"] = timed(lambda: x.half())
    x16, d16 = x.half(), (dy * (gs / in_scale)).half()
    out["mm16_dW"] = timed(lambda: cx._mm16(x16.t(), d16))
    acc = cx._mm16(x16.t(), d16)
    out["h16_epi"] = timed(lambda: h.h16_epi(acc, None, in_scale, 1.0, 1.0 / gs))
    db = dy.new_empty(O)
    out["colsum"] = timed(lambda: h.colsum_strided(dy, 1, N, O, 0, O, db, 0, False))
    dW = W.new_empty(K, O)
    for sp in (1, 4, 8, 16):
        out[f"hgemm_dW_split{sp}"] = timed(
            lambda sp=sp: h.hgemm(x, dy, dW, None, K, O, N, [1, K], [O, 1], O, 1.0, gs / in_scale, in_scale, 1.0,
                                  1.0 / gs, sp))
    for sp in (1, 4, 5, 6, 7, 8, 10, 12, 16, 19, 24, 32):
        out[f"sfc_dw_split{sp}"] = timed(
            lambda sp=sp: h.sfc_dw(x, dy, dW, db, 1.0, gs / in_scale, in_scale, 1.0 / gs, sp))
    out["sfc_dw_default_split"] = cx._sfc_dw_splits(N, K, O)
    out["torch_mm_fp32_dW"] = timed(lambda: x.t() @ dy)
    out["torch_mm_fp32_dx"] = timed(lambda: dy @ W.t())
    out["torch_sum_db"] = timed(lambda: dy.sum(0))
    # scaled_int8fc backward at its shape: the fp32 straight-through GEMMs
    N2, K2, O2 = 8192, 512, 512
    x2 = torch.randn(N2, K2, device=DEV)
    W2 = torch.randn(K2, O2, device=DEV)
    dy2 = torch.randn(N2, O2, device=DEV)
    out["i8_ksgemm_bwd"] = timed(lambda: cx._fc_backward_hip(x2, W2, dy2))
    out["i8_torch_bwd"] = timed(lambda: (dy2 @ W2.t(), x2.t() @ dy2, dy2.sum(0)))
    Wh, Wl = cx._bf16_split_of(W2)
    out["i8_f3_dx"] = timed(lambda: h.f3gemm_nt(dy2, Wh, Wl))
    dW2, db2 = W2.new_empty(K2, O2), dy2.new_empty(O2)
    for sp in (4, 8, 10, 16):
        out[f"i8_f3_dw_split{sp}"] = timed(lambda sp=sp: h.sfc_dw(x2, dy2, dW2, db2, 1.0, 1.0, 1.0, 1.0, sp, mode=1))
    out["i8_f3_dw_default_split"] = cx._sfc_dw_splits(N2, K2, O2)
    out["i8_torch_dx"] = timed(lambda: dy2 @ W2.t())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
