"""Launch only the CTR backward kernels (k_sfc_dw fp16 / bf16x3, k_f3gemm_nt)
a few times at the microbench shapes -- the program rocprofv3 --pmc passes run.

  python scripts/micro/sfc_dw_only.py [splits_fp16] [splits_bf16x3]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from paddlebox_amd import _native  # noqa: E402
from paddlebox_amd.ops import ctr_ext as cx  # noqa: E402


def main():
    s16 = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    s3 = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    dev = torch.device("cuda:0")
    h = _native.hip()
    x = torch.randn(8192, 400, device=dev)
    dy = torch.randn(8192, 400, device=dev)
    dW, db = torch.empty(400, 400, device=dev), torch.empty(400, device=dev)
    x2, dy2 = torch.randn(8192, 512, device=dev), torch.randn(8192, 512, device=dev)
    W2 = torch.randn(512, 512, device=dev)
    Wh, Wl = cx._bf16_split_of(W2)
    dW2, db2 = torch.empty(512, 512, device=dev), torch.empty(512, device=dev)
    for _ in range(5):
        h.sfc_dw(x, dy, dW, db, 1.0, 32.0, 8.0, 1.0 / 256, s16)
        h.sfc_dw(x2, dy2, dW2, db2, 1.0, 1.0, 1.0, 1.0, s3, mode=1)
        h.f3gemm_nt(dy2, Wh, Wl)
    torch.cuda.synchronize()
    print("ok", flush=True)


if __name__ == "__main__":
    main()
