"""SsdLog put / erase / get timing at a config-4 spill size (8.6M rows of 16
floats) on the box's disk: the write-back's SSD leg alone.

  PBX_SSD_TIMING=1 python scripts/micro/ssd_put_bench.py /tmp/pbx_ssd_put
"""
import os
import shutil
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from paddlebox_amd import _native  # noqa: E402


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "/tmp/pbx_ssd_put"
    shutil.rmtree(d, ignore_errors=True)
    H = _native.host()
    s = H.SsdLog(d, 16, 64 << 20)
    n = 8_600_000
    g = torch.Generator().manual_seed(0)
    k = torch.randint(0, 2 ** 62, (n,), dtype=torch.int64, generator=g)
    v = torch.randn(n, 16, generator=g)
    for rep in range(2):
        t = time.perf_counter()
        s.put(k, v)
        print(f"put {n} rows rep {rep}: {time.perf_counter() - t:.3f} s (direct io {s.direct_io()})", flush=True)
    t = time.perf_counter()
    gone = s.erase(k[: n // 4])
    print(f"erase {gone}: {time.perf_counter() - t:.3f} s", flush=True)
    shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
