"""IPC mesh exchange / all-reduce launch cost on one rank (W = 1): the fixed
part (epoch, arrive / publish / wait, depart) against the copy, by grid size,
payload and fence setting -- what the 1-rank sharded rehearsal pays per
exchange.  python scripts/micro/ipc_exchange_bench.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from paddlebox_amd.parallel.ipc import IpcMesh  # noqa: E402


def timed(fn, iters=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(20):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a.record()
    for _ in range(iters // 20):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) / iters * 1e3, 2)


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    out = []
    for fence in ("1",):
        for slot_mb, rec, used in ((1.7, 8, 68000), (10.2, 48, 68000)):
            slot = int(slot_mb * 1e6) // 16 * 16
            for blocks in (16, 32, 64, 128, 256):
                m = IpcMesh(slot, device=dev, blocks=blocks)
                send = torch.zeros(slot, dtype=torch.uint8, device=dev)
                dst = torch.empty_like(send)
                cnt = torch.tensor([used], dtype=torch.int32, device=dev)
                rc = torch.zeros(1, dtype=torch.int32, device=dev)
                us = timed(lambda: m.exchange(send.view(1, -1), dst.view(1, -1), cnt, rec, rec == 8, rc))
                out.append({"op": "exchange", "fence": fence, "slot_mb": slot_mb, "rec": rec, "records": used,
                            "blocks": blocks, "us": us})
                print(json.dumps(out[-1]), flush=True)
                m.close()
        n = 160_000  # a dense gradient arena's floats
        for blocks in (16, 32, 64, 128, 256):
            m = IpcMesh(n * 4, device=dev, blocks=blocks)
            x = torch.randn(n, device=dev)
            us = timed(lambda: m.allreduce_(x))
            print(json.dumps({"op": "allreduce", "fence": fence, "floats": n, "blocks": blocks, "us": us}), flush=True)


if __name__ == "__main__":
    main()
