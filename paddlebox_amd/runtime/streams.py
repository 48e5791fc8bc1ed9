"""Process-wide named side streams.

A HIP process gets GPU_MAX_HW_QUEUES hardware queues (4 by default); streams
created beyond that share queues round-robin, and two streams on one queue
serialise.  Components that need a side stream (the tower's dW GEMM, the
dense all-reduce, the batch copy of the graph runner) therefore take a named
stream from here instead of creating their own: rebuilding a model, or
building a second one in the same process (bench.py's secondary precision),
then reuses the same queues instead of landing a side stream on the main
stream's queue and losing the overlap (measured: fp32 step 0.44 -> 0.53 ms
when the second model's dW stream shared the compute queue).
"""
from __future__ import annotations

from typing import Dict, Tuple

import torch

_streams: Dict[Tuple[int, str], torch.cuda.Stream] = {}


def side_stream(device, name: str) -> torch.cuda.Stream:
    dev = torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    key = (idx, name)
    s = _streams.get(key)
    if s is None:
        s = torch.cuda.Stream(torch.device("cuda", idx))
        _streams[key] = s
    return s
