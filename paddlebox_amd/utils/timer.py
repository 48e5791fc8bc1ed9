"""Stage span timers (DeviceBoxData timers + PrintSyncTimer, reference
``fw/fleet/box_wrapper.h:394-419``, ``box_wrapper.cc:1085-1138``).

GPU spans are measured with HIP events on the stream (no host syncs in the
hot loop); values are read when the report is printed.  roctx ranges are
emitted around each span so ``rocprofv3 --marker-trace`` shows the pipeline.
"""
from __future__ import annotations

import time
from collections import defaultdict
from contextlib import contextmanager
from typing import Dict, List

import torch


class StageTimers:
    def __init__(self, device=None, enabled: bool = True, roctx: bool = False):
        self.device = device
        self.enabled = enabled
        self.roctx = roctx and torch.cuda.is_available()
        self.gpu_spans: Dict[str, List] = defaultdict(list)
        self.cpu_spans: Dict[str, float] = defaultdict(float)
        self.counts: Dict[str, int] = defaultdict(int)

    @contextmanager
    def span(self, name: str):
        if not self.enabled:
            yield
            return
        use_gpu = self.device is not None and torch.device(self.device).type == "cuda"
        if self.roctx:
            torch.cuda.nvtx.range_push(name)
        t0 = time.perf_counter()
        if use_gpu:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
        try:
            yield
        finally:
            if use_gpu:
                e.record()
                self.gpu_spans[name].append((s, e))
            self.cpu_spans[name] += time.perf_counter() - t0
            self.counts[name] += 1
            if self.roctx:
                torch.cuda.nvtx.range_pop()

    def report(self, reset: bool = True) -> Dict[str, Dict[str, float]]:
        out = {}
        if self.gpu_spans:
            torch.cuda.synchronize()
        for k in set(self.cpu_spans) | set(self.gpu_spans):
            g = sum(s.elapsed_time(e) for s, e in self.gpu_spans.get(k, [])) / 1e3
            out[k] = {"cpu_s": self.cpu_spans.get(k, 0.0), "gpu_s": g, "count": self.counts.get(k, 0)}
        if reset:
            self.gpu_spans.clear()
            self.cpu_spans.clear()
            self.counts.clear()
        return out

    def format(self, reset: bool = True) -> str:
        r = self.report(reset)
        return " ".join(f"{k}:{v['gpu_s'] or v['cpu_s']:.4f}s/{v['count']}" for k, v in sorted(r.items()))
