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
    def __init__(self, device=None, enabled: bool = True, roctx: bool = False, trace: bool = False,
                 rank: int = 0):
        self.device = device
        self.enabled = enabled
        self.roctx = roctx and torch.cuda.is_available()
        self.gpu_spans: Dict[str, List] = defaultdict(list)
        self.cpu_spans: Dict[str, float] = defaultdict(float)
        self.counts: Dict[str, int] = defaultdict(int)
        # chrome-trace recording (tools/timeline.py equivalent): host spans and,
        # on the GPU, event pairs timed against one origin event
        self.trace = trace
        self.rank = rank
        self._events: List[tuple] = []
        self._t0 = time.perf_counter()
        self._origin = None

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
            if self.trace and self._origin is None:
                self._origin = torch.cuda.Event(enable_timing=True)
                self._origin.record()
                self._origin_cpu = t0
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
        try:
            yield
        finally:
            t1 = time.perf_counter()
            if use_gpu:
                e.record()
                self.gpu_spans[name].append((s, e))
            if self.trace:
                self._events.append((name, t0, t1, (s, e) if use_gpu else None))
            self.cpu_spans[name] += t1 - t0
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

    def chrome_trace(self) -> Dict:
        """Recorded spans as a chrome://tracing / Perfetto JSON object: one
        "host" and one "gpu" track per rank (pid = rank)."""
        if any(ev[3] is not None for ev in self._events):
            torch.cuda.synchronize()
        out = []
        for name, t0, t1, ge in self._events:
            out.append({"name": name, "ph": "X", "pid": self.rank, "tid": "host",
                        "ts": (t0 - self._t0) * 1e6, "dur": (t1 - t0) * 1e6})
            if ge is not None and self._origin is not None:
                s, e = ge
                base = (self._origin_cpu - self._t0) * 1e6
                out.append({"name": name, "ph": "X", "pid": self.rank, "tid": "gpu",
                            "ts": base + self._origin.elapsed_time(s) * 1e3, "dur": s.elapsed_time(e) * 1e3})
        return {"traceEvents": out, "displayTimeUnit": "ms"}

    def export_chrome_trace(self, path: str) -> str:
        import json

        with open(path, "w") as f:
            json.dump(self.chrome_trace(), f)
        return path

    def format(self, reset: bool = True) -> str:
        r = self.report(reset)
        return " ".join(f"{k}:{v['gpu_s'] or v['cpu_s']:.4f}s/{v['count']}" for k, v in sorted(r.items()))
