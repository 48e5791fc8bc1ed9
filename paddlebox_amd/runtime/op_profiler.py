"""Per-op profiler of the dataset trainer (reference: BoxPSWorker's
profile mode, ``TrainFilesWithProfiler`` -- per-op time of every batch,
``boxps_worker.cc:1358-1482``).

GPU ops are timed with HIP events recorded around each lowered op's launch
(resolved once at the end, so profiling adds no per-op host sync); each
op's grad op is timed by hooks on the autograd node that produced its
outputs (``<op>_grad``), and the whole backward and the dense sync +
optimizer as phases.  CPU sessions use wall clocks."""
from __future__ import annotations

import time
from collections import defaultdict
from typing import Dict, List, Tuple

import torch


class OpProfiler:
    def __init__(self, device: torch.device):
        self.device = torch.device(device)
        self.gpu = self.device.type == "cuda"
        self._pending: List[Tuple[str, object, object]] = []
        self.total: Dict[str, float] = defaultdict(float)
        self.calls: Dict[str, int] = defaultdict(int)

    def begin(self):
        if self.gpu:
            e = torch.cuda.Event(enable_timing=True)
            e.record(torch.cuda.current_stream(self.device))
            return e
        return time.perf_counter()

    def end(self, name: str, start):
        if self.gpu:
            e = torch.cuda.Event(enable_timing=True)
            e.record(torch.cuda.current_stream(self.device))
            self._pending.append((name, start, e))
            if len(self._pending) > 4096:
                self._resolve()
        else:
            self.total[name] += (time.perf_counter() - start) * 1e3
            self.calls[name] += 1

    def watch_grad(self, name: str, outputs):
        """Time the autograd nodes that produce this op's outputs (its grad
        op): events recorded by node pre-/post-hooks, attributed as name."""
        seen = set()
        for t in outputs:
            if not isinstance(t, torch.Tensor):
                t = getattr(t, "values", None)  # Ragged
            fn = getattr(t, "grad_fn", None)
            if fn is None or id(fn) in seen:
                continue
            seen.add(id(fn))
            box = {}

            def pre(grad_outputs, box=box):
                box["t0"] = self.begin()

            def post(grad_inputs, grad_outputs, box=box, name=name):
                if "t0" in box:
                    self.end(name, box.pop("t0"))

            fn.register_prehook(pre)
            fn.register_hook(post)

    def _resolve(self):
        if not self._pending:
            return
        torch.cuda.synchronize(self.device)
        for name, a, b in self._pending:
            self.total[name] += a.elapsed_time(b)
            self.calls[name] += 1
        self._pending = []

    def report(self) -> Dict[str, Dict[str, float]]:
        """{op: {ms, calls, ms_per_call, pct}} sorted by time."""
        if self.gpu:
            self._resolve()
        tot = sum(self.total.values()) or 1.0
        rows = sorted(self.total.items(), key=lambda kv: -kv[1])
        return {k: {"ms": round(v, 4), "calls": self.calls[k], "ms_per_call": round(v / max(1, self.calls[k]), 4),
                    "pct": round(100.0 * v / tot, 2)} for k, v in rows}

    def format(self) -> str:
        rep = self.report()
        lines = [f"{'op':40s} {'calls':>7s} {'ms':>10s} {'ms/call':>9s} {'%':>6s}"]
        for k, r in rep.items():
            lines.append(f"{k[:40]:40s} {r['calls']:7d} {r['ms']:10.3f} {r['ms_per_call']:9.4f} {r['pct']:6.2f}")
        return "\n".join(lines)
