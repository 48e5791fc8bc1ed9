"""Collective / step watchdog (SURVEY §5.3 "watchdog on collectives (timeout
-> abort with rank dump)").  The reference's only hang prevention is batch
count equalisation across nodes (``data_set.cc:2692-2757``); a rank that
stalls inside NCCL hangs the job forever.

A daemon thread watches named deadlines.  ``with wd.guard("allreduce"):``
arms a deadline around a region; ``wd.beat("train")`` refreshes a periodic
heartbeat.  When a deadline passes the watchdog writes every thread's Python
stack to ``<dump_dir>/watchdog_rank<r>.txt`` (and a line to stderr) and calls
``on_timeout`` -- by default ``os._exit(124)``, so the launcher sees a failed
rank instead of a silent hang.
"""
from __future__ import annotations

import faulthandler
import os
import sys
import threading
import time
from contextlib import contextmanager
from typing import Callable, Dict, Optional


class Watchdog:
    def __init__(self, timeout_s: float = 600.0, rank: int = 0, dump_dir: str = ".",
                 on_timeout: Optional[Callable[[str], None]] = None, poll_s: float = 0.5):
        self.timeout_s = float(timeout_s)
        self.rank = rank
        self.dump_dir = dump_dir
        self.on_timeout = on_timeout or (lambda name: os._exit(124))
        self.poll_s = poll_s
        self._deadlines: Dict[str, float] = {}
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self.fired: Optional[str] = None
        self._th = threading.Thread(target=self._loop, name="pbx-watchdog", daemon=True)
        self._th.start()

    def arm(self, name: str, timeout_s: Optional[float] = None):
        with self._lock:
            self._deadlines[name] = time.monotonic() + (timeout_s or self.timeout_s)

    def disarm(self, name: str):
        with self._lock:
            self._deadlines.pop(name, None)

    def beat(self, name: str = "step", timeout_s: Optional[float] = None):
        self.arm(name, timeout_s)

    @contextmanager
    def guard(self, name: str, timeout_s: Optional[float] = None):
        self.arm(name, timeout_s)
        try:
            yield
        finally:
            self.disarm(name)

    def _loop(self):
        while not self._stop.wait(self.poll_s):
            now = time.monotonic()
            with self._lock:
                late = [n for n, d in self._deadlines.items() if now > d]
            if late:
                name = late[0]
                self.fired = name
                self.dump(name)
                with self._lock:
                    self._deadlines.pop(name, None)
                self.on_timeout(name)

    def dump(self, name: str) -> str:
        os.makedirs(self.dump_dir, exist_ok=True)
        path = os.path.join(self.dump_dir, f"watchdog_rank{self.rank}.txt")
        with open(path, "w") as f:
            f.write(f"watchdog: '{name}' exceeded its deadline on rank {self.rank} at {time.time():.3f}\n")
            f.flush()
            faulthandler.dump_traceback(file=f, all_threads=True)
        sys.stderr.write(f"[watchdog] rank {self.rank}: '{name}' timed out; stacks in {path}\n")
        sys.stderr.flush()
        return path

    def stop(self):
        self._stop.set()
        self._th.join(timeout=2 * self.poll_s + 1)
