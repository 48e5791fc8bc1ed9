"""Environment-driven fault injection (fault-injection hooks --
drop a file read, kill a rank at pass k, corrupt a shard -- exercised in
tests).  The reference has none: recovery there is operational (restart the
day/pass from the last SaveBase/SaveDelta + dense persistables,
``box_wrapper.cc:1286-1318``), and reads retry in a loop
(``data_feed.cc:3748-3750``).

``PBX_FAULT`` holds ``;``-separated rules ``<point>[@key=value,...]``:

  * ``read_fail@file=<substr>,times=<n>``  the first n opens of a matching file fail
  * ``kill_rank@rank=<r>,pass=<k>``        rank r exits with status 101 at begin_pass k
  * ``corrupt_shard@rank=<r>``             rank r's table rows are NaN-poisoned at save
  * ``nan_grad@step=<s>``                  dense gradients get a NaN at step s
  * ``hang@point=<name>,seconds=<t>``      sleep t seconds at a named point (watchdog tests)

``hit(point, **ctx)`` returns the matching rule (or None) and counts it.
"""
from __future__ import annotations

import os
import threading
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

ELASTIC_EXIT_CODE = 101  # the exit code upstream fleet/elastic restarts on


@dataclass
class Rule:
    point: str
    args: Dict[str, str] = field(default_factory=dict)
    hits: int = 0

    def matches(self, ctx: Dict[str, object]) -> bool:
        for k, v in self.args.items():
            if k in ("times", "seconds"):
                continue
            if k == "file":
                if v not in str(ctx.get("file", "")):
                    return False
                continue
            if k not in ctx or str(ctx[k]) != v:
                return False
        times = self.args.get("times")
        return times is None or self.hits < int(times)


_lock = threading.Lock()
_rules: Optional[List[Rule]] = None


def parse(spec: str) -> List[Rule]:
    rules = []
    for part in filter(None, (p.strip() for p in spec.split(";"))):
        point, _, rest = part.partition("@")
        args = {}
        for kv in filter(None, rest.split(",")):
            k, _, v = kv.partition("=")
            args[k.strip()] = v.strip()
        rules.append(Rule(point.strip(), args))
    return rules


def rules() -> List[Rule]:
    global _rules
    with _lock:
        if _rules is None:
            _rules = parse(os.environ.get("PBX_FAULT", ""))
        return _rules


def configure(spec: str):
    """Replace the active rules (tests)."""
    global _rules
    with _lock:
        _rules = parse(spec)


def hit(_point: str, **ctx) -> Optional[Rule]:
    for r in rules():
        if r.point == _point and r.matches(ctx):
            with _lock:
                r.hits += 1
            return r
    return None


class InjectedFault(RuntimeError):
    pass


def maybe_fail_read(path: str):
    if hit("read_fail", file=path) is not None:
        raise InjectedFault(f"injected read failure: {path}")


def maybe_kill(rank: int, pass_id: int):
    if hit("kill_rank", rank=rank, **{"pass": pass_id}) is not None:
        os._exit(ELASTIC_EXIT_CODE)


def maybe_hang(point: str):
    r = hit("hang", point=point)
    if r is not None:
        time.sleep(float(r.args.get("seconds", "3600")))


def maybe_corrupt(rank: int) -> bool:
    return hit("corrupt_shard", rank=rank) is not None


def maybe_nan_grad(step: int) -> bool:
    return hit("nan_grad", step=step) is not None
