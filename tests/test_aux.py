"""Auxiliary subsystems: fault injection, watchdog, chrome-trace export."""
import json
import threading
import time

import pytest

from paddlebox_amd.utils import fault
from paddlebox_amd.utils.timer import StageTimers
from paddlebox_amd.utils.watchdog import Watchdog


def test_fault_rules_parse_and_count():
    fault.configure("read_fail@file=part-1,times=2;kill_rank@rank=3,pass=2;nan_grad@step=5")
    with pytest.raises(fault.InjectedFault):
        fault.maybe_fail_read("/data/part-1.txt")
    with pytest.raises(fault.InjectedFault):
        fault.maybe_fail_read("/data/part-1.txt")
    fault.maybe_fail_read("/data/part-1.txt")  # third open succeeds (times=2)
    fault.maybe_fail_read("/data/part-2.txt")
    assert fault.hit("kill_rank", rank=3, **{"pass": 1}) is None
    assert fault.hit("kill_rank", rank=3, **{"pass": 2}) is not None
    assert fault.maybe_nan_grad(5) and not fault.maybe_nan_grad(4)
    fault.configure("")
    assert fault.hit("read_fail", file="x") is None


def test_watchdog_fires_and_dumps(tmp_path):
    fired = []
    wd = Watchdog(timeout_s=0.3, rank=7, dump_dir=str(tmp_path), on_timeout=fired.append, poll_s=0.05)
    try:
        with wd.guard("fast"):
            time.sleep(0.05)
        time.sleep(0.4)
        assert fired == []  # disarmed in time
        wd.arm("allreduce")
        deadline = time.time() + 5
        while not fired and time.time() < deadline:
            time.sleep(0.05)
        assert fired == ["allreduce"]
        txt = (tmp_path / "watchdog_rank7.txt").read_text()
        assert "allreduce" in txt and "Thread" in txt
    finally:
        wd.stop()


def test_watchdog_with_injected_hang(tmp_path):
    fault.configure("hang@point=pull,seconds=1.0")
    fired = []
    wd = Watchdog(timeout_s=0.3, rank=0, dump_dir=str(tmp_path), on_timeout=fired.append, poll_s=0.05)
    try:
        with wd.guard("pull"):
            fault.maybe_hang("pull")
        assert fired == ["pull"]
    finally:
        wd.stop()
        fault.configure("")


def test_chrome_trace_export(tmp_path):
    t = StageTimers(device=None, trace=True, rank=2)
    for _ in range(3):
        with t.span("pull"):
            time.sleep(0.002)
        with t.span("push"):
            pass
    p = t.export_chrome_trace(str(tmp_path / "trace.json"))
    d = json.load(open(p))
    ev = d["traceEvents"]
    assert len(ev) == 6 and {e["name"] for e in ev} == {"pull", "push"}
    assert all(e["ph"] == "X" and e["pid"] == 2 and e["dur"] >= 0 for e in ev)
    pulls = [e for e in ev if e["name"] == "pull"]
    assert pulls[0]["dur"] >= 1500  # us
    assert pulls[1]["ts"] > pulls[0]["ts"]
