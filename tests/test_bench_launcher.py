"""bench.py's launcher contract: ``--gpus N`` without an
outer launcher spawns N ranks from a parent that never touches the GPU, and
the JSON line reports how many ranks actually joined (``config.ranks_seen``).
Rehearsed on the CPU with gloo (``--dry-run``)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, timeout=180):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.pop("LOCAL_RANK", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    return p


def _json(stdout):
    lines = [l for l in stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


def test_spawn_two_ranks_dry():
    p = _run(["--gpus", "2", "--dry-run", "--steps", "1", "--warmup", "0"])
    assert p.returncode == 0, p.stderr[-2000:]
    out = _json(p.stdout)
    assert out["n_gpus"] == 2
    assert out["config"]["ranks_seen"] == 2
    assert out["config"]["launcher"] == "bench.py-spawn"


def test_single_rank_dry():
    p = _run(["--dry-run", "--steps", "1", "--warmup", "0"])
    assert p.returncode == 0, p.stderr[-2000:]
    out = _json(p.stdout)
    assert out["n_gpus"] == 1 and out["config"]["ranks_seen"] == 1


def test_refuses_more_gpus_than_visible():
    # no GPU in this container (and at most 8 on a node): asking for 64 must fail, not measure fewer
    p = _run(["--gpus", "64", "--steps", "1", "--warmup", "0"])
    assert p.returncode != 0
    assert "refusing" in p.stderr


def test_graph_steps_default_and_explicit():
    """Steps per captured graph: 4 on one rank / 2 multi-rank when they divide
    the timed steps, an explicit K must divide them."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("pbx_bench", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    assert b.graph_steps_for(20, 5, -1) == 4
    assert b.graph_steps_for(200, 50, -1, world=1) == 4
    assert b.graph_steps_for(20, 5, -1, world=8) == 2
    assert b.graph_steps_for(30, 5, -1) == 2
    assert b.graph_steps_for(21, 5, -1) == 1
    assert b.graph_steps_for(48, 20, 3) == 3
    with pytest.raises(SystemExit):
        b.graph_steps_for(20, 5, 3)


def test_push_run_scratch_forms(monkeypatch):
    """The fused push's straddling-run scratch: int64 per-unique arrival
    counters (one launch, default) or int32 per-wave owners (PBX_PUSH_FINISH=1)."""
    import torch

    from paddlebox_amd.ps.sparse_engine import _push_run_scratch

    monkeypatch.setenv("PBX_PUSH_FINISH", "1")
    t = _push_run_scratch(1000, "cpu")
    assert t.dtype == torch.int32 and t.numel() == (1000 + 63) // 64 + 1
    monkeypatch.delenv("PBX_PUSH_FINISH", raising=False)
    t = _push_run_scratch(1000, "cpu")
    assert t.dtype == torch.int64 and t.numel() == 1000 and int(t.abs().sum()) == 0
