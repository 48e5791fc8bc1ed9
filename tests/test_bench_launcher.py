"""bench.py's launcher contract: ``--gpus N`` without an
outer launcher spawns N ranks from a parent that never touches the GPU, and
the JSON line reports how many ranks actually joined (``config.ranks_seen``).
Rehearsed on the CPU with gloo (``--dry-run``)."""
import json
import os
import subprocess
import sys

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
