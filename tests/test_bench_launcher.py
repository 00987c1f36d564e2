"""bench.py's own rank launcher (the driver runs `python bench.py --gpus N`):
N fresh rank processes, one JSON line from rank 0, n_gpus = the world size the
collective saw and an all-gather head-count of every rank.  Rehearsed here
with --dry-run (gloo on CPU, no GPU, no kernel)."""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("world", [2, 3])
def test_bench_launches_ranks_itself(world):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    out = subprocess.run(
        [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--dry-run",
         "--steps", "3", "--warmup", "1", "--batch", "64"],
        capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == world
    assert res["ranks_seen"] == world
    assert res["dry_run"] is True
    assert res["steps"] == 3 and res["warmup"] == 3 - 2
    assert res["value"] > 0


def test_bench_single_rank_no_launcher():
    """--gpus 1 runs in-process (no launcher) and still reports one rank."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE")}
    env["MASTER_PORT"] = "29533"
    out = subprocess.run(
        [sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run", "--steps", "2",
         "--warmup", "0", "--batch", "8"],
        capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    res = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
    assert res["n_gpus"] == 1 and res["ranks_seen"] == 1
