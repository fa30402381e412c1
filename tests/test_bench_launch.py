"""bench.py's launcher logic (CPU): ``--gpus N`` either agrees with the launcher's WORLD_SIZE,
starts N rank processes itself, or fails -- it never times a different GPU count silently."""
import json
import os
import subprocess
import sys

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_launch_plan():
    assert bench.launch_plan(1, {}) == ("run", 1)
    assert bench.launch_plan(4, {}) == ("spawn", 4)
    assert bench.launch_plan(2, {"WORLD_SIZE": "2"}) == ("run", 2)
    assert bench.launch_plan(8, {"WORLD_SIZE": "8"}) == ("run", 8)
    assert bench.launch_plan(2, {"WORLD_SIZE": "1"})[0] == "error"
    assert bench.launch_plan(1, {"WORLD_SIZE": "8"})[0] == "error"
    assert bench.launch_plan(0, {})[0] == "error"


def _run(args, env_extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                          capture_output=True, text=True, timeout=300)


def test_mismatch_exits_nonzero():
    r = _run(["--gpus", "2", "--dry-launch"], {"WORLD_SIZE": "1"})
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr
    r = _run(["--gpus", "1", "--dry-launch"], {"WORLD_SIZE": "4"})
    assert r.returncode != 0


def test_spawned_world_size_equals_gpus():
    r = _run(["--gpus", "3", "--dry-launch"], {})
    assert r.returncode == 0, r.stderr
    lines = [json.loads(l) for l in r.stdout.strip().splitlines()]
    assert sorted(d["rank"] for d in lines) == [0, 1, 2]
    assert all(d["world_size"] == 3 and d["local_rank"] == d["rank"] for d in lines)
