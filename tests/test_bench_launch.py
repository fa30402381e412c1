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


def test_spawn_parent_never_initialises_hip():
    """The self-spawning parent never calls into torch.cuda (device_count() can initialise HIP
    through hipGetDeviceCount): with every torch.cuda entry point replaced by one that raises,
    spawn_ranks still starts and reaps its (dry) ranks."""
    code = """
import sys, torch
sys.path.insert(0, %r)
def boom(*a, **k):
    raise AssertionError("torch.cuda touched in the parent")
for name in ("device_count", "is_available", "init", "set_device", "current_device",
             "synchronize", "get_device_properties"):
    setattr(torch.cuda, name, boom)
torch._C._cuda_getDeviceCount = boom
import bench
sys.exit(bench.main(["--gpus", "2", "--dry-launch"]))
""" % ROOT
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr
    assert sorted(json.loads(l)["rank"] for l in r.stdout.strip().splitlines()) == [0, 1]


def test_spawn_stops_the_other_ranks_when_one_fails(tmp_path):
    """A rank that fails makes spawn_ranks terminate the rest (instead of waiting for a
    collective's timeout) and return non-zero; an overall time limit stops hung ranks."""
    import time
    script = tmp_path / "rank.py"
    script.write_text("import os, sys, time\\n"
                      "r = int(os.environ['RANK'])\\n"
                      "if r == 1: sys.exit(3)\\n"
                      "time.sleep(600)\\n")
    orig = bench.os.path.abspath
    bench.os.path.abspath = lambda p: str(script) if p == bench.__file__ else orig(p)
    try:
        t0 = time.monotonic()
        assert bench.spawn_ranks([], 3, True) != 0
        assert time.monotonic() - t0 < 60
        script.write_text("import time\\ntime.sleep(600)\\n")
        t0 = time.monotonic()
        assert bench.spawn_ranks([], 2, True, timeout_s=2) != 0
        assert time.monotonic() - t0 < 60
    finally:
        bench.os.path.abspath = orig


def test_check_world_counts_this_nodes_ranks(monkeypatch):
    """check_world compares the ranks of this node (LOCAL_WORLD_SIZE) with its GPUs, so a
    multi-node torchrun (WORLD_SIZE 16 over 2 x 8 GPUs) passes on every rank, while more local
    ranks than GPUs, or a local rank past the last GPU, fail."""
    monkeypatch.setattr(bench.torch.cuda, "device_count", lambda: 8)
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    assert bench.check_world(16, 7)
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "9")
    assert not bench.check_world(16, 0)
    monkeypatch.delenv("LOCAL_WORLD_SIZE")
    assert bench.check_world(8, 3)
    assert not bench.check_world(9, 3)
    assert not bench.check_world(4, 8)
