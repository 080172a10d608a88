"""bench.py's launch contract (no GPU): --gpus N either matches the launcher's WORLD_SIZE, or bench.py
starts torch.distributed.run with N ranks itself; a mismatch exits non-zero instead of silently
running N = 1 and reporting n_gpus 1."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(kw)
    return env


def test_launch_plan():
    assert bench.launch_plan(1, {}) == "run"
    assert bench.launch_plan(8, {}) == "spawn"
    assert bench.launch_plan(8, {"WORLD_SIZE": "8"}) == "run"
    assert bench.launch_plan(2, {"WORLD_SIZE": "1"}) == "mismatch"
    assert bench.launch_plan(1, {"WORLD_SIZE": "4"}) == "mismatch"
    assert bench.launch_plan(0, {}) == "mismatch"
    cmd = bench.spawn_command(["--gpus", "4", "--steps", "3"], 4, 29500)
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=4" in cmd
    assert "--master-addr=127.0.0.1" in cmd and cmd[-4:] == ["--gpus", "4", "--steps", "3"]


def test_mismatch_exits_nonzero():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=_env(WORLD_SIZE="1"),
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 2 and "WORLD_SIZE=1" in p.stderr
    assert '"n_gpus"' not in p.stdout


def test_gpus_spawns_one_rank_per_gpu():
    """--gpus 2 outside a launcher: two ranks, each with WORLD_SIZE = 2 (QEH_BENCH_LAUNCH_PROBE stops each
    rank before any GPU work and prints what it was started with)."""
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"],
                       env=_env(QEH_BENCH_LAUNCH_PROBE="1"), capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    seen = sorted((d["rank"], d["world"], d["gpus"]) for d in
                  (json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")))
    assert seen == [(0, 2, 2), (1, 2, 2)]
