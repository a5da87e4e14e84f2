"""bench.py's rank plumbing on CPU (no GPU): `bench.py --gpus N` started without a launcher runs
N ranks itself (torch.distributed.run, 127.0.0.1), and the JSON line's n_gpus is the world size the
ranks' process group saw; a --gpus that disagrees with a launcher's WORLD_SIZE fails.  --dry-run
exercises launch, frame sharding, the sum-reduce (gloo) and the max-over-ranks timing without
rendering (the render itself is covered by the GPU suite)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["PT_BENCH_BACKEND"] = "gloo"
    return env


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_n_spawns_n_ranks(n):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--dry-run", "--steps", "1",
                        "--spp", "16", "--width", "8", "--height", "8"], env=_env(), capture_output=True, text=True,
                       timeout=240, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    out = lines[0]
    assert out["n_gpus"] == n and out["config"]["ranks"] == n
    assert out["config"]["frames_reduced"] == 16.0  # every rank's frame share went through the reduce


def test_gpus_must_match_launcher_world_size():
    env = _env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run", "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=120, cwd="/tmp")
    assert r.returncode != 0 and "n_gpus must be the ranks that render" in r.stderr
