"""bench.py's own N-rank launcher on CPU: `python bench.py --gpus N` with no WORLD_SIZE
starts N processes (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set, before anything touches a
GPU); the ranks rendezvous (gloo here, RCCL on the GPU node) and rank 0 alone prints
the one JSON line. --dry-run stops before GPU work."""
import json
import os
import subprocess
import sys

import pytest

from helpers import ROOT


@pytest.mark.parametrize("n", [2, 3])
def test_bench_launches_its_own_ranks(n):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["YRT_BENCH_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", str(n), "--dry-run"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]  # gloo logs its connects too
    assert len(lines) == 1, r.stdout  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == n
    assert out["checked_sum"] == out["rank_sum"] == n * (n - 1) / 2


def test_bench_rank_failure_fails_the_job():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["YRT_BENCH_BACKEND"] = "no-such-backend"
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode != 0
