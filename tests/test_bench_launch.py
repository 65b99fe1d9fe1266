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


def _bench_module():
    import importlib.util

    spec = importlib.util.spec_from_file_location("yrt_bench", ROOT / "bench.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_roofline_needs_counters_of_the_timed_build(tmp_path):
    """bench.py reports an issue roofline only from counters stamped with the timed
    library's code identity; counters of another build give achieved = null"""
    b = _bench_module()
    key = "instance10000-1920x1080-s8-n1-wavefront-shadow"
    rec = {"kernel": "k_shadow_persist<0>", "source": "profiles/rX", "SQ_INSTS_SALU": 5.0e9,
           "SQ_INSTS_VALU": 12.0e9, "code_identity": "a" * 64}
    f = tmp_path / "issue.json"
    f.write_text(json.dumps({key: rec}))
    bound, pipes, _ = b.issue_roofline(f, key, 14.0, "a" * 64)
    assert bound == "valu"
    assert pipes["valu"]["achieved"] == pytest.approx(12.0e9 / 14e-3 / 1e9)
    bound, pipes, why = b.issue_roofline(f, key, 14.0, "b" * 64)
    assert bound is None and pipes is None and "another build" in why
    # an unstamped record (collected before stamps existed) is never used
    f.write_text(json.dumps({key: {k: v for k, v in rec.items() if k != "code_identity"}}))
    assert b.issue_roofline(f, key, 14.0, "a" * 64)[0] is None
    # rank share scaling from the n1 record, same identity rule
    f.write_text(json.dumps({key: rec}))
    key2 = key.replace("-n1-", "-n2-")
    bound, pipes, r2 = b.issue_roofline(f, key2, 7.0, "a" * 64, key_n1=key, share=0.5)
    assert bound == "valu" and r2["SQ_INSTS_VALU"] == pytest.approx(6.0e9)
    assert b.issue_roofline(f, key2, 7.0, "c" * 64, key_n1=key, share=0.5)[0] is None


def test_code_identity_of_the_built_library():
    import importlib.util

    spec = importlib.util.spec_from_file_location("yrt_codeid", ROOT / "yocto_raytracing_amd" / "codeid.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    lib = ROOT / "yocto_raytracing_amd" / "libyrt.so"
    ident = mod.code_identity(lib)
    assert len(ident) == 64 and ident == mod.code_identity(lib)
    assert len(mod.code_objects(lib)) == 3  # render.hip, wavefront.hip, bvh_gpu.hip
