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


def test_roofline_phase_is_a_per_ray_phase():
    """the roofline kernel of an N-rank line is the longest per-ray phase, never the per-render
    lists phase: the one-GPU N = 2 rehearsal of round 5 (two ranks contending for one card)
    timed lists at 76.7 ms and printed a roofline frac of 0.0007 for it"""
    b = _bench_module()
    rehearsal = {"primary": (9.1, 1), "shadow": (8.4, 1), "shade": (1.8, 1), "lists": (76.7, 4)}
    assert b.roofline_phase(rehearsal) == "primary"
    assert b.roofline_phase({"primary": (1.5, 1), "shadow": (1.6, 1), "lists": (0.1, 4)}) == "shadow"
    # a phase with no launch is never picked; with nothing but fixed phases, the longest
    assert b.roofline_phase({"primary": (0.0, 0), "megakernel": (3.0, 1), "lists": (9.0, 1)}) == "megakernel"
    assert b.roofline_phase({"lists": (0.2, 2)}) == "lists"
    # with the N = 1 counters of the workload, their ranking decides: the round-6 N = 2
    # rehearsal timed shadow 7.58 / primary 6.55 ms (two ranks on one card), N = 1 ranks the
    # closest hit first (9.28 vs 8.38 ms per launch)
    contended = {"primary": (6.55, 3), "shadow": (7.58, 3), "shade": (3.12, 3), "lists": (3.81, 9)}
    n1 = {"primary": 2.23e7, "shadow": 2.01e7, "shade": 4.2e6, "lists": 1.8e5}
    assert b.roofline_phase(contended) == "shadow"
    assert b.roofline_phase(contended, n1) == "primary"
    assert b.roofline_phase(contended, {"bounce": 1.0}) == "shadow"  # no N = 1 record of these phases


def test_n1_ranking_reads_only_the_timed_build(tmp_path):
    b = _bench_module()
    f = tmp_path / "issue.json"
    pre = "instance10000-1920x1080-s8-n1-wavefront-"
    f.write_text(json.dumps({pre + "primary": {"cycles": 2.2e7, "code_identity": "a" * 64},
                             pre + "shadow": {"cycles": 2.0e7, "code_identity": "a" * 64},
                             pre + "shade": {"cycles": 4.0e6, "code_identity": "b" * 64},
                             "instance10000-1920x1080-s8-n2-wavefront-primary": {"cycles": 1.1e7,
                                                                                 "code_identity": "a" * 64}}))
    assert b.n1_ranking(f, pre, "a" * 64) == {"primary": 2.2e7, "shadow": 2.0e7}
    assert b.n1_ranking(tmp_path / "missing.json", pre, "a" * 64) == {}


def test_frame_matches_n1(tmp_path):
    b = _bench_module()
    f = tmp_path / "digests.json"
    key = b.digest_key("instance10000", 1920, 1080, 8)
    assert key == "instance10000-1920x1080-s8"
    f.write_text(json.dumps({key: "ab" * 32}))
    assert b.frame_matches_n1("ab" * 32, key, f) is True
    assert b.frame_matches_n1("cd" * 32, key, f) is False
    assert b.frame_matches_n1("ab" * 32, "other-1x1-s1", f) is None
    assert b.frame_matches_n1(None, key, f) is None
    # the committed table holds the c4 digest of every round since round 2
    assert b.frame_matches_n1("391c90ce91616fe38fd0fd2781a1c9f3d2ca41ebe9011a9f3740217f7760fc89", key) is True
