"""Headline benchmark: Mrays/s + ms/frame on in/instance10000_pointlight at
1920x1080 with 8x8 = 64 samples per pixel (BASELINE.json configs[3], "c4"), on N
MI355X GPUs of one node.

One step = one full frame of the hot path (raytrace(), src/raytrace.cpp:213) over
the resident scene: every rank renders its interleaved 8-row bands of the frame with
the gfx950 kernels, then the float framebuffer is all-gathered over RCCL (xGMI) and
every rank reassembles the image (the north_star's framebuffer gather); with RCCL the
gather of frame i runs on a communication stream while frame i+1 renders. Total work
is fixed as N grows ("scaling": "strong").

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python bench.py --resolution 4096 --width 4096 --samples 16      # c5's frame
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

`python bench.py --gpus N` with N > 1 and no WORLD_SIZE in the environment launches
its own N ranks (one process per GPU, RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set) before
anything touches the GPU; rank 0 prints the one JSON line.

value     the reference's ray count over all ranks (camera + shadow + reflection rays, its
          intersect_first + intersect_any calls, src/raytrace.cpp:121-133) / wall time of K
          frames. A shadow ray whose light term is exactly zero is counted there but answered
          without a walk (the shadow cull); config.rays_traced_per_frame and
          config.Mrays_traced_per_s give the rays actually walked, config.shadow_rays_culled_per_frame
          the difference
roofline  the roofline kernel is the longest per-ray phase of this run's frame (the
          per-render lists phase, fixed work whatever a rank's share, is never picked;
          roofline_phase()): the closest hit k_primary_persist at c4. The walks are bound by
          instruction ISSUE, not by HBM (the 2.9 MB scene is cache-resident): achieved = the
          kernel's scalar- or vector-instruction count per launch (rocprofv3 SQ_INSTS_SALU /
          SQ_INSTS_VALU, committed under profiles/, tools/gpu/issue_pmc.sh) / its mean launch
          time measured live with HIP events on the launch stream, against the chip's issue
          peak (one SALU per CU per clock; one wave64 VALU per SIMD per two clocks; 256 CUs at
          2.4 GHz). The pipe with the higher fraction is the bound. The HBM fraction from the
          FETCH_SIZE/WRITE_SIZE passes is reported beside it; roofline_walks gives both walks'
          (closest hit and any hit) issue rooflines
frame     frame_sha256 of rank 0's reassembled frame, and frame_matches_n1 against the N = 1
          digest committed for this workload (profiles/frame_digests.json)
cpu_baseline  the reference itself (oracle/_ref, compiled from the unmodified sources)
          on a bounded sample of rows of the same frame, single thread, three disjoint
          row sets (value pooled, spread per set); cpu_baseline_all_cores the reference
          again on one host thread per core given to this job; cpu_baseline_port_all_cores
          the C restatement (oracle/liboracle.so, light list precomputed) on those cores
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import platform
import socket
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402

BASELINE_METRIC = "Mrays/sec + ms/frame, instance10000 1920×1080×64spp, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# issue peaks (MI355X_MICROARCH.md: 256 CUs, 4 SIMD-32 per CU, 2400 MHz max clock; a
# wave64 VALU instruction issues over 2 clocks on its SIMD; one scalar unit per CU)
N_CU, CLOCK_HZ = 256, 2.4e9
SALU_PEAK = N_CU * 1.0 * CLOCK_HZ / 1e9   # G wave-instructions/s
VALU_PEAK = N_CU * 4 * 0.5 * CLOCK_HZ / 1e9
BAND = 8
# the kernel each phase's time is dominated by on the timed path (the lists-on c4 frame;
# profiles/r*/final/pmc_c4/ks_kernel_stats.csv)
PHASE_KERNEL = {"primary": "k_primary_persist<unsigned int, 0, true>",
                "shadow": "k_shadow_persist<0>",
                "shade": "k_shade<false, true, 256, true>",
                "bounce": "k_bounce<false, true, unsigned int>",
                "megakernel": "render_kernel<false>"}
# phases whose work is fixed per render, not per ray (the camera-relative records and the
# tile lists): never the roofline kernel -- at a small rank share their launch latency can
# outlast a walk without saying anything about the walks
FIXED_PHASES = ("lists",)
DIGESTS = ROOT / "profiles" / "frame_digests.json"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--scene", default="instance10000")
    p.add_argument("--resolution", type=int, default=1080)
    p.add_argument("--width", type=int, default=0)
    p.add_argument("--samples", type=int, default=8, help="per axis: 8 -> 64 spp")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline budget per leg (0 = skip)")
    p.add_argument("--traffic-json", default=str(ROOT / "profiles" / "pmc_traffic.json"))
    p.add_argument("--issue-json", default=str(ROOT / "profiles" / "issue_counters.json"))
    p.add_argument("--algorithm", default="wavefront", choices=("wavefront", "megakernel", "wavefront_lane"))
    p.add_argument("--profile-rank", default="",
                   help="R/N: one process renders rank R's bands of an N-rank run, no gather (the counter "
                        "passes for the N-rank roofline, tools/gpu/issue_pmc.sh); its line is not a bench result")
    p.add_argument("--no-count-pass", action="store_true",
                   help="skip the untimed instrumented pass that gives SURVEY §8(d)'s algorithmic bytes")
    p.add_argument("--dry-run", action="store_true",
                   help="launch/rendezvous/report only, no GPU work (tests the N-rank launcher on CPU)")
    return p.parse_args()


# ---------------------------------------------------------------- rank launcher

def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int) -> int:
    """One process per GPU, started from this process before it touches the GPU (it
    never initialises HIP: `import torch` does not). Rank 0 prints the JSON line."""
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve()), *sys.argv[1:]], env=env))
    rc = 0
    try:
        while procs:
            for p in list(procs):
                code = p.poll()
                if code is None:
                    continue
                procs.remove(p)
                if code != 0:
                    rc = rc or code
                    for q in procs:  # a failed rank ends the job: stop the others
                        q.terminate()
            time.sleep(0.05)
    finally:
        for q in procs:
            q.kill()
    return rc


# ---------------------------------------------------------------- CPU baselines

def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def _timed_rows(run, H: int, budget_s: float, threads: int = 1, repeats: int = 1, min_rows: int = 1):
    """calibrate on the middle row, then time `repeats` disjoint sets of evenly spaced rows
    (set k offset by k / repeats of the spacing), each filling about budget_s / repeats of
    wall time on `threads` threads, with at least max(threads, min_rows) rows per set.
    Returns [(rows, rays, seconds)] per set."""
    t0 = time.perf_counter()
    run(np.array([H // 2], np.int32))
    t1 = time.perf_counter() - t0
    nrows = max(threads, min_rows, min(H // repeats, int(budget_s / repeats * threads / max(t1, 1e-6))))
    nrows = max(1, min(nrows, H // repeats))
    step = H / nrows
    sets = []
    for k in range(repeats):
        rows = np.unique(np.minimum(H - 1, (np.arange(nrows) * step + k * step / repeats).astype(np.int32)))
        t0 = time.perf_counter()
        rays = run(rows)
        sets.append((rows, rays, time.perf_counter() - t0))
    return sets


def _baseline_line(sets, W: int, H: int, spp_axis: int, threads: int, kind: str, what: str):
    """pooled Mrays/s over every timed set (the value), with the per-set spread"""
    rays = sum(r for _, r, _ in sets)
    el = sum(t for _, _, t in sets)
    nrows = sum(len(rows) for rows, _, _ in sets)
    samples = nrows * W * spp_axis * spp_axis
    per = [r / t / 1e6 for _, r, t in sets]
    return {
        "value": rays / el / 1e6,
        "unit": "Mrays/s",
        "cores": threads,
        "kind": kind,
        "repeats": [round(v, 4) for v in per],
        "min": min(per),
        "median": float(np.median(per)),
        "max": max(per),
        "cpu_model": cpu_model(),
        "sample": (f"{len(sets)} disjoint sets of evenly spaced rows ({nrows} rows in all) x {W} px x "
                   f"{spp_axis * spp_axis} spp of the same frame ({samples} camera samples, {rays} rays) in "
                   f"{el:.1f} s on {threads} thread(s) of {cpu_model()} ({what}); value = all sets pooled, "
                   f"repeats = each set's own rate; extrapolated full frame {el / samples * W * H * spp_axis ** 2:.0f} s"),
    }


def _reference(scene_file: Path, res: int):
    """the reference build (oracle/_ref/libyrtref.so) with the scene loaded, or None"""
    ref_so = ROOT / "oracle" / "_ref" / "libyrtref.so"
    if not ref_so.exists():
        return None
    lib = ctypes.CDLL(str(ref_so))
    lib.ref_read_scene.restype = ctypes.c_void_p
    lib.ref_read_scene.argtypes = [ctypes.c_char_p]
    lib.ref_image_size.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    lib.ref_render_rows_mt.restype = ctypes.c_longlong
    lib.ref_render_rows_mt.argtypes = [ctypes.c_void_p, ctypes.c_float, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    scn = lib.ref_read_scene(str(scene_file).encode())
    w, h = ctypes.c_int(), ctypes.c_int()
    lib.ref_image_size(scn, res, ctypes.byref(w), ctypes.byref(h))
    return lib, scn, w.value, h.value


def _host_cores() -> int:
    """the cores this job has: OMP_NUM_THREADS when the host sets it (16 per GPU on the GPU
    box), else every CPU"""
    return int(os.environ.get("OMP_NUM_THREADS") or 0) or (os.cpu_count() or 1)


def cpu_baseline(scene_file: Path, res: int, width: int, spp_axis: int, budget_s: float):
    """The reference's own code (oracle/_ref/libyrtref.so) on 1 thread: three disjoint sets
    of at least 16 evenly spaced rows of the same frame; the C restatement (1 thread) if the
    reference build did not travel. Test/baseline infrastructure only."""
    ref = None if width else _reference(scene_file, res)
    if ref is not None:
        lib, scn, W, H = ref

        def run(rows):
            out = np.zeros((len(rows), W, 4), np.float32)
            r = np.ascontiguousarray(rows, np.int32)
            return lib.ref_render_rows_mt(scn, 0.1, res, spp_axis, r.ctypes.data, len(r), out.ctypes.data, 1)
        kind, what = "reference", "the reference's eval_camera/shade, oracle/_ref"
    else:
        o = _oracle(scene_file, 1)
        W, H = o.image_size(res)
        W = width or W

        def run(rows):
            return o.render(res, spp_axis, rows=rows, width=width)[1]
        kind, what = "port", "oracle/oracle.c"
    sets = _timed_rows(run, H, budget_s, repeats=3, min_rows=16)
    return _baseline_line(sets, W, H, spp_axis, 1, kind, what)


def _oracle(scene_file: Path, threads: int):
    sys.path.insert(0, str(ROOT / "tests"))
    from helpers import Oracle, oracle_lib  # test infrastructure, baseline legs only

    lib = oracle_lib()
    lib.oracle_set_threads.restype = ctypes.c_int
    lib.oracle_set_threads.argtypes = [ctypes.c_int]
    lib.oracle_set_threads(threads)
    return Oracle(str(scene_file))


def cpu_baseline_all_cores(scene_file: Path, res: int, width: int, spp_axis: int, budget_s: float):
    """The reference itself on every core this job has (ref_render_rows_mt: one host thread
    per core, each running the reference's per-pixel loop body on the next row), three
    disjoint row sets. None when the reference build did not travel or the frame has an
    explicit width (the reference cannot express one)."""
    ref = None if width else _reference(scene_file, res)
    if ref is None:
        return None
    lib, scn, W, H = ref
    cores = _host_cores()

    def run(rows):
        out = np.zeros((len(rows), W, 4), np.float32)
        r = np.ascontiguousarray(rows, np.int32)
        return lib.ref_render_rows_mt(scn, 0.1, res, spp_axis, r.ctypes.data, len(r), out.ctypes.data, cores)
    sets = _timed_rows(run, H, budget_s, threads=cores, repeats=3)
    return _baseline_line(sets, W, H, spp_axis, cores, "reference",
                          "the reference's eval_camera/shade on one host thread per core, oracle/_ref")


def cpu_baseline_port_all_cores(scene_file: Path, res: int, width: int, spp_axis: int, budget_s: float):
    """The C restatement (oracle.c, OpenMP over rows) on every core this job has. Its light
    loop visits a precomputed light list instead of scanning all instances as shade() does
    (raytrace.cpp:121-126), so it is NOT the reference's throughput: a labelled third leg."""
    cores = _host_cores()
    o = _oracle(scene_file, cores)
    W, H = o.image_size(res)
    W = width or W

    def run(rows):
        return o.render(res, spp_axis, rows=rows, width=width)[1]
    sets = _timed_rows(run, H, budget_s, threads=cores, repeats=3)
    o.lib.oracle_set_threads(1)
    return _baseline_line(sets, W, H, spp_axis, cores, "port",
                          "oracle/oracle.c, OpenMP over rows, light list precomputed")


# ---------------------------------------------------------------- roofline

def algorithmic_bytes(st: dict, pixels: int) -> float:
    """SURVEY §8(d)'s fixed yardstick: the reference's traversal and shading work on its
    own AoS layout, in bytes"""
    return float(32 * st["box_tests"] + 56 * st["instance_entries"] + 52 * st["prim_tests"] +
                 216 * st["shaded_hits"] + 16 * st["texture_lookups"] + 16 * pixels)


def frame_digest(frame) -> str:
    """sha256 of a float32 RGBA frame's bytes in image order (host copy, untimed)"""
    import hashlib

    return hashlib.sha256(frame.detach().contiguous().cpu().numpy().tobytes()).hexdigest()


def load_counters(path: Path, key: str, identity: str):
    """the committed counter record for `key`, if it was collected from a library with
    this code identity: (record, None), else (None, why not)"""
    try:
        table = json.loads(Path(path).read_text())
    except (OSError, ValueError):
        return None, f"no counter file {path}"
    rec = table.get(key)
    if rec is None:
        return None, f"no committed counters for {key}"
    if rec.get("code_identity") != identity:
        return None, (f"committed counters for {key} come from another build (code identity "
                      f"{str(rec.get('code_identity'))[:12]}, timed library {identity[:12]})")
    return rec, None


def issue_roofline(issue_json: Path, key: str, kernel_ms: float, identity: str, key_n1: str = "",
                   share: float = 1.0):
    """achieved issue rate of the dominant kernel: its committed per-launch instruction
    counts / the live launch time -- only when the counters were collected from a library
    with the timed library's code identity. At N > 1 ranks without counters of that exact
    run, the single-GPU counts of the same frame are scaled by this rank's share of the
    frame's rays (the walks' instruction counts follow the rays they trace; the result
    says so). Returns (bound, pipes, record) or (None, None, why not)."""
    rec, why = load_counters(issue_json, key, identity)
    if rec is None and key_n1:
        rec1, why1 = load_counters(issue_json, key_n1, identity)
        if rec1 is not None:
            rec = dict(rec1)
            for c in ("SQ_INSTS_SALU", "SQ_INSTS_VALU"):
                rec[c] = rec[c] * share
            rec["source"] = f"{rec.get('source')} (n1 counts x this rank's ray share {share:.4f})"
    if rec is None:
        return None, None, why
    if kernel_ms <= 0:
        return None, None, "no launch time"
    s = kernel_ms / 1e3
    salu = rec["SQ_INSTS_SALU"] / s / 1e9
    valu = rec["SQ_INSTS_VALU"] / s / 1e9
    pipes = {"salu": {"achieved": salu, "peak": SALU_PEAK, "frac": salu / SALU_PEAK},
             "valu": {"achieved": valu, "peak": VALU_PEAK, "frac": valu / VALU_PEAK}}
    bound = max(pipes, key=lambda k: pipes[k]["frac"])
    return bound, pipes, rec


def roofline_phase(phases: dict, n1_cycles: dict | None = None) -> str:
    """the phase whose kernel the line's roofline describes, among this frame's per-ray phases
    ({phase: (ms, launches)}; never a fixed per-render phase, FIXED_PHASES): the one that
    dominates the same workload at N = 1 (its cycles per launch in the committed counters,
    n1_ranking(), times its launches), so that an N-rank line -- whose phases can be contended
    or latency-bound at a small share -- reports the kernel the N = 1 line does; without N = 1
    counters, the longest phase of this run"""
    per_ray = {k: v for k, v in phases.items() if k not in FIXED_PHASES and v[1] > 0}
    pool = per_ray or phases
    # (cycles per launch at N = 1 x this run's launches: a phase's launches per frame are the
    # workload's, whatever the rank count)
    ranked = {k: n1_cycles[k] * pool[k][1] for k in pool if n1_cycles and k in n1_cycles}
    if ranked:
        return max(ranked, key=ranked.get)
    return max(pool, key=lambda k: pool[k][0])


def n1_ranking(issue_json: Path, prefix: str, identity: str) -> dict:
    """{phase: GPU cycles per launch} of the workload at N = 1 from the committed counters
    (keys prefix + phase, prefix = scene-WxH-s<samples>-n1-<algorithm>-), only records of the
    timed library's code identity"""
    try:
        table = json.loads(Path(issue_json).read_text())
    except (OSError, ValueError):
        return {}
    out = {}
    for k, rec in table.items():
        if k.startswith(prefix) and rec.get("code_identity") == identity and rec.get("cycles"):
            out[k[len(prefix):]] = float(rec["cycles"])
    return out


def digest_key(scene: str, W: int, H: int, samples: int) -> str:
    return f"{scene}-{W}x{H}-s{samples}"


def frame_matches_n1(digest, key: str, path: Path = DIGESTS):
    """whether this frame's sha256 equals the committed N = 1 digest of the workload (None
    when there is no digest to compare: no frame, or no committed entry)"""
    if digest is None:
        return None
    try:
        want = json.loads(Path(path).read_text()).get(key)
    except (OSError, ValueError):
        return None
    return None if want is None else digest == want


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(launch_ranks(a.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")

    import torch
    import torch.distributed as dist

    backend = os.environ.get("YRT_BENCH_BACKEND", "nccl")  # nccl = RCCL over xGMI
    if a.dry_run:
        if world > 1:
            dist.init_process_group("gloo" if backend == "gloo" else backend)
            t = torch.tensor([float(rank)])
            dist.all_reduce(t)
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": world,
                              "rank_sum": world * (world - 1) / 2 if world > 1 else 0.0,
                              "checked_sum": float(t[0]) if world > 1 else 0.0}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return

    # rehearsal of the N-rank path on fewer GPUs (e.g. 2 ranks on one card with gloo):
    # YRT_BENCH_DEVICES=1 maps rank r to device r % 1; the driver's runs never set it
    ndev_override = int(os.environ.get("YRT_BENCH_DEVICES", "0"))
    if ndev_override > 0:
        local = local % ndev_override
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    import yocto_raytracing_amd as yrt
    from yocto_raytracing_amd import _native as yrt_native
    from yocto_raytracing_amd.codeid import code_identity

    scene_file = ROOT / "tests" / "golden" / "scenes" / f"{a.scene}.yrtscene"
    scn = yrt.load_scene(str(scene_file))
    yrt.build_bvh(scn)
    ds = scn.upload(local)

    from yocto_raytracing_amd.shard import BandLayout, gather_frame, render_params_band

    params = yrt.render_params(0.1, a.resolution, a.samples, width=a.width, algorithm=a.algorithm)
    W, H = ds.image_size(params)
    band_world, band_rank = world, rank
    if a.profile_rank:
        if world > 1:
            raise SystemExit("--profile-rank is a single-process mode")
        band_rank, band_world = (int(v) for v in a.profile_rank.split("/"))
        if not 0 <= band_rank < band_world:
            raise SystemExit(f"--profile-rank {a.profile_rank}: want R/N with 0 <= R < N")
    layout = BandLayout(H, band_world, BAND)
    band, local_rows = render_params_band(layout, band_rank)
    params.band, params.band_stride, params.band_offset = band
    params.tile_h = local_rows  # every rank renders the same padded count (rows past H read 0)
    # two frames in flight at N > 1 over RCCL: frame i's all_gather + reassembly run on a
    # communication stream while frame i+1 renders (double-buffered shards and frames)
    backend_name = dist.get_backend() if world > 1 else None
    overlap = world > 1 and (backend_name == "nccl" or os.environ.get("YRT_BENCH_OVERLAP") == "1")
    nbuf = 2 if overlap else 1
    shards = [torch.empty((local_rows, W, 4), dtype=torch.float32, device=dev) for _ in range(nbuf)]
    gathered = [torch.empty((world * local_rows, W, 4), dtype=torch.float32, device=dev) if world > 1 else None
                for _ in range(nbuf)]
    # (one rank: the shard is the frame in image order, no reassembly copy)
    identity = world == 1 and local_rows == H
    frames = [shards[i] if identity else torch.empty((H, W, 4), dtype=torch.float32, device=dev)
              for i in range(nbuf)]
    index = torch.as_tensor(layout.gather_index(), device=dev)
    stream = torch.cuda.current_stream(dev)
    comm = torch.cuda.Stream(dev) if overlap else None
    rendered = [torch.cuda.Event() for _ in range(nbuf)]
    gathered_ev = [None] * nbuf

    def step(i, timing=0):
        b = i % nbuf
        params.timing = timing
        if not overlap:
            ds.render_into(params, shards[b].data_ptr(), stream=stream.cuda_stream)
            if not a.profile_rank and not identity:
                gather_frame(shards[b], layout, index, gathered[b], frames[b])
            return b
        if gathered_ev[b] is not None:  # shards[b] is free once its previous gather has read it
            stream.wait_event(gathered_ev[b])
        ds.render_into(params, shards[b].data_ptr(), stream=stream.cuda_stream)
        rendered[b].record(stream)
        with torch.cuda.stream(comm):
            comm.wait_event(rendered[b])
            gather_frame(shards[b], layout, index, gathered[b], frames[b])
            gathered_ev[b] = torch.cuda.Event()
            gathered_ev[b].record(comm)
        return b

    for i in range(a.warmup):
        step(i)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(a.steps):
        # HIP events around every kernel launch, on the launch stream (library-side)
        step(i, timing=1 if i == 0 else 2)
    torch.cuda.synchronize(dev)  # every stream of the device: renders and gathers
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    st = ds.last_stats()
    phases = ds.last_timings()  # {phase: (ms over the K steps, launches)}
    try:
        identity = code_identity(yrt_native.LIB_PATH)
    except (OSError, ValueError, subprocess.CalledProcessError) as e:  # no binutils/bundler: no roofline
        identity = f"unavailable ({type(e).__name__})"
    dom = roofline_phase(phases, n1_ranking(Path(a.issue_json), f"{a.scene}-{W}x{H}-s{a.samples}-n1-{a.algorithm}-",
                                            identity))
    dom_ms = phases[dom][0] / a.steps  # per frame
    dom_launches = phases[dom][1] / a.steps
    render_ms = sum(v[0] for v in phases.values()) / a.steps

    # ---- end to end (untimed above): render + gather + the float frame to host memory
    # (what raytrace() returns, image4f) + the device tonemap of save_hdr_or_ldr's PNG
    e2e_frames = max(1, min(a.steps, 3))
    host_frame = torch.empty((H, W, 4), dtype=torch.float32, pin_memory=True) if rank == 0 else None
    ldr = torch.empty((H, W, 4), dtype=torch.uint8, device=dev) if rank == 0 else None
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    for i in range(e2e_frames):
        b = step(a.steps + i)
        if rank == 0:
            if overlap:
                stream.wait_event(gathered_ev[b])
            yrt.tonemap_device(frames[b].data_ptr(), H * W, ldr.data_ptr(), stream=stream.cuda_stream)
            host_frame.copy_(frames[b], non_blocking=True)
            torch.cuda.synchronize(dev)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    e2e_ms = (time.perf_counter() - t1) / e2e_frames * 1e3
    # rank 0's reassembled float frame (every step renders the same frame): an N-rank
    # line can be checked bit for bit against the N = 1 line
    frame_sha256 = None
    if rank == 0 and not a.profile_rank:
        frame_sha256 = frame_digest(frames[b])

    # SURVEY §8(d)'s algorithmic yardstick, from one instrumented (untimed) pass of this
    # rank's share: the reference's work counts x the reference layout's bytes per unit
    algo_bytes = 0.0
    if not a.no_count_pass:
        params.count_work, params.timing = 1, 0
        ds.render_into(params, shards[0].data_ptr(), stream=stream.cuda_stream)
        torch.cuda.synchronize(dev)
        algo_bytes = algorithmic_bytes(ds.last_stats(), local_rows * W)
        params.count_work = 0

    t = torch.tensor([elapsed, dom_ms, render_ms, e2e_ms], dtype=torch.float64, device=dev)
    rays = torch.tensor([st["rays"] * a.steps, st["camera_samples"] * a.steps, algo_bytes,
                         st["shadow_rays_culled"] * a.steps], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(rays, op=dist.ReduceOp.SUM)
    elapsed, dom_ms, render_ms, e2e_ms = (float(v) for v in t)
    total_rays, total_samples, total_algo_bytes = float(rays[0]), float(rays[1]), float(rays[2])
    total_culled = float(rays[3])

    if rank == 0:
        spp = a.samples * a.samples
        is_c4 = (a.scene, a.resolution, a.width, a.samples) == ("instance10000", 1080, 0, 8)
        metric = BASELINE_METRIC if is_c4 else f"Mrays/sec + ms/frame, {a.scene} {W}×{H}×{spp}spp, {world} MI355X"
        key = f"{a.scene}-{W}x{H}-s{a.samples}-n{band_world}-{a.algorithm}-{dom}"
        kernel_ms = dom_ms / dom_launches
        tr, _ = load_counters(Path(a.traffic_json), key, identity)
        traffic = tr.get("hbm_bytes_per_launch") if tr else None
        key_n1 = f"{a.scene}-{W}x{H}-s{a.samples}-n1-{a.algorithm}-{dom}"
        share = (st["rays"] * a.steps) / total_rays if total_rays else 1.0  # rank 0's share of the frame
        bound, pipes, rec = issue_roofline(Path(a.issue_json), key, kernel_ms, identity, key_n1, share)
        # both walks' issue rooflines (the closest hit and the any hit), whichever is longer
        walks = {}
        for ph in ("primary", "shadow"):
            if ph not in phases or not phases[ph][1]:
                continue
            ph_ms = phases[ph][0] / phases[ph][1]
            wb, wp, wr = issue_roofline(Path(a.issue_json), f"{a.scene}-{W}x{H}-s{a.samples}-n{band_world}-"
                                        f"{a.algorithm}-{ph}", ph_ms, identity,
                                        f"{a.scene}-{W}x{H}-s{a.samples}-n1-{a.algorithm}-{ph}", share)
            walks[ph] = ({"kernel": wr.get("kernel", PHASE_KERNEL.get(ph, ph)), "kernel_ms": ph_ms, "bound": wb,
                          "frac": wp[wb]["frac"], "salu_frac": wp["salu"]["frac"], "valu_frac": wp["valu"]["frac"]}
                         if wb else {"kernel": PHASE_KERNEL.get(ph, ph), "kernel_ms": ph_ms, "frac": None,
                                     "note": wr})
        if bound:
            roof = {"bound": "issue", "pipe": bound, "achieved": pipes[bound]["achieved"],
                    "peak": pipes[bound]["peak"], "unit": "G wave-instructions/s", "frac": pipes[bound]["frac"],
                    "traffic": traffic, "kernel": rec.get("kernel", PHASE_KERNEL.get(dom, dom)), "kernel_ms": kernel_ms,
                    "pipes": pipes, "counters": rec.get("source"),
                    "code_identity": identity,
                    "hbm": {"bytes_per_launch": traffic,
                            "achieved_GBs": traffic / (kernel_ms / 1e3) / 1e9 if traffic else None,
                            "peak_GBs": HBM_PEAK_GBS,
                            "frac": traffic / (kernel_ms / 1e3) / 1e9 / HBM_PEAK_GBS if traffic else None},
                    "note": ("SQ_INSTS_* per launch from the committed rocprofv3 counters of this exact "
                             "configuration / live HIP-event launch time; peak at the 2.4 GHz max clock")}
        else:
            roof = {"bound": "issue", "achieved": None, "peak": None, "unit": "G wave-instructions/s",
                    "frac": None, "traffic": traffic, "kernel": PHASE_KERNEL.get(dom, dom),
                    "kernel_ms": kernel_ms, "code_identity": identity,
                    "note": f"{rec} (tools/gpu/issue_pmc.sh collects them)"}
        line = {
            "metric": metric,
            "value": total_rays / elapsed / 1e6,
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"in/{a.scene} scene (reference input, .yrtscene); deterministic camera samples",
            "config": {"workload": f"{a.scene} {W}x{H} {a.samples}x{a.samples} spp, amb 0.1, one frame per step",
                       "scene": a.scene, "width": W, "height": H, "spp": spp,
                       "parallelism": (f"image bands x{world} + {backend_name} all_gather" +
                                       (" overlapped with the next frame" if overlap else "")) if world > 1
                       else "single GPU",
                       "rays_per_frame": total_rays / a.steps,
                       "rays_traced_per_frame": (total_rays - total_culled) / a.steps,
                       "shadow_rays_culled_per_frame": total_culled / a.steps,
                       "Mrays_traced_per_s": (total_rays - total_culled) / elapsed / 1e6,
                       "rays_note": ("value counts the reference's rays (intersect_first + intersect_any "
                                     "calls); rays_traced_per_frame excludes the shadow rays whose light "
                                     "term is exactly zero, answered without a walk (identical image)"),
                       "camera_samples_per_frame": total_samples / a.steps,
                       "gpu_ms_per_frame": render_ms,
                       "ms_per_frame_end_to_end": e2e_ms,
                       "end_to_end": "render + gather + float frame to pinned host memory + device tonemap",
                       "phase_ms_per_frame": {k: v[0] / a.steps for k, v in phases.items()},
                       "camera_Msamples_per_s": total_samples / elapsed / 1e6,
                       "algorithm": a.algorithm},
            "roofline": roof,
            "algorithmic_yardstick": None if a.no_count_pass else {
                "bytes_per_frame": total_algo_bytes,
                "GBs": total_algo_bytes / (elapsed / a.steps) / 1e9,
                "frac_of_hbm_peak": total_algo_bytes / (elapsed / a.steps) / 1e9 / HBM_PEAK_GBS / world,
                "note": ("SURVEY §8(d): 32 B per box test, 56 B per instance entry, 52 B per primitive test, "
                         "216 B per shaded hit, 16 B per texture lookup, 16 B per pixel, with the reference's "
                         "own work counts (one instrumented pass, untimed), over the timed ms/frame. The "
                         "reference's per-ray fetches of its AoS layout, not this path's traffic: the packet "
                         "walks fetch each record once per 64-ray wave from a cache-resident scene, so this "
                         "exceeds the HBM peak; roofline above is the bound that applies.")},
            "roofline_walks": walks,
            "frame_sha256": frame_sha256,
            "frame_matches_n1": frame_matches_n1(frame_sha256, digest_key(a.scene, W, H, a.samples)),
        }
        if a.profile_rank:  # a counter-collection run, not a bench result
            line["metric"] = f"profile of rank {a.profile_rank} (bands only, no gather): {metric}"
            line["config"]["parallelism"] = f"rank {a.profile_rank} of an image-band split, rendered alone"
        if world == 1 and a.cpu_seconds > 0 and not a.profile_rank:
            line["cpu_baseline"] = cpu_baseline(scene_file, a.resolution, a.width, a.samples, a.cpu_seconds)
            line["cpu_baseline_all_cores"] = cpu_baseline_all_cores(scene_file, a.resolution, a.width, a.samples,
                                                                    a.cpu_seconds)
            line["cpu_baseline_port_all_cores"] = cpu_baseline_port_all_cores(scene_file, a.resolution, a.width,
                                                                              a.samples, a.cpu_seconds)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
