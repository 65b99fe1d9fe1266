"""Headline benchmark: Mrays/s + ms/frame on in/instance10000_pointlight at
1920x1080 with 8x8 = 64 samples per pixel (BASELINE.json configs[3], "c4"), on N
MI355X GPUs of one node.

One step = one full frame of the hot path (raytrace(), src/raytrace.cpp:213) over
the resident scene, end to end: every rank renders its interleaved 8-row bands of
the frame with the gfx950 kernel, then the float framebuffer is all-gathered over
RCCL (xGMI) and every rank reassembles the image (the north_star's framebuffer gather);
with RCCL the gather of frame i runs on a communication stream while frame i+1 renders.
Total work is fixed as N grows ("scaling": "strong").

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

value   = all rays traced by all ranks (camera + shadow + reflection, the
          reference's intersect_first + intersect_any calls) / wall time of K frames
roofline: the render kernel's ALGORITHMIC bytes per launch (SURVEY §8d cost model x
          the work counters of an instrumented, untimed pass) / its mean launch time
          measured with HIP events on the launch stream, against 8 TB/s HBM
cpu_baseline: the reference itself (oracle/_ref, compiled from the unmodified
          sources) on a bounded sample of rows of the same frame, single thread
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import platform
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# algorithmic bytes of the reference's traversal on its own AoS layout
BYTES_BOX, BYTES_INST, BYTES_PRIM, BYTES_HIT, BYTES_TEX, BYTES_PIXEL = 32, 56, 52, 216, 16, 16
BAND = 8


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--scene", default="instance10000")
    p.add_argument("--resolution", type=int, default=1080)
    p.add_argument("--width", type=int, default=0)
    p.add_argument("--samples", type=int, default=8, help="per axis: 8 -> 64 spp")
    p.add_argument("--cpu-seconds", type=float, default=15.0, help="CPU baseline budget (0 = skip)")
    p.add_argument("--traffic-json", default=str(ROOT / "profiles" / "pmc_traffic.json"))
    p.add_argument("--algorithm", default="wavefront", choices=("wavefront", "megakernel", "wavefront_lane"))
    return p.parse_args()


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_baseline(scene_file: Path, res: int, spp_axis: int, budget_s: float):
    """The reference's own code (oracle/_ref/libyrtref.so) on rows of the same frame.
    Falls back to the C restatement (oracle/liboracle.so, 1 thread) if the reference
    build did not travel. Test/baseline infrastructure only."""
    ref_so = ROOT / "oracle" / "_ref" / "libyrtref.so"
    if ref_so.exists():
        lib = ctypes.CDLL(str(ref_so))
        lib.ref_read_scene.restype = ctypes.c_void_p
        lib.ref_read_scene.argtypes = [ctypes.c_char_p]
        lib.ref_image_size.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        lib.ref_render_rows.restype = ctypes.c_longlong
        lib.ref_render_rows.argtypes = [ctypes.c_void_p, ctypes.c_float, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
        scn = lib.ref_read_scene(str(scene_file).encode())
        w, h = ctypes.c_int(), ctypes.c_int()
        lib.ref_image_size(scn, res, ctypes.byref(w), ctypes.byref(h))
        W, H = w.value, h.value

        def run(rows):
            out = np.zeros((len(rows), W, 4), np.float32)
            r = np.ascontiguousarray(rows, np.int32)
            return lib.ref_render_rows(scn, 0.1, res, spp_axis, r.ctypes.data, len(r), out.ctypes.data)
        kind = "reference"
    else:
        sys.path.insert(0, str(ROOT / "tests"))
        from helpers import Oracle  # test infrastructure, baseline leg only

        os.environ["OMP_NUM_THREADS"] = "1"
        o = Oracle(str(scene_file))
        W, H = o.image_size(res)

        def run(rows):
            return o.render(res, spp_axis, rows=rows)[1]
        kind = "port"
    # calibrate on the middle row, then sample evenly spaced rows to fill the budget
    t0 = time.perf_counter()
    rays = run([H // 2])
    t1 = time.perf_counter() - t0
    nrows = max(1, min(H, int(budget_s / max(t1, 1e-6))))
    rows = np.linspace(0, H - 1, nrows).astype(np.int32)
    t0 = time.perf_counter()
    rays = run(rows)
    el = time.perf_counter() - t0
    samples = len(rows) * W * spp_axis * spp_axis
    return {
        "value": rays / el / 1e6,
        "unit": "Mrays/s",
        "cores": 1,
        "kind": kind,
        "sample": (f"{len(rows)} evenly spaced rows x {W} px x {spp_axis * spp_axis} spp of the same "
                   f"frame ({samples} camera samples, {rays} rays) in {el:.1f} s on 1 thread of "
                   f"{cpu_model()}; extrapolated full frame {el / samples * W * H * spp_axis ** 2:.0f} s"),
    }


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the N-rank path on fewer GPUs (e.g. 2 ranks on one card with gloo):
    # YRT_BENCH_DEVICES=1 maps rank r to device r % 1; the driver's runs never set it
    ndev_override = int(os.environ.get("YRT_BENCH_DEVICES", "0"))
    if ndev_override > 0:
        local = local % ndev_override
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            raise SystemExit("--gpus N>1 needs one process per GPU: launch with torch.distributed.run")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        backend = os.environ.get("YRT_BENCH_BACKEND", "nccl")  # nccl = RCCL over xGMI
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    import yocto_raytracing_amd as yrt

    scene_file = ROOT / "tests" / "golden" / "scenes" / f"{a.scene}.yrtscene"
    scn = yrt.load_scene(str(scene_file))
    yrt.build_bvh(scn)
    ds = scn.upload(local)

    from yocto_raytracing_amd.shard import BandLayout, gather_frame, render_params_band

    params = yrt.render_params(0.1, a.resolution, a.samples, width=a.width, algorithm=a.algorithm)
    W, H = ds.image_size(params)
    layout = BandLayout(H, world, BAND)
    band, local_rows = render_params_band(layout, rank)
    params.band, params.band_stride, params.band_offset = band
    params.tile_h = local_rows  # every rank renders the same padded count (rows past H read 0)
    # two frames in flight at N > 1 over RCCL: frame i's all_gather + reassembly run on a
    # communication stream while frame i+1 renders (double-buffered shards and frames)
    overlap = world > 1 and (dist.get_backend() == "nccl" or os.environ.get("YRT_BENCH_OVERLAP") == "1")
    nbuf = 2 if overlap else 1
    shards = [torch.empty((local_rows, W, 4), dtype=torch.float32, device=dev) for _ in range(nbuf)]
    gathered = [torch.empty((world * local_rows, W, 4), dtype=torch.float32, device=dev) if world > 1 else None
                for _ in range(nbuf)]
    frames = [torch.empty((H, W, 4), dtype=torch.float32, device=dev) for _ in range(nbuf)]
    shard = shards[0]
    index = torch.as_tensor(layout.gather_index(), device=dev)
    stream = torch.cuda.current_stream(dev)
    comm = torch.cuda.Stream(dev) if overlap else None
    rendered = [torch.cuda.Event() for _ in range(nbuf)]
    gathered_ev = [None] * nbuf

    # untimed instrumented pass: algorithmic work counts for the roofline bytes
    pc = yrt.render_params(0.1, a.resolution, a.samples, width=a.width, band=band, count_work=True,
                           algorithm=a.algorithm)
    pc.tile_h = local_rows
    ds.render_into(pc, shard.data_ptr(), stream=stream.cuda_stream)
    work = ds.last_stats()
    # per kernel phase: SURVEY §8d cost model on the phase's own traversal counts, plus
    # the wavefront buffers the phase reads/writes (shadow: 16 B hit point in, 1 B out)
    sh = {k: work[f"shadow_{k}"] for k in ("box_tests", "instance_entries", "prim_tests", "rays")}
    alg = {
        "shadow": sh["box_tests"] * BYTES_BOX + sh["instance_entries"] * BYTES_INST +
                  sh["prim_tests"] * BYTES_PRIM + sh["rays"] * 17,
        "primary": (work["box_tests"] - sh["box_tests"]) * BYTES_BOX +
                   (work["instance_entries"] - sh["instance_entries"]) * BYTES_INST +
                   (work["prim_tests"] - sh["prim_tests"]) * BYTES_PRIM + work["camera_samples"] * 36,
        "megakernel": work["box_tests"] * BYTES_BOX + work["instance_entries"] * BYTES_INST +
                      work["prim_tests"] * BYTES_PRIM + work["shaded_hits"] * BYTES_HIT +
                      work["texture_lookups"] * BYTES_TEX + local_rows * W * BYTES_PIXEL,
    }
    # rocprof names of the timed (COUNT=false) kernels: <COUNT, PACKET, stack entry>
    targs = {"wavefront": "<false, true, unsigned int>", "wavefront_lane": "<false, false, unsigned short>"}
    kernel_names = {"megakernel": "render_kernel<false>"}
    for ph in ("primary", "shadow", "bounce"):
        kernel_names[ph] = f"k_{ph}{targs.get(a.algorithm, '')}"
    if a.algorithm == "wavefront":  # the timed shadow kernel walks the 4-wide collapse
        kernel_names["shadow"] = "k_shadow<false, true, unsigned int, true>"

    def step(i, timing=0):
        b = i % nbuf
        params.timing = timing
        if not overlap:
            ds.render_into(params, shards[b].data_ptr(), stream=stream.cuda_stream)
            gather_frame(shards[b], layout, index, gathered[b], frames[b])
            return
        if gathered_ev[b] is not None:  # shards[b] is free once its previous gather has read it
            stream.wait_event(gathered_ev[b])
        ds.render_into(params, shards[b].data_ptr(), stream=stream.cuda_stream)
        rendered[b].record(stream)
        with torch.cuda.stream(comm):
            comm.wait_event(rendered[b])
            gather_frame(shards[b], layout, index, gathered[b], frames[b])
            gathered_ev[b] = torch.cuda.Event()
            gathered_ev[b].record(comm)

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
    dom = max(phases, key=lambda k: phases[k][0])
    dom_ms = phases[dom][0] / a.steps  # per frame; one launch per frame at N=1 (one chunk)
    dom_launches = phases[dom][1] / a.steps
    render_ms = sum(v[0] for v in phases.values()) / a.steps

    t = torch.tensor([elapsed, dom_ms, render_ms], dtype=torch.float64, device=dev)
    rays = torch.tensor([st["rays"] * a.steps, st["camera_samples"] * a.steps], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(rays, op=dist.ReduceOp.SUM)
    elapsed, dom_ms, render_ms = float(t[0]), float(t[1]), float(t[2])
    total_rays, total_samples = float(rays[0]), float(rays[1])
    alg_bytes = alg.get(dom)

    if rank == 0:
        # per launch: algorithmic bytes of one frame's launch(es) / their mean duration
        achieved = (alg_bytes / dom_launches) / (dom_ms / dom_launches / 1e3) / 1e9 if alg_bytes else None
        traffic = None
        tj = Path(a.traffic_json)
        if tj.exists():
            try:
                tr = json.loads(tj.read_text())
                key = f"{a.scene}-r{a.resolution}-s{a.samples}-n{world}-{a.algorithm}-{dom}"
                traffic = tr.get(key, {}).get("hbm_bytes_per_launch")
            except (OSError, ValueError):
                traffic = None
        line = {
            "metric": "Mrays/sec + ms/frame, instance10000 1920x1080x64spp, 1/2/4/8 MI355X",
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
            "data": "in/instance10000_pointlight scene (reference input, .yrtscene); deterministic camera samples",
            "config": {"workload": f"{a.scene} {W}x{H} {a.samples}x{a.samples} spp, amb 0.1, one frame per step",
                       "scene": a.scene, "width": W, "height": H, "spp": a.samples * a.samples,
                       "parallelism": (f"image bands x{world} + RCCL all_gather" +
                                       (" overlapped with the next frame" if overlap else "")) if world > 1
                       else "single GPU",
                       "rays_per_frame": total_rays / a.steps,
                       "camera_samples_per_frame": total_samples / a.steps,
                       "gpu_ms_per_frame": render_ms,
                       "phase_ms_per_frame": {k: v[0] / a.steps for k, v in phases.items()},
                       "camera_Msamples_per_s": total_samples / elapsed / 1e6,
                       "algorithm": a.algorithm},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS if achieved else None, "traffic": traffic,
                         "kernel": kernel_names.get(dom, dom), "kernel_ms": dom_ms / dom_launches,
                         "algorithmic_bytes_per_launch": alg_bytes / dom_launches if alg_bytes else None},
        }
        if world == 1 and a.cpu_seconds > 0:
            line["cpu_baseline"] = cpu_baseline(scene_file, a.resolution, a.samples, a.cpu_seconds)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
