"""A/B several builds of libyrt in ONE process, interleaved rounds (cdna guide §5.4
rule 24: cross-process timings are not comparable).

    python tools/build_variants.py NAME:DEFINES ...      # build the .so files
    python tools/ab_variants.py --rounds 5 lib_a.so lib_b.so ...
    python tools/ab_variants.py lib.so@on lib.so@off        # the same library, tile lists forced

Each library is loaded with RTLD_LOCAL (own kernels, shared HIP runtime), renders
the c4 frame (instance10000, 1080p, 8x8 spp) into a device buffer on its own
stream, and reports per-phase GPU ms (library HIP events) per round, their total, and
the wall time of the call through the end of its kernels ("wall": host gaps included).
"""
from __future__ import annotations

import argparse
import ctypes as C
import hashlib
import json
import os
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def bind(path):
    from yocto_raytracing_amd import _native as N  # struct layouts only

    lib = C.CDLL(str(path), mode=os.RTLD_LOCAL)
    vp = C.c_void_p
    lib.yrt_scene_load.argtypes = [C.c_char_p, C.POINTER(vp)]
    lib.yrt_host_scene_build_bvh.argtypes = [vp, C.c_int]
    lib.yrt_scene_upload.argtypes = [vp, C.c_int, C.POINTER(vp)]
    lib.yrt_render_params_default.argtypes = [C.POINTER(N.RenderParams)]
    lib.yrt_image_size.argtypes = [vp, C.POINTER(N.RenderParams), C.POINTER(C.c_int), C.POINTER(C.c_int)]
    lib.yrt_render.argtypes = [vp, C.POINTER(N.RenderParams), vp, C.c_int, vp]
    lib.yrt_last_timings.argtypes = [vp, C.POINTER(N.Timings)]
    lib.yrt_last_stats.argtypes = [vp, C.POINTER(N.Stats)]
    lib.yrt_last_error.restype = C.c_char_p
    return lib, N


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--scene", default="instance10000")
    ap.add_argument("--resolution", type=int, default=1080)
    ap.add_argument("--samples", type=int, default=8)
    ap.add_argument("--width", type=int, default=0, help="image width (0: the camera's aspect)")
    ap.add_argument("--algorithm", type=int, default=0)
    ap.add_argument("--count", action="store_true", help="also print the work counters of one pass")
    ap.add_argument("--share", default="0/1", help="R/N: render rank R's 8-row bands of an N-rank split")
    a = ap.parse_args()
    import torch  # device buffer + streams

    torch.cuda.set_device(0)
    out = None
    runs = []
    scene = str(ROOT / "tests" / "golden" / "scenes" / f"{a.scene}.yrtscene").encode()
    for spec in a.libs:
        # lib.so@auto|on|off: yrt_scene_set_tile_lists; lib.so@lds: yrt_scene_set_lds_staging
        path, _, lists = spec.partition("@")
        lib, N = bind(path)
        hs, ds = C.c_void_p(), C.c_void_p()
        assert lib.yrt_scene_load(scene, C.byref(hs)) == 0, lib.yrt_last_error()
        assert lib.yrt_host_scene_build_bvh(hs, 0) == 0
        assert lib.yrt_scene_upload(hs, 0, C.byref(ds)) == 0, lib.yrt_last_error()
        if lists == "lds":
            lib.yrt_scene_set_lds_staging.argtypes = [C.c_void_p, C.c_int]
            assert lib.yrt_scene_set_lds_staging(ds, 1) == 0
        elif lists:
            lib.yrt_scene_set_tile_lists.argtypes = [C.c_void_p, C.c_int]
            assert lib.yrt_scene_set_tile_lists(ds, {"auto": 0, "on": 1, "off": 2}[lists]) == 0
        p = N.RenderParams()
        lib.yrt_render_params_default(C.byref(p))
        p.resolution, p.samples, p.algorithm, p.timing = a.resolution, a.samples, a.algorithm, 1
        p.width = a.width
        w, h = C.c_int(), C.c_int()
        lib.yrt_image_size(ds, C.byref(p), C.byref(w), C.byref(h))
        rank, world = (int(v) for v in a.share.split("/"))
        if world > 1:  # bench.py --profile-rank R/N's bands
            from yocto_raytracing_amd.shard import BandLayout, render_params_band

            layout = BandLayout(h.value, world, 8)
            (p.band, p.band_stride, p.band_offset), p.tile_h = render_params_band(layout, rank)
            h = C.c_int(p.tile_h)
        if out is None:
            out = torch.empty((h.value, w.value, 4), dtype=torch.float32, device="cuda")
        runs.append((Path(path).name + (f"@{lists}" if lists else ""), lib, N, ds, p, torch.cuda.Stream()))
    res = {name: {} for name, *_ in runs}
    digest = {}
    for r in range(a.rounds + 1):  # round 0 = warmup
        for name, lib, N, ds, p, stream in runs:
            stream.synchronize()
            t0 = time.perf_counter()
            rc = lib.yrt_render(ds, C.byref(p), C.c_void_p(out.data_ptr()), 1, C.c_void_p(stream.cuda_stream))
            assert rc == 0, lib.yrt_last_error()
            stream.synchronize()
            wall = (time.perf_counter() - t0) * 1e3  # the call and its kernels, idle gaps included
            t = N.Timings()
            lib.yrt_last_timings(ds, C.byref(t))
            if r == 0:  # warmup; the image digest shows whether the variants agree bit for bit
                stream.synchronize()
                digest[name] = hashlib.sha1(out.cpu().numpy().tobytes()).hexdigest()[:16]
                continue
            for k, ph in enumerate(N.PHASES):
                if t.launches[k]:
                    res[name].setdefault(ph, []).append(t.ms[k])
            res[name].setdefault("total", []).append(sum(t.ms))
            res[name].setdefault("wall", []).append(wall)
    if a.count:
        for name, lib, N, ds, p, stream in runs:
            p.count_work, p.timing = 1, 0
            lib.yrt_render(ds, C.byref(p), C.c_void_p(out.data_ptr()), 1, C.c_void_p(stream.cuda_stream))
            s = N.Stats()
            lib.yrt_last_stats(ds, C.byref(s))
            print(name, "work", {f: getattr(s, f) for f, _ in N.Stats._fields_})
    summary = {}
    for name, d in res.items():
        summary[name] = {ph: {"median": statistics.median(v), "min": min(v)} for ph, v in d.items()}
        print(name, {ph: round(v["median"], 2) for ph, v in summary[name].items()}, "image", digest[name])
    print(json.dumps(summary))


if __name__ == "__main__":
    main()
