"""Per-wave phase times of the list builders, from a YRT_LIST_TIMING build:

    python tools/build_variants.py lt:-DYRT_LIST_TIMING
    python tools/list_timing.py yocto_raytracing_amd/variants/libyrt_lt.so [--share 0/8]

Renders the c4 frame (or --scene / --share) twice and prints, per builder, the mean /
median / p90 of each phase in microseconds (the constant clock's 10 ns ticks):
k_camera_lists {setup, frontier rounds, masks + output} and its rounds and entries;
k_bundle_super {hit-point box + light, hull walk} and its list length; k_bundle_lists
{box + candidates, sort + masks, records} and its list length (waves 0-65535 only;
early-out waves write nothing and are skipped).
"""
from __future__ import annotations

import argparse
import ctypes as C
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tools"))

from ab_variants import bind  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--scene", default="instance10000")
    ap.add_argument("--resolution", type=int, default=1080)
    ap.add_argument("--samples", type=int, default=8)
    ap.add_argument("--share", default="0/1")
    a = ap.parse_args()
    import torch

    torch.cuda.set_device(0)
    lib, N = bind(a.lib)
    lib.yrt_debug_list_time.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int]
    scene = str(ROOT / "tests" / "golden" / "scenes" / f"{a.scene}.yrtscene").encode()
    hs, ds = C.c_void_p(), C.c_void_p()
    assert lib.yrt_scene_load(scene, C.byref(hs)) == 0, lib.yrt_last_error()
    assert lib.yrt_host_scene_build_bvh(hs, 0) == 0
    assert lib.yrt_scene_upload(hs, 0, C.byref(ds)) == 0, lib.yrt_last_error()
    p = N.RenderParams()
    lib.yrt_render_params_default(C.byref(p))
    p.resolution, p.samples = a.resolution, a.samples
    w, h = C.c_int(), C.c_int()
    lib.yrt_image_size(ds, C.byref(p), C.byref(w), C.byref(h))
    rank, world = (int(v) for v in a.share.split("/"))
    if world > 1:
        from yocto_raytracing_amd.shard import BandLayout, render_params_band

        layout = BandLayout(h.value, world, 8)
        (p.band, p.band_stride, p.band_offset), p.tile_h = render_params_band(layout, rank)
        h = C.c_int(p.tile_h)
    out = torch.empty((h.value, w.value, 4), dtype=torch.float32, device="cuda")
    buf = np.zeros((65536, 4), np.uint64)
    for rep in range(2):
        for k in range(3):
            assert lib.yrt_debug_list_time(buf.ctypes.data, k, 65536, 1) == 0
        assert lib.yrt_render(ds, C.byref(p), C.c_void_p(out.data_ptr()), 1, None) == 0, lib.yrt_last_error()
        torch.cuda.synchronize()
    names = {0: ("k_camera_lists", ["setup", "rounds", "masks+out"]),
             1: ("k_bundle_super", ["box+light", "hull walk"]),
             2: ("k_bundle_lists", ["box+cand", "sort+masks", "records"])}
    for k, (name, phases) in names.items():
        assert lib.yrt_debug_list_time(buf.ctypes.data, k, 65536, 0) == 0
        rows = buf[buf[:, :3].sum(axis=1) > 0]
        if not len(rows):
            print(name, "no waves")
            continue
        msg = [f"{name}: {len(rows)} waves"]
        for j, ph in enumerate(phases):
            v = rows[:, j].astype(np.float64) / 100.0  # us
            msg.append(f"{ph} mean {v.mean():.2f} med {np.median(v):.2f} p90 {np.percentile(v, 90):.2f}")
        tot = rows[:, :len(phases)].astype(np.float64).sum(axis=1) / 100.0
        msg.append(f"total mean {tot.mean():.2f} p90 {np.percentile(tot, 90):.2f} max {tot.max():.2f}")
        if k == 0:
            r = (rows[:, 3] >> np.uint64(32)).astype(np.int64)
            n = (rows[:, 3] & np.uint64(0xffffffff)).astype(np.int64)
            msg.append(f"rounds mean {r.mean():.1f} max {r.max()}; entries mean {n.mean():.1f}")
        else:
            n = rows[:, 3].astype(np.int64)
            n = np.where(n > 0x7fffffff, n - (1 << 32), n)
            msg.append(f"list length mean {n[n >= 0].mean():.1f}; overflow {(n < 0).sum()}")
        print("\n  ".join(msg))


if __name__ == "__main__":
    main()
