"""Diagnostic: where the persistent grids' time goes at the end of a launch -- per wave
start / end on the 100 MHz constant clock, items taken, XCD -- from a YRT_TAIL_STATS build.

    python tools/build_variants.py tail:-DYRT_TAIL_STATS
    python tools/tail_stats.py yocto_raytracing_amd/variants/libyrt_tail.so [--share R/N] [--scene S]
"""
import argparse
import ctypes as C
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tools"))
sys.path.insert(0, str(ROOT))
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

    lib, N = bind(a.lib)
    lib.yrt_debug_tail.argtypes = [C.c_void_p, C.c_int]
    torch.cuda.set_device(0)
    hs, ds = C.c_void_p(), C.c_void_p()
    scene = str(ROOT / "tests" / "golden" / "scenes" / f"{a.scene}.yrtscene").encode()
    assert lib.yrt_scene_load(scene, C.byref(hs)) == 0
    assert lib.yrt_host_scene_build_bvh(hs, 0) == 0
    assert lib.yrt_scene_upload(hs, 0, C.byref(ds)) == 0
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
    for _ in range(3):  # the last render's records stay
        assert lib.yrt_render(ds, C.byref(p), C.c_void_p(out.data_ptr()), 1, None) == 0
    torch.cuda.synchronize()
    buf = np.zeros((8192, 4), np.uint64)
    for k, name in enumerate(("k_primary_persist", "k_shadow_persist")):
        assert lib.yrt_debug_tail(buf.ctypes.data, k) == 0
        t = buf[buf[:, 1] > 0].astype(np.int64)
        if not len(t):
            print(name, "did not run")
            continue
        t0 = t[:, 0].min()
        start, end, items, xcd = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0, t[:, 2], t[:, 3]  # us
        span = end.max()
        idle = float(np.sum(span - end) / (len(end) * span))
        q = lambda v: " ".join(f"{x:.0f}" for x in np.percentile(v, [0, 10, 50, 90, 99, 100]))
        print(f"{a.scene} {a.share} {name}: {len(t)} waves, span {span:.0f} us, starts spread {start.max():.0f} us, "
              f"idle after own end {100 * idle:.1f} % of wave-time, items/wave {items.mean():.1f}")
        print(f"  wave end us percentiles 0/10/50/90/99/100: {q(end)}")
        for x in range(8):
            m = xcd == x
            print(f"  xcd {x}: waves {m.sum()}, items {items[m].sum()}, last end {end[m].max():.0f}, "
                  f"median end {np.median(end[m]):.0f} us")


if __name__ == "__main__":
    main()
