"""Diagnostic: per-walk work of the wide any-hit walk from a YRT_WIDE_STATS build
(every shadow walk of one 64-ray wave adds its counts).

    python tools/build_variants.py ws:-DYRT_WIDE_STATS
    python tools/wide_stats.py yocto_raytracing_amd/variants/libyrt_ws.so [scene res s]
"""
import ctypes as C
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tools"))
sys.path.insert(0, str(ROOT))
from ab_variants import bind  # noqa: E402

import torch  # noqa: E402

NAMES = ["walks", "steps_top", "steps_shape", "inst_entries", "leaves", "prim_tests", "pops", "empty_pops",
         "live_lanes", "occluded_lanes", "walks_all_occluded", "steps_in_all_occluded", "entries_root_missed", "-", "-", "-"]


FIRST_NAMES = ["walks", "list_entries", "spine_records", "inst_entries", "entries_root_missed", "shape_leaves",
               "prim_tests", "-", "live_lanes", "hit_lanes", "-", "-", "-", "-", "-", "-"]


def main():
    lib, N = bind(sys.argv[1])
    name, res, s = (sys.argv[2], int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else ("instance10000", 1080, 8)
    lib.yrt_debug_wide_stats.argtypes = [C.c_void_p, C.c_int]
    torch.cuda.set_device(0)
    hs, ds = C.c_void_p(), C.c_void_p()
    scene = str(ROOT / "tests" / "golden" / "scenes" / f"{name}.yrtscene").encode()
    assert lib.yrt_scene_load(scene, C.byref(hs)) == 0
    assert lib.yrt_host_scene_build_bvh(hs, 0) == 0
    assert lib.yrt_scene_upload(hs, 0, C.byref(ds)) == 0
    p = N.RenderParams()
    lib.yrt_render_params_default(C.byref(p))
    p.resolution, p.samples = res, s
    w, h = C.c_int(), C.c_int()
    lib.yrt_image_size(ds, C.byref(p), C.byref(w), C.byref(h))
    out = torch.empty((h.value, w.value, 4), dtype=torch.float32, device="cuda")
    st = (C.c_ulonglong * 16)()
    lib.yrt_debug_wide_stats(st, 1)
    lib.yrt_debug_first_stats.argtypes = [C.c_void_p, C.c_int]
    lib.yrt_debug_first_stats((C.c_ulonglong * 16)(), 1)  # reset
    rc = lib.yrt_render(ds, C.byref(p), C.c_void_p(out.data_ptr()), 1, None)
    torch.cuda.synchronize()
    lib.yrt_debug_wide_stats(st, 1)
    v = {k: x for k, x in zip(NAMES, list(st)) if k != "-"}
    walks = max(1, v["walks"])
    print(json.dumps({"scene": name, "res": res, "s": s, "rc": rc, "totals": v,
                      "per_walk": {k: round(x / walks, 2) for k, x in v.items()}}))
    # the closest-hit walk's (camera rays, packet_first)
    lib.yrt_debug_first_stats.argtypes = [C.c_void_p, C.c_int]
    fs = (C.c_ulonglong * 16)()
    lib.yrt_debug_first_stats(fs, 1)  # (the render above filled it; read and reset)
    f = {k: x for k, x in zip(FIRST_NAMES, list(fs)) if k != "-"}
    fw = max(1, f["walks"])
    print(json.dumps({"closest_hit_totals": f, "per_walk": {k: round(x / fw, 2) for k, x in f.items()}}))


if __name__ == "__main__":
    main()
