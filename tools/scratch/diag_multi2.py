import sys; sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import numpy as np
import yocto_raytracing_amd as yrt
from helpers import scene_path
def load(n):
    s = yrt.load_scene(str(scene_path(n))); yrt.build_bvh(s); return s
si = load("instance10000"); sr = load("refl")
ref_img, ref_st = yrt.raytrace(sr.upload(0), (0.1,)*3, 90, 3, return_stats=True)
bad = 0
for it in range(6):
    for devs in [(0,), (0, 0), (0, 0, 0), (0,) * 8]:
        ms = yrt.MultiScene(si, devs); o = np.zeros((100, 178, 4), np.float32)
        ms.render_into(yrt.render_params(0.1, 100, 2), o.ctypes.data); ms.close()
    for devs in [(0,), (0, 0, 0)]:
        ms = yrt.MultiScene(sr, devs)
        o = np.zeros_like(ref_img)
        ms.render_into(yrt.render_params(0.1, 90, 3), o.ctypes.data)
        st = ms.last_stats(); ms.close()
        same = np.array_equal(o.view(np.uint32), ref_img.view(np.uint32))
        if st != ref_st or not same:
            bad += 1
            print("MISMATCH", it, devs, same, {k: (st[k], ref_st[k]) for k in st if st[k] != ref_st[k]})
    img, st = yrt.raytrace(sr.upload(0), (0.1,)*3, 90, 3, return_stats=True)
    if st != ref_st:
        print("SINGLE MISMATCH", it, {k: (st[k], ref_st[k]) for k in st if st[k] != ref_st[k]})
print("bad", bad)
