import sys; sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import numpy as np
import yocto_raytracing_amd as yrt
from helpers import scene_path
s = yrt.load_scene(str(scene_path("refl"))); yrt.build_bvh(s)
ds = s.upload(0)
img, st1 = yrt.raytrace(ds, (0.1,)*3, 90, 3, return_stats=True)
img2, st2 = yrt.raytrace(ds, (0.1,)*3, 90, 3, return_stats=True)
print("single", st1); print("single again", st2)
q = yrt.render_params(0.1, 90, 3, band=(8, 1, 0)); q.tile_h = 96; q.out_stride = 160
out = np.zeros((96, 160, 4), np.float32)
ds.render_into(q, out.ctypes.data, device_memory=False)
print("band", ds.last_stats(), np.array_equal(out[:90], img))
ms = yrt.MultiScene(s, [0])
o2 = np.zeros_like(img); ms.render_into(yrt.render_params(0.1, 90, 3), o2.ctypes.data)
print("multi", ms.last_stats(), np.array_equal(o2, img))
ds2 = yrt.DeviceScene(s, 0)
img3, st3 = yrt.raytrace(ds2, (0.1,)*3, 90, 3, return_stats=True)
print("second upload", st3)
