import ctypes as C, sys
sys.path.insert(0, '/root/repo/tools'); sys.path.insert(0, '/root/repo')
from ab_variants import bind
import torch
lib, N = bind(sys.argv[1])
lib.yrt_debug_wide_stats.argtypes = [C.c_void_p, C.c_int]
torch.cuda.set_device(0)
hs, ds = C.c_void_p(), C.c_void_p()
scene = b'/root/repo/tests/golden/scenes/instance10000.yrtscene'
assert lib.yrt_scene_load(scene, C.byref(hs)) == 0
assert lib.yrt_host_scene_build_bvh(hs, 0) == 0
assert lib.yrt_scene_upload(hs, 0, C.byref(ds)) == 0
p = N.RenderParams(); lib.yrt_render_params_default(C.byref(p)); p.resolution, p.samples = 1080, 8
w, h = C.c_int(), C.c_int(); lib.yrt_image_size(ds, C.byref(p), C.byref(w), C.byref(h))
out = torch.empty((h.value, w.value, 4), dtype=torch.float32, device='cuda')
st = (C.c_ulonglong * 8)()
lib.yrt_render(ds, C.byref(p), C.c_void_p(out.data_ptr()), 1, None); torch.cuda.synchronize()
lib.yrt_debug_wide_stats(st, 1)
lib.yrt_render(ds, C.byref(p), C.c_void_p(out.data_ptr()), 1, None); torch.cuda.synchronize()
lib.yrt_debug_wide_stats(st, 1)
print(dict(zip(['wide_visits', 'inst_leaves', 'prim_leaves', 'inst_entries', 'pops'], list(st)[:5])))
