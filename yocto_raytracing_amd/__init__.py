"""yocto_raytracing_amd -- MI355X-native renderer for the yocto_raytracing hot path.

Python mirror of the reference's host interface (names, argument meaning and
error behaviour of src/scene.h and src/raytrace.cpp), over the C-ABI of
include/yrt.h implemented by libyrt.so (C++ host code + gfx950 HIP kernels):

    scn = load_scene("in/basic_pointlight/basic_pointlight.obj")   # scene.cpp:113
    build_bvh(scn, False)                                          # scene.cpp:554
    img = raytrace(scn, (0.1, 0.1, 0.1), 720, 1)                   # raytrace.cpp:213
    save_hdr_or_ldr("out.png", img)                                # image.cpp:81

`img` is the reference's image4f: float32 RGBA, shape (H, W, 4), pixels[j][i].
There is no CPU fallback: without a GPU the render calls raise.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Sequence

import numpy as np

from . import _native as N
from ._native import RenderParams, Stats, YrtError, check

__all__ = [
    "Scene", "DeviceScene", "load_scene", "build_bvh", "raytrace", "intersect_first",
    "intersect_any", "tonemap", "save_hdr_or_ldr", "render_params", "device_count", "YrtError",
]

ALGORITHMS = {"wavefront": 0, "megakernel": 1, "wavefront_lane": 2}
TILE_LISTS = {"auto": 0, "on": 1, "off": 2}
INFO_FIELDS = ("cameras", "textures", "materials", "shapes", "instances", "lights",
               "bvh_nodes", "bvh_depth", "shape_bvh_depth", "triangles", "lines", "points")


class Scene:
    """Host scene (the reference's `scene*`), owned by libyrt."""

    def __init__(self, handle: int):
        self._h = C.c_void_p(handle)
        self._device_scenes = {}

    @property
    def handle(self):
        return self._h

    def __del__(self):
        try:
            for ds in self._device_scenes.values():
                ds.close()
            if self._h:
                N.lib.yrt_host_scene_free(self._h)
                self._h = C.c_void_p()
        except Exception:
            pass

    # ---- building a scene in memory (yrt_host_scene_add_*: the reference's scene*
    # filled field by field, scene.h:26-155) ----
    @classmethod
    def create(cls) -> "Scene":
        h = C.c_void_p()
        check(N.lib.yrt_host_scene_create(C.byref(h)), "yrt_host_scene_create")
        return cls(h.value)

    @staticmethod
    def _frame(frame) -> np.ndarray:
        f = np.ascontiguousarray(frame, np.float32).reshape(-1)
        if f.size != 12:
            raise ValueError("frame must be 12 floats: x.xyz, y.xyz, z.xyz, o.xyz")
        return f

    def _added(self, status, what, idx) -> int:
        check(status, what)
        for ds in self._device_scenes.values():
            ds.close()
        self._device_scenes.clear()
        return idx.value

    def add_camera(self, frame, fovy: float, aspect: float, focus: float, aperture: float = 0.0) -> int:
        f, idx = self._frame(frame), C.c_int()
        return self._added(N.lib.yrt_host_scene_add_camera(self._h, f.ctypes.data, fovy, aspect, aperture, focus,
                                                           C.byref(idx)), "add_camera", idx)

    def add_texture(self, rgba8: np.ndarray) -> int:
        t = np.ascontiguousarray(rgba8, np.uint8)
        if t.ndim != 3 or t.shape[2] != 4:
            raise ValueError("texture must be (h, w, 4) uint8")
        idx = C.c_int()
        return self._added(N.lib.yrt_host_scene_add_texture(self._h, t.shape[1], t.shape[0], t.ctypes.data,
                                                            C.byref(idx)), "add_texture", idx)

    def add_material(self, kd=(0, 0, 0), ks=(0, 0, 0), kr=(0, 0, 0), ke=(0, 0, 0), rs: float = 0.0,
                     kd_txt: int = -1, ks_txt: int = -1) -> int:
        m = N.MaterialDesc()
        for name, v in (("ke", ke), ("kd", kd), ("ks", ks), ("kr", kr)):
            getattr(m, name)[:] = [float(x) for x in v]
        m.rs, m.kd_txt, m.ks_txt = float(rs), int(kd_txt), int(ks_txt)
        idx = C.c_int()
        return self._added(N.lib.yrt_host_scene_add_material(self._h, C.byref(m), C.byref(idx)), "add_material", idx)

    def add_shape(self, pos, norm=None, texcoord=None, radius=None, points=None, lines=None, triangles=None) -> int:
        keep = []

        def arr(a, dtype, cols):
            if a is None:
                return None, 0
            x = np.ascontiguousarray(a, dtype)
            x = x.reshape(-1, cols) if cols > 1 else x.reshape(-1)
            keep.append(x)
            return x.ctypes.data, x.shape[0]

        d = N.ShapeDesc()
        d.pos, d.npos = arr(pos, np.float32, 3)
        d.norm, _ = arr(norm, np.float32, 3)
        d.texcoord, _ = arr(texcoord, np.float32, 2)
        d.radius, _ = arr(radius, np.float32, 1)
        d.points, d.npoints = arr(points, np.int32, 1)
        d.lines, d.nlines = arr(lines, np.int32, 2)
        d.triangles, d.ntriangles = arr(triangles, np.int32, 3)
        for name, n in (("norm", 3), ("texcoord", 2), ("radius", 1)):
            a = locals()[name]
            if a is not None and np.asarray(a).size != d.npos * n:
                raise ValueError(f"{name} must have one entry per vertex")
        idx = C.c_int()
        return self._added(N.lib.yrt_host_scene_add_shape(self._h, C.byref(d), C.byref(idx)), "add_shape", idx)

    def add_instance(self, frame, shape: int, material: int) -> int:
        f, idx = self._frame(frame), C.c_int()
        return self._added(N.lib.yrt_host_scene_add_instance(self._h, f.ctypes.data, shape, material, C.byref(idx)),
                           "add_instance", idx)

    def info(self) -> dict:
        buf = (C.c_longlong * 12)()
        check(N.lib.yrt_host_scene_info(self._h, buf), "yrt_host_scene_info")
        return dict(zip(INFO_FIELDS, list(buf)))

    def image_size(self, resolution: int, camera: int = 0):
        w, h = C.c_int(), C.c_int()
        check(N.lib.yrt_host_image_size(self._h, camera, resolution, C.byref(w), C.byref(h)),
              "yrt_host_image_size")
        return w.value, h.value

    def save(self, path: str) -> None:
        check(N.lib.yrt_scene_save(self._h, str(path).encode()), "yrt_scene_save")

    def save_bvh(self, path: str) -> None:
        check(N.lib.yrt_host_scene_save_bvh(self._h, str(path).encode()), "yrt_host_scene_save_bvh")

    def upload(self, device: int = 0) -> "DeviceScene":
        if device not in self._device_scenes:
            self._device_scenes[device] = DeviceScene(self, device)
        return self._device_scenes[device]


class DeviceScene:
    """A scene resident in one GPU's HBM (yrt_scene*)."""

    def __init__(self, scene: Scene, device: int = 0):
        h = C.c_void_p()
        check(N.lib.yrt_scene_upload(scene.handle, device, C.byref(h)), "yrt_scene_upload")
        self._h = h
        self.device = device
        self.host = scene

    @property
    def handle(self):
        return self._h

    def close(self):
        if self._h:
            N.lib.yrt_scene_free(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_trace_algorithm(self, algorithm: str) -> None:
        """walks used by intersect_first/intersect_any on this scene (identical results)"""
        check(N.lib.yrt_scene_set_trace_algorithm(self._h, ALGORITHMS[algorithm]), "set_trace_algorithm")

    def set_tile_lists(self, mode: str) -> None:
        """per-tile candidate lists of render_into: "on" builds them whenever the scene allows,
        "auto" (default) the same from 9 samples per pixel, "off" never -- identical images
        either way"""
        check(N.lib.yrt_scene_set_tile_lists(self._h, TILE_LISTS[mode]), "set_tile_lists")

    def tile_lists(self) -> dict:
        """the lists the last render used, and the sums of the last render that built any"""
        cam, bun, sums = C.c_int(), C.c_int(), (C.c_ulonglong * 4)()
        check(N.lib.yrt_scene_tile_lists(self._h, C.byref(cam), C.byref(bun), sums), "tile_lists")
        ex = (C.c_ulonglong * 2)()
        check(N.lib.yrt_scene_tile_list_masks(self._h, ex), "tile_list_masks")
        return {"camera": bool(cam.value), "bundles": bool(bun.value), "camera_entries": int(sums[0]),
                "camera_lists": int(sums[1]), "bundle_entries": int(sums[2]), "bundle_lists": int(sums[3]),
                "camera_instances_masked": int(ex[0]), "bundle_instances_masked": int(ex[1])}

    def set_lds_staging(self, on: bool) -> None:
        """LDS staging of the instance tree's top in render_into's persistent walks (the tile
        lists are not built while it is on; identical images; off by default, measured slower:
        DESIGN.md §5)"""
        check(N.lib.yrt_scene_set_lds_staging(self._h, 1 if on else 0), "set_lds_staging")

    def lds_staging(self) -> dict:
        """which walks of the last render read the staged records"""
        v = C.c_int()
        check(N.lib.yrt_scene_lds_staging(self._h, C.byref(v)), "lds_staging")
        return {"closest_hit": bool(v.value & 1), "any_hit": bool(v.value & 2)}

    @property
    def device_bytes(self) -> int:
        return int(N.lib.yrt_scene_device_bytes(self._h))

    def image_size(self, params: RenderParams):
        w, h = C.c_int(), C.c_int()
        check(N.lib.yrt_image_size(self._h, C.byref(params), C.byref(w), C.byref(h)), "yrt_image_size")
        return w.value, h.value

    def render_into(self, params: RenderParams, out_ptr: int, device_memory: bool = True,
                    stream: Optional[int] = None) -> None:
        """Launch raytrace() into a caller buffer (device pointer by default), stream ordered."""
        mem = N.YRT_MEM_DEVICE if device_memory else N.YRT_MEM_HOST
        check(N.lib.yrt_render(self._h, C.byref(params), C.c_void_p(out_ptr), mem,
                               C.c_void_p(stream or 0)), "yrt_render")

    def last_timings(self) -> dict:
        """per-phase GPU ms of the last render with timing=True: {phase: (ms, launches)}"""
        t = N.Timings()
        check(N.lib.yrt_last_timings(self._h, C.byref(t)), "yrt_last_timings")
        return {name: (float(t.ms[k]), int(t.launches[k])) for k, name in enumerate(N.PHASES)
                if t.launches[k]}

    def last_stats(self) -> dict:
        s = Stats()
        check(N.lib.yrt_last_stats(self._h, C.byref(s)), "yrt_last_stats")
        return {name: int(getattr(s, name)) for name, _ in Stats._fields_}


class MultiScene:
    """A scene replicated on several GPUs of this node (yrt_multi*): raytrace() of a
    whole frame split into interleaved 8-row bands, gathered to devices[0] over RCCL
    (or plain copies when a device is listed twice -- a rehearsal on one GPU)."""

    def __init__(self, scene: "Scene", devices: Sequence[int]):
        ids = (C.c_int * len(devices))(*[int(d) for d in devices])
        h = C.c_void_p()
        check(N.lib.yrt_multi_create(scene.handle, ids, len(devices), C.byref(h)), "yrt_multi_create")
        self._h = h
        self.devices = tuple(int(d) for d in devices)
        n, tr = C.c_int(), C.c_int()
        check(N.lib.yrt_multi_info(self._h, C.byref(n), C.byref(tr)), "yrt_multi_info")
        self.transport = "rccl" if tr.value == N.YRT_TRANSPORT_RCCL else "copy"

    def close(self):
        if self._h:
            N.lib.yrt_multi_free(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def render_into(self, params: RenderParams, out_ptr: int, device_memory: bool = False) -> None:
        """raytrace() of the whole frame into a host buffer, or a device buffer on devices[0]"""
        mem = N.YRT_MEM_DEVICE if device_memory else N.YRT_MEM_HOST
        check(N.lib.yrt_multi_render(self._h, C.byref(params), C.c_void_p(out_ptr), mem), "yrt_multi_render")

    def last_stats(self) -> dict:
        s = Stats()
        check(N.lib.yrt_multi_last_stats(self._h, C.byref(s)), "yrt_multi_last_stats")
        return {name: int(getattr(s, name)) for name, _ in Stats._fields_}

    def last_timings(self) -> dict:
        r, g = C.c_float(), C.c_float()
        check(N.lib.yrt_multi_last_timings(self._h, C.byref(r), C.byref(g)), "yrt_multi_last_timings")
        return {"render_ms": r.value, "gather_ms": g.value}


def device_count() -> int:
    n = C.c_int(0)
    N.lib.yrt_device_count(C.byref(n))
    return n.value


def load_scene(filename: str) -> Scene:
    """load_scene (src/scene.cpp:113): Yocto OBJ or .yrtscene. Raises on failure
    (the reference prints "could not load scene" and exits)."""
    h = C.c_void_p()
    check(N.lib.yrt_scene_load(str(filename).encode(), C.byref(h)), f"load_scene({filename})")
    return Scene(h.value)


def build_bvh(scn: Scene, equal_num: bool = False, device: Optional[int] = None) -> Optional[float]:
    """build_bvh (src/scene.cpp:554): per-shape BVHs, then the instance BVH. With
    `device`, the tree construction runs on that GPU (the same nodes byte for byte) and
    the GPU milliseconds of its level passes are returned."""
    if device is None:
        check(N.lib.yrt_host_scene_build_bvh(scn.handle, 1 if equal_num else 0), "build_bvh")
        return None
    ms = C.c_float(0)
    check(N.lib.yrt_host_scene_build_bvh_gpu(scn.handle, 1 if equal_num else 0, int(device), C.byref(ms)),
          "build_bvh(device)")
    return float(ms.value)


def render_params(amb=(0.1, 0.1, 0.1), resolution: int = 720, samples: int = 1, *,
                  width: int = 0, max_depth: int = 16, camera: int = 0, window=None,
                  band=(1, 1, 0), count_work: bool = False, algorithm: str = "wavefront",
                  timing: int = 0) -> RenderParams:
    p = RenderParams()
    N.lib.yrt_render_params_default(C.byref(p))
    if np.isscalar(amb):
        amb = (amb, amb, amb)
    for k in range(3):
        p.ambient[k] = float(amb[k])
    p.resolution, p.samples, p.width = int(resolution), int(samples), int(width)
    p.max_depth, p.camera = int(max_depth), int(camera)
    if window is not None:
        p.x0, p.y0, p.tile_w, p.tile_h = (int(v) for v in window)
    p.band, p.band_stride, p.band_offset = (int(v) for v in band)
    p.count_work = 1 if count_work else 0
    p.algorithm = ALGORITHMS[algorithm]
    p.timing = int(timing)
    return p


def _device_scene(scn, device: int = 0) -> DeviceScene:
    if isinstance(scn, DeviceScene):
        return scn
    return scn.upload(device)


def raytrace(scn, amb: Sequence[float] = (0.1, 0.1, 0.1), resolution: int = 720, samples: int = 1,
             *, width: int = 0, max_depth: int = 16, camera: int = 0, window=None,
             count_work: bool = False, return_stats: bool = False, algorithm: str = "wavefront",
             devices: Optional[Sequence[int]] = None):
    """raytrace (src/raytrace.cpp:213): RGBA float32 image (H, W, 4), row-major.

    `samples` is per axis (s*s samples per pixel), `resolution` the vertical size.
    `window` = (x0, y0, w, h) renders a sub-rectangle only. `devices` (a Scene, whole
    frames) splits the frame over those GPUs (MultiScene)."""
    if devices is not None:
        if window is not None or isinstance(scn, DeviceScene):
            raise ValueError("devices= renders whole frames of a host Scene")
        ms = MultiScene(scn, devices)
        try:
            p = render_params(amb, resolution, samples, width=width, max_depth=max_depth, camera=camera,
                              count_work=count_work, algorithm=algorithm)
            W, H = scn.image_size(resolution, camera)  # host-side: no extra replica on devices[0]
            W = int(width) or W
            img = np.zeros((H, W, 4), np.float32)
            ms.render_into(p, img.ctypes.data)
            stats = ms.last_stats()
        finally:
            ms.close()
        return (img, stats) if return_stats else img
    ds = _device_scene(scn)
    p = render_params(amb, resolution, samples, width=width, max_depth=max_depth, camera=camera,
                      window=window, count_work=count_work, algorithm=algorithm)
    W, H = ds.image_size(p)
    if window is None:
        w, h = W, H
    else:
        w, h = window[2] or W - window[0], window[3] or H - window[1]
    img = np.zeros((h, w, 4), np.float32)
    ds.render_into(p, img.ctypes.data, device_memory=False)
    if return_stats:
        return img, ds.last_stats()
    return img


def _rays_array(rays) -> np.ndarray:
    r = np.ascontiguousarray(rays, dtype=np.float32)
    if r.ndim != 2 or r.shape[1] != 8:
        raise ValueError("rays must be (n, 8): o.xyz, d.xyz, tmin, tmax")
    return r


def intersect_first(scn, rays) -> dict:
    """Batch intersect_first (src/scene.cpp:483): per ray hit, instance, ei, ew[4], dist."""
    ds = _device_scene(scn)
    r = _rays_array(rays)
    n = r.shape[0]
    out = {"hit": np.zeros(n, np.uint8), "inst": np.zeros(n, np.int32), "ei": np.zeros(n, np.int32),
           "ew": np.zeros((n, 4), np.float32), "dist": np.zeros(n, np.float32)}
    check(N.lib.yrt_trace_first(ds.handle, r.ctypes.data, n, out["hit"].ctypes.data,
                                out["inst"].ctypes.data, out["ei"].ctypes.data, out["ew"].ctypes.data,
                                out["dist"].ctypes.data, N.YRT_MEM_HOST, None), "intersect_first")
    out["hit"] = out["hit"].astype(bool)
    return out


def intersect_any(scn, rays) -> np.ndarray:
    """Batch intersect_any (src/scene.cpp:489): occluded flag per ray."""
    ds = _device_scene(scn)
    r = _rays_array(rays)
    hit = np.zeros(r.shape[0], np.uint8)
    check(N.lib.yrt_trace_any(ds.handle, r.ctypes.data, r.shape[0], hit.ctypes.data, N.YRT_MEM_HOST,
                              None), "intersect_any")
    return hit.astype(bool)


def tonemap(img: np.ndarray) -> np.ndarray:
    """tonemap (src/image.cpp:55, exposure 0, srgb): RGBA8 of the same shape."""
    a = np.ascontiguousarray(img, dtype=np.float32)
    out = np.zeros(a.shape, np.uint8)
    check(N.lib.yrt_tonemap(a.ctypes.data, a.size // 4, out.ctypes.data, N.YRT_MEM_HOST, None), "tonemap")
    return out


def save_image_device(filename: str, ptr: int, width: int, height: int, stream: Optional[int] = None) -> None:
    """save_hdr_or_ldr of a frame in device memory: the PNG tonemap runs on the GPU"""
    check(N.lib.yrt_save_image_mem(str(filename).encode(), C.c_void_p(ptr), int(width), int(height),
                                   N.YRT_MEM_DEVICE, C.c_void_p(stream or 0)), "save_image_device")


def tonemap_device(rgba_ptr: int, n: int, out_ptr: int, stream: Optional[int] = None) -> None:
    """tonemap (src/image.cpp:55) of n RGBA f32 pixels in device memory into RGBA8 (device)"""
    check(N.lib.yrt_tonemap(C.c_void_p(rgba_ptr), int(n), C.c_void_p(out_ptr), N.YRT_MEM_DEVICE,
                            C.c_void_p(stream or 0)), "tonemap_device")


def save_hdr_or_ldr(filename: str, img: np.ndarray) -> None:
    """save_hdr_or_ldr (src/image.cpp:81): .hdr -> RGBE, otherwise tonemapped PNG."""
    a = np.ascontiguousarray(img, dtype=np.float32)
    check(N.lib.yrt_save_image(str(filename).encode(), a.ctypes.data, a.shape[1], a.shape[0]),
          "save_hdr_or_ldr")
