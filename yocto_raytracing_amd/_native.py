"""ctypes binding of include/yrt.h (libyrt.so, built in-tree).

The library is the product: nothing here falls back to Python or to the CPU. If
libyrt.so is missing or fails to load, importing this module raises.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

_PKG = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("YRT_LIB", _PKG / "libyrt.so"))

if not LIB_PATH.exists():
    raise ImportError(
        f"{LIB_PATH} not found: build it with `python yocto_raytracing_amd/build.py` "
        "(or __graft_entry__.build()); there is no fallback path")

# One HIP runtime per process. PyTorch-ROCm bundles its own libamdhip64 (SONAME
# libamdhip64.so.7, but torch asks for it as "libamdhip64.so"): if libyrt.so is loaded
# first, /opt/rocm's runtime is mapped, torch then maps its bundled copy on top of the
# same HSA runtime and finds no GPU ("No HIP GPUs are available"). With torch loaded
# first, libyrt.so's libamdhip64.so.7 resolves to torch's copy and both share it. torch
# is plumbing here (device buffers, streams, torch.distributed), so when it is installed
# it is imported before the library; YRT_NO_TORCH_PRELOAD=1 skips this for processes
# that never import torch.
if os.environ.get("YRT_NO_TORCH_PRELOAD") != "1":
    try:
        import torch  # noqa: F401
    except ImportError:
        pass

lib = C.CDLL(str(LIB_PATH))

YRT_OK = 0
YRT_MEM_HOST = 0
YRT_MEM_DEVICE = 1
YRT_TRANSPORT_COPY = 0
YRT_TRANSPORT_RCCL = 1


class RenderParams(C.Structure):
    _fields_ = [
        ("ambient", C.c_float * 3),
        ("resolution", C.c_int),
        ("width", C.c_int),
        ("samples", C.c_int),
        ("max_depth", C.c_int),
        ("camera", C.c_int),
        ("x0", C.c_int),
        ("y0", C.c_int),
        ("tile_w", C.c_int),
        ("tile_h", C.c_int),
        ("band", C.c_int),
        ("band_stride", C.c_int),
        ("band_offset", C.c_int),
        ("out_stride", C.c_int),
        ("count_work", C.c_int),
        ("algorithm", C.c_int),
        ("timing", C.c_int),
    ]


class Stats(C.Structure):
    _fields_ = [(n, C.c_ulonglong) for n in (
        "rays", "camera_samples", "depth_truncated", "stack_overflow", "box_tests",
        "instance_entries", "prim_tests", "shaded_hits", "texture_lookups", "shadow_rays",
        "shadow_box_tests", "shadow_instance_entries", "shadow_prim_tests", "wave_node_visits",
        "wave_prim_visits", "shadow_wave_node_visits", "shadow_rays_culled")]


PHASES = ("primary", "shadow", "shade", "bounce", "fold", "accumulate", "megakernel", "lists")


class Timings(C.Structure):
    _fields_ = [("ms", C.c_float * 8), ("launches", C.c_int * 8)]


class MaterialDesc(C.Structure):
    _fields_ = [("ke", C.c_float * 3), ("kd", C.c_float * 3), ("ks", C.c_float * 3), ("kr", C.c_float * 3),
                ("rs", C.c_float), ("kd_txt", C.c_int), ("ks_txt", C.c_int)]


class ShapeDesc(C.Structure):
    _fields_ = [("npos", C.c_int), ("pos", C.c_void_p), ("norm", C.c_void_p), ("texcoord", C.c_void_p),
                ("radius", C.c_void_p), ("npoints", C.c_int), ("points", C.c_void_p), ("nlines", C.c_int),
                ("lines", C.c_void_p), ("ntriangles", C.c_int), ("triangles", C.c_void_p)]


_vp = C.c_void_p
_ip = C.POINTER(C.c_int)
_sig = {
    "yrt_abi_version": (C.c_int, []),
    "yrt_status_string": (C.c_char_p, [C.c_int]),
    "yrt_last_error": (C.c_char_p, []),
    "yrt_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "yrt_scene_load": (C.c_int, [C.c_char_p, C.POINTER(_vp)]),
    "yrt_scene_save": (C.c_int, [_vp, C.c_char_p]),
    "yrt_host_scene_build_bvh": (C.c_int, [_vp, C.c_int]),
    "yrt_host_scene_build_bvh_gpu": (C.c_int, [_vp, C.c_int, C.c_int, C.POINTER(C.c_float)]),
    "yrt_host_scene_save_bvh": (C.c_int, [_vp, C.c_char_p]),
    "yrt_host_scene_info": (C.c_int, [_vp, C.POINTER(C.c_longlong)]),
    "yrt_host_image_size": (C.c_int, [_vp, C.c_int, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "yrt_host_scene_free": (None, [_vp]),
    "yrt_host_scene_create": (C.c_int, [C.POINTER(_vp)]),
    "yrt_host_scene_add_camera": (C.c_int, [_vp, _vp, C.c_float, C.c_float, C.c_float, C.c_float, _ip]),
    "yrt_host_scene_add_texture": (C.c_int, [_vp, C.c_int, C.c_int, _vp, _ip]),
    "yrt_host_scene_add_material": (C.c_int, [_vp, C.POINTER(MaterialDesc), _ip]),
    "yrt_host_scene_add_shape": (C.c_int, [_vp, C.POINTER(ShapeDesc), _ip]),
    "yrt_host_scene_add_instance": (C.c_int, [_vp, _vp, C.c_int, C.c_int, _ip]),
    "yrt_scene_upload": (C.c_int, [_vp, C.c_int, C.POINTER(_vp)]),
    "yrt_scene_device_bytes": (C.c_size_t, [_vp]),
    "yrt_scene_free": (None, [_vp]),
    "yrt_render_params_default": (None, [C.POINTER(RenderParams)]),
    "yrt_image_size": (C.c_int, [_vp, C.POINTER(RenderParams), C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "yrt_render": (C.c_int, [_vp, C.POINTER(RenderParams), _vp, C.c_int, _vp]),
    "yrt_trace_first": (C.c_int, [_vp, _vp, C.c_int, _vp, _vp, _vp, _vp, _vp, C.c_int, _vp]),
    "yrt_trace_any": (C.c_int, [_vp, _vp, C.c_int, _vp, C.c_int, _vp]),
    "yrt_scene_set_trace_algorithm": (C.c_int, [_vp, C.c_int]),
    "yrt_scene_set_tile_lists": (C.c_int, [_vp, C.c_int]),
    "yrt_scene_tile_lists": (C.c_int, [_vp, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_ulonglong)]),
    "yrt_scene_tile_list_masks": (C.c_int, [_vp, C.POINTER(C.c_ulonglong)]),
    "yrt_scene_set_lds_staging": (C.c_int, [_vp, C.c_int]),
    "yrt_scene_lds_staging": (C.c_int, [_vp, C.POINTER(C.c_int)]),
    "yrt_last_stats": (C.c_int, [_vp, C.POINTER(Stats)]),
    "yrt_last_timings": (C.c_int, [_vp, C.POINTER(Timings)]),
    "yrt_tonemap": (C.c_int, [_vp, C.c_int, _vp, C.c_int, _vp]),
    "yrt_save_image": (C.c_int, [C.c_char_p, _vp, C.c_int, C.c_int]),
    "yrt_save_image_mem": (C.c_int, [C.c_char_p, _vp, C.c_int, C.c_int, C.c_int, _vp]),
    "yrt_multi_create": (C.c_int, [_vp, _ip, C.c_int, C.POINTER(_vp)]),
    "yrt_multi_free": (None, [_vp]),
    "yrt_multi_info": (C.c_int, [_vp, _ip, _ip]),
    "yrt_multi_render": (C.c_int, [_vp, C.POINTER(RenderParams), _vp, C.c_int]),
    "yrt_multi_last_stats": (C.c_int, [_vp, C.POINTER(Stats)]),
    "yrt_multi_last_timings": (C.c_int, [_vp, C.POINTER(C.c_float), C.POINTER(C.c_float)]),
    "yrt_render_multi": (C.c_int, [_vp, _ip, C.c_int, C.POINTER(RenderParams), _vp, C.c_int]),
}
EXPORTS = tuple(_sig)

for _name, (_res, _args) in _sig.items():
    try:
        _f = getattr(lib, _name)
    except AttributeError as e:
        raise ImportError(f"{LIB_PATH} is stale (missing {_name}): rebuild it") from e
    _f.restype = _res
    _f.argtypes = _args


class YrtError(RuntimeError):
    def __init__(self, status: int, what: str):
        msg = lib.yrt_last_error().decode() or lib.yrt_status_string(status).decode()
        super().__init__(f"{what}: {lib.yrt_status_string(status).decode()}: {msg}")
        self.status = status


def check(status: int, what: str) -> None:
    if status != YRT_OK:
        raise YrtError(status, what)
