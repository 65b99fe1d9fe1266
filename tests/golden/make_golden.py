"""Generate the committed golden fixtures from the REFERENCE ITSELF.

Run in the container that has /root/reference (never on the GPU box):

    make -C oracle ref && python tests/golden/make_golden.py

It drives oracle/_ref/libyrtref.so -- the unmodified reference sources compiled by
oracle/Makefile plus the ctypes harness oracle/ref_harness.cpp -- and writes:

  scenes/<name>.yrtscene   the reference loader's scene (load_scene, scene.cpp:113),
                           serialised to the .yrtscene interchange format
  ref_render_<name>.npz    raytrace() float images (raytrace.cpp:213) at small sizes,
                           plus the number of rays the reference traced
  ref_rays_<name>.npz      intersect_first / intersect_any records (scene.cpp:483-494)
                           for camera rays and seeded random rays
  ref_digests.json         sha256 of the reference's BVH (.yrtbvh) and scene bytes
  ref_images.npz           the reference's own shipped renders (out/*.png, author's
                           build at -r 720 -s 3) and the course images (check/*.png),
                           decoded to RGB u8 -- data only, for PSNR reporting

Every fixture is data (inputs and expected outputs); no reference source is copied.
"""
from __future__ import annotations

import ctypes as C
import gzip
import hashlib
import json
import os
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
REF = Path(os.environ.get("YRT_REFERENCE", "/root/reference"))
SCENES = {
    "basic": "in/basic_pointlight/basic_pointlight.obj",
    "simple": "in/simple_pointlight/simple_pointlight.obj",
    "refl": "in/refl_pointlight/refl_pointlight.obj",
    "instance10000": "in/instance10000_pointlight/instance10000_pointlight.obj",
}
# (resolution, samples-per-axis) rendered by the reference for each scene
RENDERS = {
    "basic": [(64, 1), (48, 2), (36, 3)],
    "simple": [(64, 1), (48, 2)],
    "refl": [(64, 1), (48, 2)],
    "instance10000": [(64, 1), (36, 3)],
}


def load_ref():
    lib = C.CDLL(str(ROOT / "oracle/_ref/libyrtref.so"))
    lib.ref_load_scene.restype = C.c_void_p
    lib.ref_load_scene.argtypes = [C.c_char_p]
    lib.ref_write_scene.argtypes = [C.c_void_p, C.c_char_p]
    lib.ref_write_bvh.argtypes = [C.c_void_p, C.c_char_p]
    lib.ref_image_size.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
    lib.ref_render.restype = C.c_longlong
    lib.ref_render.argtypes = [C.c_void_p, C.c_float, C.c_int, C.c_int, C.c_void_p]
    lib.ref_trace.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int] + [C.c_void_p] * 5
    lib.ref_camera_ray.argtypes = [C.c_void_p] + [C.c_int] * 6 + [C.c_void_p]
    return lib


def sample_rays(lib, scn, rng, n_cam=2048, n_rand=2048):
    """camera rays on a jittered pixel grid + random rays aimed into the scene box"""
    rays = []
    res, s = 90, 2
    w, h = C.c_int(), C.c_int()
    lib.ref_image_size(scn, res, C.byref(w), C.byref(h))
    for _ in range(n_cam):
        i, j = rng.integers(0, w.value), rng.integers(0, h.value)
        ii, jj = rng.integers(0, s), rng.integers(0, s)
        r = np.zeros(8, np.float32)
        lib.ref_camera_ray(scn, res, s, int(i), int(j), int(ii), int(jj), r.ctypes.data)
        rays.append(r)
    cam_rays = np.array(rays, np.float32)
    # random rays: origins near the camera rays' origin region, random directions
    o = cam_rays[:, :3]
    lo, hi = o.min(0) - 20, o.max(0) + 20
    orig = rng.uniform(lo, hi, size=(n_rand, 3)).astype(np.float32)
    d = rng.normal(size=(n_rand, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rr = np.zeros((n_rand, 8), np.float32)
    rr[:, :3], rr[:, 3:6], rr[:, 6], rr[:, 7] = orig, d, 1e-4, np.float32(3.4028234663852886e38)
    # a band of finite tmax values exercises the slab test's tmax scaling
    rr[: n_rand // 4, 7] = rng.uniform(1, 100, size=n_rand // 4).astype(np.float32)
    return np.concatenate([cam_rays, rr])


def trace(lib, scn, rays, any_hit):
    n = len(rays)
    hit = np.zeros(n, np.uint8)
    inst = np.zeros(n, np.int32)
    ei = np.zeros(n, np.int32)
    ew = np.zeros((n, 4), np.float32)
    dist = np.zeros(n, np.float32)
    lib.ref_trace(scn, rays.ctypes.data, n, int(any_hit), hit.ctypes.data, inst.ctypes.data,
                  ei.ctypes.data, ew.ctypes.data, dist.ctypes.data)
    return hit, inst, ei, ew, dist


def main():
    lib = load_ref()
    (HERE / "scenes").mkdir(exist_ok=True)
    digests = {}
    rng = np.random.default_rng(20171015)
    for name, rel in SCENES.items():
        scn = lib.ref_load_scene(str(REF / rel).encode())
        spath = HERE / "scenes" / f"{name}.yrtscene"
        lib.ref_write_scene(scn, str(spath).encode())
        bpath = Path(f"/tmp/{name}_ref.yrtbvh")
        lib.ref_write_bvh(scn, str(bpath).encode())
        digests[name] = {
            "scene_sha256": hashlib.sha256(gzip.open(spath).read()).hexdigest(),
            "bvh_sha256": hashlib.sha256(gzip.open(bpath).read()).hexdigest(),
        }
        out = {}
        for res, s in RENDERS[name]:
            w, h = C.c_int(), C.c_int()
            lib.ref_image_size(scn, res, C.byref(w), C.byref(h))
            img = np.zeros((h.value, w.value, 4), np.float32)
            nrays = lib.ref_render(scn, 0.1, res, s, img.ctypes.data)
            out[f"img_r{res}_s{s}"] = img
            out[f"rays_r{res}_s{s}"] = np.int64(nrays)
        np.savez_compressed(HERE / f"ref_render_{name}.npz", **out)
        rays = sample_rays(lib, scn, rng)
        hit, inst, ei, ew, dist = trace(lib, scn, rays, False)
        ahit = trace(lib, scn, rays, True)[0]
        np.savez_compressed(HERE / f"ref_rays_{name}.npz", rays=rays, hit=hit, inst=inst, ei=ei, ew=ew,
                            dist=dist, any_hit=ahit)
        print(name, digests[name], {k: v.shape for k, v in out.items() if hasattr(v, "shape")})
    (HERE / "ref_digests.json").write_text(json.dumps(digests, indent=1) + "\n")

    # the reference's shipped images (data), decoded by the reference's own loader
    lib.ref_load_image4b.argtypes = [C.c_char_p, C.c_void_p, C.c_void_p, C.c_void_p]
    imgs = {}
    for kind in ("out", "check"):
        for png in sorted((REF / kind).glob("*.png")):
            w, h = C.c_int(), C.c_int()
            lib.ref_load_image4b(str(png).encode(), C.byref(w), C.byref(h), None)
            buf = np.zeros((h.value, w.value, 4), np.uint8)
            lib.ref_load_image4b(str(png).encode(), C.byref(w), C.byref(h), buf.ctypes.data)
            imgs[f"{kind}_{png.stem}"] = buf[..., :3].copy()
    np.savez_compressed(HERE / "ref_images.npz", **imgs)
    print("images", {k: v.shape for k, v in imgs.items()})


if __name__ == "__main__":
    main()
