"""The reference-side binding (oracle/ref_integration.cpp): the
reference's own in-memory scene handed to libyrt through the yrt.h builder.

* CPU (needs /root/reference): what the binding hands over is byte-identical to the
  reference's scene (same .yrtscene digest) and gives the reference's BVH.
* GPU: raytrace_gpu() -- raytrace()'s signature over the MI355X path -- renders the
  reference's scene to the reference's image (golden fixtures)."""
import ctypes as C
import gzip
import hashlib

import numpy as np
import pytest

from helpers import GOLDEN, OBJ_SCENES, REF_OBJ, ROOT, close_mask, digests, have_reference, scene_path

INT_SO = ROOT / "oracle" / "_ref" / "libyrtref_int.so"


def int_lib():
    import yocto_raytracing_amd  # noqa: F401  (libyrt.so first, same file the binding links)

    lib = C.CDLL(str(INT_SO))
    for f in ("ref_load_scene", "ref_read_scene"):
        getattr(lib, f).restype = C.c_void_p
        getattr(lib, f).argtypes = [C.c_char_p]
    lib.ref_int_save_scene.argtypes = [C.c_void_p, C.c_char_p]
    lib.ref_int_save_bvh.argtypes = [C.c_void_p, C.c_char_p]
    lib.ref_int_render.argtypes = [C.c_void_p, C.c_float, C.c_int, C.c_int, C.c_void_p]
    lib.ref_free_scene.argtypes = [C.c_void_p]
    lib.ref_int_release.argtypes = [C.c_void_p]
    return lib


@pytest.mark.reference
@pytest.mark.skipif(not (have_reference() and INT_SO.exists()), reason="needs /root/reference and oracle/_ref")
@pytest.mark.parametrize("name", OBJ_SCENES)
def test_binding_hands_over_the_reference_scene(name, tmp_path):
    lib = int_lib()
    scn = lib.ref_load_scene(str(REF_OBJ[name]).encode())
    try:
        out, bvh = tmp_path / "s.yrtscene", tmp_path / "s.yrtbvh"
        assert lib.ref_int_save_scene(scn, str(out).encode()) == 0
        assert lib.ref_int_save_bvh(scn, str(bvh).encode()) == 0
    finally:
        lib.ref_free_scene(scn)
    assert hashlib.sha256(gzip.open(out).read()).hexdigest() == digests()[name]["scene_sha256"]
    assert hashlib.sha256(gzip.open(bvh).read()).hexdigest() == digests()[name]["bvh_sha256"]


@pytest.mark.gpu
@pytest.mark.skipif(not INT_SO.exists(), reason="oracle/_ref/libyrtref_int.so not built (make -C oracle ref)")
@pytest.mark.parametrize("name", ["basic", "simple", "refl", "instance10000", "lines"])
def test_raytrace_gpu_from_reference_scene(name):
    lib = int_lib()
    z = np.load(GOLDEN / f"ref_render_{name}.npz")
    key = max((k for k in z.files if k.startswith("img_")), key=lambda k: z[k].size)  # the largest fixture
    _, r, s = key.split("_")
    res, spp = int(r[1:]), int(s[1:])
    ref = z[key]
    scn = lib.ref_read_scene(str(scene_path(name)).encode())  # reference structs + reference build_bvh
    try:
        img = np.zeros_like(ref)
        assert lib.ref_int_render(scn, 0.1, res, spp, img.ctypes.data) == 0
    finally:
        lib.ref_int_release(scn)  # the device copy is keyed by the scene's address
        lib.ref_free_scene(scn)
    assert close_mask(img, ref).all()
    assert np.mean(img.view(np.uint32) == ref.view(np.uint32)) > 0.99
