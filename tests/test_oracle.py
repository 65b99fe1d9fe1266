"""Pin the oracle (oracle/oracle.c, test infrastructure) to the reference: its BVH,
per-ray intersection records and rendered images must equal the reference's own
outputs bit for bit -- the committed golden fixtures everywhere, and the live
reference build (oracle/_ref) where /root/reference is present."""
import ctypes as C
import gzip
import hashlib

import numpy as np
import pytest

from helpers import GOLDEN, ROOT, SCENE_NAMES, Oracle, assert_same_floats, digests, have_reference, scene_path


@pytest.mark.parametrize("name", SCENE_NAMES)
def test_oracle_bvh_matches_reference(name, tmp_path):
    o = Oracle(name)
    out = tmp_path / "o.yrtbvh"
    o.lib.oracle_write_bvh(o.h, str(out).encode())
    assert hashlib.sha256(gzip.open(out).read()).hexdigest() == digests()[name]["bvh_sha256"]


def _cases():
    for name in SCENE_NAMES:
        z = np.load(GOLDEN / f"ref_render_{name}.npz")
        for key in z.files:
            if key.startswith("img_"):
                _, r, s = key.split("_")
                yield name, int(r[1:]), int(s[1:])


@pytest.mark.parametrize("name,res,spp", list(_cases()))
def test_oracle_render_bitexact_vs_reference_fixture(name, res, spp):
    z = np.load(GOLDEN / f"ref_render_{name}.npz")
    ref = z[f"img_r{res}_s{spp}"]
    img, nrays, trunc = Oracle(name).render(res, spp)
    assert trunc == 0
    assert nrays == int(z[f"rays_r{res}_s{spp}"])
    np.testing.assert_array_equal(img.view(np.uint32), ref.view(np.uint32))


def _edge_cases():
    z = np.load(GOLDEN / "ref_render_edges.npz")
    for key in z.files:
        name, kind, r, s = key.rsplit("_", 3)
        if kind == "img":
            yield name, int(r[1:]), int(s[1:])


@pytest.mark.parametrize("name,res,spp", list(_edge_cases()))
def test_oracle_edge_scenes_vs_reference_fixture(name, res, spp):
    """no lights, every ray a miss, no instances at all, only a point light; 2x1 and 12x7
    frames (tests/golden/make_edges.py)"""
    z = np.load(GOLDEN / "ref_render_edges.npz")
    img, nrays, trunc = Oracle(str(scene_path(f"edge_{name}"))).render(res, spp)
    assert nrays == int(z[f"{name}_rays_r{res}_s{spp}"])
    np.testing.assert_array_equal(img.view(np.uint32), z[f"{name}_img_r{res}_s{spp}"].view(np.uint32))


@pytest.mark.parametrize("name", SCENE_NAMES)
def test_oracle_trace_bitexact_vs_reference_fixture(name):
    z = np.load(GOLDEN / f"ref_rays_{name}.npz")
    o = Oracle(name)
    got = o.trace(z["rays"])
    np.testing.assert_array_equal(got["hit"], z["hit"].astype(bool))
    np.testing.assert_array_equal(got["ei"], z["ei"])
    h = z["hit"] > 0
    np.testing.assert_array_equal(got["inst"][h], z["inst"][h])
    np.testing.assert_array_equal(got["ew"].view(np.uint32), z["ew"].view(np.uint32))
    np.testing.assert_array_equal(got["dist"].view(np.uint32), z["dist"].view(np.uint32))
    anyh = o.trace(z["rays"], any_hit=True)["hit"]
    np.testing.assert_array_equal(anyh, z["any_hit"].astype(bool))
    assert h.mean() > 0.3 and (~h).mean() > 0.05  # fixtures cover hits and misses


def test_oracle_rows_subset_equals_full_render():
    o = Oracle("refl")
    full, n_full, _ = o.render(40, 2)
    rows = np.array([3, 17, 39], np.int32)
    part, _, _ = o.render(40, 2, rows=rows, x0=11, ncols=20)
    np.testing.assert_array_equal(part, full[rows, 11:31])
    assert n_full > 0


@pytest.mark.reference
@pytest.mark.skipif(not have_reference(), reason="needs /root/reference and oracle/_ref")
@pytest.mark.parametrize("name,res,spp", [("simple", 72, 2), ("refl", 60, 3), ("instance10000", 45, 2)])
def test_oracle_vs_live_reference(name, res, spp):
    lib = C.CDLL(str(ROOT / "oracle/_ref/libyrtref.so"))
    lib.ref_read_scene.restype = C.c_void_p
    lib.ref_read_scene.argtypes = [C.c_char_p]
    lib.ref_image_size.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
    lib.ref_render.restype = C.c_longlong
    lib.ref_render.argtypes = [C.c_void_p, C.c_float, C.c_int, C.c_int, C.c_void_p]
    scn = lib.ref_read_scene(str(scene_path(name)).encode())
    w, h = C.c_int(), C.c_int()
    lib.ref_image_size(scn, res, C.byref(w), C.byref(h))
    ref = np.zeros((h.value, w.value, 4), np.float32)
    n = lib.ref_render(scn, 0.1, res, spp, ref.ctypes.data)
    img, nrays, _ = Oracle(name).render(res, spp)
    assert nrays == n
    np.testing.assert_array_equal(img.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("name", ["basic", "refl", "instance10000", "lines"])
def test_oracle_trace_degenerate_rays_vs_reference(name):
    """axis-parallel rays (0*inf slabs), rays on box planes, NaN/inf/zero components,
    empty and inverted [tmin, tmax]: the reference's answers (make_degenerate.py)"""
    z = np.load(GOLDEN / f"ref_rays_degenerate_{name}.npz")
    o = Oracle(name)
    got = o.trace(z["rays"])
    np.testing.assert_array_equal(got["hit"], z["hit"].astype(bool))
    h = z["hit"] > 0
    np.testing.assert_array_equal(got["ei"][h], z["ei"][h])
    np.testing.assert_array_equal(got["inst"][h], z["inst"][h])
    assert_same_floats(got["ew"][h], z["ew"][h])
    assert_same_floats(got["dist"][h], z["dist"][h])
    np.testing.assert_array_equal(o.trace(z["rays"], any_hit=True)["hit"], z["any_hit"].astype(bool))


@pytest.mark.reference
@pytest.mark.skipif(not have_reference(), reason="needs /root/reference and oracle/_ref")
@pytest.mark.parametrize("name,res,spp", [("refl", 40, 2), ("instance10000", 36, 2)])
def test_reference_all_cores_rows_equal_full_render(name, res, spp):
    """bench.py's cpu_baseline_all_cores runs the reference's loop body on many host threads
    (ref_render_rows_mt): its rows and ray count equal the reference's own raytrace()"""
    lib = C.CDLL(str(ROOT / "oracle/_ref/libyrtref.so"))
    lib.ref_read_scene.restype = C.c_void_p
    lib.ref_read_scene.argtypes = [C.c_char_p]
    lib.ref_image_size.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
    lib.ref_render.restype = C.c_longlong
    lib.ref_render.argtypes = [C.c_void_p, C.c_float, C.c_int, C.c_int, C.c_void_p]
    lib.ref_render_rows_mt.restype = C.c_longlong
    lib.ref_render_rows_mt.argtypes = [C.c_void_p, C.c_float, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_void_p,
                                       C.c_int]
    scn = lib.ref_read_scene(str(scene_path(name)).encode())
    w, h = C.c_int(), C.c_int()
    lib.ref_image_size(scn, res, C.byref(w), C.byref(h))
    full = np.zeros((h.value, w.value, 4), np.float32)
    n_full = lib.ref_render(scn, 0.1, res, spp, full.ctypes.data)
    rows = np.arange(h.value, dtype=np.int32)
    for threads in (1, 5):
        part = np.zeros_like(full)
        n = lib.ref_render_rows_mt(scn, 0.1, res, spp, rows.ctypes.data, len(rows), part.ctypes.data, threads)
        assert n == n_full
        np.testing.assert_array_equal(part.view(np.uint32), full.view(np.uint32))
