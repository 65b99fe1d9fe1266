"""GPU parity on edge-case scenes (tests/golden/make_edges.py, rendered by the reference
itself): no lights (shade()'s light loop empty, no shadow rays), every camera ray a miss,
a scene with no instances at all (the reference renders it black), a point light alone;
frames of 2x1 and 12x7 pixels, ragged against every tile and block size. Every algorithm
through the C-ABI, bit-exact against the fixture, ray counts exact."""
import gzip
import hashlib

import numpy as np
import pytest

from helpers import EDGE_SCENES, GOLDEN, digests, scene_path

pytestmark = pytest.mark.gpu

ALGOS = ("wavefront", "megakernel", "wavefront_lane")


@pytest.fixture(scope="module")
def yrt():
    import yocto_raytracing_amd as y

    if y.device_count() < 1:
        pytest.fail("no GPU visible: the -m gpu suite must run on the MI355X box")
    return y


def _cases():
    z = np.load(GOLDEN / "ref_render_edges.npz")
    for key in z.files:
        name, kind, r, s = key.rsplit("_", 3)
        if kind == "img":
            yield name, int(r[1:]), int(s[1:])


_scenes = {}


def dev_scene(yrt, name):
    if name not in _scenes:
        s = yrt.load_scene(str(scene_path(f"edge_{name}")))
        yrt.build_bvh(s)
        _scenes[name] = (s, s.upload(0))
    return _scenes[name][1]


@pytest.mark.parametrize("algo", ALGOS)
@pytest.mark.parametrize("name,res,spp", list(_cases()))
def test_edge_scene_matches_reference_fixture(yrt, name, res, spp, algo):
    z = np.load(GOLDEN / "ref_render_edges.npz")
    ref = z[f"{name}_img_r{res}_s{spp}"]
    img, st = yrt.raytrace(dev_scene(yrt, name), (0.1, 0.1, 0.1), res, spp, return_stats=True, algorithm=algo)
    assert img.shape == ref.shape
    assert st["rays"] == int(z[f"{name}_rays_r{res}_s{spp}"])
    np.testing.assert_array_equal(img.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("algo", ["wavefront", "megakernel"])
def test_empty_scene_queries_find_nothing(yrt, algo):
    """intersect_first / intersect_any on a scene without instances: no hit, any ray"""
    rng = np.random.default_rng(5)
    rays = np.zeros((1000, 8), np.float32)
    rays[:, :3] = rng.uniform(-10, 10, (1000, 3))
    d = rng.normal(size=(1000, 3))
    rays[:, 3:6] = d / np.linalg.norm(d, axis=1, keepdims=True)
    rays[:, 6], rays[:, 7] = 1e-4, np.float32(3.4028235e38)
    ds = dev_scene(yrt, "empty")
    ds.set_trace_algorithm(algo)
    try:
        assert not yrt.intersect_first(ds, rays)["hit"].any()
        assert not yrt.intersect_any(ds, rays).any()
    finally:
        ds.set_trace_algorithm("wavefront")


@pytest.mark.parametrize("name", EDGE_SCENES)
def test_edge_scene_gpu_bvh_build_equals_reference(yrt, name, tmp_path):
    """the GPU BVH build on these scenes (no instances: one empty leaf) gives the
    reference's BVH bytes"""
    s = yrt.load_scene(str(scene_path(f"edge_{name}")))
    yrt.build_bvh(s, device=0)
    out = tmp_path / "gpu.yrtbvh"
    s.save_bvh(str(out))
    assert hashlib.sha256(gzip.open(out).read()).hexdigest() == digests()[f"edge_{name}"]["bvh_sha256"]


def test_upload_refuses_a_shape_mixing_primitive_kinds(yrt, tmp_path):
    """A group mixing `f` and `l` (test_library.write_mixed_obj) loads as the reference's
    one mixed shape, but the reference's answer for it is undefined (its traversal tests
    the line as a triangle, its shading reads the triangle hit as lines[ei], out of range;
    test_mixed_kind_group_is_the_references_and_its_lines_are_invisible): the upload refuses
    it with YRT_ERR_UNSUPPORTED and a message, instead of rendering something."""
    from test_library import write_mixed_obj

    s = yrt.load_scene(str(write_mixed_obj(tmp_path)))
    yrt.build_bvh(s)
    with pytest.raises(yrt.YrtError) as e:
        s.upload(0)
    assert "mixes primitive types" in str(e.value)


def test_mirror_depth_beyond_hbm_is_refused(yrt):
    """max_depth = INT_MAX (a natural 'unbounded'): the mirror levels' records (64 B per
    sample and level) cannot fit even at the smallest chunk, so the render is refused with
    YRT_ERR_UNSUPPORTED and the sizes, not hipErrorOutOfMemory; a deep but fitting depth
    renders, and equals the default depth's frame (in/refl's paths are at most 2 deep)"""
    s = yrt.load_scene(str(scene_path("refl")))
    yrt.build_bvh(s)
    ds = s.upload(0)
    with pytest.raises(yrt.YrtError) as e:
        yrt.raytrace(ds, (0.1, 0.1, 0.1), 24, 1, max_depth=2**31 - 1)
    assert "max_depth" in str(e.value) and "MiB" in str(e.value)
    deep = yrt.raytrace(ds, (0.1, 0.1, 0.1), 24, 1, max_depth=4096)
    base = yrt.raytrace(ds, (0.1, 0.1, 0.1), 24, 1)
    np.testing.assert_array_equal(deep.view(np.uint32), base.view(np.uint32))
