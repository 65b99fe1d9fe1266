"""Shadow rays whose light term is exactly zero are not traced (wavefront.hip light_term_zero,
YRT_SHADOW_CULL): the light's term in shade() (raytrace.cpp:133-183) is +-0 for a hit facing
away from the light on a material without specular (class 1) or with an exponent high enough
that pow(max(0, n.h), ns) is exactly 0 (classes >= 2), so the occlusion cannot change the
pixel. These scenes put every material class, and the cases that must NOT be culled, in one
frame, and compare with the oracle (the reference's raytrace() through the C restatement):

- matte (Ks = 0), glossy with ns ~ 1e6 (rs = 0), ns ~ 245 (rs = 0.3), low ns (rs = 0.9,
  never culled), a huge Kd (|Kd| > 2^20, never culled), and textured Kd / Ks (the texture
  factor in [0, 1] scales a term that is already +-0);
- a light under the floor (the whole floor faces away from it), a light 1e-3 off a box face
  (short shadow rays, a large ke / r^2) and a light inside a box (every face of that box
  faces away from it, and its shadow rays start inside the box);
- a line shape (always traced: its lighting uses sqrt(1 - |n.l|), not max(0, n.l));
- the camera sees back faces of boxes and the floor from above.

Each frame is rendered with the tile lists forced on (the persistent any-hit grid: whole waves
are culled) and off (the one-wave-block kernel: single lanes are culled); both must equal
each other and the oracle. The cull must leave the image bit for bit as tracing every ray does:
the instrumented count_work pass walks every shadow ray (no cull), and its image must equal the
default render's exactly, not just within the oracle tolerance. yrt_stats.shadow_rays_culled
reports how many rays were answered without a walk: > 0 on these scenes, 0 on the count pass,
and walked + culled = the reference's count."""
from __future__ import annotations

import numpy as np
import pytest

from helpers import Oracle, close_mask

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def yrt():
    import yocto_raytracing_amd as y

    if not y.device_count():
        pytest.fail("no GPU visible: the -m gpu suite needs one")
    return y


def _cull_scene(yrt, tmp_path, tag, near_light):
    s = yrt.Scene.create()
    fr = np.r_[1, 0, 0, 0, 0.8, -0.6, 0, 0.6, 0.8, [0.5, 9.0, 13.0]]
    s.add_camera(fr.astype(np.float32), fovy=0.9, aspect=16 / 9, focus=15.0)
    mats = [
        s.add_material(kd=(0.6, 0.5, 0.4)),                                # class 1
        s.add_material(kd=(0.5, 0.6, 0.4), ks=(0.04, 0.04, 0.04), rs=0.0),  # ns 1e6
        s.add_material(kd=(0.4, 0.5, 0.6), ks=(0.2, 0.2, 0.2), rs=0.3),    # ns ~245
        s.add_material(kd=(0.6, 0.6, 0.3), ks=(0.5, 0.4, 0.3), rs=0.9),    # ns ~1: never culled
        s.add_material(kd=(3e6, 0.2, 0.2)),                                # |Kd| > 2^20: never culled
        s.add_material(kd=(0.3, 0.6, 0.6), ks=(0.3, 0.3, 0.3), rs=0.05),   # ns ~3.2e5
    ]
    rng = np.random.default_rng(5)
    tex = s.add_texture(rng.integers(0, 256, size=(8, 8, 4), dtype=np.uint8))
    mats.append(s.add_material(kd=(0.7, 0.7, 0.7), kd_txt=tex))                                # class 1, textured
    mats.append(s.add_material(kd=(0.7, 0.6, 0.5), ks=(0.1, 0.1, 0.1), rs=0.1, kd_txt=tex, ks_txt=tex))  # ns ~2e4
    mf = s.add_material(kd=(0.4, 0.4, 0.4))
    q = np.array([[-12, 0, -12], [12, 0, -12], [12, 0, 12], [-12, 0, 12]], np.float32)
    floor = s.add_shape(q, norm=[[0, 1, 0]] * 4, texcoord=[[0, 0]] * 4, triangles=[[0, 1, 2], [0, 2, 3]])
    s.add_instance(np.r_[1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0].astype(np.float32), floor, mf)
    c = np.array([[x, y, z] for x in (-0.6, 0.6) for y in (0, 1.2) for z in (-0.6, 0.6)], np.float64)
    faces = [[0, 1, 3], [0, 3, 2], [4, 6, 7], [4, 7, 5], [0, 4, 5], [0, 5, 1],
             [2, 3, 7], [2, 7, 6], [0, 2, 6], [0, 6, 4], [1, 5, 7], [1, 7, 3]]
    # per-face normals would need split vertices: smooth corner normals, as the margin scenes
    box = s.add_shape(c.astype(np.float32), norm=(c / np.linalg.norm(c, axis=1, keepdims=True)).astype(np.float32),
                      texcoord=[[0, 0]] * 8, triangles=faces)
    k = 0
    for i in range(6):
        for j in range(6):
            s.add_instance(np.r_[1, 0, 0, 0, 1, 0, 0, 0, 1, -7.5 + 3 * i, 0, -7.5 + 3 * j].astype(np.float32), box,
                           mats[k % len(mats)])
            k += 1
    # a line shape on the floor
    lines = s.add_shape(np.array([[-9, 0.3, 9], [9, 0.3, 9], [-9, 0.3, 8], [9, 0.3, 8]], np.float32),
                        norm=[[0, 1, 0]] * 4, texcoord=[[0, 0]] * 4, radius=[0.2] * 4, lines=[[0, 1], [2, 3]])
    s.add_instance(np.r_[1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0].astype(np.float32), lines, mats[0])
    pt = s.add_shape([[0, 0, 0]], radius=[0.001], points=[0])
    lights = [[-6, 8, -3], [5, -3, 2], [-1.5 + 0.0, 0.6, -4.5]]  # above; under the floor; inside a box
    if near_light:
        lights.append([4.5 + 0.6 + 1e-3, 0.6, 1.5])  # almost on a box face (x = 4.5 + 0.6)
    for o in lights:
        lm = s.add_material(ke=(40.0, 35.0, 30.0))
        s.add_instance(np.r_[1, 0, 0, 0, 1, 0, 0, 0, 1, o].astype(np.float32), pt, lm)
    path = tmp_path / f"cull_{tag}.yrtscene"
    s.save(str(path))
    yrt.build_bvh(s)
    return s, path


@pytest.mark.parametrize("near_light", [False, True])
def test_shadow_cull_equals_oracle(yrt, tmp_path, near_light):
    s, path = _cull_scene(yrt, tmp_path, f"near{int(near_light)}", near_light)
    ds = s.upload(0)
    res, spp = 96, 4
    out = {}
    for mode in ("on", "off"):
        ds.set_tile_lists(mode)
        img, st = yrt.raytrace(ds, (0.1, 0.1, 0.1), res, spp, return_stats=True)
        out[mode] = (img, st)
    (on, st_on), (off, st_off) = out["on"], out["off"]
    np.testing.assert_array_equal(on.view(np.uint32), off.view(np.uint32))
    assert st_on == st_off
    # culled rays exist here, and the count pass (every shadow ray walked) gives the same bits
    assert 0 < st_on["shadow_rays_culled"] < st_on["shadow_rays"]
    for mode in ("on", "off"):
        ds.set_tile_lists(mode)
        walked, st_w = yrt.raytrace(ds, (0.1, 0.1, 0.1), res, spp, return_stats=True, count_work=True)
        np.testing.assert_array_equal(walked.view(np.uint32), on.view(np.uint32))
        assert st_w["shadow_rays_culled"] == 0 and st_w["rays"] == st_on["rays"]
        assert st_w["shadow_rays"] == st_on["shadow_rays"]
    ref, n, trunc = Oracle(str(path)).render(res, spp)
    assert trunc == 0 and n == st_on["rays"]  # culled rays are counted: the reference's count
    walked_rays = st_on["rays"] - st_on["shadow_rays_culled"]
    assert walked_rays + st_on["shadow_rays_culled"] == n and walked_rays < n
    differ = int(np.sum(on.view(np.uint32) != ref.view(np.uint32)))
    print(f"near_light={near_light}: {differ} of {on.size} channels not bit-exact vs oracle")
    assert close_mask(on, ref).all()
    assert np.mean(on.view(np.uint32) == ref.view(np.uint32)) > 0.99


def test_shadow_cull_counts_at_c4_scale(yrt):
    """instance10000 at 1080p, 1 spp (the c4 frame's geometry): culled rays are reported, the
    count pass walks every one of them, and both images are the same bits"""
    scn = yrt.load_scene(str(__import__("helpers").scene_path("instance10000")))
    yrt.build_bvh(scn)
    ds = scn.upload(0)
    img, st = yrt.raytrace(ds, (0.1, 0.1, 0.1), 1080, 1, return_stats=True)
    walked, st_w = yrt.raytrace(ds, (0.1, 0.1, 0.1), 1080, 1, return_stats=True, count_work=True)
    np.testing.assert_array_equal(walked.view(np.uint32), img.view(np.uint32))
    assert st["rays"] == st_w["rays"] == 4 * st["camera_samples"]  # the reference's 4.000 per sample
    assert st_w["shadow_rays_culled"] == 0
    frac = st["shadow_rays_culled"] / st["shadow_rays"]
    print(f"instance10000 1080p 1 spp: {st['shadow_rays_culled']} of {st['shadow_rays']} shadow rays culled "
          f"({frac:.3f})")
    assert 0.0 < frac < 1.0
