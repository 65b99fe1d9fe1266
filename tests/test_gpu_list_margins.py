"""The per-tile lists' margins under stress (VERDICT r4 "what's weak" 1). Both kinds of list
drop an instance-level box only when it lies outside a cone or hull plane by more than
eps = 1e-3 + 3e-5 M (M: the largest coordinate of the scene root, the camera and the light;
wavefront.hip make_hull / k_camera_lists). A false separation would silently change a
closest hit or an occlusion, so these scenes put the geometry where fp32 rounding is largest
relative to the margin:

- the grid scene scaled by 1e-3 (every box a few thousandths wide, eps dominated by 1e-3)
  and by 1e3 (coordinates ~1e4, eps dominated by the 3e-5 M term);
- the grid translated to (1e4, 0, 1e4), where the float spacing is ~1e-3 and every slab
  distance carries that rounding;
- a camera whose origin lies in the plane of a row of box tops, looking along the row, with
  the frame's middle tile boundary on the horizon: one cone plane of every tile at that
  boundary contains the top faces (the slab test's t values of those grazing rays are
  0 * inf and ties, scene.cpp:371-382), and the camera also sits in the side plane of a box
  column.

Each scene is rendered with the lists forced on and forced off; the two images must be
bitwise equal and equal the oracle (the reference's raytrace(), raytrace.cpp:213-254, through
the C restatement pinned to it). The list sums are printed so the log shows the lists were
built and used (pytest -s)."""
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


def _margin_scene(yrt, tmp_path, scale, offset, grazing, tag):
    """32 x 32 boxes on a floor (1 024 identity-rotation instances) and three point lights,
    every coordinate mapped p -> scale * p + offset (shapes scaled in their vertices, so the
    instance frames stay rotation-free translations)"""
    off = np.asarray(offset, np.float64)

    def P(p):
        return (scale * np.asarray(p, np.float64) + off).astype(np.float32)

    s = yrt.Scene.create()
    if grazing:
        # eye on the box tops' plane (y = 0.9) and on the side plane x = xs of box column 20,
        # looking along -z over the row
        xs = -25.6 + 1.6 * 20 + 0.4
        fr = np.r_[1, 0, 0, 0, 1, 0, 0, 0, 1, P([xs, 0.9, 30.0])]
        s.add_camera(fr.astype(np.float32), fovy=0.5, aspect=16 / 9, focus=22.0 * scale)
    else:
        fr = np.r_[1, 0, 0, 0, 0.8, -0.6, 0, 0.6, 0.8, P([0, 20, 26])]
        s.add_camera(fr.astype(np.float32), fovy=0.8, aspect=16 / 9, focus=30.0 * scale)
    m = s.add_material(kd=(0.6, 0.5, 0.4), ks=(0.2, 0.2, 0.2), rs=0.3)
    mf = s.add_material(kd=(0.4, 0.4, 0.4))
    q = scale * np.array([[-30, 0, -30], [30, 0, -30], [30, 0, 30], [-30, 0, 30]], np.float64)
    floor = s.add_shape(q.astype(np.float32), norm=[[0, 1, 0]] * 4, texcoord=[[0, 0]] * 4,
                        triangles=[[0, 1, 2], [0, 2, 3]])
    s.add_instance(np.r_[1, 0, 0, 0, 1, 0, 0, 0, 1, off].astype(np.float32), floor, mf)
    c = np.array([[x, y, z] for x in (-0.4, 0.4) for y in (0, 0.9) for z in (-0.4, 0.4)], np.float64)
    faces = [[0, 1, 3], [0, 3, 2], [4, 6, 7], [4, 7, 5], [0, 4, 5], [0, 5, 1],
             [2, 3, 7], [2, 7, 6], [0, 2, 6], [0, 6, 4], [1, 5, 7], [1, 7, 3]]
    box = s.add_shape((scale * c).astype(np.float32), norm=(c / np.linalg.norm(c, axis=1, keepdims=True)).astype(np.float32),
                      texcoord=[[0, 0]] * 8, triangles=faces)
    for i in range(32):
        for j in range(32):
            s.add_instance(np.r_[1, 0, 0, 0, 1, 0, 0, 0, 1, P([-25.6 + 1.6 * i, 0, -25.6 + 1.6 * j])], box, m)
    pt = s.add_shape([[0, 0, 0]], radius=[0.001 * scale], points=[0])
    for k, o in enumerate(([-8, 9, -6], [10, 12, 4], [2, 7, 14])):
        lm = s.add_material(ke=(60.0 * scale * scale, 50.0 * scale * scale, 40.0 * scale * scale))
        s.add_instance(np.r_[1, 0, 0, 0, 1, 0, 0, 0, 1, P(o)].astype(np.float32), pt, lm)
    path = tmp_path / f"margin_{tag}.yrtscene"
    s.save(str(path))
    yrt.build_bvh(s)
    return s, path


@pytest.mark.parametrize("tag,scale,offset,grazing", [
    ("scale_1e-3", 1e-3, (0, 0, 0), False),
    ("scale_1e3", 1e3, (0, 0, 0), False),
    ("translated_1e4", 1.0, (1e4, 0, 1e4), False),
    ("grazing", 1.0, (0, 0, 0), True),
    ("grazing_translated_1e4", 1.0, (1e4, 0, 1e4), True),
])
def test_list_margins_on_off_equal_oracle(yrt, tmp_path, tag, scale, offset, grazing):
    s, path = _margin_scene(yrt, tmp_path, scale, offset, grazing, tag)
    ds = s.upload(0)
    res, spp = 96, 4  # 96 rows: the horizon (v = 0.5) is the boundary of tile rows 5 and 6
    out = {}
    for mode in ("on", "off"):
        ds.set_tile_lists(mode)
        img, st = yrt.raytrace(ds, (0.1, 0.1, 0.1), res, spp, return_stats=True)
        out[mode] = (img, st, ds.tile_lists())
    (on, st_on, l_on), (off, st_off, l_off) = out["on"], out["off"]
    print(f"{tag}: lists on {l_on}")
    assert l_on["camera"] and l_on["bundles"], l_on
    assert l_on["camera_lists"] > 0 and l_on["bundle_lists"] > 0
    assert not l_off["camera"] and not l_off["bundles"]
    np.testing.assert_array_equal(on.view(np.uint32), off.view(np.uint32))
    assert st_on == st_off and st_on["shadow_rays"] > 0
    ref, n, trunc = Oracle(str(path)).render(res, spp)
    assert trunc == 0 and n == st_on["rays"]
    differ = int(np.sum(on.view(np.uint32) != ref.view(np.uint32)))
    print(f"{tag}: {differ} of {on.size} channels not bit-exact vs oracle")
    assert close_mask(on, ref).all()
    assert np.mean(on.view(np.uint32) == ref.view(np.uint32)) > 0.99
