"""The list builders' instance masks (YRT_INSTANCE_MASKS): k_camera_lists
and k_bundle_lists mark the instances of a listed leaf whose world box (dev_scene_view ibox)
their cone or hull excludes, drop leaves whose every instance is excluded, and the walks pass
over the marked instances. Exact only if the world box holds everything the instance's
root box test in instance space can pass -- so these scenes mix what the box construction
has to get right:

- rotated instances (orthonormal frames about several axes: the box is the root box's
  corners through (R^T)^-1);
- scaled and sheared instances (non-orthonormal frames: NaN boxes, never excluded, because
  the walk reuses the world tmax along the renormalised local direction);
- instances whose shape sits far from its local origin, and a shape with an empty BVH;
- dense clusters, so that leaves hold several instances and rays pass between them;
- a camera inside the instance cloud, one far outside it, one far away with a narrow view of
  the dense cluster (its tiles' lists reach single leaves), and lights among the
  instances.

Each frame is rendered with the lists forced on (masks built) and off (no lists, no masks);
both must be bit-identical and equal the oracle (the reference's raytrace(),
raytrace.cpp:213-254, through the C restatement). The masks must also have fired: the lists
report how many instances their cones and hulls excluded (yrt_scene_tile_list_masks), and a
test whose masks never excluded anything would not test them."""
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


def _rot(axis, a):
    c, s = np.cos(a), np.sin(a)
    if axis == 0:
        return np.array([[1, 0, 0], [0, c, -s], [0, s, c]])
    if axis == 1:
        return np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])
    return np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]])


def _frame(R, o):
    # columns of R are the frame's axes x, y, z
    return np.r_[R[:, 0], R[:, 1], R[:, 2], o].astype(np.float32)


def _mask_scene(yrt, tmp_path, camera):
    rng = np.random.default_rng(17)
    s = yrt.Scene.create()
    if camera == "far":
        s.add_camera(_frame(_rot(0, -0.5), [0.0, 60.0, 110.0]), fovy=0.25, aspect=16 / 9, focus=120.0)
    elif camera == "zoom":  # far away with a narrow view of the dense cluster: a tile's cone meets few leaves
        s.add_camera(_frame(_rot(0, -0.56), [2.0, 40.0, 60.0]), fovy=0.06, aspect=16 / 9, focus=74.0)
    else:  # inside the cloud
        s.add_camera(_frame(_rot(1, 0.3) @ _rot(0, -0.2), [1.0, 2.5, 6.0]), fovy=1.0, aspect=16 / 9, focus=8.0)
    mats = [s.add_material(kd=(0.6, 0.5, 0.4)),
            s.add_material(kd=(0.4, 0.6, 0.5), ks=(0.2, 0.2, 0.2), rs=0.3),
            s.add_material(kd=(0.5, 0.4, 0.6), ks=(0.04, 0.04, 0.04), rs=0.0)]
    q = np.array([[-30, 0, -30], [30, 0, -30], [30, 0, 30], [-30, 0, 30]], np.float32)
    floor = s.add_shape(q, norm=[[0, 1, 0]] * 4, texcoord=[[0, 0]] * 4, triangles=[[0, 1, 2], [0, 2, 3]])
    s.add_instance(_frame(np.eye(3), [0, 0, 0]), floor, mats[0])
    c = np.array([[x, y, z] for x in (-0.4, 0.4) for y in (0, 0.8) for z in (-0.3, 0.3)], np.float64)
    faces = [[0, 1, 3], [0, 3, 2], [4, 6, 7], [4, 7, 5], [0, 4, 5], [0, 5, 1],
             [2, 3, 7], [2, 7, 6], [0, 2, 6], [0, 6, 4], [1, 5, 7], [1, 7, 3]]
    nrm = (c / np.linalg.norm(c, axis=1, keepdims=True)).astype(np.float32)
    box = s.add_shape(c.astype(np.float32), norm=nrm, texcoord=[[0, 0]] * 8, triangles=faces)
    # the same box far from its local origin (its root box does not contain the origin)
    offbox = s.add_shape((c + [3.0, 0.5, -2.0]).astype(np.float32), norm=nrm, texcoord=[[0, 0]] * 8, triangles=faces)
    empty = s.add_shape([[0, 0, 0]], triangles=np.zeros((0, 3), np.int32))
    for k in range(900):
        o = rng.uniform([-14, 0, -14], [14, 3, 14])
        if k % 9 == 0:  # a dense cluster around some instances
            o = np.array([2.0, 0.5, -3.0]) + rng.normal(scale=0.6, size=3)
        kind = k % 6
        if kind == 0:
            R = np.eye(3)
        elif kind in (1, 2):
            R = _rot(kind - 1, rng.uniform(0, 6.28)) @ _rot(2, rng.uniform(0, 6.28))
        elif kind == 3:
            R = _rot(1, rng.uniform(0, 6.28)) * rng.uniform(0.5, 1.6)  # scaled: NaN box
        elif kind == 4:
            R = np.array([[1, 0.3, 0], [0, 1, 0], [0, 0.2, 1]]) @ _rot(1, rng.uniform(0, 6.28))  # sheared
        else:
            R = _rot(0, rng.uniform(0, 6.28))
        shape = offbox if k % 7 == 0 else box
        s.add_instance(_frame(R, o), shape, mats[k % 3])
    s.add_instance(_frame(np.eye(3), [0, 1, 0]), empty, mats[0])
    pt = s.add_shape([[0, 0, 0]], radius=[0.001], points=[0])
    for o in ([-6, 9, -4], [8, 12, 5], [1.5, 1.2, -2.5]):  # the last one among the instances
        lm = s.add_material(ke=(40.0, 35.0, 30.0))
        s.add_instance(_frame(np.eye(3), o), pt, lm)
    path = tmp_path / f"masks_{camera}.yrtscene"
    s.save(str(path))
    yrt.build_bvh(s)
    return s, path


@pytest.mark.parametrize("camera", ["near", "far", "zoom"])
def test_instance_masks_on_off_equal_oracle(yrt, tmp_path, camera):
    s, path = _mask_scene(yrt, tmp_path, camera)
    ds = s.upload(0)
    res, spp = 96, 4
    out = {}
    for mode in ("on", "off"):
        ds.set_tile_lists(mode)
        img, st = yrt.raytrace(ds, (0.1, 0.1, 0.1), res, spp, return_stats=True)
        out[mode] = (img, st, ds.tile_lists())
    (on, st_on, l_on), (off, st_off, _) = out["on"], out["off"]
    print(f"camera={camera}: lists on {l_on}")
    assert l_on["camera"] and l_on["bundles"], l_on
    # the masks excluded instances (else the on/off comparison proves nothing): the bundles' in
    # every frame; the camera lists' in the zoomed view, whose tiles' cones reach single leaves
    # (in the near and far views every tile's cone meets more leaves than a list holds, its
    # frontier is 32 subtrees, and only a listed leaf carries skip bits)
    assert l_on["bundle_instances_masked"] > 0, l_on
    if camera == "zoom":
        assert l_on["camera_instances_masked"] > 0 and l_on["camera_entries"] < 32 * l_on["camera_lists"], l_on
    np.testing.assert_array_equal(on.view(np.uint32), off.view(np.uint32))
    assert st_on == st_off and st_on["shadow_rays"] > 0
    ref, n, trunc = Oracle(str(path)).render(res, spp)
    assert trunc == 0 and n == st_on["rays"]
    differ = int(np.sum(on.view(np.uint32) != ref.view(np.uint32)))
    print(f"camera={camera}: {differ} of {on.size} channels not bit-exact vs oracle")
    assert close_mask(on, ref).all()
    assert np.mean(on.view(np.uint32) == ref.view(np.uint32)) > 0.99
