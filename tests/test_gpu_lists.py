"""The per-tile candidate lists of the render path: camera lists
(k_camera_lists, packet_first's list mode) and shadow bundles (k_bundle_lists). Lists are
an acceleration only: with them forced on, forced off, or in the default (auto) mode the
image is the same, and it equals the oracle (the reference's raytrace(),
src/raytrace.cpp:213-254) -- on ragged frames whose 8x8-pixel tiles are cut by the frame's
edge, sample counts whose 64-sample items straddle pixels, windows, lists that overflow
their capacity and fall back to the tree, rotated lights and more lights than a bundle
takes."""
from __future__ import annotations

import numpy as np
import pytest

from helpers import Oracle, close_mask, scene_path

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def yrt():
    import yocto_raytracing_amd as y

    if not y.device_count():
        pytest.fail("no GPU visible: the -m gpu suite needs one")
    return y


_hosts = {}


def host(yrt, name):
    if name not in _hosts:
        s = yrt.load_scene(str(scene_path(name)))
        yrt.build_bvh(s)
        _hosts[name] = s
    return _hosts[name]


def render(yrt, ds, mode, res, spp, window=None):
    ds.set_tile_lists(mode)
    img, st = yrt.raytrace(ds, (0.1, 0.1, 0.1), res, spp, window=window, return_stats=True)
    return img, st, ds.tile_lists()


def check_oracle(img, ref, what):
    differ = int(np.sum(img.view(np.uint32) != ref.view(np.uint32)))
    print(f"{what}: {differ} of {img.size} channels not bit-exact vs oracle")
    assert close_mask(img, ref).all()
    assert np.mean(img.view(np.uint32) == ref.view(np.uint32)) > 0.99


@pytest.mark.parametrize("name,res,spp", [
    ("instance10000", 90, 8),    # 160x90: the bottom tile row is cut by the frame
    ("instance10000", 37, 3),    # 66x37, 9 spp: 64-sample items straddle pixels
    ("instance10000", 200, 1),   # 1 spp: one item spans 64 pixels
    ("instance1k", 120, 5),
    ("instance100k", 72, 8),     # long lists: some overflow their capacity (tree fallback)
])
def test_lists_on_off_same_image_as_oracle(yrt, name, res, spp):
    ds = host(yrt, name).upload(0)
    on, st_on, l_on = render(yrt, ds, "on", res, spp)
    off, st_off, l_off = render(yrt, ds, "off", res, spp)
    assert l_on["camera"] and l_on["bundles"], l_on
    assert not l_off["camera"] and not l_off["bundles"], l_off
    assert l_on["camera_lists"] > 0 and l_on["bundle_lists"] > 0
    np.testing.assert_array_equal(on.view(np.uint32), off.view(np.uint32))
    assert st_on == st_off
    ref, n, trunc = Oracle(name).render(res, spp)
    assert trunc == 0 and n == st_on["rays"]
    check_oracle(on, ref, f"{name} {res}p {spp}x{spp} lists on")


def test_lists_on_in_a_window(yrt):
    """a window whose origin is not on the 8x8 tile grid: the tiles' cones follow the
    window's own pixels"""
    name, res, spp = "instance10000", 180, 4
    ds = host(yrt, name).upload(0)
    win = (37, 21, 101, 67)
    on, _, l_on = render(yrt, ds, "on", res, spp, window=win)
    off, _, _ = render(yrt, ds, "off", res, spp, window=win)
    assert l_on["camera"] and l_on["bundles"]
    np.testing.assert_array_equal(on.view(np.uint32), off.view(np.uint32))
    x0, y0, w, h = win
    ref, _, _ = Oracle(name).render(res, spp, rows=np.arange(y0, y0 + h), x0=x0, ncols=w)
    check_oracle(on, ref, "instance10000 window lists on")


def test_lists_auto(yrt):
    """auto builds both kinds of list on the instance scenes at c4 settings -- the camera lists
    are frontiers of at most camera_list_max entries, so none falls back to the tree -- and
    the image is the forced-off image (instance100k: 17.8 leaves per tile as leaf lists, which
    round 4's probe turned off; as frontiers they take its closest hit 26.6 -> 25.3 ms)"""
    for name in ("instance10000", "instance100k"):
        ds = host(yrt, name).upload(0)
        auto, _, la = render(yrt, ds, "auto", 1080, 8)
        assert la["camera"] and la["bundles"], (name, la)
        assert 0 < la["camera_entries"] <= 32 * la["camera_lists"], (name, la)
        print(name, la)
        off, _, _ = render(yrt, ds, "off", 1080, 8)
        np.testing.assert_array_equal(auto.view(np.uint32), off.view(np.uint32))
        del ds


def test_lists_auto_by_samples(yrt):
    """auto builds the lists from 9 samples per pixel (YRT_LISTS_MIN_SPP: their cost is per
    pixel tile, their gain per sample); below that it renders without them, the same image"""
    ds = host(yrt, "instance10000").upload(0)
    for s, used in ((1, False), (2, False), (3, True)):
        auto, _, la = render(yrt, ds, "auto", 180, s)
        assert la["camera"] == used, (s, la)
        on, _, _ = render(yrt, ds, "on", 180, s)
        np.testing.assert_array_equal(auto.view(np.uint32), on.view(np.uint32))


def _grid_scene(yrt, tmp_path, nlights, rotated_light):
    """16 x 16 boxes on a floor (an instance tree of well over 8 wide records) lit by point
    lights; optionally one light's frame rotated (its shadow rays leave p along
    R (pos0 - p) + o, raytrace.cpp:129-130: the bundle hull does not hold, so the bundles
    of that light walk the tree)"""
    s = yrt.Scene.create()
    s.add_camera(np.r_[1, 0, 0, 0, 0.8, -0.6, 0, 0.6, 0.8, 0, 14, 18], fovy=0.7, aspect=16 / 9, focus=22.0)
    m = s.add_material(kd=(0.6, 0.5, 0.4), ks=(0.2, 0.2, 0.2), rs=0.3)
    mf = s.add_material(kd=(0.4, 0.4, 0.4))
    floor = s.add_shape([[-20, 0, -20], [20, 0, -20], [20, 0, 20], [-20, 0, 20]], norm=[[0, 1, 0]] * 4,
                        texcoord=[[0, 0]] * 4, triangles=[[0, 1, 2], [0, 2, 3]])
    s.add_instance(np.r_[1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0], floor, mf)
    c = np.array([[x, y, z] for x in (-0.4, 0.4) for y in (0, 0.9) for z in (-0.4, 0.4)], np.float32)
    faces = [[0, 1, 3], [0, 3, 2], [4, 6, 7], [4, 7, 5], [0, 4, 5], [0, 5, 1],
             [2, 3, 7], [2, 7, 6], [0, 2, 6], [0, 6, 4], [1, 5, 7], [1, 7, 3]]
    box = s.add_shape(c, norm=c / np.linalg.norm(c, axis=1, keepdims=True), texcoord=[[0, 0]] * 8,
                      triangles=faces)
    for i in range(16):
        for j in range(16):
            s.add_instance(np.r_[1, 0, 0, 0, 1, 0, 0, 0, 1, -12 + 1.6 * i, 0, -12 + 1.6 * j], box, m)
    pt = s.add_shape([[0.5, 0.2, -0.3]], radius=[0.001], points=[0])
    rng = np.random.default_rng(5)
    for k in range(nlights):
        lm = s.add_material(ke=(40 + k, 40, 40 - k))
        o = rng.uniform([-10, 6, -10], [10, 12, 10])
        if rotated_light and k == 0:
            a = 0.7
            fr = np.r_[np.cos(a), 0, -np.sin(a), 0, 1, 0, np.sin(a), 0, np.cos(a), o]
        else:
            fr = np.r_[1, 0, 0, 0, 1, 0, 0, 0, 1, o]
        s.add_instance(fr.astype(np.float32), pt, lm)
    path = tmp_path / f"grid_{nlights}_{int(rotated_light)}.yrtscene"
    s.save(str(path))
    yrt.build_bvh(s)
    return s, path


@pytest.mark.parametrize("nlights,rotated,bundles", [(3, False, True), (3, True, True), (9, False, False)])
def test_lists_synthetic_lights(yrt, tmp_path, nlights, rotated, bundles):
    """a rotated light (its bundles fall back to the tree) and nine lights (more than the
    bundles take: no bundles at all, camera lists still on) give the oracle's image"""
    s, path = _grid_scene(yrt, tmp_path, nlights, rotated)
    ds = s.upload(0)
    res, spp = 144, 4
    on, st_on, l_on = render(yrt, ds, "on", res, spp)
    off, st_off, _ = render(yrt, ds, "off", res, spp)
    assert l_on["camera"] and l_on["bundles"] == bundles, l_on
    np.testing.assert_array_equal(on.view(np.uint32), off.view(np.uint32))
    assert st_on == st_off and st_on["shadow_rays"] > 0
    ref, n, _ = Oracle(str(path)).render(res, spp)
    assert n == st_on["rays"]
    check_oracle(on, ref, f"grid {nlights} lights rotated={rotated}")


def test_tile_lists_argument_errors(yrt):
    ds = yrt.DeviceScene(host(yrt, "instance1k"), 0)  # a handle of its own (upload() caches one)
    # a handle that has not rendered, and one whose renders never built lists, read back zeros
    assert ds.tile_lists() == {"camera": False, "bundles": False, "camera_entries": 0, "camera_lists": 0,
                               "bundle_entries": 0, "bundle_lists": 0, "camera_instances_masked": 0,
                               "bundle_instances_masked": 0}
    ds.set_tile_lists("off")
    yrt.raytrace(ds, (0.1, 0.1, 0.1), 90, 2)
    assert ds.tile_lists()["camera"] is False and ds.tile_lists()["camera_lists"] == 0
    with pytest.raises(KeyError):
        ds.set_tile_lists("sometimes")
    from yocto_raytracing_amd import _native as N

    assert N.lib.yrt_scene_set_tile_lists(ds.handle, 3) == 1  # YRT_ERR_INVALID_ARG
    assert N.lib.yrt_scene_set_tile_lists(None, 0) == 1  # YRT_ERR_INVALID_ARG


def test_lists_follow_the_view(yrt):
    """one scene handle rendered from each of instance10000's five cameras in turn and back
    to the first (`camera` selects scn->cameras[k]; the reference always takes the first,
    raytrace.cpp:225): each new view gets its own lists, and every frame -- auto, forced on
    or off -- equals the oracle's render from that camera"""
    name, res, spp = "instance10000", 180, 4
    ds = host(yrt, name).upload(0)
    orc = Oracle(name)
    for cam in (0, 1, 2, 3, 4, 0):
        ref, n, _ = orc.render(res, spp, camera=cam)
        imgs = []
        for mode in ("auto", "on", "off"):
            ds.set_tile_lists(mode)
            img, st = yrt.raytrace(ds, (0.1, 0.1, 0.1), res, spp, camera=cam, return_stats=True)
            assert st["rays"] == n
            imgs.append(img)
        for img in imgs[1:]:
            np.testing.assert_array_equal(img.view(np.uint32), imgs[0].view(np.uint32))
        check_oracle(imgs[0], ref, f"instance10000 camera {cam}")

