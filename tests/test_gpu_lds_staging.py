"""LDS staging of the instance tree's top (yrt_scene_set_lds_staging; the north_star's "hot
node tiles staged in LDS"): the persistent closest-hit grid copies the first
YRT_PRIMARY_LDS_RECORDS camera-relative spine records into LDS once per block and its walk
reads them from there (packet_trace.h first_descend); the persistent any-hit grid does the
same with the first YRT_SHADOW_LDS_RECORDS 4-wide records (wide_descend) on scenes that
have that many. Only where a record is read from changes, so the image and the work counts
are those of the unstaged walks (tile lists off: the staging turns them off), and the image
equals the oracle (the reference's raytrace(), src/raytrace.cpp:213-254, through the C
restatement)."""
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


def render(yrt, ds, staged, res, spp, lists="off"):
    ds.set_tile_lists(lists)
    ds.set_lds_staging(staged)
    img, st = yrt.raytrace(ds, (0.1, 0.1, 0.1), res, spp, return_stats=True)
    return img, st, ds.lds_staging(), ds.tile_lists()


@pytest.mark.parametrize("name,res,spp,any_hit", [
    ("instance10000", 90, 8, True),   # 160x90, 64 spp: the bottom tile row cut by the frame
    ("instance1k", 120, 5, None),
    ("instance100k", 72, 8, True),    # the instance tree deeper than the staged top
    ("refl", 96, 3, False),           # mirror levels; 5 instances: the whole tree staged
    ("simple", 64, 2, False),         # textures
])
def test_staged_walks_same_image_as_oracle(yrt, name, res, spp, any_hit):
    ds = host(yrt, name).upload(0)
    off, st_off, s_off, _ = render(yrt, ds, False, res, spp)
    on, st_on, s_on, l_on = render(yrt, ds, True, res, spp)
    print(f"{name}: staged {s_on}")
    assert s_off == {"closest_hit": False, "any_hit": False}
    assert s_on["closest_hit"], s_on
    if any_hit is not None:
        assert s_on["any_hit"] == any_hit, s_on
    assert not l_on["camera"] and not l_on["bundles"], l_on
    np.testing.assert_array_equal(on.view(np.uint32), off.view(np.uint32))
    assert st_on == st_off
    ref, n, trunc = Oracle(name).render(res, spp)
    assert trunc == 0 and n == st_on["rays"]
    differ = int(np.sum(on.view(np.uint32) != ref.view(np.uint32)))
    print(f"{name} {res}p {spp}x{spp} staged: {differ} of {on.size} channels not bit-exact vs oracle")
    assert close_mask(on, ref).all()
    assert np.mean(on.view(np.uint32) == ref.view(np.uint32)) > 0.99


def test_staging_turns_the_lists_off_and_back(yrt):
    """with the lists forced on, staging wins (no lists built); turning it off restores them;
    the three images are the same"""
    ds = host(yrt, "instance10000").upload(0)
    lists, _, s0, l0 = render(yrt, ds, False, 120, 4, lists="on")
    staged, _, s1, l1 = render(yrt, ds, True, 120, 4, lists="on")
    again, _, s2, l2 = render(yrt, ds, False, 120, 4, lists="on")
    assert l0["camera"] and l0["bundles"] and not s0["closest_hit"]
    assert not l1["camera"] and not l1["bundles"] and s1["closest_hit"] and s1["any_hit"]
    assert l2["camera"] and l2["bundles"] and not s2["closest_hit"]
    np.testing.assert_array_equal(lists.view(np.uint32), staged.view(np.uint32))
    np.testing.assert_array_equal(lists.view(np.uint32), again.view(np.uint32))


def test_staged_c4_frame_equals_default(yrt):
    """the c4 frame (instance10000, 1920x1080, 8x8 spp) with the staged walks equals the
    default render's (tile lists on), bit for bit -- the frame test_full_size_c4_properties
    compares with the oracle"""
    ds = host(yrt, "instance10000").upload(0)
    base, st_b, _, l_b = render(yrt, ds, False, 1080, 8, lists="auto")
    staged, st_s, s_s, _ = render(yrt, ds, True, 1080, 8, lists="auto")
    assert l_b["camera"] and s_s == {"closest_hit": True, "any_hit": True}
    np.testing.assert_array_equal(base.view(np.uint32), staged.view(np.uint32))
    assert st_b["rays"] == st_s["rays"]


def test_staging_argument_errors(yrt):
    from yocto_raytracing_amd import _native as N

    ds = host(yrt, "basic").upload(0)
    assert ds.lds_staging() == {"closest_hit": False, "any_hit": False}
    assert N.lib.yrt_scene_set_lds_staging(ds.handle, 2) == 1  # YRT_ERR_INVALID_ARG
    assert N.lib.yrt_scene_lds_staging(ds.handle, None) == 1
