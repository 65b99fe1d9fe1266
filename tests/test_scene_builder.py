"""The in-memory scene builder (yrt_host_scene_add_*, include/yrt.h): the reference's
scene* (scene.h:26-155) handed over field by field instead of through a file."""
import gzip
import sys

import numpy as np
import pytest

from helpers import GOLDEN, digests, scene_path

sys.path.insert(0, str(GOLDEN))


@pytest.fixture(scope="module")
def yrt():
    import yocto_raytracing_amd as y

    return y


def tiny(yrt):
    s = yrt.Scene.create()
    s.add_camera(np.r_[1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 1, 5], fovy=0.5, aspect=1.5, focus=5)
    m = s.add_material(kd=(0.5, 0.5, 0.5))
    tri = s.add_shape([[-1, 0, -1], [1, 0, -1], [0, 0, 1]], norm=[[0, 1, 0]] * 3, texcoord=[[0, 0]] * 3,
                      triangles=[[0, 1, 2]])
    s.add_instance(np.r_[1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0], tri, m)
    return s, m, tri


def test_builder_counts_and_roundtrip(yrt, tmp_path):
    s, m, tri = tiny(yrt)
    info = s.info()
    assert (info["cameras"], info["materials"], info["shapes"], info["instances"], info["triangles"]) == (1, 1, 1, 1, 1)
    yrt.build_bvh(s)
    assert s.info()["bvh_nodes"] == 1
    a = tmp_path / "a.yrtscene"
    s.save(str(a))
    b = tmp_path / "b.yrtscene"
    yrt.load_scene(str(a)).save(str(b))
    assert gzip.open(a).read() == gzip.open(b).read()
    assert s.image_size(100) == (150, 100)


def test_builder_rejects_bad_input(yrt):
    s, m, tri = tiny(yrt)
    with pytest.raises(yrt.YrtError, match="invalid argument"):
        s.add_shape([[0, 0, 0]], triangles=[[0, 1, 2]])  # index past the vertex array
    with pytest.raises(yrt.YrtError, match="unsupported"):
        s.add_shape([[0, 0, 0], [1, 0, 0]], radius=[1, 1], points=[0], lines=[[0, 1]])
    with pytest.raises(yrt.YrtError, match="invalid argument"):
        s.add_shape([[0, 0, 0], [1, 0, 0]], lines=[[0, 1]])  # lines need radii
    with pytest.raises(yrt.YrtError, match="invalid argument"):
        s.add_material(kd_txt=3)  # no such texture
    with pytest.raises(yrt.YrtError, match="invalid argument"):
        s.add_instance(np.eye(4)[:, :3].reshape(-1), 7, m)  # no such shape
    with pytest.raises(ValueError):
        s.add_shape([[0, 0, 0], [1, 0, 0]], norm=[[0, 1, 0]], radius=[1, 1], points=[0, 1])
    assert s.info()["shapes"] == 1  # nothing half-added


def test_synthetic_fixture_is_reproducible(yrt, tmp_path):
    """tests/golden/scenes/lines.yrtscene is exactly what make_synthetic.build_scene
    builds, and its digest is the one the reference read back (ref_digests.json)."""
    import hashlib

    from make_synthetic import build_scene

    out = tmp_path / "lines.yrtscene"
    build_scene(out)
    assert gzip.open(out).read() == gzip.open(scene_path("lines")).read()
    assert hashlib.sha256(gzip.open(out).read()).hexdigest() == digests()["lines"]["scene_sha256"]


def test_nan_bounded_instance_is_refused_by_the_build(yrt):
    """An instance whose box carries a NaN (a shape whose root box keeps a NaN vertex: the
    reference's ?: folds keep a NaN that comes last) makes the instance level's centroid box
    NaN, every midpoint comparison false and the split empty: the reference's make_node then
    recurses forever (scene.cpp:572-603, its assert compiled out); the build refuses it. So no
    buildable scene has a NaN-bounded instance-level leaf, and the candidate lists never list
    one (wavefront.hip k_bundle_lists still folds a chain box NaN-sticky, so a NaN bound could
    only widen it)."""
    s, m, tri = tiny(yrt)
    bad = s.add_shape(np.array([[0, 0.2, 0], [0.3, 0.2, 0], [0.1, np.nan, 0.1]], np.float32),
                      norm=[[0, 1, 0]] * 3, texcoord=[[0, 0]] * 3, triangles=[[0, 1, 2]])
    for k in range(8):
        s.add_instance(np.r_[1, 0, 0, 0, 1, 0, 0, 0, 1, k, 0, 0].astype(np.float32), tri, m)
    s.add_instance(np.r_[1, 0, 0, 0, 1, 0, 0, 0, 1, 3, 0, 1].astype(np.float32), bad, m)
    with pytest.raises(yrt.YrtError, match="degenerate centroids"):
        yrt.build_bvh(s)
