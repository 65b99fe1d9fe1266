"""GPU: build_bvh with the tree construction on the GPU (bvh_gpu.hip,
yrt_host_scene_build_bvh_gpu) produces the reference's nodes and leaf order byte for
byte: against the host builder (itself pinned to the reference's BVH digests) on every
scene, against the reference's digests directly, and on inputs where the reference's
sequential ?: folds are order sensitive (signed-zero ties, NaN coordinates, coincident
centroids, a point/line shape, an empty shape)."""
import gzip
import hashlib

import numpy as np
import pytest

from helpers import SCENE_NAMES, digests, scene_path

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def yrt():
    import yocto_raytracing_amd as y

    if y.device_count() < 1:
        pytest.fail("no GPU visible: the -m gpu suite must run on the MI355X box")
    return y


def bvh_bytes(s, tmp_path, tag):
    out = tmp_path / f"{tag}.yrtbvh"
    s.save_bvh(str(out))
    return gzip.open(out).read()


@pytest.mark.parametrize("name", SCENE_NAMES)
def test_gpu_build_equals_reference_bvh(yrt, name, tmp_path):
    host = yrt.load_scene(str(scene_path(name)))
    yrt.build_bvh(host)
    gpu = yrt.load_scene(str(scene_path(name)))
    ms = yrt.build_bvh(gpu, device=0)
    assert ms is not None and ms > 0
    a, b = bvh_bytes(host, tmp_path, "host"), bvh_bytes(gpu, tmp_path, "gpu")
    assert a == b
    assert hashlib.sha256(b).hexdigest() == digests()[name]["bvh_sha256"]
    print(f"{name}: GPU build passes {ms:.3f} ms")


def synthetic(yrt, pos, tris=None, points=None, lines=None, radius=None, extra_empty=False):
    s = yrt.Scene.create()
    s.add_camera(np.r_[1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 1, 5], fovy=0.5, aspect=1.5, focus=5)
    m = s.add_material(kd=(0.5, 0.5, 0.5))
    sh = s.add_shape(pos, triangles=tris, points=points, lines=lines, radius=radius)
    rng = np.random.default_rng(7)
    for k in range(40):  # instances with coincident and signed-zero translations
        o = [(-0.0 if k % 3 == 0 else 0.0) + (k // 7), 0.0 if k % 2 else -0.0, float(k % 5)]
        s.add_instance(np.r_[1, 0, 0, 0, 1, 0, 0, 0, 1, o], sh, m)
    if extra_empty:
        e = s.add_shape([[0, 0, 0]], triangles=np.zeros((0, 3), np.int32))
        s.add_instance(np.r_[1, 0, 0, 0, 1, 0, 0, 0, 1, rng.normal(size=3)], e, m)
    return s


def both_builds(yrt, make, tmp_path):
    host, gpu = make(), make()
    err_h = err_g = None
    try:
        yrt.build_bvh(host)
    except yrt.YrtError as e:
        err_h = str(e)
    try:
        yrt.build_bvh(gpu, device=0)
    except yrt.YrtError as e:
        err_g = str(e)
    assert (err_h is None) == (err_g is None), (err_h, err_g)
    if err_h is None:
        assert bvh_bytes(host, tmp_path, "h") == bvh_bytes(gpu, tmp_path, "g")
    return err_h


def test_gpu_build_signed_zero_ties(yrt, tmp_path):
    # a grid of triangles whose vertices alternate -0.0 and +0.0 on every axis: the node
    # boxes' zero signs depend on the fold order
    n = 24
    pos, tris = [], []
    for i in range(n):
        for j in range(n):
            z = -0.0 if (i + j) % 2 else 0.0
            pos += [[i * 0.5, z, j * 0.5], [i * 0.5 + 0.5, -z, j * 0.5], [i * 0.5, z, j * 0.5 + 0.5]]
            b = 3 * (i * n + j)
            tris.append([b, b + 1, b + 2])
    pos += [[-0.0, -0.0, -0.0], [0.0, 0.0, 0.0], [-0.0, 0.0, -0.0]]
    tris.append([len(pos) - 3, len(pos) - 2, len(pos) - 1])
    assert both_builds(yrt, lambda: synthetic(yrt, pos, tris=tris, extra_empty=True), tmp_path) is None


def test_gpu_build_nan_and_coincident(yrt, tmp_path):
    rng = np.random.default_rng(3)
    pos = rng.normal(size=(300, 3)).astype(np.float32)
    pos[17] = np.nan
    pos[40:60] = pos[40]  # coincident centroids
    tris = rng.integers(0, 300, size=(100, 3))
    tris[:20] = [40, 41, 42]
    both_builds(yrt, lambda: synthetic(yrt, pos, tris=tris), tmp_path)  # same result or same error


def test_gpu_build_points_and_lines(yrt, tmp_path):
    rng = np.random.default_rng(5)
    pos = rng.normal(size=(200, 3)).astype(np.float32)
    r = np.abs(rng.normal(size=200)).astype(np.float32) * 0.01
    assert both_builds(yrt, lambda: synthetic(yrt, pos, points=np.arange(200), radius=r), tmp_path) is None
    lines = np.stack([np.arange(199), np.arange(1, 200)], 1)
    assert both_builds(yrt, lambda: synthetic(yrt, pos, lines=lines, radius=r), tmp_path) is None


def test_gpu_build_equal_num_unsupported(yrt):
    s = yrt.load_scene(str(scene_path("basic")))
    with pytest.raises(yrt.YrtError, match="unsupported"):
        yrt.build_bvh(s, equal_num=True, device=0)
