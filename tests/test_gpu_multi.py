"""GPU: the multi-device boundary (yrt_multi_*, include/yrt.h), the device tonemap and
save path, and the BASELINE configs at their full stated sizes (c1, c3, c5).

Multi-device: one host process, the scene replicated per device, 8-row bands dealt
round-robin, gathered to devices[0] (RCCL between distinct devices; plain copies when a
device is listed more than once, which is how the band geometry and reassembly are
rehearsed on a one-GPU box) -- the assembled frame must equal the single-device render
bit for bit. The RCCL transport itself is exercised at n = 1 (YRT_MULTI_TRANSPORT=rccl:
the root's shard goes through an RCCL self send/receive); N > 1 over xGMI is the
driver's 8-GPU run.
"""
import numpy as np
import pytest

from helpers import GOLDEN, ROOT, Oracle, assert_same_floats, close_mask, psnr_u8, scene_path, tonemap_ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def yrt():
    import yocto_raytracing_amd as y

    if y.device_count() < 1:
        pytest.fail("no GPU visible: the -m gpu suite must run on the MI355X box")
    return y


_scenes = {}


def host_scene(yrt, name):
    if name not in _scenes:
        s = yrt.load_scene(str(scene_path(name)))
        yrt.build_bvh(s)
        _scenes[name] = s
    return _scenes[name]


# (scene, resolution, spp axis): 100 and 90 rows leave a partial last band (100 % 8, 90 % 8)
MULTI_CASES = [("instance10000", 100, 2), ("refl", 90, 3), ("simple", 64, 2), ("lines", 120, 2)]


@pytest.mark.parametrize("devices", [(0,), (0, 0), (0, 0, 0), (0, 0, 0, 0, 0, 0, 0, 0)])
@pytest.mark.parametrize("name,res,spp", MULTI_CASES)
def test_multi_render_equals_single_device(yrt, name, res, spp, devices):
    s = host_scene(yrt, name)
    single, st1 = yrt.raytrace(s.upload(0), (0.1, 0.1, 0.1), res, spp, return_stats=True)
    ms = yrt.MultiScene(s, devices)
    assert ms.transport == "copy"  # a device listed more than once (or one device)
    p = yrt.render_params(0.1, res, spp)
    img = np.full_like(single, np.nan)
    ms.render_into(p, img.ctypes.data)
    np.testing.assert_array_equal(img.view(np.uint32), single.view(np.uint32))
    st = ms.last_stats()
    assert st == st1, {k: (st[k], st1[k]) for k in st if st[k] != st1.get(k)}
    t = ms.last_timings()
    assert t["render_ms"] > 0 and t["gather_ms"] >= 0
    ms.close()


def test_multi_render_rccl_transport(yrt, monkeypatch):
    """the RCCL path (dlopen'd librccl, ncclCommInitAll, grouped ncclSend/ncclRecv to the
    root, strided reassembly) at n = 1: a self send/receive on this box"""
    monkeypatch.setenv("YRT_MULTI_TRANSPORT", "rccl")
    s = host_scene(yrt, "instance10000")
    single = yrt.raytrace(s.upload(0), (0.1, 0.1, 0.1), 100, 2)
    ms = yrt.MultiScene(s, [0])
    assert ms.transport == "rccl"
    img = np.zeros_like(single)
    for _ in range(2):  # buffers and communicators are reused across frames
        img[:] = 0
        ms.render_into(yrt.render_params(0.1, 100, 2), img.ctypes.data)
        np.testing.assert_array_equal(img.view(np.uint32), single.view(np.uint32))
    ms.close()


def test_multi_transport_errors(yrt, monkeypatch):
    s = host_scene(yrt, "basic")
    monkeypatch.setenv("YRT_MULTI_TRANSPORT", "rccl")
    with pytest.raises(yrt.YrtError, match="distinct devices"):
        yrt.MultiScene(s, [0, 0])
    monkeypatch.setenv("YRT_MULTI_TRANSPORT", "bogus")
    with pytest.raises(yrt.YrtError, match="invalid argument"):
        yrt.MultiScene(s, [0])
    monkeypatch.delenv("YRT_MULTI_TRANSPORT")
    with pytest.raises(yrt.YrtError, match="invalid argument"):
        yrt.MultiScene(s, [0, 99])
    ms = yrt.MultiScene(s, [0, 0])
    p = yrt.render_params(0.1, 32, 1, band=(4, 2, 1))  # whole frames only
    out = np.zeros((32, 57, 4), np.float32)
    with pytest.raises(yrt.YrtError, match="invalid argument"):
        ms.render_into(p, out.ctypes.data)
    ms.close()


def test_multi_render_into_device_memory(yrt):
    import torch

    s = host_scene(yrt, "refl")
    single = yrt.raytrace(s.upload(0), (0.1, 0.1, 0.1), 72, 2)
    ms = yrt.MultiScene(s, [0, 0, 0])
    out = torch.zeros(single.shape, dtype=torch.float32, device="cuda:0")
    ms.render_into(yrt.render_params(0.1, 72, 2), out.data_ptr(), device_memory=True)
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), single.view(np.uint32))
    ms.close()


def test_raytrace_devices_keyword(yrt):
    s = host_scene(yrt, "basic")
    a, sa = yrt.raytrace(s, (0.1, 0.1, 0.1), 80, 2, return_stats=True)
    b, sb = yrt.raytrace(s, (0.1, 0.1, 0.1), 80, 2, return_stats=True, devices=[0, 0])
    np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))
    assert sa["rays"] == sb["rays"]


# ---- device tonemap (render.hip tonemap_kernel, image.cpp:55-77) and save ----

def tonemap_inputs(yrt):
    """rendered pixels + a strided sweep of float bit patterns over [0, 2] + specials"""
    s = host_scene(yrt, "simple")
    img = yrt.raytrace(s.upload(0), (0.1, 0.1, 0.1), 90, 2).reshape(-1)
    sweep = np.arange(0, 0x40000000, 97, dtype=np.uint32).view(np.float32)  # 0 .. 2.0
    special = np.array([np.nan, -np.nan, np.inf, -np.inf, -0.0, 0.0, -1.0, -1e-30, 1e-45, 1.0,
                        np.nextafter(np.float32(1), np.float32(0)), 3.4e38, -3.4e38], np.float32)
    v = np.concatenate([img, sweep, np.tile(special, 4)]).astype(np.float32)
    v = v[: v.size // 4 * 4]
    return v.reshape(-1, 4)


def test_device_tonemap_matches_host_and_image_cpp(yrt):
    import torch

    px = tonemap_inputs(yrt)
    host = yrt.tonemap(px)  # host restatement of image.cpp:55-77 (glibc powf)
    d_in = torch.from_numpy(px).cuda()
    d_out = torch.zeros((px.shape[0], 4), dtype=torch.uint8, device="cuda")
    yrt.tonemap_device(d_in.data_ptr(), px.shape[0], d_out.data_ptr())
    torch.cuda.synchronize()
    dev = d_out.cpu().numpy()
    np.testing.assert_array_equal(dev, host)
    # numpy's float32 power is its own SIMD routine, not libm's powf: a handful of level
    # boundaries differ by one from image.cpp's pow (the host restatement above is the bar)
    assert np.mean(dev[:, :3] == tonemap_ref(px)) > 0.99999
    # NaN and negatives -> 0, >= 1 -> 255 (the select clamp of image.cpp)
    nan_rows = np.isnan(px[:, 0])
    assert (dev[nan_rows, 0] == 0).all()
    assert (dev[px[:, 0] >= 1, 0] == 255).all()


@pytest.mark.parametrize("ext", ["png", "hdr"])
def test_save_image_device_equals_host_save(yrt, tmp_path, ext):
    import torch

    s = host_scene(yrt, "simple")
    img = yrt.raytrace(s.upload(0), (0.1, 0.1, 0.1), 72, 2)
    h, w = img.shape[:2]
    yrt.save_hdr_or_ldr(str(tmp_path / f"host.{ext}"), img)
    d = torch.from_numpy(img).cuda()
    yrt.save_image_device(str(tmp_path / f"dev.{ext}"), d.data_ptr(), w, h)
    assert (tmp_path / f"dev.{ext}").read_bytes() == (tmp_path / f"host.{ext}").read_bytes()


@pytest.mark.parametrize("ext", ["hdr", "png"])
def test_save_image_device_equals_reference_writer(yrt, tmp_path, ext):
    """the device save path (RGBE / tonemap on the GPU, rgbe.h) against the bytes the
    reference's stbi_write_hdr wrote (.hdr) and the pixels of its stbi_write_png (.png)
    for frames with NaN, +-inf, negative, denormal and huge components
    (tests/golden/ref_hdr.npz)"""
    import torch

    from helpers import decode_png_rgba8

    gold = np.load(ROOT / "tests" / "golden" / "ref_hdr.npz")
    for name in sorted(k[3:] for k in gold.files if k.startswith("in_")):
        img = gold[f"in_{name}"]
        h, w = img.shape[:2]
        d = torch.from_numpy(np.ascontiguousarray(img)).cuda()
        out = tmp_path / f"{name}.{ext}"
        yrt.save_image_device(str(out), d.data_ptr(), w, h)
        if ext == "hdr":
            assert out.read_bytes() == gold[f"hdr_{name}"].tobytes(), name
        else:
            np.testing.assert_array_equal(decode_png_rgba8(out.read_bytes()),
                                          decode_png_rgba8(gold[f"png_{name}"].tobytes()), err_msg=name)


# ---- BASELINE configs at their full stated sizes ----

def test_full_size_c1_simple_default(yrt):
    """c1: in/simple_pointlight at the CLI defaults (-r 720 -s 1 -> 1280x720x1), the whole
    frame against the oracle, and PSNR vs check/simple.png equal to the oracle's own
    (the reference scores ~27 dB there; that gap is a property of the reference)"""
    s = host_scene(yrt, "simple")
    img, st = yrt.raytrace(s.upload(0), (0.1, 0.1, 0.1), 720, 1, return_stats=True)
    assert img.shape == (720, 1280, 4)
    ref, nrays, trunc = Oracle("simple").render(720, 1)
    assert st["rays"] == nrays and trunc == 0
    assert close_mask(img, ref).all()
    assert np.mean(img.view(np.uint32) == ref.view(np.uint32)) > 0.99
    check = np.load(GOLDEN / "ref_images.npz")["check_simple"]
    p_gpu, p_oracle = psnr_u8(tonemap_ref(img), check), psnr_u8(tonemap_ref(ref), check)
    print(f"c1 PSNR vs check/simple.png: GPU {p_gpu:.3f} dB, oracle {p_oracle:.3f} dB")
    assert abs(p_gpu - p_oracle) < 0.01 and p_gpu > 25.0


def test_full_size_c2_basic(yrt):
    """c2: in/basic_pointlight 1280x720 at 1 sample per pixel (BASELINE.json configs[1]):
    the whole frame against the oracle, the ray count equal to the oracle's, and PSNR vs
    check/basic.png equal to the oracle's own"""
    s = host_scene(yrt, "basic")
    img, st = yrt.raytrace(s.upload(0), (0.1, 0.1, 0.1), 720, 1, return_stats=True)
    assert img.shape == (720, 1280, 4)
    assert st["camera_samples"] == 1280 * 720
    ref, nrays, trunc = Oracle("basic").render(720, 1)
    assert st["rays"] == nrays and trunc == 0
    assert close_mask(img, ref).all()
    assert np.mean(img.view(np.uint32) == ref.view(np.uint32)) > 0.99
    check = np.load(GOLDEN / "ref_images.npz")["check_basic"]
    p_gpu, p_oracle = psnr_u8(tonemap_ref(img), check), psnr_u8(tonemap_ref(ref), check)
    print(f"c2 PSNR vs check/basic.png: GPU {p_gpu:.3f} dB, oracle {p_oracle:.3f} dB")
    assert abs(p_gpu - p_oracle) < 0.01


def test_full_size_c3_refl(yrt):
    """c3: refl 1920x1080 at 4x4 spp, mirror depth 8 (parity-neutral: max depth 2): the
    whole frame against the oracle (OpenMP over rows) and the oracle's ray count"""
    s = host_scene(yrt, "refl")
    img, st = yrt.raytrace(s.upload(0), (0.1, 0.1, 0.1), 1080, 4, max_depth=8, return_stats=True)
    assert img.shape == (1080, 1920, 4)
    assert st["camera_samples"] == 1920 * 1080 * 16 and st["depth_truncated"] == 0
    assert np.isfinite(img).all() and (img[..., 3] == 1).all()
    ref, nrays, trunc = Oracle("refl").render(1080, 4, max_depth=8)
    assert trunc == 0 and st["rays"] == nrays
    assert close_mask(img, ref).all()
    assert np.mean(img.view(np.uint32) == ref.view(np.uint32)) > 0.99


def test_full_size_c5_properties(yrt):
    """c5: instance10000 at 4096x4096 (--width 4096; the camera's aspect is 16:9, so the
    literal square frame needs the explicit width, raytrace.cpp:215-216), 16x16 spp on one
    GPU: 4.29 G camera samples in chunks; every sample traces 1 primary ray and every hit
    3 shadow rays (a handful of corner samples miss the floor at this sampling), nothing
    truncated, 128 evenly spaced whole rows and every non-finite pixel equal the oracle"""
    s = host_scene(yrt, "instance10000")
    img, st = yrt.raytrace(s.upload(0), (0.1, 0.1, 0.1), 4096, 16, width=4096, return_stats=True)
    assert img.shape == (4096, 4096, 4)
    assert st["camera_samples"] == 4096 * 4096 * 256
    assert st["rays"] == st["camera_samples"] + st["shadow_rays"]
    assert st["shadow_rays"] % 3 == 0 and st["shadow_rays"] // 3 >= 0.9999 * st["camera_samples"]
    assert st["depth_truncated"] == 0 and st["stack_overflow"] == 0
    assert (img[..., 3] == 1).all()
    o = Oracle("instance10000")
    # non-finite pixels (a sample whose shading divides by a zero distance or normalises a
    # zero vector sums to NaN/inf in the reference too): EVERY one must be the oracle's
    bad = np.argwhere(~np.isfinite(img[..., :3]).all(-1))
    print(f"c5: {len(bad)} non-finite pixels of {4096 * 4096}")
    assert len(bad) < 4096
    for row in np.unique(bad[:, 0]):
        cols = bad[bad[:, 0] == row, 1]
        x0, x1 = int(cols.min()), int(cols.max()) + 1
        ref, _, _ = o.render(4096, 16, rows=[row], x0=x0, ncols=x1 - x0, width=4096)
        assert_same_floats(img[row:row + 1, cols], ref[:, cols - x0])
    # 128 evenly spaced WHOLE rows against the oracle (OpenMP over rows, ~18 s on the box)
    rows = np.linspace(0, 4095, 128).astype(np.int32)
    ref, _, trunc = o.render(4096, 16, rows=rows, width=4096)
    assert trunc == 0
    seg = img[rows]
    differ = int(np.sum(seg.view(np.uint32) != ref.view(np.uint32)))
    print(f"c5 128 rows vs oracle: {differ} of {seg.size} channels not bit-exact")
    assert close_mask(seg, ref).all()
    assert np.mean(seg.view(np.uint32) == ref.view(np.uint32)) > 0.99


# ---- instance scaling (instance10000's `i`-line pattern, 1 K / 100 K) ----

@pytest.mark.parametrize("name,ninst,depth", [("instance1k", 1004, 10), ("instance100k", 100004, 18)])
def test_instance_scaling_c4_frame(yrt, name, ninst, depth):
    """the scaling scenes at c4's settings (1920x1080, 8x8 spp): every camera sample traces
    one ray and every hit one shadow ray per light, nothing is truncated or overflows, the
    instance BVH depth plus the deepest shape BVH (15) stays within the walks' stack
    (traversal_stack_cap = 40), and 64 evenly spaced whole rows equal the oracle"""
    s = host_scene(yrt, name)
    info = s.info()
    assert info["instances"] == ninst and info["bvh_depth"] == depth and info["shape_bvh_depth"] == 15
    assert depth + 15 <= 40
    img, st = yrt.raytrace(s.upload(0), (0.1, 0.1, 0.1), 1080, 8, return_stats=True)
    assert img.shape == (1080, 1920, 4)
    assert st["camera_samples"] == 1920 * 1080 * 64
    assert st["rays"] == st["camera_samples"] + st["shadow_rays"] and st["shadow_rays"] % 3 == 0
    assert st["depth_truncated"] == 0 and st["stack_overflow"] == 0
    rows = np.linspace(0, 1079, 64).astype(np.int32)
    ref, _, trunc = Oracle(name).render(1080, 8, rows=rows)
    assert trunc == 0
    differ = int(np.sum(img[rows].view(np.uint32) != ref.view(np.uint32)))
    print(f"{name} 64 rows vs oracle: {differ} of {img[rows].size} channels not bit-exact")
    assert close_mask(img[rows], ref).all()
    assert np.mean(img[rows].view(np.uint32) == ref.view(np.uint32)) > 0.99


def test_upload_rejects_bvh_deeper_than_the_stack(yrt):
    """instances on an exponential sequence make the reference's midpoint split peel one
    instance per level: an instance BVH 49 deep, past traversal_stack_cap (40), which the
    upload refuses (YRT_ERR_UNSUPPORTED) instead of letting a walk overflow its stack"""
    s = yrt.Scene.create()
    s.add_camera(np.r_[1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 1, 5], fovy=0.5, aspect=1.5, focus=5)
    m = s.add_material(kd=(0.5, 0.5, 0.5))
    tri = s.add_shape([[-1, 0, -1], [1, 0, -1], [0, 0, 1]], norm=[[0, 1, 0]] * 3, texcoord=[[0, 0]] * 3,
                      triangles=[[0, 1, 2]])
    for k in range(80):
        s.add_instance(np.r_[1, 0, 0, 0, 1, 0, 0, 0, 1, 2.0 ** k, 0, 0], tri, m)
    yrt.build_bvh(s)
    assert s.info()["bvh_depth"] > 40
    with pytest.raises(yrt.YrtError, match="too deep"):
        s.upload(0)


# ---- mirror recursion deeper than 16 levels (the reference's recursion has no cap) ----

def test_mirror_corridor_deep_recursion(yrt):
    """tests/golden/scenes/mirrors.yrtscene: camera rays bounce between two mirror walls
    up to 37-40 times. With max_depth 64 the wavefront pipeline keeps every level's records
    in HBM and the whole 640x360x4 frame equals the oracle's unbounded recursion (ray
    count included, nothing truncated); with max_depth 30 the cut paths count as misses,
    exactly as the oracle's depth cap counts them"""
    s = host_scene(yrt, "mirrors")
    ds = s.upload(0)
    o = Oracle("mirrors")
    ref, nrays, trunc = o.render(360, 2)
    assert trunc == 0
    img, st = yrt.raytrace(ds, (0.1, 0.1, 0.1), 360, 2, max_depth=64, return_stats=True)
    assert st["depth_truncated"] == 0 and st["rays"] == nrays
    assert nrays / st["camera_samples"] > 60  # ~26 levels of 1 + 2 shadow rays on average
    assert close_mask(img, ref).all()
    assert np.mean(img.view(np.uint32) == ref.view(np.uint32)) > 0.99
    ref30, n30, t30 = o.render(360, 2, max_depth=30)
    img30, st30 = yrt.raytrace(ds, (0.1, 0.1, 0.1), 360, 2, max_depth=30, return_stats=True)
    assert t30 > 0 and st30["depth_truncated"] == t30 and st30["rays"] == n30
    assert close_mask(img30, ref30).all()
