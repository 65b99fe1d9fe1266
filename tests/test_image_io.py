"""save_hdr_or_ldr (src/image.cpp:81-88) against the REFERENCE's own writer.

tests/golden/ref_hdr.npz (tests/golden/make_hdr.py) holds frames with NaN, +-inf,
negative, denormal, tiny and huge components, long runs and run-free stretches, widths
on both sides of the RLE threshold, and a real render, with the bytes the reference
wrote for each: stbi_write_hdr's .hdr file and stbi_write_png's .png after its tonemap.
The .hdr files must be byte-identical (header lines, run-length scanlines, the x86
build's truncations, rgbe.h). PNG bytes depend on each zlib's choices, so the .png
check is on the decoded pixels.
"""
import ctypes
import os

import numpy as np
import pytest

from helpers import ROOT, decode_png_rgba8, have_reference

GOLD = np.load(ROOT / "tests" / "golden" / "ref_hdr.npz")
FRAMES = sorted(k[3:] for k in GOLD.files if k.startswith("in_"))


@pytest.fixture(scope="module")
def yrt():
    import yocto_raytracing_amd as y

    return y


def test_fixture_covers_the_corners():
    assert {"special_w40", "runs_w300", "flat_w1", "flat_w5", "flat_w7", "flat_w8", "render_basic"} <= set(FRAMES)
    allv = np.concatenate([GOLD[f"in_{f}"][..., :3].ravel() for f in FRAMES])
    assert np.isnan(allv).any() and np.isposinf(allv).any() and np.isneginf(allv).any()
    assert (allv < 0).any() and ((allv != 0) & (np.abs(allv) < 1.2e-38)).any() and (allv > 2.0 ** 31).any()


@pytest.mark.parametrize("name", FRAMES)
def test_hdr_bytes_equal_reference(yrt, tmp_path, name):
    img = GOLD[f"in_{name}"]
    out = tmp_path / f"{name}.hdr"
    yrt.save_hdr_or_ldr(str(out), img)
    got = np.frombuffer(out.read_bytes(), np.uint8)
    want = GOLD[f"hdr_{name}"]
    assert got.size == want.size and (got == want).all(), f"first difference at byte {np.argmax(got[:want.size] != want[:got.size])}"


@pytest.mark.parametrize("name", FRAMES)
def test_png_pixels_equal_reference(yrt, tmp_path, name):
    img = GOLD[f"in_{name}"]
    out = tmp_path / f"{name}.png"
    yrt.save_hdr_or_ldr(str(out), img)
    np.testing.assert_array_equal(decode_png_rgba8(out.read_bytes()), decode_png_rgba8(GOLD[f"png_{name}"].tobytes()))


@pytest.mark.reference
@pytest.mark.skipif(not have_reference(), reason="needs /root/reference and oracle/_ref")
def test_hdr_bytes_equal_live_reference(yrt, tmp_path):
    """random frames through the reference build itself (this container only)"""
    lib = ctypes.CDLL(str(ROOT / "oracle" / "_ref" / "libyrtref.so"))
    lib.ref_save_image.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    rng = np.random.default_rng(7)
    special = np.array([np.nan, np.inf, -np.inf, -2.5, 0.0, 1e-40, 1e-32, 3e38, 2.0 ** 33], np.float32)
    for w, h in [(3, 2), (8, 3), (9, 2), (129, 3), (400, 2)]:
        img = rng.uniform(-0.5, 8.0, (h, w, 4)).astype(np.float32)
        m = rng.random(img.shape) < 0.2
        img[m] = rng.choice(special, m.sum())
        img[0, : w // 2, :3] = 1.5
        ref = tmp_path / f"ref_{w}.hdr"
        assert lib.ref_save_image(str(ref).encode(), img.ctypes.data, w, h) == 0
        out = tmp_path / f"got_{w}.hdr"
        yrt.save_hdr_or_ldr(str(out), img)
        assert out.read_bytes() == ref.read_bytes(), (w, h)
