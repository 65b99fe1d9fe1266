"""Shared test helpers: the oracle binding (test infrastructure), fixture paths and
image metrics. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
touch oracle/."""
from __future__ import annotations

import ctypes as C
import json
import subprocess
from functools import lru_cache
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
GOLDEN = ROOT / "tests" / "golden"
SCENES = GOLDEN / "scenes"
# the reference's four `in/*` scenes + "lines", a synthetic lines/points/texture scene,
# and "mirrors", a mirror corridor whose paths recurse 20-40 levels deep (both built by
# tests/golden/make_synthetic.py) + the instance-scaling scenes (instance10000's `i`-line
# pattern with 1 000 / 100 000 instances, tests/golden/make_scaling.py), all loaded,
# rendered and traced by the reference itself
SCENE_NAMES = ("basic", "simple", "refl", "instance10000", "lines", "instance1k", "instance100k", "mirrors")
# the max_depth the GPU renders the mirror corridor with (its deepest path: 37-40 levels;
# the reference's recursion has no cap)
MIRROR_DEPTH = 64
# edge-case scenes (tests/golden/make_edges.py): no lights, every ray a miss, no
# instances, a point light alone -- scenes/edge_<name>.yrtscene
EDGE_SCENES = ("unlit", "sky", "empty", "lightsonly")
OBJ_SCENES = ("basic", "simple", "refl", "instance10000")
REFERENCE = Path("/root/reference")
REF_OBJ = {
    "basic": REFERENCE / "in/basic_pointlight/basic_pointlight.obj",
    "simple": REFERENCE / "in/simple_pointlight/simple_pointlight.obj",
    "refl": REFERENCE / "in/refl_pointlight/refl_pointlight.obj",
    "instance10000": REFERENCE / "in/instance10000_pointlight/instance10000_pointlight.obj",
}

# Per-channel float tolerance of the GPU path against the reference / oracle
# (DESIGN.md §6): the only libm call left on the device is pow() in the specular
# term; everything else is bit-exact by construction.
ATOL = 1e-6
RTOL = 2e-6


def scene_path(name: str) -> Path:
    return SCENES / f"{name}.yrtscene"


def digests() -> dict:
    return json.loads((GOLDEN / "ref_digests.json").read_text())


@lru_cache(maxsize=None)
def oracle_lib():
    so = ROOT / "oracle" / "liboracle.so"
    if not so.exists():
        subprocess.run(["make", "-C", str(ROOT / "oracle"), "liboracle.so"], check=True,
                       capture_output=True)
    lib = C.CDLL(str(so))
    lib.oracle_load.restype = C.c_void_p
    lib.oracle_load.argtypes = [C.c_char_p]
    lib.oracle_free.argtypes = [C.c_void_p]
    lib.oracle_write_bvh.argtypes = [C.c_void_p, C.c_char_p]
    lib.oracle_image_size.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
    lib.oracle_render_rows.restype = C.c_longlong
    lib.oracle_render_rows.argtypes = [C.c_void_p, C.c_float, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                       C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
    lib.oracle_trace.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int] + [C.c_void_p] * 5
    lib.oracle_camera_ray.argtypes = [C.c_void_p] + [C.c_int] * 8 + [C.c_void_p]
    return lib


class Oracle:
    """CPU restatement of the reference (oracle/oracle.c) on a .yrtscene file."""

    def __init__(self, name_or_path):
        p = scene_path(name_or_path) if name_or_path in SCENE_NAMES else Path(name_or_path)
        self.lib = oracle_lib()
        self.h = self.lib.oracle_load(str(p).encode())
        if not self.h:
            raise RuntimeError(f"oracle could not load {p}")

    def __del__(self):
        try:
            self.lib.oracle_free(self.h)
        except Exception:
            pass

    def image_size(self, resolution, camera=0):
        w, h = C.c_int(), C.c_int()
        self.lib.oracle_image_size(self.h, camera, resolution, C.byref(w), C.byref(h))
        return w.value, h.value

    def render(self, resolution, samples, amb=0.1, rows=None, x0=0, ncols=None, width=0, max_depth=0,
               camera=0):
        W, H = self.image_size(resolution, camera)
        if width:
            W = width
        rows = np.arange(H, dtype=np.int32) if rows is None else np.ascontiguousarray(rows, np.int32)
        ncols = W - x0 if ncols is None else ncols
        out = np.zeros((len(rows), ncols, 4), np.float32)
        trunc = C.c_longlong(0)
        n = self.lib.oracle_render_rows(self.h, amb, camera, resolution, width, samples, max_depth,
                                        rows.ctypes.data, len(rows), x0, ncols, out.ctypes.data,
                                        C.byref(trunc))
        if n < 0:
            raise RuntimeError("oracle render failed")
        return out, int(n), int(trunc.value)

    def trace(self, rays, any_hit=False):
        rays = np.ascontiguousarray(rays, np.float32)
        n = len(rays)
        hit = np.zeros(n, np.uint8)
        inst = np.zeros(n, np.int32)
        ei = np.zeros(n, np.int32)
        ew = np.zeros((n, 4), np.float32)
        dist = np.zeros(n, np.float32)
        self.lib.oracle_trace(self.h, rays.ctypes.data, n, 1 if any_hit else 0, hit.ctypes.data,
                              inst.ctypes.data, ei.ctypes.data, ew.ctypes.data, dist.ctypes.data)
        return {"hit": hit.astype(bool), "inst": inst, "ei": ei, "ew": ew, "dist": dist}


def tonemap_ref(img: np.ndarray) -> np.ndarray:
    """tonemap (image.cpp:55-77) in numpy: pow(x, 1/2.2), select clamp, truncate *255."""
    x = img[..., :3].astype(np.float32)
    with np.errstate(invalid="ignore"):
        g = np.power(x, np.float32(1 / 2.2)).astype(np.float32)
    g[np.isneginf(x)] = np.inf  # C pow(-inf, y > 0, y not an odd integer) = +inf; numpy gives NaN
    g = np.where(g > 0, g, np.float32(0))  # max(x, 0): NaN -> 0
    g = np.where(g < 1, g, np.float32(1))
    return (g * np.float32(255)).astype(np.uint8)


def psnr_u8(a: np.ndarray, b: np.ndarray) -> float:
    d = a.astype(np.float64) - b.astype(np.float64)
    mse = float(np.mean(d * d))
    return float("inf") if mse == 0 else 10 * np.log10(255.0 ** 2 / mse)


def close_mask(a: np.ndarray, b: np.ndarray, atol=ATOL, rtol=RTOL) -> np.ndarray:
    return np.abs(a.astype(np.float64) - b.astype(np.float64)) <= atol + rtol * np.abs(b.astype(np.float64))


def have_reference() -> bool:
    return (REFERENCE / "src" / "raytrace.cpp").exists() and (ROOT / "oracle/_ref/libyrtref.so").exists()


def read_png_rgba8(path) -> np.ndarray:
    """Decode an RGBA8 PNG written by yrt_save_image (filter type 0 on every row)."""
    import struct
    import zlib

    data = Path(path).read_bytes()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, w, h = 8, b"", 0, 0
    while pos < len(data):
        n = struct.unpack(">I", data[pos:pos + 4])[0]
        typ = data[pos + 4:pos + 8]
        if typ == b"IHDR":
            w, h = struct.unpack(">II", data[pos + 8:pos + 16])
        elif typ == b"IDAT":
            idat += data[pos + 8:pos + 8 + n]
        pos += 12 + n
    raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(h, w * 4 + 1)
    assert (raw[:, 0] == 0).all(), "unexpected PNG row filter"
    return raw[:, 1:].reshape(h, w, 4)


def decode_png_rgba8(data: bytes) -> np.ndarray:
    """Decode an 8-bit RGBA, non-interlaced PNG with any of the five row filters
    (stbi_write_png picks one per row, yrt_save_image writes filter 0)."""
    import struct
    import zlib

    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, w, h = 8, b"", 0, 0
    while pos < len(data):
        n = struct.unpack(">I", data[pos:pos + 4])[0]
        typ = data[pos + 4:pos + 8]
        if typ == b"IHDR":
            w, h, depth, ctype, _, _, interlace = struct.unpack(">IIBBBBB", data[pos + 8:pos + 21])
            assert (depth, ctype, interlace) == (8, 6, 0), "only RGBA8, non-interlaced"
        elif typ == b"IDAT":
            idat += data[pos + 8:pos + 8 + n]
        pos += 12 + n
    raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(h, w * 4 + 1)
    out = np.zeros((h, w * 4), np.int32)
    for y in range(h):
        f, cur = raw[y, 0], raw[y, 1:].astype(np.int32)
        up = out[y - 1] if y else np.zeros(w * 4, np.int32)
        if f in (0, 2):
            out[y] = (cur + (up if f == 2 else 0)) & 255
            continue
        row = np.zeros(w * 4, np.int32)
        for x in range(w * 4):
            a = row[x - 4] if x >= 4 else 0
            b = up[x]
            c = up[x - 4] if x >= 4 else 0
            if f == 1:
                pred = a
            elif f == 3:
                pred = (a + b) // 2
            else:  # Paeth
                p = a + b - c
                pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
                pred = a if pa <= pb and pa <= pc else (b if pb <= pc else c)
            row[x] = (cur[x] + pred) & 255
        out[y] = row
    return out.astype(np.uint8).reshape(h, w, 4)


def assert_same_floats(got, want):
    """bit-for-bit equality, except that a NaN only has to be a NaN: its sign and
    payload follow the GPU's NaN propagation, not x86's"""
    got = np.asarray(got, np.float32)
    want = np.asarray(want, np.float32)
    assert got.shape == want.shape
    gn, wn = np.isnan(got), np.isnan(want)
    np.testing.assert_array_equal(gn, wn)
    np.testing.assert_array_equal(got[~gn].view(np.uint32), want[~wn].view(np.uint32))
