"""Golden fixtures of the reference's image writer (save_hdr_or_ldr, src/image.cpp:81-88).

Run in the container that has /root/reference (never on the GPU box):

    make -C oracle ref && python tests/golden/make_hdr.py

It writes tests/golden/ref_hdr.npz: seeded RGBA float frames holding the values that
exercise the writer's corners -- NaN in each channel, +-inf, negatives next to positive
maxima, denormals, values around the 1e-32 cut-off, huge values, long constant runs and
long run-free stretches (RLE run and dump lengths past 127/128), widths on both sides
of the RLE threshold (8) -- and for each frame the bytes the REFERENCE wrote through
stbi_write_hdr (.hdr) and stbi_write_png (.png, after its tonemap). Data only.
"""
from __future__ import annotations

import ctypes as C
import os
import tempfile
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent

SPECIAL = np.array([np.nan, np.inf, -np.inf, -1.0, -0.0, 0.0, 1e-45, 1e-40, 1e-33, 1e-32, 1.1e-32, 0.5, 1.0,
                    255.0, 3.4e38, 2.0 ** 31, 7.25, 1e-20], np.float32)


def frames(rng):
    out = {}
    # RLE path, special values in every channel position, mixed with ordinary ones
    w, h = 40, 8
    f = rng.uniform(0, 2, (h, w, 4)).astype(np.float32)
    mask = rng.random((h, w, 4)) < 0.3
    f[mask] = rng.choice(SPECIAL, mask.sum())
    f[0, :, :3] = 0.25  # a constant row: runs
    f[1, :20, :3] = rng.choice(SPECIAL, (20, 3))
    out["special_w40"] = f
    # run and dump lengths past 127 / 128
    w, h = 300, 4
    f = np.zeros((h, w, 4), np.float32)
    f[0] = 0.7                                                  # one run of 300
    f[1] = rng.uniform(0.01, 50, (w, 4))                        # no runs
    f[2, :150] = 3.0
    f[2, 150:] = rng.uniform(0, 1, (150, 4))
    f[3] = np.repeat(rng.uniform(0, 4, (w // 3, 4)), 3, axis=0)  # runs of exactly 3
    out["runs_w300"] = f
    # the flat (no RLE) path: width < 8, and the threshold itself
    for w in (1, 5, 7, 8):
        f = rng.uniform(-1, 3, (3, w, 4)).astype(np.float32)
        f[1, :, :3] = rng.choice(SPECIAL, (w, 3))
        out[f"flat_w{w}"] = f
    # a real frame: the reference's own render of basic (64 px, 1 spp)
    ref = np.load(HERE / "ref_render_basic.npz")
    key = [k for k in ref.files if k.startswith("img")][0]
    out["render_basic"] = ref[key].astype(np.float32)
    return out


def main():
    lib = C.CDLL(str(ROOT / "oracle" / "_ref" / "libyrtref.so"))
    lib.ref_save_image.argtypes = [C.c_char_p, C.c_void_p, C.c_int, C.c_int]
    rng = np.random.default_rng(20261017)
    data = {}
    with tempfile.TemporaryDirectory() as td:
        for name, f in frames(rng).items():
            f = np.ascontiguousarray(f, np.float32)
            h, w = f.shape[:2]
            data[f"in_{name}"] = f
            for ext in ("hdr", "png"):
                p = os.path.join(td, f"{name}.{ext}")
                assert lib.ref_save_image(p.encode(), f.ctypes.data, w, h) == 0
                data[f"{ext}_{name}"] = np.frombuffer(Path(p).read_bytes(), np.uint8)
    np.savez_compressed(HERE / "ref_hdr.npz", **data)
    print({k: v.shape for k, v in data.items()})


if __name__ == "__main__":
    main()
