"""Instance-scaling scenes (SURVEY.md §8d "optional synthetic scaling scenes"), pinned by
the REFERENCE ITSELF:

    make -C oracle ref && python tests/golden/make_scaling.py

in/instance10000_pointlight places 10 000 `i` lines on a jittered 100 x 100 grid over
the floor (x, z in [-100, 100], y = 1, identity rotation, one of the ten shapes shp000
.. shp009 each). This script writes the same OBJ with that grid replaced by N instances
in the same pattern (a jittered ceil(sqrt N)^2 grid, the first N cells, seeded shape
choice, coordinates printed to 6 significant digits like the original), N = 1 000 and
100 000, and then:

1. has the reference load it with its own loader (oracle/_ref ref_load_scene:
   load_scene, scene.cpp:113 -> yocto_obj `i` lines -> yocto_scn instances) and writes
   scenes/instance{1k,100k}.yrtscene plus the scene/BVH digests (ref_digests.json);
2. checks that the product's OBJ loader reads the same OBJ into the same bytes;
3. renders (raytrace.cpp:213) and traces (scene.cpp:483-494) with the reference into
   ref_render_<name>.npz / ref_rays_<name>.npz, exactly like make_golden.py.

Data only; the generated OBJ stays in /tmp.
"""
from __future__ import annotations

import ctypes as C
import gzip
import hashlib
import json
import shutil
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(HERE))

SRC = Path("/root/reference/in/instance10000_pointlight")
SCALES = {"instance1k": 1000, "instance100k": 100000}
RENDERS = {"instance1k": [(64, 1), (36, 3)], "instance100k": [(64, 1), (36, 2)]}


def grid_lines(n: int, rng) -> list:
    side = int(np.ceil(np.sqrt(n)))
    step = 200.0 / side
    out = []
    for k in range(n):
        gx, gz = k % side, k // side
        x = -100.0 + (gx + 0.5) * step + rng.uniform(-0.2, 0.2) * step
        z = -100.0 + (gz + 0.5) * step + rng.uniform(-0.2, 0.2) * step
        out.append(f"i ist{k:06d}  shp{int(rng.integers(0, 10)):03d}  1 0 0 0 1 0 0 0 1 {x:.6g} 1 {z:.6g}\n")
    return out


def write_obj(name: str, n: int, rng) -> Path:
    dst = Path("/tmp") / f"{name}_pointlight"
    dst.mkdir(exist_ok=True)
    shutil.copy(SRC / "instance10000_pointlight.mtl", dst / f"{name}_pointlight.mtl")
    lines = (SRC / "instance10000_pointlight.obj").read_text().splitlines(keepends=True)
    out, placed = [], False
    for line in lines:
        if line.startswith("mtllib "):
            out.append(f"mtllib {name}_pointlight.mtl\n")
        elif line.startswith("i ist"):
            if not placed:
                out += grid_lines(n, rng)
                placed = True
        else:
            out.append(line)
    p = dst / f"{name}_pointlight.obj"
    p.write_text("".join(out))
    return p


def main():
    from make_golden import load_ref, sample_rays, trace

    import yocto_raytracing_amd as yrt

    lib = load_ref()
    dig = json.loads((HERE / "ref_digests.json").read_text())
    for name, n in SCALES.items():
        rng = np.random.default_rng(8000 + n)
        obj = write_obj(name, n, rng)
        scn = lib.ref_load_scene(str(obj).encode())
        assert scn, f"reference could not load {obj}"
        spath = HERE / "scenes" / f"{name}.yrtscene"
        lib.ref_write_scene(scn, str(spath).encode())
        bpath = Path(f"/tmp/{name}_ref.yrtbvh")
        lib.ref_write_bvh(scn, str(bpath).encode())
        dig[name] = {"scene_sha256": hashlib.sha256(gzip.open(spath).read()).hexdigest(),
                     "bvh_sha256": hashlib.sha256(gzip.open(bpath).read()).hexdigest()}
        # the product's loader on the same OBJ: the same scene bytes
        mine = Path(f"/tmp/{name}_mine.yrtscene")
        yrt.load_scene(str(obj)).save(str(mine))
        assert gzip.open(mine).read() == gzip.open(spath).read(), f"{name}: product loader differs"
        out = {}
        for res, s in RENDERS[name]:
            w, h = C.c_int(), C.c_int()
            lib.ref_image_size(scn, res, C.byref(w), C.byref(h))
            img = np.zeros((h.value, w.value, 4), np.float32)
            out[f"rays_r{res}_s{s}"] = np.int64(lib.ref_render(scn, 0.1, res, s, img.ctypes.data))
            out[f"img_r{res}_s{s}"] = img
        np.savez_compressed(HERE / f"ref_render_{name}.npz", **out)
        rays = sample_rays(lib, scn, np.random.default_rng(n))
        hit, inst, ei, ew, dist = trace(lib, scn, rays, False)
        ahit = trace(lib, scn, rays, True)[0]
        np.savez_compressed(HERE / f"ref_rays_{name}.npz", rays=rays, hit=hit, inst=inst, ei=ei, ew=ew, dist=dist,
                            any_hit=ahit)
        print(name, dig[name], "hit fraction", hit.mean(), "any", ahit.mean(), spath.stat().st_size, "bytes")
    (HERE / "ref_digests.json").write_text(json.dumps(dig, indent=1) + "\n")


if __name__ == "__main__":
    main()
