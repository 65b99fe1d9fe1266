"""Degenerate-ray fixtures from the REFERENCE ITSELF (run where /root/reference is):

    make -C oracle ref && python tests/golden/make_degenerate.py

For each scene, rays that exercise the slab test's and the triangle test's edge cases
-- axis-parallel directions (1/d = +-inf, 0*inf = NaN slabs), rays starting exactly on
box planes, zero / NaN / inf components, empty and inverted [tmin, tmax] ranges,
tmax = 0, huge and tiny magnitudes -- traced with intersect_first / intersect_any
(scene.cpp:483-494) through oracle/_ref. Writes ref_rays_degenerate_<scene>.npz (data
only)."""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))

SCENES = ("basic", "refl", "instance10000", "lines")


def degenerate_rays(rng, scene_box_lo, scene_box_hi, n_random=1500):
    inf, nan, fmax = np.float32(np.inf), np.float32(np.nan), np.float32(3.4028234663852886e38)
    lo, hi = scene_box_lo.astype(np.float32), scene_box_hi.astype(np.float32)
    center = ((lo + hi) / 2).astype(np.float32)
    rays = []

    def add(o, d, tmin=1e-4, tmax=fmax):
        rays.append(np.array([*o, *d, tmin, tmax], np.float32))

    # axis-parallel rays through the scene from each side, and from inside
    for axis in range(3):
        for sgn in (1, -1):
            d = np.zeros(3, np.float32)
            d[axis] = sgn
            for _ in range(60):
                o = rng.uniform(lo, hi).astype(np.float32)
                o[axis] = lo[axis] - 1 if sgn > 0 else hi[axis] + 1
                add(o, d)
                o2 = rng.uniform(lo, hi).astype(np.float32)
                add(o2, d)
            # negative zero components
            d2 = d.copy()
            d2[(axis + 1) % 3] = -0.0
            add(center, d2)
    # rays starting exactly on the scene box planes, axis-parallel and oblique
    for axis in range(3):
        for v in (lo[axis], hi[axis]):
            for _ in range(30):
                o = rng.uniform(lo, hi).astype(np.float32)
                o[axis] = v
                d = rng.normal(size=3).astype(np.float32)
                d[(axis + 1 + rng.integers(2)) % 3] = 0
                n = np.linalg.norm(d)
                add(o, d / n if n else np.array([0, 0, 1], np.float32))
    # zero, NaN and infinite directions / origins, odd ranges
    specials = [
        (center, [0, 0, 0]), (center, [nan, 0, 1]), (center, [0, -1, nan]), (center, [inf, 0, 0]),
        (center, [0, -inf, 0]), ([nan, 0, 0], [0, -1, 0]), ([inf, 1, 1], [-1, 0, 0]),
        (center + [0, 50, 0], [0, -1, 0]), (center + [0, 50, 0], [1e-30, -1, 1e-30]),
        (center + [0, 50, 0], [1e30, -1e30, 0]),
    ]
    for o, d in specials:
        add(np.asarray(o, np.float32), np.asarray(d, np.float32))
    for tmin, tmax in [(0, 0), (1, 0.5), (5, 5), (-1, 1e-3), (nan, 10), (0, nan), (0, inf), (-inf, inf), (1e-4, 1e-30)]:
        add(center + [0, 40, 0], np.array([0, -1, 0], np.float32), tmin, tmax)
        add(center + [3, 40, -2], np.array([0.1, -1, 0.05], np.float32) / np.float32(1.0062), tmin, tmax)
    # random rays toward the scene, a third with finite tmax
    for _ in range(n_random):
        o = (center + rng.normal(size=3) * (hi - lo)).astype(np.float32)
        tgt = rng.uniform(lo, hi).astype(np.float32)
        d = tgt - o
        d = (d / np.linalg.norm(d)).astype(np.float32)
        tmax = fmax if rng.random() < 0.66 else np.float32(rng.uniform(0.1, 200))
        add(o, d, 1e-4, tmax)
    return np.stack(rays)


def main():
    import gzip
    import struct

    from make_golden import load_ref, trace

    lib = load_ref()
    lib.ref_read_scene.restype = lib.ref_load_scene.restype
    lib.ref_read_scene.argtypes = lib.ref_load_scene.argtypes
    rng = np.random.default_rng(5150)
    for name in SCENES:
        path = HERE / "scenes" / f"{name}.yrtscene"
        scn = lib.ref_read_scene(str(path).encode())
        assert scn
        # scene bounds from the reference's own top-level BVH root (dump via ref_write_bvh)
        tmp = Path(f"/tmp/{name}_deg.yrtbvh")
        lib.ref_write_bvh(scn, str(tmp).encode())
        raw = gzip.open(tmp).read()
        # .yrtbvh: magic, u32 shapes, per shape {u32 n, n nodes of 32 B, u32 m, m ints},
        # then the instance level the same way: its root node is the scene's box
        pos = 8
        nshapes = struct.unpack_from("I", raw, pos)[0]
        pos += 4
        for _ in range(nshapes + 1):
            n = struct.unpack_from("I", raw, pos)[0]
            top_nodes = pos + 4
            pos += 4 + 32 * n
            m = struct.unpack_from("I", raw, pos)[0]
            pos += 4 + 4 * m
        root = raw[top_nodes:top_nodes + 24]
        lo = np.array(struct.unpack("3f", root[:12]), np.float32)
        hi = np.array(struct.unpack("3f", root[12:24]), np.float32)
        rays = degenerate_rays(rng, lo, hi)
        hit, inst, ei, ew, dist = trace(lib, scn, rays, False)
        ahit = trace(lib, scn, rays, True)[0]
        np.savez_compressed(HERE / f"ref_rays_degenerate_{name}.npz", rays=rays, hit=hit, inst=inst, ei=ei, ew=ew,
                            dist=dist, any_hit=ahit)
        print(name, len(rays), "hits", int(hit.sum()), "any", int(ahit.sum()), "box", lo, hi)


if __name__ == "__main__":
    main()
