"""Probe: does rendering consecutive c4 frames on two streams (two device replicas of
the scene, i.e. two workspaces) raise throughput over one stream? Frames are identical
work; the image digests of both replicas are printed.

    python tools/overlap_probe.py [--frames 12] [--share R/N]
"""
from __future__ import annotations

import argparse
import hashlib
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=12)
    ap.add_argument("--scene", default="instance10000")
    ap.add_argument("--resolution", type=int, default=1080)
    ap.add_argument("--share", default="0/1", help="R/N: rank R's 8-row bands of an N-rank split (bench.py)")
    a = ap.parse_args()
    import torch

    import yocto_raytracing_amd as yrt

    torch.cuda.set_device(0)
    scn = yrt.load_scene(str(ROOT / "tests" / "golden" / "scenes" / f"{a.scene}.yrtscene"))
    yrt.build_bvh(scn)
    reps = [yrt.DeviceScene(scn, 0), yrt.DeviceScene(scn, 0)]  # two workspaces (upload() caches one)
    from yocto_raytracing_amd.shard import BandLayout, render_params_band

    p = yrt.render_params(0.1, a.resolution, 8)
    W, H = reps[0].image_size(p)
    rank, world = (int(v) for v in a.share.split("/"))
    layout = BandLayout(H, world, 8)
    band, local_rows = render_params_band(layout, rank)
    if world > 1:
        p.band, p.band_stride, p.band_offset = band
        p.tile_h = local_rows
        H = local_rows
    outs = [torch.empty((H, W, 4), dtype=torch.float32, device="cuda") for _ in range(2)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for k in range(2):  # warm both replicas (workspace allocation)
        reps[k].render_into(p, outs[k].data_ptr(), stream=streams[k].cuda_stream)
    torch.cuda.synchronize()
    for nstreams in (1, 2, 1, 2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.frames):
            k = i % nstreams
            reps[k].render_into(p, outs[k].data_ptr(), stream=streams[k].cuda_stream)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        print(f"streams={nstreams}: {el / a.frames * 1e3:.2f} ms/frame")
    for k in range(2):
        print("replica", k, hashlib.sha1(outs[k].cpu().numpy().tobytes()).hexdigest()[:16])


if __name__ == "__main__":
    main()
