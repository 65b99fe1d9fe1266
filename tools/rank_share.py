"""Per-rank efficiency of the N-rank band split on one GPU: render rank r's 8-row bands of
the c4 frame (what `bench.py --gpus N` gives rank r) and compare each phase's GPU time with
1/N of the full frame's.

    python tools/rank_share.py [--ranks 2 4 8] [--steps 10]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--scene", default="instance10000")
    a = ap.parse_args()
    import torch

    import yocto_raytracing_amd as yrt
    from yocto_raytracing_amd.shard import BandLayout, render_params_band

    s = yrt.load_scene(str(ROOT / "tests" / "golden" / "scenes" / f"{a.scene}.yrtscene"))
    yrt.build_bvh(s)
    ds = s.upload(0)
    stream = torch.cuda.current_stream()

    def run(world, rank):
        p = yrt.render_params(0.1, 1080, 8)
        W, H = ds.image_size(p)
        L = BandLayout(H, world, 8)
        band, rows = render_params_band(L, rank)
        p.band, p.band_stride, p.band_offset = band
        p.tile_h = rows
        out = torch.empty((rows, W, 4), dtype=torch.float32, device="cuda")
        for i in range(3):
            ds.render_into(p, out.data_ptr(), stream=stream.cuda_stream)
        for i in range(a.steps):
            p.timing = 1 if i == 0 else 2
            ds.render_into(p, out.data_ptr(), stream=stream.cuda_stream)
        torch.cuda.synchronize()
        return {k: v[0] / a.steps for k, v in ds.last_timings().items()}

    full = run(1, 0)
    res = {"full": full}
    for n in a.ranks:
        t = run(n, 0)
        res[f"rank0_of_{n}"] = {k: {"ms": v, "vs_1_over_n": v / (full[k] / n)} for k, v in t.items()}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
